#!/usr/bin/env python3
"""Does the 2^20 host-buffer call (hsv_verify from numpy) run slower when the
process's first such call comes after bench.py's device work (torch tensors,
C4 launches on three streams, the mad peak probe) than when it comes first?
One child process per order, same box; each prints the median of 7 calls and
the per-call times.

python tools/host_api_late_probe.py
"""
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r"""
import json, sys, time
import numpy as np
sys.path.insert(0, {root!r} + "/hotstuff-digital-signature-benchmarking_amd")
import torch
from hsverify import _lib, _testing, synth, verifier
order = {order!r}
n = 1 << 20
dev = torch.device("cuda", 0)
_lib.load()
verifier.bind_device(0)
w = synth.independent_triples(n, seed=0xC4 * 1000, corrupt_frac=0.05, nthreads=16)

def host(tag):
    verifier.verify_flags(w.pk, w.sig, w.msg)
    ts = []
    for _ in range(7):
        t0 = time.perf_counter()
        verifier.verify_flags(w.pk, w.sig, w.msg)
        ts.append((time.perf_counter() - t0) * 1e3)
    print(json.dumps({{"order": order, "tag": tag, "median_ms": float(np.median(ts)),
                      "ms": [round(t, 3) for t in ts]}}), flush=True)

if order == "early":
    host("first")
pk, sig, msg = (torch.from_numpy(x).to(dev) for x in (w.pk, w.sig, w.msg))
streams = [torch.cuda.current_stream(dev)] + [torch.cuda.Stream(dev) for _ in range(2)]
outs = [(torch.zeros(n, dtype=torch.uint8, device=dev), torch.zeros((n + 31) // 32, dtype=torch.int32, device=dev))
        for _ in range(3)]
for i in range(15):
    o = outs[i % 3]
    verifier.verify_device(pk, sig, msg, o[0], o[1], stream=streams[i % 3].cuda_stream)
torch.cuda.synchronize(dev)
verifier.measure_mad_peak()
host("after_device_work")
"""


def main():
    for rnd in range(2):
        for order, eager in (("late", "1"), ("late", "0"), ("early", "1")):
            r = subprocess.run([sys.executable, "-c", CHILD.format(root=ROOT, order=order)], capture_output=True,
                               text=True, timeout=300, env=dict(os.environ, HSV_EAGER_STREAMS=eager))
            if r.returncode != 0:
                print(json.dumps({"order": order, "rc": r.returncode, "err": r.stderr[-400:]}), flush=True)
                return r.returncode
            for line in r.stdout.strip().splitlines():
                if line.startswith("{"):
                    print(json.dumps(dict(json.loads(line), HSV_EAGER_STREAMS=eager)), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
