#!/usr/bin/env python3
"""A/B timing of kernel builds: every library named on the command line (files
in hsverify/, e.g. libhsv.so libhsv_base.so) is loaded in a fresh process,
checked bit-exact against the golden records, and timed on the C4 workload
(2^20 triples in HBM, HIP events, default variant).  Runs alternate A, B, A, B
so clock drift hits both; medians per library are printed at the end.

python tools/ab_probe.py [--rounds 3] [--reps 10] LIB [LIB ...]
"""
import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CACHE = "/tmp/hsv_ab_c4.npz"

CHILD = r"""
import json, os, sys, numpy as np
sys.path.insert(0, os.path.join({root!r}, "hotstuff-digital-signature-benchmarking_amd"))
sys.path.insert(0, os.path.join({root!r}, "tools"))
import torch
from hsverify import verifier, synth, _lib
from gpu_probe import golden
pk, sig, msg, exp = golden()
got = verifier.verify_flags(pk, sig, msg)
bad = int((got != exp).sum())
if os.path.exists({cache!r}):
    z = np.load({cache!r})
    P, S, M = z["pk"], z["sig"], z["msg"]
else:
    w = synth.independent_triples(1 << 20, seed=0xC4 * 1000, corrupt_frac=0.05, nthreads=16)
    P, S, M = w.pk, w.sig, w.msg
    np.savez({cache!r}, pk=P, sig=S, msg=M)
dev = torch.device("cuda:0")
tp, ts, tm = (torch.from_numpy(x).to(dev) for x in (P, S, M))
fl = torch.zeros(P.shape[0], dtype=torch.uint8, device=dev)
bits = torch.zeros(P.shape[0] // 32, dtype=torch.int32, device=dev)
st = torch.cuda.current_stream(dev)
for _ in range(2):
    verifier.verify_device(tp, ts, tm, fl, bits)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record(st)
for _ in range({reps}):
    verifier.verify_device(tp, ts, tm, fl, bits)
e1.record(st)
torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / {reps}
print(json.dumps({{"lib": os.environ.get("HSV_LIB"), "golden_mismatches": bad, "ms": ms,
                  "accepted": int((fl.cpu().numpy() & 1).sum())}}), flush=True)
"""


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("libs", nargs="+")
    a = ap.parse_args()
    res = {lib: [] for lib in a.libs}
    code = CHILD.format(root=ROOT, cache=CACHE, reps=a.reps)
    for r in range(a.rounds):
        for lib in a.libs:
            env = dict(os.environ, HSV_LIB=lib)
            out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
            line = [l for l in out.stdout.splitlines() if l.startswith("{")]
            if out.returncode != 0 or not line:
                print(f"{lib}: FAILED rc={out.returncode}\n{out.stderr[-2000:]}", flush=True)
                sys.exit(1)
            j = json.loads(line[0])
            res[lib].append(j)
            print(f"round {r} {lib}: {j['ms']:.3f} ms  golden mismatches {j['golden_mismatches']}  "
                  f"accepted {j['accepted']}", flush=True)
    for lib, js in res.items():
        ms = sorted(j["ms"] for j in js)
        print(f"{lib}: median {ms[len(ms) // 2]:.3f} ms  ({(1 << 20) / (ms[len(ms) // 2] * 1e-3) / 1e6:.2f} M verif/s) "
              f"all {['%.3f' % m for m in ms]}", flush=True)


if __name__ == "__main__":
    main()
