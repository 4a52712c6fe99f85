#!/usr/bin/env python3
"""Why the host-buffer call measures slower inside bench.py than in a fresh
process (tools/host_pipeline_probe.py): the same 2^20-item hsv_verify call in a
fresh child per case --

  npz        inputs loaded from a cached .npz by the main thread;
  synth      inputs generated in-process by synth (16 threads, as bench.py);
  synth_copy the synth arrays copied once by the main thread;
  after_c4   npz inputs, after ten HBM-resident 2^20 launches on three streams;
  after_load npz inputs, right after 2 s of back-to-back resident launches;
  after_rest the same, then 2 s idle before the host calls.

python tools/host_env_probe.py [--reps 9]
"""
import argparse
import json
import os
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "hotstuff-digital-signature-benchmarking_amd"))
CACHE = "/tmp/hsv_host_pipe_c4.npz"
N = 1 << 20
CASES = ("npz", "synth", "synth_copy", "after_c4", "after_load", "after_rest")


def arrays(case):
    from hsverify import synth
    if case.startswith("synth"):
        w = synth.independent_triples(N, seed=0xC4 * 1000, corrupt_frac=0.05, nthreads=16)
        a = (w.pk, w.sig, w.msg)
        return tuple(x.copy() for x in a) if case == "synth_copy" else a
    if not os.path.exists(CACHE):
        w = synth.independent_triples(N, seed=0xC4 * 1000, corrupt_frac=0.05, nthreads=16)
        np.savez(CACHE, pk=w.pk, sig=w.sig, msg=w.msg)
    z = np.load(CACHE)
    return z["pk"], z["sig"], z["msg"]


def child(case, reps):
    from hsverify import _testing, verifier
    pk, sig, msg = arrays(case)
    if case.startswith("after"):
        import torch
        dev = torch.device("cuda", 0)
        tp, ts, tm = (torch.from_numpy(x).to(dev) for x in (pk, sig, msg))
        streams = [torch.cuda.Stream(dev) for _ in range(3)]
        flags = [torch.zeros(N, dtype=torch.uint8, device=dev) for _ in range(3)]
        t_end = time.perf_counter() + (2.0 if case != "after_c4" else 0.0)
        k = 0
        while k < 10 or time.perf_counter() < t_end:
            verifier.verify_device(tp, ts, tm, flags[k % 3], stream=streams[k % 3].cuda_stream)
            k += 1
            if k % 30 == 0:
                torch.cuda.synchronize(dev)
        torch.cuda.synchronize(dev)
        if case == "after_rest":
            time.sleep(2.0)
    verifier.verify_flags(pk, sig, msg)
    res = []
    for _ in range(reps):
        t0 = time.perf_counter()
        verifier.verify_flags(pk, sig, msg)
        res.append(((time.perf_counter() - t0) * 1e3, _testing.host_call_stats()))
    res.sort(key=lambda r: r[0])
    ms, st = res[len(res) // 2]
    print(json.dumps({"case": case, "ms": round(ms, 3), "call_ms": round(st["call_ms"], 3),
                      "pack_ms": round(st["pack_ms"], 3), "min_ms": round(res[0][0], 3)}), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=9)
    ap.add_argument("--child", choices=CASES)
    a = ap.parse_args()
    if a.child:
        return child(a.child, a.reps)
    arrays("npz")
    for case in ("npz", "after_c4", "after_load", "after_rest", "npz", "after_load"):
        r = subprocess.run([sys.executable, __file__, "--child", case, "--reps", str(a.reps)],
                           capture_output=True, text=True, timeout=300)
        print(r.stdout.strip().splitlines()[-1] if r.returncode == 0 else f"{case}: rc={r.returncode} {r.stderr[-300:]}",
              flush=True)


if __name__ == "__main__":
    main()
