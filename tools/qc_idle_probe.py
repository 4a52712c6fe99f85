#!/usr/bin/env python3
"""Does a long GPU idle (or a long host-CPU load) before the QC legs change
the drop-in C3 latency?  bench.py runs its CPU baseline (10-30 s of host
work, GPU idle) right before the QC legs.  Measures the drop-in C3 p50 and
phases: warm, after S seconds of GPU idle (sleep), after S seconds of a
16-thread host load, each followed by an immediate re-measurement.

python tools/qc_idle_probe.py [--idle 20] [--reps 300]
"""
import argparse
import json
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "hotstuff-digital-signature-benchmarking_amd"))
sys.path.insert(0, ROOT)


def cpu_load(seconds, threads=16):
    stop = time.time() + seconds

    def spin():
        a = np.random.default_rng(0).random((256, 256))
        while time.time() < stop:
            a = a @ a
            a /= np.abs(a).max() + 1.0

    ts = [threading.Thread(target=spin) for _ in range(threads)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--idle", type=float, default=20.0)
    ap.add_argument("--reps", type=int, default=300)
    ap.add_argument("--generic", action="store_true", help="committee cache off: the generic kernels")
    a = ap.parse_args()
    import bench
    from hsverify import _lib, synth
    lib = _lib.load()
    lib.hsv_set_auto_committee(0 if a.generic else 1)
    calls = {}
    for size in (4, 1000):
        w = synth.qc_votes(size, seed=size)
        packed = np.concatenate([w.pk, w.sig], axis=1).tobytes()
        d = bytes(w.msg)
        calls[f"qc_votes{w.n}"] = lambda d=d, p=packed, n=w.n: lib.hsv_verify_batch_packed(d, p, n)
        for _ in range(3):
            calls[f"qc_votes{w.n}"]()
        lib.hsv_auto_committee_wait(60000)

    def rep(tag):
        for name, call in calls.items():
            t = bench._timed_lib(call, a.reps)
            print(json.dumps({"case": tag, "call": name, "p50_ms": round(t["p50_ms"], 4),
                              "p99_ms": round(t["p99_ms"], 4),
                              "sync_ms": (t.get("median_phases_ms") or {}).get("sync")}), flush=True)

    rep("warm")
    rep("warm_again")
    time.sleep(a.idle)
    rep(f"after_{a.idle:.0f}s_gpu_idle")
    rep("then_again")
    cpu_load(a.idle)
    rep(f"after_{a.idle:.0f}s_host_load")
    rep("then_again")
    return 0


if __name__ == "__main__":
    sys.exit(main())
