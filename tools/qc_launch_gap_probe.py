#!/usr/bin/env python3
"""Does the launch phase of a drop-in QC call depend on how soon it follows
the previous call?  C1 (3 votes) and C3 (667): p50 of the wall time and of the
library's host phases (hsv_host_call_marks), back to back and with a busy
gap of G microseconds between calls.

python tools/qc_launch_gap_probe.py [--reps 400] [--gaps 0,20,50,200]"""
import argparse
import ctypes
import gc
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "hotstuff-digital-signature-benchmarking_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=400)
    ap.add_argument("--gaps", default="0,20,50,200")
    a = ap.parse_args()
    import bench
    from hsverify import _lib, synth
    import torch
    bench.pin_to_gpu_node(0)
    lib = _lib.load()
    lib.hsv_set_auto_committee(1)
    buf = (ctypes.c_double * 8)()
    for size in (4, 1000):
        w = synth.qc_votes(size, seed=size)
        p = np.concatenate([w.pk, w.sig], 1).tobytes()
        d = bytes(w.msg)
        call = lambda: lib.hsv_verify_batch_packed(d, p, w.n)
        for _ in range(3):
            call()
        lib.hsv_auto_committee_wait(60000)
        for gap in (int(x) for x in a.gaps.split(",")):
            ts, marks = [], []
            gc.disable()
            for _ in range(a.reps):
                t_end = time.perf_counter() + gap * 1e-6
                while time.perf_counter() < t_end:
                    pass
                t0 = time.perf_counter()
                call()
                ts.append(time.perf_counter() - t0)
                n = lib.hsv_host_call_marks(buf, 8)
                marks.append([buf[i] for i in range(n)])
            gc.enable()
            m = np.array(marks)
            step = np.diff(np.concatenate([np.zeros((len(m), 1)), np.maximum(m, 0)], axis=1), axis=1)
            med = np.median(step, axis=0)
            print(json.dumps({"votes": w.n, "gap_us": gap, "p50_ms": round(float(np.median(ts)) * 1e3, 4),
                              "phases_ms": [round(float(x), 4) for x in med]}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
