#!/usr/bin/env python3
"""A/B of the pipelined host call's launch schedule (hsv_verify from numpy
arrays, PCIe included) through libhsv_test.so's hsv_test_pipe_schedule, in
one warm process, schedules alternating round by round.  Beside them: one
device-resident launch of the same batch alone (the GPU time without PCIe or
chunk boundaries) and three back-to-back launches on alternating streams.

python tools/host_sched_ab.py [--n 1048576] [--rounds 5] [--reps 5]
"""
import argparse
import ctypes
import json
import os
import statistics
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "hotstuff-digital-signature-benchmarking_amd"))

SCHEDULES = {
    "default": [],                                   # 2^16, then 3x everything before
    "r05_pieces": [1 << 16, 1 << 17],                # round 5: 2^16, then 2^17 per launch
    "full1": [3 << 16, 3 << 16, 1 << 20],            # one 64-item batch per wave of the grid first
    "full1b": [3 << 16, 1 << 20],
    "half_full": [3 << 15, 3 << 16, 1 << 20],
    "geo_15": [1 << 15, 3 << 15, 12 << 15, 1 << 20],
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1 << 20)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("schedules", nargs="*", default=list(SCHEDULES))
    a = ap.parse_args()
    import torch
    from hsverify import _testing, synth, verifier
    w = synth.independent_triples(a.n, seed=5, corrupt_frac=0.05)
    res = {s: [] for s in a.schedules}
    marks = {}
    with _testing.test_library() as lib:
        def set_sched(name):
            sz = (ctypes.c_uint64 * max(1, len(SCHEDULES[name])))(*SCHEDULES[name])
            assert lib.hsv_test_pipe_schedule(sz, len(SCHEDULES[name])) == 0

        ref = None
        for r in range(a.rounds):
            for name in a.schedules:
                set_sched(name)
                f = verifier.verify_flags(w.pk, w.sig, w.msg)  # warm this schedule's workspaces
                if ref is None:
                    ref = f
                assert (f == ref).all(), name
                ts = []
                for _ in range(a.reps):
                    t0 = time.perf_counter()
                    verifier.verify_flags(w.pk, w.sig, w.msg)
                    ts.append(time.perf_counter() - t0)
                res[name].append(statistics.median(ts) * 1e3)
                marks[name] = _testing.host_call_marks()
                print(r, name, round(res[name][-1], 3), "ms", flush=True)
        set_sched("default")
    dev = torch.device("cuda:0")
    pk, sig, msg = (torch.from_numpy(x).to(dev) for x in (w.pk, w.sig, w.msg))
    flags = torch.zeros(a.n, dtype=torch.uint8, device=dev)
    st = [torch.cuda.current_stream(dev), torch.cuda.Stream(dev), torch.cuda.Stream(dev)]
    outs = [torch.zeros(a.n, dtype=torch.uint8, device=dev) for _ in st]
    for _ in range(2):
        verifier.verify_device(pk, sig, msg, flags)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(3):
        verifier.verify_device(pk, sig, msg, flags)
    e1.record()
    torch.cuda.synchronize()
    iso = e0.elapsed_time(e1) / 3
    e0.record(st[0])
    for s in st[1:]:
        s.wait_event(e0)
    for i in range(9):
        verifier.verify_device(pk, sig, msg, outs[i % 3], stream=st[i % 3].cuda_stream)
    for s in st[1:]:
        ev = torch.cuda.Event()
        ev.record(s)
        st[0].wait_event(ev)
    e1.record(st[0])
    torch.cuda.synchronize()
    steady = e0.elapsed_time(e1) / 9
    out = {"n": a.n, "device_isolated_launch_ms": round(iso, 4), "device_3stream_step_ms": round(steady, 4),
           "median_ms": {k: round(statistics.median(v), 4) for k, v in res.items()},
           "rounds_ms": {k: [round(x, 3) for x in v] for k, v in res.items()},
           "vs_3stream_step": {k: round(steady / statistics.median(v), 4) for k, v in res.items()},
           "marks_last_call": marks}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
