#!/usr/bin/env python3
"""A few pipelined host calls (hsv_verify from numpy arrays, 2^20 items) for
a kernel and copy trace:

cd /tmp && rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d OUT -o host -- \
    python3 tools/host_call_trace.py
then tools/host_call_trace.py --analyze OUT: the last call's timeline (copies, prepass and point
pass launches, gaps), from the trace's own timestamps.
"""
import csv
import glob
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "hotstuff-digital-signature-benchmarking_amd"))


def run(n=1 << 20, calls=4):
    from hsverify import synth, verifier
    w = synth.independent_triples(n, seed=5, corrupt_frac=0.05)
    verifier.verify_flags(w.pk, w.sig, w.msg)
    for _ in range(calls):
        time.sleep(0.05)  # separates the calls in the trace
        t0 = time.perf_counter()
        verifier.verify_flags(w.pk, w.sig, w.msg)
        print("call_ms", round((time.perf_counter() - t0) * 1e3, 3), flush=True)


def analyze(d):
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            rows.append(("K", r["Kernel_Name"].split("(")[0][:40], int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                         r.get("Stream_Id", r.get("Queue_Id", ""))))
    for f in glob.glob(os.path.join(d, "**", "*memory_copy_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            rows.append(("C", r.get("Direction", "copy"), int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                         r.get("Size", r.get("Bytes", ""))))
    rows.sort(key=lambda x: x[2])
    # the last call: everything after the last gap of > 20 ms
    starts = [r[2] for r in rows]
    cut = 0
    for i in range(1, len(starts)):
        if starts[i] - max(r[3] for r in rows[:i]) > 20_000_000:
            cut = i
    last = rows[cut:]
    t0 = last[0][2]
    out = []
    for kind, name, s, e, extra in last:
        out.append({"kind": kind, "name": name, "start_us": round((s - t0) / 1e3, 1), "end_us": round((e - t0) / 1e3, 1),
                    "dur_us": round((e - s) / 1e3, 1), "extra": extra})
    span = (max(r[3] for r in last) - t0) / 1e3
    print(json.dumps({"events": out, "span_us": round(span, 1)}, indent=0))


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--analyze":
        analyze(sys.argv[2])
    else:
        run()
