#!/usr/bin/env python3
"""Where the mempool line's time goes against the C4 line (round-5 VERDICT
item 4): bench.py's mempool leg (2^20 transactions of 512 B in HBM, two
alternating streams) and its C4 leg (2^20 triples, three streams), run under

cd /tmp && rocprofv3 --kernel-trace --output-format csv -d OUT -o mp -- python3 tools/mempool_trace.py
python3 tools/mempool_trace.py --analyze OUT

The analysis takes each leg's timed window from the trace (the kernels
between its markers), and reports per kernel the average duration and the
share of the window during which at least one kernel of each kind runs.
"""
import csv
import glob
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "hotstuff-digital-signature-benchmarking_amd"))


def run():
    import numpy as np
    import torch
    import bench
    from hsverify import synth, verifier
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    n = 1 << 20
    w = synth.independent_triples(n, seed=0xC4, corrupt_frac=0.05)
    pk, sig, msg = (torch.from_numpy(x).to(dev) for x in (w.pk, w.sig, w.msg))
    streams = [torch.cuda.current_stream(dev)] + [torch.cuda.Stream(dev) for _ in range(2)]
    outs = [(torch.zeros(n, dtype=torch.uint8, device=dev), torch.zeros((n + 31) // 32, dtype=torch.int32, device=dev))
            for _ in streams]
    for i in range(3):
        verifier.verify_device(pk, sig, msg, outs[i][0], outs[i][1], stream=streams[i].cuda_stream)
    torch.cuda.synchronize()
    time.sleep(0.1)  # marks the C4 window in the trace
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(streams[0])
    for s in streams[1:]:
        s.wait_event(e0)
    for i in range(10):
        verifier.verify_device(pk, sig, msg, outs[i % 3][0], outs[i % 3][1], stream=streams[i % 3].cuda_stream)
    for s in streams[1:]:
        ev = torch.cuda.Event()
        ev.record(s)
        streams[0].wait_event(ev)
    e1.record(streams[0])
    torch.cuda.synchronize()
    c4 = e0.elapsed_time(e1) / 10
    time.sleep(0.1)  # marks the mempool window
    mp = bench.mempool_bench(dev, cpu_sample=0, streams=streams[:2])
    print(json.dumps({"c4_ms_per_step": c4, "mempool_ms_per_step": mp["ms_per_step"],
                      "mempool_rounds": mp["rounds_ms_per_step"]}), flush=True)


def analyze(d):
    ks = []
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            ks.append((r["Kernel_Name"].split("(")[0].replace("void ", "").split("<")[0], int(r["Start_Timestamp"]),
                       int(r["End_Timestamp"])))
    ks.sort(key=lambda x: x[1])
    # windows: groups separated by > 50 ms of idle
    groups, cur, end = [], [], 0
    for k in ks:
        if cur and k[1] - end > 50_000_000:
            groups.append(cur)
            cur = []
        cur.append(k)
        end = max(end, k[2])
    groups.append(cur)

    def summary(g, steps):
        t0, t1 = g[0][1], max(k[2] for k in g)
        span = (t1 - t0) / 1e6
        by = {}
        for name, s, e in g:
            by.setdefault(name, []).append((s, e))
        out = {"span_ms": round(span, 3), "ms_per_step": round(span / steps, 4), "kernels": {}}
        for name, iv in by.items():
            iv.sort()
            busy, cs, ce = 0, None, None
            for s, e in iv:  # union of this kernel's intervals
                if ce is None or s > ce:
                    if ce is not None:
                        busy += ce - cs
                    cs, ce = s, e
                else:
                    ce = max(ce, e)
            busy += ce - cs
            out["kernels"][name] = {"count": len(iv), "avg_us": round(sum(e - s for s, e in iv) / len(iv) / 1e3, 1),
                                    "busy_share": round(busy / (t1 - t0), 4)}
        return out

    # the C4 window: the 10 timed steps (the group before the mempool); the
    # mempool window: its last round of 10 steps
    res = {"groups": len(groups)}
    c4 = [g for g in groups if any(k[0] == "hsv::hsv_prep_kernel" for k in g)]
    mp = [g for g in groups if any("tx_record" in k[0] for k in g)]
    if c4:  # the timed group: ten launches of prepass + point pass
        res["c4_10_steps"] = summary(c4[-1], sum(1 for k in c4[-1] if "hp_kernel" in k[0]))
    if mp:
        g = mp[-1]
        rec = [i for i, k in enumerate(g) if "tx_record" in k[0]]
        last = g[rec[-10]:] if len(rec) >= 10 else g
        res["mempool_last_10_steps"] = summary(last, 10)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--analyze":
        analyze(sys.argv[2])
    else:
        run()
