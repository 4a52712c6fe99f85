#!/usr/bin/env python3
"""The mempool line (bench.mempool_bench, 2^20 transactions of 512 B) on two
against three of the C4 line's streams, alternating in one process after the
three streams exist: prints ms per 2^20 transactions for each, then medians.
The library is the one HSV_LIB names (default libhsv.so).
python tools/mempool_nstreams_ab.py [--rounds 4]"""
import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "hotstuff-digital-signature-benchmarking_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=4)
    a = ap.parse_args()
    import torch
    import bench
    dev = torch.device("cuda", 0)
    c4_streams = [torch.cuda.current_stream(dev)] + [torch.cuda.Stream(dev) for _ in range(2)]
    res = {2: [], 3: []}
    for _ in range(a.rounds):
        for k in (2, 3):
            r = bench.mempool_bench(dev, cpu_sample=0, streams=c4_streams[:k])
            r.pop("_check", None)
            ok = r["honest_all_accepted"] and r["corrupted_all_rejected"]
            res[k].append(r["ms_per_step"])
            print(json.dumps({"streams": k, "ms": round(r["ms_per_step"], 4), "ok": ok}), flush=True)
    print(json.dumps({"lib": os.environ.get("HSV_LIB", "libhsv.so"),
                      "median_ms": {k: round(statistics.median(v), 4) for k, v in res.items()}}))
    return 0


if __name__ == "__main__":
    sys.exit(main())
