#!/usr/bin/env python3
"""The mempool line on the C4 line's streams against streams of its own
(bench.mempool_bench), in one process after a C4-style warm-up that creates
three streams first: prints ms per 2^20 transactions for both, alternating.
python tools/mempool_streams_ab.py [--rounds 3] [--own 3]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "hotstuff-digital-signature-benchmarking_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--own", type=int, default=3, help="streams of the mempool line's own")
    a = ap.parse_args()
    import torch
    import bench
    dev = torch.device("cuda", 0)
    c4_streams = [torch.cuda.current_stream(dev)] + [torch.cuda.Stream(dev) for _ in range(2)]
    for _ in range(a.rounds):
        shared = bench.mempool_bench(dev, cpu_sample=0, nstreams=3, streams=c4_streams)
        own = bench.mempool_bench(dev, cpu_sample=0, nstreams=a.own)
        print(json.dumps({"c4_streams_ms": round(shared["ms_per_step"], 4), "own_streams_ms": round(own["ms_per_step"], 4),
                          "ok": shared["honest_all_accepted"] and own["corrupted_all_rejected"]}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
