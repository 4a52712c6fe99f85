#!/usr/bin/env python3
"""One run of bench.mempool_bench (2^20 transactions of 512 B in HBM, three
streams) without the CPU leg, for a rocprofv3 kernel trace of the mempool
line: python tools/mempool_once.py"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "hotstuff-digital-signature-benchmarking_amd"))


def main():
    import torch
    import bench
    r = bench.mempool_bench(torch.device("cuda", 0), cpu_sample=0)
    print(json.dumps({"ms": r["ms_per_step"], "ok": r["honest_all_accepted"] and r["corrupted_all_rejected"]}))
    return 0


if __name__ == "__main__":
    sys.exit(main())
