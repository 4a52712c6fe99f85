#!/usr/bin/env python3
"""Mempool line scheduling sweep (round-4 VERDICT item 8): ms per 2^20
transactions for 1-4 alternating streams at normal and at high stream
priority, beside the C4 line (3 streams) in the same process.

python tools/mempool_sched_probe.py [--rounds 2]"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "hotstuff-digital-signature-benchmarking_amd"))


def c4_ms(dev, w, streams, steps=10):
    import torch
    from hsverify import verifier
    pk, sig, msg = (torch.from_numpy(x).to(dev) for x in (w.pk, w.sig, w.msg))
    flags = [torch.zeros(w.n, dtype=torch.uint8, device=dev) for _ in streams]
    for i in range(2):
        verifier.verify_device(pk, sig, msg, flags[i % len(streams)], stream=streams[i % len(streams)].cuda_stream)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for i in range(steps):
        s = streams[i % len(streams)]
        verifier.verify_device(pk, sig, msg, flags[i % len(streams)], stream=s.cuda_stream)
    torch.cuda.synchronize(dev)
    return (time.perf_counter() - t0) / steps * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=2)
    a = ap.parse_args()
    import torch
    import bench
    from hsverify import synth
    dev = torch.device("cuda", 0)
    w = synth.independent_triples(1 << 20, seed=3, corrupt_frac=0.05, nthreads=16)
    c4_streams = [torch.cuda.Stream(dev) for _ in range(3)]
    for r in range(a.rounds):
        out = {"round": r, "c4_3streams_ms": round(c4_ms(dev, w, c4_streams), 4)}
        for prio in (0, -1):
            for k in (1, 2, 3, 4):
                ss = [torch.cuda.Stream(dev, priority=prio) for _ in range(k)]
                res = bench.mempool_bench(dev, cpu_sample=0, nstreams=k, streams=ss)
                out[f"mempool_{k}s_prio{prio}_ms"] = round(res["ms_per_step"], 4)
        print(json.dumps(out), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
