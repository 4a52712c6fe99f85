#!/usr/bin/env python3
"""Back-to-back C4 launches (2^20 triples in HBM) on one stream against the
same launches alternating over two or more streams, where a launch can start in the
previous launch's grid end.  Both forms produce the
same flags; prints ms per launch (median of rounds) for each.

python tools/pipeline_probe.py [--n 1048576] [--steps 20] [--rounds 3] [--max-streams 3]
"""
import argparse
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "hotstuff-digital-signature-benchmarking_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1 << 20)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--max-streams", type=int, default=3)
    a = ap.parse_args()
    import torch
    from hsverify import _lib, synth, verifier
    _lib.load()
    dev = torch.device("cuda", 0)
    w = synth.independent_triples(a.n, seed=0xC4 * 1000, corrupt_frac=0.05, nthreads=16)
    pk, sig, msg = (torch.from_numpy(x).to(dev) for x in (w.pk, w.sig, w.msg))
    ks = list(range(1, a.max_streams + 1))
    streams = [torch.cuda.Stream(dev) for _ in ks]
    outs = [(torch.zeros(a.n, dtype=torch.uint8, device=dev),
             torch.zeros((a.n + 31) // 32, dtype=torch.int32, device=dev)) for _ in streams]

    def run(nstreams):
        torch.cuda.synchronize(dev)
        t = time.perf_counter()
        for i in range(a.steps):
            j = i % nstreams
            verifier.verify_device(pk, sig, msg, outs[j][0], outs[j][1], stream=streams[j].cuda_stream)
        torch.cuda.synchronize(dev)
        return (time.perf_counter() - t) * 1e3 / a.steps

    for k in ks:  # warm-up (workspace pools, tables)
        run(k)
    res = {k: [] for k in ks}
    for _ in range(a.rounds):
        for k in ks:
            res[k].append(run(k))
    same = all(torch.equal(outs[0][0], o[0]) and torch.equal(outs[0][1], o[1]) for o in outs[1:])
    for k in ks:
        med = statistics.median(res[k])
        print(f"{k} stream(s): {med:.3f} ms per launch ({a.n / med / 1e3:.2f} M verif/s) "
              f"all {[round(x, 3) for x in res[k]]}")
    print("outputs identical across streams:", same)
    return 0 if same else 1


if __name__ == "__main__":
    sys.exit(main())
