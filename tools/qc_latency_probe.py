#!/usr/bin/env python3
"""QC verify latency per kernel variant (p50/p99 of hsv_verify_batch_packed,
host buffers: H2D + kernels + D2H), for the C2 / C3 quorums and a few larger
batches.  Measurement tool, run on the GPU box:

    python tools/qc_latency_probe.py [--variants 19,21] [--reps 200]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "hotstuff-digital-signature-benchmarking_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="19,21")
    ap.add_argument("--reps", type=int, default=200)
    a = ap.parse_args()
    from hsverify import _lib, synth, verifier
    lib = _lib.load()
    cases = [(100, synth.qc_votes(100, seed=100)), (1000, synth.qc_votes(1000, seed=1000))]
    out = {}
    for v in (int(x) for x in a.variants.split(",")):
        verifier.set_variant(v)
        res = {}
        for committee, w in cases:
            packed = np.concatenate([w.pk, w.sig], axis=1).tobytes()
            digest = bytes(w.msg)
            for _ in range(10):
                assert lib.hsv_verify_batch_packed(digest, packed, w.n) == 1
            ts = []
            for _ in range(a.reps):
                t0 = time.perf_counter()
                rc = lib.hsv_verify_batch_packed(digest, packed, w.n)
                ts.append(time.perf_counter() - t0)
                assert rc == 1
            ts = np.array(ts) * 1e3
            res[f"n{committee}_votes{w.n}"] = {"p50_ms": float(np.percentile(ts, 50)),
                                                "p99_ms": float(np.percentile(ts, 99))}
        for n in (4096, 32768):
            w = synth.independent_triples(n, seed=n, corrupt_frac=0.0)
            for _ in range(3):
                verifier.verify_flags(w.pk, w.sig, w.msg)
            ts = []
            for _ in range(10):
                t0 = time.perf_counter()
                f = verifier.verify_flags(w.pk, w.sig, w.msg)
                ts.append(time.perf_counter() - t0)
            assert (f & 1).all()
            res[f"batch{n}"] = {"p50_ms": float(np.median(ts) * 1e3)}
        out[f"variant{v}"] = res
        print(json.dumps({f"variant{v}": res}), flush=True)


if __name__ == "__main__":
    main()
