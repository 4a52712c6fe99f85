#!/usr/bin/env python3
"""Six host-buffer calls of 2^20 items (hsv_verify from numpy arrays, the
chunked copy pipeline), for a rocprofv3 kernel + memory-copy trace of the
pipeline: python tools/host_api_once.py [--n-log2 20] [--reps 6]"""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "hotstuff-digital-signature-benchmarking_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n-log2", type=int, default=20)
    ap.add_argument("--reps", type=int, default=6)
    a = ap.parse_args()
    from hsverify import synth, verifier
    w = synth.independent_triples(1 << a.n_log2, seed=5, corrupt_frac=0.05)
    for r in range(a.reps):
        t0 = time.perf_counter()
        f = verifier.verify_flags(w.pk, w.sig, w.msg)
        print(f"rep {r}: {(time.perf_counter() - t0) * 1e3:.3f} ms", flush=True)
    ok = bool((f[w.accept] & 1).all()) and not bool((f[~w.accept] & 1).any())
    print("ok" if ok else "MISMATCH", flush=True)
    return 0 if ok else 1


if __name__ == "__main__":
    rc = main()
    if os.environ.get("HSV_PROBE_FAST_EXIT") == "1":  # skip static destructors
        sys.stdout.flush()
        os._exit(rc)
    sys.exit(rc)
