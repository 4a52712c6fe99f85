#!/usr/bin/env python3
"""200 cold one-item hsv_verify calls (committee cache off) for a
rocprofv3 --kernel-trace --stats run: the latency kernel's duration per build
(HSV_LIB selects the library)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "hotstuff-digital-signature-benchmarking_amd"))
from hsverify import _lib, synth, verifier  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1
lib = _lib.load()
lib.hsv_set_auto_committee(0)
w = synth.independent_triples(max(n, 1), seed=5, corrupt_frac=0.0, nthreads=4)
for _ in range(200):
    verifier.verify_flags(w.pk[:n], w.sig[:n], w.msg[:n])
print("ok")
