#!/usr/bin/env python3
"""Diagnostics of the resident service path (HSV_QC_RESIDENT=1): marks and
timings of single cached-key verifies."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "hotstuff-digital-signature-benchmarking_amd"))
from hsverify import _lib, _testing, synth, verifier  # noqa: E402

lib = _lib.load()
lib.hsv_set_auto_committee(1)
w = synth.qc_votes(100, seed=5)
packed = np.concatenate([w.pk, w.sig], axis=1).tobytes()
for _ in range(3):
    lib.hsv_verify_batch_packed(bytes(w.msg), packed, w.n)
print("wait", lib.hsv_auto_committee_wait(60000), "size", lib.hsv_auto_committee_size(), flush=True)
for k in (1, 3, 4):
    for rep in range(3):
        t0 = time.perf_counter()
        f = verifier.verify_flags(w.pk[:k], w.sig[:k], w.msg)
        dt = (time.perf_counter() - t0) * 1e3
        print(k, rep, f.tolist(), round(dt, 4), _testing.host_call_marks()[:6], flush=True)
print("env", os.environ.get("HSV_QC_RESIDENT"))
