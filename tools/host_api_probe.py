#!/usr/bin/env python3
"""Host-buffer API throughput (hsv_verify from numpy arrays, PCIe-inclusive)
at 2^20 items; run twice, with and without HSV_NO_PIPELINE, to compare the
two-stream pipeline against the one-chunk path:

    python tools/host_api_probe.py ; HSV_NO_PIPELINE=1 python tools/host_api_probe.py
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "hotstuff-digital-signature-benchmarking_amd"))

from hsverify import synth, verifier  # noqa: E402

n = 1 << 20
w = synth.independent_triples(n, seed=5, corrupt_frac=0.05)
verifier.verify_flags(w.pk, w.sig, w.msg)
ts = []
for _ in range(5):
    t0 = time.perf_counter()
    f = verifier.verify_flags(w.pk, w.sig, w.msg)
    ts.append(time.perf_counter() - t0)
ms = float(np.median(ts) * 1e3)
import ctypes  # noqa: E402
from hsverify import _lib  # noqa: E402
lib = _lib.load()
marks = (ctypes.c_double * 256)()
cnt = lib.hsv_host_call_marks(marks, 256)
print("per-chunk host marks (ms: staged-wait done, packed, copies enqueued, launch enqueued):")
for k in range(0, cnt, 4):
    print("  chunk %d: %s" % (k // 4, " ".join("%.3f" % marks[k + j] for j in range(4) if k + j < cnt)))
print(json.dumps({"pipeline": "HSV_NO_PIPELINE" not in os.environ, "items": n, "ms": ms,
                  "verif_per_s": n / (ms * 1e-3), "ok": bool((f[w.accept] & 1).all())}))
