#!/usr/bin/env python3
"""Phase stamps of the quad-form latency kernel (hsv_verify_quad_kernel),
block 0, medians over reps of a one-item cold verify (cache off):
HSV_LIB=libhsv_quadclk.so python tools/quad_clocks.py
(build: tools/build_ab_libs.sh quadclk "-DHSV_QUAD_CLOCKS")."""
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "hotstuff-digital-signature-benchmarking_amd"))
from hsverify import _lib, synth, verifier  # noqa: E402

lib = _lib.load()
fn = lib.hsv_quad_clocks
fn.restype = ctypes.c_int
fn.argtypes = [ctypes.c_void_p]
lib.hsv_set_auto_committee(0)
w = synth.qc_votes(4, seed=4)
buf = np.zeros((4, 9), np.uint64)
rows = []
for i in range(80):
    verifier.verify_flags(w.pk[:1], w.sig[:1], w.msg)
    assert fn(buf.ctypes.data) == 0
    if i >= 10:
        c = buf[:, :8].astype(np.int64)
        t0 = c[:, 0].min()
        rows.append((c - t0) * 0.01)  # us
        hwid = [int(x) for x in buf[:, 8]]
r = np.median(np.array(rows), axis=0)
names = ["entry", "decomp|prep", "table", "barrier1", "straus", "comb", "barrier2", "exit"]
for wv, role in enumerate(("R", "A", "prepass + R low windows + B comb", "A low windows")):
    print(json.dumps({"wave": role, "simd": (hwid[wv] >> 4) & 3, "cu": (hwid[wv] >> 8) & 15,
                      **{n: round(float(r[wv][j]), 2) for j, n in enumerate(names)}}))
