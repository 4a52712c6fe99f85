#!/usr/bin/env python3
"""Per-wave phases of one cached verify_strict through the resident service
(HSV_QC_RESIDENT=1) or a launch (unset), with the clock-stamp build:
HSV_LIB=libhsv_qcclk.so [HSV_QC_RESIDENT=1] python tools/resident_clocks.py"""
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "hotstuff-digital-signature-benchmarking_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
from hsverify import _lib, synth, verifier  # noqa: E402
import qc_wave_clocks as q  # noqa: E402

lib = _lib.load()
fn = lib.hsv_qc_wave_clocks_nosync
fn.restype = ctypes.c_int
fn.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
lib.hsv_set_auto_committee(1)
w = synth.qc_votes(100, seed=5)
packed = np.concatenate([w.pk, w.sig], axis=1).tobytes()
for _ in range(3):
    lib.hsv_verify_batch_packed(bytes(w.msg), packed, w.n)
lib.hsv_auto_committee_wait(60000)
buf = np.zeros((4096, q.SLOTS), dtype=np.uint64)
rows = []
for i in range(60):
    verifier.verify_flags(w.pk[:1], w.sig[:1], w.msg)
    wpb = fn(buf.ctypes.data, 4)
    if i >= 10:
        rows.append(q.analyse(buf, 1, wpb))
keys = ("span_us", "r_load_us", "r_alu_us", "hash_load_us", "hash_alu_us", "comb_s_half_us",
        "comb_k_half_swaps_us", "comb_tail_us", "shader_clock_mhz")
print(json.dumps({"resident": os.environ.get("HSV_QC_RESIDENT") == "1",
                  **{k: round(float(np.median([r[k] for r in rows])), 3) for k in keys}}))
