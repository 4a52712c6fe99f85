"""Row form of the field (csrc/hsv_fe16x16.hpp): one element spread over a
16-lane DPP row, used by the committee QC kernel's R waves
(hsv_comb_verify_quad_fused_kernel).

CPU: the bit-exact model of the row product (tools/lanesplit_model.py) keeps
every instruction's operand bound over worst-case limbs.
GPU: the row form (one element per row, and two rows per element as the
committee R waves run it) against the one-lane radix-2^25.5 form (the path the
golden vectors pin) on random elements and on edge encodings -- products, the
root chain x^((p-5)/8), and CompressedEdwardsY::decompress (flag, x, y) of every
public key and R of the golden records plus constructed y values (0, 1,
p - 1, p, p + 1, 2^255 - 1, both sign bits).
"""
import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

P = 2**255 - 19


def test_row_product_bounds_model():
    import lanesplit_model
    st = lanesplit_model.run(trials=200, seed=7)
    assert st["out"] < 2**16.1
    assert st["acc"] < 2**43


def test_row_point_formula_bounds_model():
    import lanesplit_model
    st = lanesplit_model.run_points(trials=40, seed=11)
    assert st["out"] < 2**16.3


def test_two_row_product_bounds_model():
    """The two-row product (RowLane2) keeps every instruction bound and gives
    the one-row product's limbs exactly, for operands up to 2^18.4."""
    import lanesplit_model
    st = lanesplit_model.run_two_row(trials=120, seed=9)
    assert st["out"] < 2**16.7


def _words(v):
    return [(v >> (32 * i)) & 0xFFFFFFFF for i in range(8)]


def _edge_encodings():
    encs = []
    for y in (0, 1, 2, P - 1, P, P + 1, P + 18, 2**255 - 1, 2**255 - 20):
        for sign in (0, 1):
            encs.append(_words((y & (2**255 - 1)) | (sign << 255)))
    with open(os.path.join(ROOT, "tests", "golden", "edge_vectors.json")) as f:
        vecs = json.load(f)["vectors"]
    for v in vecs:
        for hexs in (v["pk"], v["sig"][:64]):
            encs.append(list(np.frombuffer(bytes.fromhex(hexs), "<u4")))
    return encs


@pytest.mark.gpu
def test_row_form_matches_one_lane_form():
    from hsverify import _testing
    rng = np.random.default_rng(16)
    edges = _edge_encodings()
    n = 4096
    words = rng.integers(0, 2**32, size=(n, 16), dtype=np.uint64).astype(np.uint32)
    words[: len(edges), :8] = np.array(edges, dtype=np.uint32)
    with _testing.test_library():
        bad = _testing.lanesplit_check(words)
    assert not bad.any(), f"rows {np.nonzero(bad)[0][:8].tolist()} differ (bits {bad[bad != 0][:8].tolist()})"
