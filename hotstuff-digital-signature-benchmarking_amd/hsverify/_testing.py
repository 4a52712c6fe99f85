"""Test and measurement hooks of libhsv.so (not part of include/hsv.h).

Kept out of the public modules: each changes process-wide behaviour of the
library for every thread, so only tests, bench.py and tools/ use them.
"""
from __future__ import annotations

import contextlib
import ctypes

from . import _lib

# fault injection modes (csrc/hsv_verify_core.hpp kInject*)
INJECT_NONE = 0
INJECT_ZERO_TABLES = 1   # table entries read back as zeros
INJECT_CANARY = 2        # a lane's workspace canary is overwritten mid-batch
INJECT_FLIP_TABLES = 3   # one bit of table entries flipped


def set_lattice_bits(bits: int) -> int:
    """The lattice bound of the comb-path prepass (0 = default, 138; 133 sends
    the tests/golden/lattice_fallback.bin challenges down the full-length
    path).  Returns the previous bound."""
    prev = _lib.load().hsv_set_lattice_bits(bits)
    if prev < 0:
        raise ValueError(f"lattice bound out of range: {bits}")
    return prev


def inject_fault(mode: int) -> int:
    """Corrupt what the following launches read back (INJECT_*; 0 = off).
    Returns the previous mode."""
    prev = _lib.load().hsv_test_inject_fault(mode)
    if prev < 0:
        raise ValueError(f"unknown fault injection mode {mode}")
    return prev


@contextlib.contextmanager
def injected_fault(mode: int):
    prev = inject_fault(mode)
    try:
        yield
    finally:
        inject_fault(prev)


def host_call_stats() -> dict:
    """The calling thread's last host-buffer verification: pack time (host ms
    spent copying into pinned staging), bytes copied host-to-device, wall ms."""
    v = [ctypes.c_double() for _ in range(3)]
    _lib.load().hsv_host_call_stats(*[ctypes.byref(x) for x in v])
    return {"pack_ms": v[0].value, "h2d_bytes": v[1].value, "call_ms": v[2].value}


def host_call_marks() -> list:
    """Per-chunk host marks of the calling thread's last pipelined call, ms
    from its start: staging buffer free, packed, copy enqueued, launch
    enqueued (4 per chunk; empty for calls below the pipeline's size)."""
    buf = (ctypes.c_double * 256)()
    n = _lib.load().hsv_host_call_marks(buf, 256)
    return [round(buf[i], 4) for i in range(max(0, n))]


def pack_threads() -> int:
    """Helper threads of the library's staging-copy pool (HSV_PACK_THREADS)."""
    return _lib.load().hsv_pack_threads()


def lanesplit_check(words):
    """Row-form field arithmetic against the one-lane form on the GPU
    (hsv_test_lanesplit_check): words is an (n, 16) uint32 array of element
    pairs a | b; returns per-row mismatch bits (1 product, 2 root chain,
    4 decompression of a as an encoding) of the one-row form, and the same
    three shifted by 3 (8, 16, 32) for the two-row form (RowLane2)."""
    import numpy as np
    w = np.ascontiguousarray(words, dtype=np.uint32)
    out = np.zeros(len(w), np.uint32)
    lib = _lib.load()
    rc = lib.hsv_test_lanesplit_check(ctypes.c_void_p(w.ctypes.data), ctypes.c_uint32(len(w)),
                                      ctypes.c_void_p(out.ctypes.data))
    if rc != 0:
        raise RuntimeError(f"hsv_test_lanesplit_check failed: hipError {rc}")
    return out
