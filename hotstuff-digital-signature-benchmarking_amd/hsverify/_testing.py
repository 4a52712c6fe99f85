"""Test and measurement hooks (csrc/hsv_test_hooks.h), exported by
libhsv_test.so only -- the product libhsv.so exports exactly include/hsv.h.

libhsv_test.so is a second, independent instance of the library (same
objects plus the hooks).  ``test_library()`` routes every hsverify call made
inside it to that instance, so a test injects faults into, or changes the
variant of, the very library its calls run on -- and nothing it does reaches
the product instance other tests use.  The hook functions below require it
(they enter it themselves where that is unambiguous).
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
INJECT_NO_PUBLISH = 4    # fused transaction launch: record batch 0 never published (bounded wait -> fault)


@contextlib.contextmanager
def test_library():
    """Route hsverify calls to libhsv_test.so for the duration (re-entrant)."""
    lib = _lib.load_test()
    prev = _lib.set_override(lib)
    try:
        yield lib
    finally:
        _lib.set_override(prev)


def set_lattice_bits(bits: int) -> int:
    """The lattice bound of the comb-path prepass (0 = default, 138; 133 sends
    the tests/golden/lattice_fallback.bin challenges down the full-length
    path).  Returns the previous bound."""
    prev = _lib.hook("hsv_set_lattice_bits")(bits)
    if prev < 0:
        raise ValueError(f"lattice bound out of range: {bits}")
    return prev


def inject_fault(mode: int) -> int:
    """Corrupt what the calling thread's following launches read back
    (INJECT_*; 0 = off; other threads are unaffected).  Returns the previous mode."""
    prev = _lib.hook("hsv_test_inject_fault")(mode)
    if prev < 0:
        raise ValueError(f"unknown fault injection mode {mode}")
    return prev


@contextlib.contextmanager
def injected_fault(mode: int):
    """test_library() with `mode` injected into this thread's launches."""
    with test_library():
        prev = inject_fault(mode)
        try:
            yield
        finally:
            inject_fault(prev)


def corrupt_auto_committee() -> int:
    """Zero the automatic committee cache's tables in HBM (test library);
    returns the number of cached keys."""
    return _lib.check(_lib.hook("hsv_test_corrupt_auto_committee")(), "hsv_test_corrupt_auto_committee")


def pipe_nocopy(on: bool) -> bool:
    """Measurement only (test library): pipelined host calls of the same size
    as the slot's previous one skip the pack and the copies and verify what
    that call left in HBM.  Returns the previous setting."""
    return bool(_lib.hook("hsv_test_pipe_nocopy")(1 if on else 0))


def host_call_stats() -> dict:
    """The calling thread's last host-buffer verification: pack time (host ms
    spent copying into pinned staging), bytes copied host-to-device, wall ms."""
    v = [ctypes.c_double() for _ in range(3)]
    _lib.load().hsv_host_call_stats(*[ctypes.byref(x) for x in v])
    return {"pack_ms": v[0].value, "h2d_bytes": v[1].value, "call_ms": v[2].value}


def host_call_marks() -> list:
    """Host timeline of the calling thread's last call, ms from its entry
    (hsv_host_call_marks): HSV_MARK_* points for a latency call (see
    latency_marks), four per chunk for a pipelined call."""
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
    rc = _lib.hook("hsv_test_lanesplit_check")(ctypes.c_void_p(w.ctypes.data), ctypes.c_uint32(len(w)),
                                               ctypes.c_void_p(out.ctypes.data))
    if rc != 0:
        raise RuntimeError(f"hsv_test_lanesplit_check failed: hipError {rc}")
    return out
