"""ctypes binding of libhsv.so (the C ABI declared in include/hsv.h).

The shared library is built in-tree (``make`` in the package root, or
``__graft_entry__.build()``) and is loaded from this directory only.  If it
is missing, every entry point raises :class:`HsvLibraryError` -- there is no
CPU fallback for verification.

PyTorch, when importable, is imported *before* the library so that the HIP
runtime (``libamdhip64.so.7``) already mapped by torch is the one libhsv
binds to: one runtime per process, so device pointers from torch tensors can
be passed to ``hsv_verify_device``.
"""
from __future__ import annotations

import ctypes
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
# HSV_LIB selects another build of the library for tools (e.g. a clock-stamp
# build from tools/build_ab_libs.sh); it must live in this directory as well.
LIB_PATH = os.path.join(_HERE, os.path.basename(os.environ.get("HSV_LIB", "libhsv.so")))
# The same objects plus the exported test hooks (csrc/hsv_test_hooks.h);
# loaded only by tests and tools through hsverify._testing.
TEST_LIB_PATH = os.path.join(_HERE, "libhsv_test.so")
# Exported by libhsv_test.so only, never by libhsv.so.
HOOKS = ("hsv_test_inject_fault", "hsv_test_inject_mode", "hsv_test_corrupt_auto_committee",
         "hsv_test_lanesplit_check", "hsv_set_lattice_bits", "hsv_set_variant", "hsv_variant_list",
         "hsv_variant_available", "hsv_num_variants", "hsv_set_virtual_shards", "hsv_test_pipe_nocopy",
         "hsv_test_resident_counts", "hsv_test_resident_post_bad", "hsv_test_tx_records",
         "hsv_test_pipe_schedule", "hsv_test_numa_plan", "hsv_test_pinned_thread_cpus")

# flag bits (include/hsv.h)
STRICT_OK = 0x01
EQ_OK = 0x02
PARSE_OK = 0x04
SMALL_A = 0x08
SMALL_R = 0x10
S_OK = 0x20
A_OK = 0x40
R_OK = 0x80

HSV_OK = 0
ERRORS = {
    -1: "HSV_ERR_NO_DEVICE",
    -2: "HSV_ERR_HIP",
    -3: "HSV_ERR_INVALID_ARG",
    -4: "HSV_ERR_ALLOC",
    -5: "HSV_ERR_ALIGN",
    -6: "HSV_ERR_PARSE",
    -7: "HSV_ERR_DEVICE_FAULT",
}
HSV_ERR_DEVICE_FAULT = -7


class HsvLibraryError(RuntimeError):
    """libhsv.so missing, or an infrastructure error (never a signature rejection)."""


_lock = threading.Lock()
_lib = None        # the library every hsverify call uses (LIB_PATH)
_test_lib = None   # libhsv_test.so, a second instance, loaded on demand
_override = None   # hsverify._testing.test_library(): calls go to _test_lib


def _declare(lib):
    c_u8p = ctypes.c_void_p
    sz = ctypes.c_size_t
    sig = {
        "hsv_init": (ctypes.c_int, [ctypes.c_int]),
        "hsv_bound_device": (ctypes.c_int, []),
        "hsv_set_virtual_shards": (ctypes.c_int, [ctypes.c_int]),
        "hsv_test_pipe_nocopy": (ctypes.c_int, [ctypes.c_int]),
        "hsv_test_pipe_schedule": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
        "hsv_test_numa_plan": (ctypes.c_int, [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_char_p, ctypes.c_int,
                                              ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]),
        "hsv_test_pinned_thread_cpus": (ctypes.c_int, [ctypes.c_char_p, ctypes.c_void_p, ctypes.c_int]),
        "hsv_test_resident_counts": (None, [ctypes.POINTER(ctypes.c_uint64)] * 2),
        "hsv_test_resident_post_bad": (ctypes.c_int, [ctypes.c_uint32]),
        "hsv_test_tx_records": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_size_t,
                                               ctypes.c_void_p, ctypes.c_void_p]),
        "hsv_auto_committee_wait": (ctypes.c_int, [ctypes.c_int]),
        "hsv_auto_committee_faults": (ctypes.c_uint64, []),
        "hsv_variant_list": (ctypes.c_int, [ctypes.POINTER(ctypes.c_int), ctypes.c_int]),
        "hsv_variant_available": (ctypes.c_int, [ctypes.c_int]),
        "hsv_shutdown": (None, []),
        "hsv_device_count": (ctypes.c_int, []),
        "hsv_last_error": (ctypes.c_char_p, []),
        "hsv_version": (ctypes.c_char_p, []),
        "hsv_abi_version": (ctypes.c_int, []),
        "hsv_verify": (ctypes.c_int, [c_u8p, c_u8p, c_u8p, sz, sz, c_u8p]),
        "hsv_verify_strict": (ctypes.c_int, [c_u8p, c_u8p, c_u8p]),
        "hsv_verify_batch": (ctypes.c_int, [c_u8p, c_u8p, c_u8p, sz]),
        "hsv_verify_batch_packed": (ctypes.c_int, [c_u8p, c_u8p, sz]),
        "hsv_verify_device": (ctypes.c_int, [c_u8p, sz, c_u8p, sz, c_u8p, sz, sz, c_u8p, ctypes.c_void_p]),
        "hsv_verify_device_bits": (ctypes.c_int, [c_u8p, sz, c_u8p, sz, c_u8p, sz, sz, c_u8p, c_u8p,
                                                  ctypes.c_void_p, ctypes.c_void_p]),
        "hsv_verify_transactions": (ctypes.c_int, [c_u8p, c_u8p, sz, c_u8p]),
        "hsv_verify_transactions_fixed": (ctypes.c_int, [c_u8p, sz, sz, c_u8p]),
        "hsv_verify_transactions_device": (ctypes.c_int, [c_u8p, c_u8p, sz, sz, c_u8p, c_u8p, ctypes.c_void_p,
                                                          ctypes.c_void_p]),
        "hsv_qc_verify_bincode": (ctypes.c_int, [c_u8p, sz, ctypes.POINTER(ctypes.c_size_t), c_u8p]),
        "hsv_tc_verify_bincode": (ctypes.c_int, [c_u8p, sz, ctypes.POINTER(ctypes.c_size_t), c_u8p]),
        "hsv_set_auto_committee": (ctypes.c_int, [ctypes.c_int]),
        "hsv_set_resident_service": (ctypes.c_int, [ctypes.c_int]),
        "hsv_auto_committee_size": (sz, []),
        "hsv_public_key": (ctypes.c_int, [c_u8p, c_u8p]),
        "hsv_sign": (ctypes.c_int, [c_u8p, c_u8p, sz, c_u8p]),
        "hsv_sign_many": (ctypes.c_int, [c_u8p, c_u8p, sz, sz, c_u8p, c_u8p, ctypes.c_int]),
        "hsv_measure_mad_peak": (ctypes.c_double, []),
        "hsv_committee_create": (ctypes.c_int, [c_u8p, sz, ctypes.POINTER(ctypes.c_void_p)]),
        "hsv_committee_destroy": (None, [ctypes.c_void_p]),
        "hsv_committee_size": (sz, [ctypes.c_void_p]),
        "hsv_committee_index": (ctypes.c_int64, [ctypes.c_void_p, c_u8p]),
        "hsv_committee_verify": (ctypes.c_int, [ctypes.c_void_p, c_u8p, c_u8p, c_u8p, sz, sz, c_u8p]),
        "hsv_committee_verify_batch_packed": (ctypes.c_int, [ctypes.c_void_p, c_u8p, c_u8p, sz]),
        "hsv_committee_verify_device": (ctypes.c_int, [ctypes.c_void_p, c_u8p, c_u8p, sz, c_u8p, sz, sz, c_u8p,
                                                       ctypes.c_void_p, ctypes.c_void_p]),
        "hsv_set_variant": (ctypes.c_int, [ctypes.c_int]),
        "hsv_get_variant": (ctypes.c_int, []),
        "hsv_set_lattice_bits": (ctypes.c_int, [ctypes.c_int]),
        "hsv_num_variants": (ctypes.c_int, []),
        "hsv_device_faults": (ctypes.c_int, [ctypes.c_int, ctypes.c_int]),
        "hsv_test_inject_fault": (ctypes.c_int, [ctypes.c_int]),
        "hsv_test_inject_mode": (ctypes.c_int, []),
        "hsv_test_corrupt_auto_committee": (ctypes.c_int, []),
        "hsv_test_lanesplit_check": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p]),
        "hsv_host_call_stats": (None, [ctypes.POINTER(ctypes.c_double)] * 3),
        "hsv_host_call_marks": (ctypes.c_int, [ctypes.POINTER(ctypes.c_double), ctypes.c_int]),
        "hsv_pack_threads": (ctypes.c_int, []),
        "hsv_sign_mixed_order": (ctypes.c_int, [c_u8p, c_u8p, sz, ctypes.c_int, ctypes.c_int, c_u8p, c_u8p]),
    }
    # hooks (libhsv_test.so only) and entry points absent from older A/B builds (tools/ab_probe.py)
    optional = set(HOOKS) | {"hsv_host_call_stats", "hsv_host_call_marks", "hsv_pack_threads", "hsv_device_faults",
                             "hsv_sign_mixed_order", "hsv_auto_committee_faults"}
    for name, (res, args) in sig.items():
        fn = getattr(lib, name, None) if name in optional else getattr(lib, name)
        if fn is None:
            continue
        fn.restype = res
        fn.argtypes = args


def _open(path, require):
    if not os.path.exists(path):
        if require:
            raise HsvLibraryError(
                f"{path} not built: run `make` in {os.path.dirname(_HERE)} "
                "or __graft_entry__.build(); there is no CPU fallback")
        return None
    if os.environ.get("HSV_NO_TORCH") != "1":
        try:
            import torch  # noqa: F401  (share torch's HIP runtime)
        except Exception:  # pragma: no cover - torch absent is fine
            pass
    # RTLD_LOCAL: libhsv.so and libhsv_test.so export the same names and may
    # both be loaded (two independent instances); neither may bind the other's.
    lib = ctypes.CDLL(path, mode=ctypes.RTLD_LOCAL)
    _declare(lib)
    return lib


def load(require: bool = True):
    """Return the library hsverify calls go to (cached): LIB_PATH, or
    libhsv_test.so inside hsverify._testing.test_library().  Raises
    HsvLibraryError if absent."""
    global _lib
    with _lock:
        if _override is not None:
            return _override
        if _lib is None:
            _lib = _open(LIB_PATH, require)
        return _lib


def load_test():
    """libhsv_test.so: the product's objects plus the exported test hooks.  If
    the library already loaded exports them (HSV_LIB=libhsv_test.so), that
    instance is returned instead of a second one."""
    global _test_lib
    main = load()
    if getattr(main, "hsv_test_inject_fault", None) is not None:
        return main
    with _lock:
        if _test_lib is None:
            _test_lib = _open(TEST_LIB_PATH, True)
        return _test_lib


def set_override(lib):
    """Route every hsverify call to `lib` (None: back to LIB_PATH); returns the
    previous override.  Used by hsverify._testing.test_library()."""
    global _override
    with _lock:
        prev, _override = _override, lib
        return prev


def hook(name: str):
    """A test / measurement hook of the library in use; raises when it is the
    product library, which exports none (csrc/hsv_test_hooks.h)."""
    fn = getattr(load(), name, None)
    if fn is None:
        raise HsvLibraryError(f"{name} is a test hook: libhsv.so does not export it; run inside "
                              "hsverify._testing.test_library() (libhsv_test.so)")
    return fn


def check(rc: int, what: str) -> int:
    if rc < 0:
        lib = load()
        msg = lib.hsv_last_error().decode(errors="replace")
        raise HsvLibraryError(f"{what}: {ERRORS.get(rc, rc)}: {msg}")
    return rc


def last_error() -> str:
    return load().hsv_last_error().decode(errors="replace")


def device_count() -> int:
    return load().hsv_device_count()


def version() -> str:
    return load().hsv_version().decode()
