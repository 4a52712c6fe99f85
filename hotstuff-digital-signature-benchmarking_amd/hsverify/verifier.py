"""Array-level entry points over the C ABI (throughput path).

* :func:`verify_flags`   host numpy arrays -> per-item flag bytes (hsv_verify)
* :func:`verify_device`  device-resident torch tensors, stream-ordered
                          (hsv_verify_device[_bits]); no synchronisation
* :func:`sign_many`      bulk RFC 8032 signing on host threads (input synthesis)

Record layout is the reference's byte layout: pk 32 B, sig 64 B (R || s),
msg 32 B (a consensus Digest).
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib


def _ptr(a: np.ndarray):
    return ctypes.c_void_p(a.ctypes.data)


def verify_flags(pk: np.ndarray, sig: np.ndarray, msg: np.ndarray) -> np.ndarray:
    """pk (n,32) u8, sig (n,64) u8, msg (n,32) u8 or (32,) shared -> flags (n,) u8."""
    pk = np.ascontiguousarray(pk, dtype=np.uint8).reshape(-1, 32)
    sig = np.ascontiguousarray(sig, dtype=np.uint8).reshape(-1, 64)
    n = pk.shape[0]
    if sig.shape[0] != n:
        raise ValueError("pk/sig length mismatch")
    msg = np.ascontiguousarray(msg, dtype=np.uint8)
    if msg.size == 32 and (msg.ndim == 1 or n != 1):
        stride = 0
    else:
        msg = msg.reshape(-1, 32)
        if msg.shape[0] != n:
            raise ValueError("msg length mismatch")
        stride = 32
    out = np.zeros(n, dtype=np.uint8)
    if n == 0:
        return out
    lib = _lib.load()
    _lib.check(lib.hsv_verify(_ptr(pk), _ptr(sig), _ptr(msg), stride, n, _ptr(out)), "hsv_verify")
    return out


def verify_device(pk, sig, msg, flags=None, strict_bits=None, stream=None, fault=None) -> None:
    """Enqueue verification of device tensors (uint8, contiguous rows).

    pk: (n,32), sig: (n,64), msg: (n,32) or (32,) shared; flags: (n,) uint8
    and/or strict_bits: (ceil(n/32),) int32 outputs.  ``stream`` is a raw
    hipStream_t handle (int) -- default: torch's current stream.  ``fault``
    (optional): an int32 device tensor of >= 2 words owned by this call; the
    library zeroes it on the stream and the kernels set it on a self-check
    failure (read it with :func:`fault_bits` after synchronising).  Without
    it the launches report into the per-device word (:func:`device_faults`).
    """
    import torch

    n = pk.shape[0]
    for t in (sig, msg, flags, strict_bits, fault):
        if t is not None and t.device != pk.device:
            raise ValueError(f"all tensors must live on {pk.device}, got {t.device}")
    with torch.cuda.device(pk.device):  # the library launches on the inputs' device
        if stream is None:
            stream = torch.cuda.current_stream(pk.device).cuda_stream
        msg_stride = 0 if msg.dim() == 1 else msg.stride(0)
        lib = _lib.load()
        rc = lib.hsv_verify_device_bits(
            ctypes.c_void_p(pk.data_ptr()), pk.stride(0), ctypes.c_void_p(sig.data_ptr()), sig.stride(0),
            ctypes.c_void_p(msg.data_ptr()), msg_stride, n,
            ctypes.c_void_p(flags.data_ptr()) if flags is not None else None,
            ctypes.c_void_p(strict_bits.data_ptr()) if strict_bits is not None else None,
            _fault_ptr(fault), ctypes.c_void_p(stream))
    _lib.check(rc, "hsv_verify_device_bits")


def _fault_ptr(fault):
    if fault is None:
        return None
    if fault.numel() * fault.element_size() < 8:
        raise ValueError("a fault tensor needs two 32-bit words")
    return ctypes.c_void_p(fault.data_ptr())


def fault_bits(fault) -> int:
    """Bits of a call's own fault words (after synchronising its stream):
    1 = a final point failed the curve check, 2 = a workspace canary changed."""
    w = fault.view(-1)[:2].cpu().tolist()
    return (1 if w[0] else 0) | (2 if w[1] else 0)


def device_faults(device: int = -1, clear: bool = True) -> int:
    """Self-check results of the device-resident calls (hsv_device_faults):
    0, or fault bits (1: a final point failed the curve check, 2: a workspace
    canary changed).  Call after synchronising the streams the calls ran on."""
    return _lib.check(_lib.load().hsv_device_faults(device, 1 if clear else 0), "hsv_device_faults")


def check_device_faults(device: int = -1) -> None:
    """Raise HsvLibraryError (HSV_ERR_DEVICE_FAULT) if the device-resident calls
    since the last check tripped a self-check; clears the record."""
    bits = device_faults(device, True)
    if bits:
        raise _lib.HsvLibraryError(f"HSV_ERR_DEVICE_FAULT: device self-check bits {bits:#x}: "
                                   "the flags of those launches are not a verdict")


def sign_many(seeds: np.ndarray, msgs: np.ndarray, nthreads: int = 0):
    """seeds (n,32), msgs (n,L) -> (pk (n,32), sig (n,64)) via host threads."""
    seeds = np.ascontiguousarray(seeds, dtype=np.uint8).reshape(-1, 32)
    n = seeds.shape[0]
    msgs = np.ascontiguousarray(msgs, dtype=np.uint8).reshape(n, -1)
    pk = np.zeros((n, 32), dtype=np.uint8)
    sig = np.zeros((n, 64), dtype=np.uint8)
    if n:
        lib = _lib.load()
        _lib.check(lib.hsv_sign_many(_ptr(seeds), _ptr(msgs), msgs.shape[1], n, _ptr(pk), _ptr(sig),
                                     nthreads), "hsv_sign_many")
    return pk, sig


def measure_mad_peak() -> float:
    """Measured v_mad_u64_u32 rate of the current device (MAC/s)."""
    return float(_lib.load().hsv_measure_mad_peak())


def set_variant(v: int) -> None:
    """Test/measurement hook (libhsv_test.so only)."""
    _lib.check(_lib.hook("hsv_set_variant")(v), "hsv_set_variant")


def get_variant() -> int:
    return _lib.load().hsv_get_variant()


def num_variants() -> int:
    """Size of the variant id space (not all ids are built: see variants())."""
    return _lib.hook("hsv_num_variants")()


def variants() -> list:
    """Kernel variant ids built into the loaded library (product build: 19, 21)."""
    fn = _lib.hook("hsv_variant_list")
    n = fn(None, 0)
    buf = (ctypes.c_int * n)()
    fn(buf, n)
    return list(buf)


def bind_device(device: int) -> int:
    """hsv_init: -1 = every visible GPU (large host batches sharded), d >= 0 = GPU d only."""
    return _lib.check(_lib.load().hsv_init(device), "hsv_init")


def set_virtual_shards(k: int) -> None:
    """Test hook: split host batches of >= 2^16 items into k shards (0 = default)."""
    _lib.check(_lib.hook("hsv_set_virtual_shards")(k), "hsv_set_virtual_shards")
