"""Committee key cache over the C ABI.

A HotStuff committee's keys are fixed per epoch (reference
consensus/src/config.rs: Committee, looked up by stake(name) in
QC::verify / TC::verify, consensus/src/messages.rs:186,296).  ``Committee``
builds a 384 KiB fixed-base comb table of -A per key in HBM once; votes by
members are then verified with 64 mixed additions and no doublings.  Results
are bit-identical to the generic path (same flag byte per vote).
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib


def _ptr(a: np.ndarray):
    return ctypes.c_void_p(a.ctypes.data)


class Committee:
    def __init__(self, public_keys):
        keys = [k.data if hasattr(k, "data") and isinstance(k.data, bytes) else bytes(k) for k in public_keys] \
            if not isinstance(public_keys, np.ndarray) else None
        arr = np.ascontiguousarray(public_keys, np.uint8).reshape(-1, 32) if keys is None else \
            np.frombuffer(b"".join(keys), np.uint8).reshape(-1, 32).copy()
        self._lib = _lib.load()
        self._h = ctypes.c_void_p()
        _lib.check(self._lib.hsv_committee_create(_ptr(arr) if arr.size else None, arr.shape[0],
                                                  ctypes.byref(self._h)), "hsv_committee_create")
        self._n = arr.shape[0]

    def __len__(self) -> int:
        return self._n

    def index(self, pk) -> int:
        b = pk.data if hasattr(pk, "data") and isinstance(pk.data, bytes) else bytes(pk)
        return int(self._lib.hsv_committee_index(self._h, ctypes.c_char_p(b)))

    def verify_flags(self, key_idx, sig, msg) -> np.ndarray:
        """key_idx (m,) member indices, sig (m,64), msg (m,32) or (32,) -> flags (m,)."""
        idx = np.ascontiguousarray(key_idx, np.uint32).reshape(-1)
        sig = np.ascontiguousarray(sig, np.uint8).reshape(-1, 64)
        msg = np.ascontiguousarray(msg, np.uint8)
        m = idx.size
        stride = 0 if (msg.ndim == 1 and msg.size == 32) else 32
        out = np.zeros(m, np.uint8)
        if m:
            _lib.check(self._lib.hsv_committee_verify(self._h, _ptr(idx), _ptr(sig), _ptr(msg), stride, m, _ptr(out)),
                       "hsv_committee_verify")
        return out

    def verify_batch(self, digest, votes):
        """crypto::Signature::verify_batch for votes by (mostly) members -> crypto.Result."""
        from .crypto import OK, CryptoError, Result
        votes = list(votes)
        packed = b"".join(pk.data + sig.flatten() for pk, sig in votes)
        d = digest.data if hasattr(digest, "data") else bytes(digest)
        rc = _lib.check(self._lib.hsv_committee_verify_batch_packed(
            self._h, ctypes.c_char_p(d), ctypes.c_char_p(packed) if packed else None, len(votes)),
            "hsv_committee_verify_batch_packed")
        return OK if rc == 1 else Result(CryptoError("signature error"))

    def verify_device(self, key_idx, sig, msg, flags, stream=None, fault=None) -> None:
        """Device tensors: key_idx (m,) int32, sig (m,64) u8, msg (m,32) or (32,), flags (m,) u8;
        fault: optional per-call fault words (verifier.verify_device)."""
        from .verifier import _fault_ptr
        import torch
        m = key_idx.shape[0]
        if stream is None:
            stream = torch.cuda.current_stream(sig.device).cuda_stream
        rc = self._lib.hsv_committee_verify_device(
            self._h, ctypes.c_void_p(key_idx.data_ptr()), ctypes.c_void_p(sig.data_ptr()), sig.stride(0),
            ctypes.c_void_p(msg.data_ptr()), 0 if msg.dim() == 1 else msg.stride(0), m,
            ctypes.c_void_p(flags.data_ptr()), _fault_ptr(fault), ctypes.c_void_p(stream))
        _lib.check(rc, "hsv_committee_verify_device")

    def close(self) -> None:
        if self._h:
            self._lib.hsv_committee_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
