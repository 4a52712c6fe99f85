"""Mempool transaction-signature verification.

The reference's client transactions are ``message || pk (32 B) || sig (64 B)``
and the check it carries (commented out in the shipped code) is, per
transaction (``mempool/src/batch_maker.rs:79-85``)::

    message   = tx[..len-96]
    digest    = Digest(SHA-512(message)[..32])
    signature = Signature::from_bytes(sig[..32], sig[32..64])
    signature.verify(&digest, &PublicKey(pk)).is_ok()

``BatchMaker::run`` keeps only transactions that pass; ``Core::make_vote``
(``consensus/src/core.rs:121-131``) refuses to vote for a block whose batch
holds any transaction that fails.  Those two call shapes are
:func:`filter_transactions` and :func:`verify_batch_transactions` below, over
the GPU path (``hsv_verify_transactions*`` in ``include/hsv.h``): digests are
computed on the device by ``hsv_tx_record_kernel``, then verified by the
generic verification kernels.  There is no CPU fallback.
"""
from __future__ import annotations

import ctypes
from typing import Iterable, List, Sequence

import numpy as np

from . import _lib

TX_OVERHEAD = 96  # pk (32) || signature (64) at the end of every transaction


def _ptr(a: np.ndarray):
    return ctypes.c_void_p(a.ctypes.data)


def make_transaction(message: bytes, pk: bytes, sig: bytes) -> bytes:
    """Client-side layout: message || pk || part1 (R) || part2 (s)."""
    if len(pk) != 32 or len(sig) != 64:
        raise ValueError("pk must be 32 bytes and sig 64 bytes")
    return bytes(message) + bytes(pk) + bytes(sig)


def pack(txs: Sequence[bytes]):
    """Ragged list of transactions -> (concatenated u8 buffer, n+1 u64 offsets)."""
    lens = np.fromiter((len(t) for t in txs), dtype=np.uint64, count=len(txs))
    offsets = np.zeros(len(txs) + 1, dtype=np.uint64)
    np.cumsum(lens, out=offsets[1:])
    buf = np.frombuffer(b"".join(txs), dtype=np.uint8) if txs else np.zeros(0, np.uint8)
    return np.ascontiguousarray(buf), offsets


def verify_transactions(txs: Sequence[bytes]) -> np.ndarray:
    """Per-transaction flag bytes (``HSV_*`` bits; STRICT_OK = the reference's
    ``verify(..).is_ok()``).  Raises HsvLibraryError for a transaction shorter
    than 96 bytes, where the reference's slice would panic."""
    n = len(txs)
    out = np.zeros(n, dtype=np.uint8)
    if n == 0:
        return out
    buf, offsets = pack(txs)
    lib = _lib.load()
    _lib.check(lib.hsv_verify_transactions(_ptr(buf), _ptr(offsets), n, _ptr(out)), "hsv_verify_transactions")
    return out


def verify_transactions_fixed(txs: np.ndarray) -> np.ndarray:
    """(n, tx_size) u8 array of equal-size transactions -> (n,) flag bytes."""
    txs = np.ascontiguousarray(txs, dtype=np.uint8)
    if txs.ndim != 2:
        raise ValueError("expected an (n, tx_size) array")
    n, size = txs.shape
    out = np.zeros(n, dtype=np.uint8)
    if n == 0:
        return out
    lib = _lib.load()
    _lib.check(lib.hsv_verify_transactions_fixed(_ptr(txs), size, n, _ptr(out)), "hsv_verify_transactions_fixed")
    return out


def verify_transactions_device(txs, offsets=None, tx_size: int = 0, n: int | None = None, flags=None,
                               strict_bits=None, stream=None, fault=None) -> None:
    """Enqueue verification of device-resident transactions (torch uint8 tensor
    ``txs``; ``offsets`` an int64 tensor of n+1 byte offsets, or None with
    ``tx_size`` for fixed-size transactions).  Outputs: ``flags`` (n,) uint8
    and/or ``strict_bits`` (ceil(n/32),) int32; ``fault`` optional per-call
    fault words (verifier.verify_device).  No synchronisation."""
    from .verifier import _fault_ptr
    import torch

    if n is None:
        n = offsets.numel() - 1 if offsets is not None else txs.numel() // tx_size
    if stream is None:
        stream = torch.cuda.current_stream(txs.device).cuda_stream
    lib = _lib.load()
    rc = lib.hsv_verify_transactions_device(
        ctypes.c_void_p(txs.data_ptr()), ctypes.c_void_p(offsets.data_ptr()) if offsets is not None else None,
        tx_size, n, ctypes.c_void_p(flags.data_ptr()) if flags is not None else None,
        ctypes.c_void_p(strict_bits.data_ptr()) if strict_bits is not None else None, _fault_ptr(fault),
        ctypes.c_void_p(stream))
    _lib.check(rc, "hsv_verify_transactions_device")


def filter_transactions(txs: Sequence[bytes]) -> List[bytes]:
    """``BatchMaker::run`` with the check enabled (batch_maker.rs:79-97): the
    transactions whose signature verifies, in order."""
    flags = verify_transactions(txs)
    return [t for t, f in zip(txs, flags) if f & _lib.STRICT_OK]


def verify_batch_transactions(txs: Iterable[bytes]) -> bool:
    """``Core::make_vote`` batch re-check (core.rs:121-131): True iff every
    transaction of the batch verifies (an empty batch passes)."""
    txs = list(txs)
    if not txs:
        return True
    return bool((verify_transactions(txs) & _lib.STRICT_OK).all())
