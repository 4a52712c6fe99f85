"""Wire formats: QC / TC certificates as bincode bytes.

Encoders restate bincode 1.3's default encoding of the reference's serde
derives (little-endian fixed-width integers, u64 length prefixes; PublicKey
serialises as its base64 string, crypto/src/lib.rs:94-101):

    QC = hash (32) | round u64 | votes: u64 n, n x (PublicKey str, R (32), s (32))
                                                  consensus/src/messages.rs:162-167
    TC = round u64 | votes: u64 n, n x (PublicKey str, R, s, high_qc_round u64)
                                                  consensus/src/messages.rs:281-285

:func:`qc_verify` / :func:`tc_verify` hand the bytes to
``hsv_qc_verify_bincode`` / ``hsv_tc_verify_bincode``, which parse them in C++
and verify on the GPU (QC: ``verify_batch`` over ``qc.digest()``; TC: one
strict verification per vote over SHA-512(round_le || high_qc_round_le)[..32]).
"""
from __future__ import annotations

import base64
import ctypes
import struct
from typing import Sequence, Tuple

import numpy as np

from . import _lib


def _str(s: bytes) -> bytes:
    return struct.pack("<Q", len(s)) + s


def encode_public_key(pk: bytes) -> bytes:
    """bincode of PublicKey: its base64 (standard, padded) string."""
    return _str(base64.b64encode(bytes(pk)))


def encode_qc(block_hash: bytes, round_: int, votes: Sequence[Tuple[bytes, bytes]]) -> bytes:
    """bincode of consensus::QC{hash, round, votes: [(pk, sig R||s)]}."""
    out = [bytes(block_hash), struct.pack("<QQ", round_, len(votes))]
    for pk, sig in votes:
        out.append(encode_public_key(pk))
        out.append(bytes(sig))
    return b"".join(out)


def encode_tc(round_: int, votes: Sequence[Tuple[bytes, bytes, int]]) -> bytes:
    """bincode of consensus::TC{round, votes: [(pk, sig, high_qc_round)]}."""
    out = [struct.pack("<QQ", round_, len(votes))]
    for pk, sig, hqc in votes:
        out.append(encode_public_key(pk))
        out.append(bytes(sig))
        out.append(struct.pack("<Q", hqc))
    return b"".join(out)


def qc_verify(buf: bytes):
    """-> (ok: bool, decoded public keys (n, 32) u8).  Raises HsvLibraryError on
    malformed bytes (HSV_ERR_PARSE) or an infrastructure error."""
    lib = _lib.load()
    n = ctypes.c_size_t(0)
    # keys are written only after a successful parse; size the buffer generously
    pks = np.zeros((max(1, len(buf) // 115), 32), np.uint8)
    rc = _lib.check(lib.hsv_qc_verify_bincode(buf, len(buf), ctypes.byref(n), ctypes.c_void_p(pks.ctypes.data)),
                    "hsv_qc_verify_bincode")
    return rc == 1, pks[: n.value]


def tc_verify(buf: bytes):
    """-> (ok: bool, per-vote flag bytes)."""
    lib = _lib.load()
    n = ctypes.c_size_t(0)
    flags = np.zeros(max(1, len(buf) // 123), np.uint8)
    rc = _lib.check(lib.hsv_tc_verify_bincode(buf, len(buf), ctypes.byref(n), ctypes.c_void_p(flags.ctypes.data)),
                    "hsv_tc_verify_bincode")
    return rc == 1, flags[: n.value]
