"""Python mirror of the reference's ``crypto`` crate (crypto/src/lib.rs).

Same type names, byte layouts, argument meaning and error behaviour as the
Rust API, so the parity tests read like the reference's own tests
(crypto/src/tests/crypto_tests.rs).  Verification goes through the C ABI of
libhsv.so onto the GPU; signing is host code in the same library (as in the
reference, where signing is CPU dalek).

Rust -> Python:
  Result<(), CryptoError>          -> Result (is_ok / is_err / unwrap)
  Digest(pub [u8;32])              -> Digest(bytes)            lib.rs:22
  PublicKey(pub [u8;32])           -> PublicKey(bytes)         lib.rs:66
  SecretKey([u8;64])               -> SecretKey(bytes)         lib.rs:121
  Signature{part1, part2}          -> Signature(part1, part2)  lib.rs:179-182
  Signature::verify                -> Signature.verify         lib.rs:204-208
  Signature::verify_batch          -> Signature.verify_batch   lib.rs:210-223
  generate_keypair(csprng)         -> generate_keypair(rng)    lib.rs:167-175
  SignatureService                 -> SignatureService (asyncio) lib.rs:229-254
"""
from __future__ import annotations

import asyncio
import base64
import ctypes
import os
from typing import Iterable, Tuple

from . import _lib


class CryptoError(Exception):
    """``ed25519::Error`` -- opaque, as in the reference (lib.rs:18)."""


class Result:
    """``Result<(), CryptoError>``."""

    __slots__ = ("_err",)

    def __init__(self, err: CryptoError | None = None):
        self._err = err

    def is_ok(self) -> bool:
        return self._err is None

    def is_err(self) -> bool:
        return self._err is not None

    def unwrap(self) -> None:
        if self._err is not None:
            raise self._err

    def __repr__(self) -> str:
        return "Ok(())" if self._err is None else f"Err({self._err})"


OK = Result()


def _buf(b: bytes):
    return ctypes.c_char_p(b)


class Digest:
    __slots__ = ("data",)

    def __init__(self, data: bytes = bytes(32)):
        data = bytes(data)
        if len(data) != 32:
            raise ValueError("Digest is 32 bytes")
        self.data = data

    def to_vec(self) -> bytes:
        return self.data

    def size(self) -> int:
        return 32

    def __eq__(self, other) -> bool:
        return isinstance(other, Digest) and other.data == self.data

    def __hash__(self) -> int:
        return hash(self.data)

    def __repr__(self) -> str:
        return base64.b64encode(self.data).decode()


class PublicKey:
    __slots__ = ("data",)

    def __init__(self, data: bytes = bytes(32)):
        data = bytes(data)
        if len(data) != 32:
            raise ValueError("PublicKey is 32 bytes")
        self.data = data

    def encode_base64(self) -> str:
        return base64.b64encode(self.data).decode()

    @classmethod
    def decode_base64(cls, s: str) -> "PublicKey":
        raw = base64.b64decode(s)
        if len(raw) < 32:
            raise ValueError("InvalidLength")
        return cls(raw[:32])

    def __eq__(self, other) -> bool:
        return isinstance(other, PublicKey) and other.data == self.data

    def __hash__(self) -> int:
        return hash(self.data)

    def __repr__(self) -> str:
        return self.encode_base64()


class SecretKey:
    """64 bytes: secret seed (32) || public key (32), dalek Keypair::to_bytes."""

    __slots__ = ("data",)

    def __init__(self, data: bytes):
        data = bytes(data)
        if len(data) != 64:
            raise ValueError("SecretKey is 64 bytes")
        self.data = data

    def encode_base64(self) -> str:
        return base64.b64encode(self.data).decode()

    @classmethod
    def decode_base64(cls, s: str) -> "SecretKey":
        raw = base64.b64decode(s)
        if len(raw) < 64:
            raise ValueError("InvalidLength")
        return cls(raw[:64])

    def __eq__(self, other) -> bool:
        return isinstance(other, SecretKey) and other.data == self.data


def public_key_from_seed(seed: bytes) -> PublicKey:
    lib = _lib.load()
    out = ctypes.create_string_buffer(32)
    _lib.check(lib.hsv_public_key(_buf(bytes(seed)), out), "hsv_public_key")
    return PublicKey(out.raw)


def generate_keypair(rng) -> Tuple[PublicKey, SecretKey]:
    """``generate_keypair(csprng)``: 32 secret bytes from ``rng`` (anything with
    ``fill_bytes(n)``, ``randbytes(n)`` or a callable ``rng(n)``)."""
    if hasattr(rng, "fill_bytes"):
        seed = bytes(rng.fill_bytes(32))
    elif hasattr(rng, "randbytes"):
        seed = rng.randbytes(32)
    else:
        seed = bytes(rng(32))
    pk = public_key_from_seed(seed)
    return pk, SecretKey(seed + pk.data)


def generate_production_keypair() -> Tuple[PublicKey, SecretKey]:
    return generate_keypair(os.urandom)


class Signature:
    __slots__ = ("part1", "part2")

    def __init__(self, part1: bytes = bytes(32), part2: bytes = bytes(32)):
        self.part1 = bytes(part1)
        self.part2 = bytes(part2)
        if len(self.part1) != 32 or len(self.part2) != 32:
            raise ValueError("Unexpected signature length")

    @classmethod
    def default(cls) -> "Signature":
        """``Signature::default()``: 64 zero bytes."""
        return cls()

    @classmethod
    def new(cls, digest: Digest, secret: SecretKey) -> "Signature":
        """``Signature::new`` (lib.rs:185-191): RFC 8032 over ``digest.0``."""
        lib = _lib.load()
        out = ctypes.create_string_buffer(64)
        _lib.check(lib.hsv_sign(_buf(secret.data[:32]), _buf(digest.data), 32, out), "hsv_sign")
        return cls(out.raw[:32], out.raw[32:])

    @classmethod
    def from_bytes(cls, part1: bytes, part2: bytes) -> "Signature":
        return cls(part1, part2)

    def flatten(self) -> bytes:
        return self.part1 + self.part2

    def verify(self, digest: Digest, public_key: PublicKey) -> Result:
        """``Signature::verify`` (lib.rs:204-208): ed25519-dalek verify_strict semantics."""
        lib = _lib.load()
        rc = _lib.check(lib.hsv_verify_strict(_buf(digest.data), _buf(public_key.data),
                                              _buf(self.flatten())), "hsv_verify_strict")
        return OK if rc == 1 else Result(CryptoError("signature error"))

    @staticmethod
    def verify_batch(digest: Digest, votes: Iterable[Tuple[PublicKey, "Signature"]]) -> Result:
        """``Signature::verify_batch`` (lib.rs:210-223): all votes over one digest."""
        votes = list(votes)
        packed = b"".join(pk.data + sig.flatten() for pk, sig in votes)
        lib = _lib.load()
        rc = _lib.check(lib.hsv_verify_batch_packed(_buf(digest.data), _buf(packed) if packed else None,
                                                    len(votes)), "hsv_verify_batch_packed")
        return OK if rc == 1 else Result(CryptoError("signature error"))

    @staticmethod
    def verify_many(items: Iterable[Tuple[Digest, PublicKey, "Signature"]]) -> list:
        """Batched strict API: per-item verify_strict results."""
        items = list(items)
        if not items:
            return []
        lib = _lib.load()
        pk = b"".join(p.data for _, p, _ in items)
        sg = b"".join(s.flatten() for _, _, s in items)
        mg = b"".join(d.data for d, _, _ in items)
        out = ctypes.create_string_buffer(len(items))
        _lib.check(lib.hsv_verify(_buf(pk), _buf(sg), _buf(mg), 32, len(items), out), "hsv_verify")
        return [bool(b & _lib.STRICT_OK) for b in out.raw]

    def __repr__(self) -> str:
        return f"Signature({self.part1.hex()}, {self.part2.hex()})"


class SignatureService:
    """``SignatureService`` (lib.rs:229-254): a task that owns the secret key and
    answers signature requests over a channel (asyncio instead of tokio)."""

    def __init__(self, secret: SecretKey):
        self._secret = secret
        self._queue: asyncio.Queue = asyncio.Queue(100)
        self._task = asyncio.get_event_loop().create_task(self._run())

    async def _run(self):
        while True:
            digest, fut = await self._queue.get()
            if not fut.done():
                fut.set_result(Signature.new(digest, self._secret))

    async def close(self) -> None:
        self._task.cancel()
        try:
            await self._task
        except asyncio.CancelledError:
            pass

    async def request_signature(self, digest: Digest) -> Signature:
        fut = asyncio.get_event_loop().create_future()
        await self._queue.put((digest, fut))
        return await fut
