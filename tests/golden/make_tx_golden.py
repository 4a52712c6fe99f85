#!/usr/bin/env python3
"""Golden vectors for mempool transaction verification.

Transaction layout and check follow the reference's transaction path
(mempool/src/batch_maker.rs:79-85, consensus/src/core.rs:121-127):
    tx = message || pk (32) || sig (64, R || s)
    accept  <=>  Signature::verify(Digest(SHA-512(message)[..32]), pk)
Expected flags come from oracle/ed25519_ref.py (verify_flags over the 32-byte
digest); every STRICT_OK bit is cross-checked against libsodium's
crypto_sign_verify_detached when it is present, and the generator aborts on a
disagreement.

Output: tx_vectors.json = {"vectors": [{"case", "tx" (hex), "flags"}]}.
Message lengths cover every SHA-512 padding boundary (111/112 bytes: one vs
two blocks) and the reference benchmark's 512-byte transactions (416-byte
message, benchmark/fabfile.py 'tx_size': 512).

Run from the repo root:  python tests/golden/make_tx_golden.py
"""
import hashlib
import json
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.abspath(os.path.join(HERE, "..", ".."))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, HERE)
import ed25519_ref as o  # noqa: E402
from make_golden import load_sodium, seed_bytes, sodium_verify  # noqa: E402

MLENS = [0, 1, 7, 8, 9, 31, 32, 33, 64, 100, 110, 111, 112, 113, 127, 128, 129, 200, 238, 239, 240, 241,
         255, 256, 257, 416, 600, 1000]


def digest(message: bytes) -> bytes:
    return hashlib.sha512(message).digest()[:32]


def main():
    rnd = random.Random(85)
    sodium = load_sodium()
    vecs = []

    def add(case, message, pk, sig):
        tx = message + pk + sig
        f = o.verify_flags(pk, sig, digest(message))
        if sodium is not None and bool(f & 1) != sodium_verify(sodium, pk, sig, digest(message)):
            raise SystemExit(f"libsodium disagrees with the oracle on {case}")
        vecs.append({"case": case, "tx": tx.hex(), "flags": f})

    for j, mlen in enumerate(MLENS):
        seed = seed_bytes(5000 + j, b"hsv-tx")
        pk = o.public_key(seed)
        message = rnd.randbytes(mlen)
        sig = o.sign(seed, digest(message))
        add(f"honest_m{mlen}", message, pk, sig)
    seed = seed_bytes(6000, b"hsv-tx")
    pk = o.public_key(seed)
    message = rnd.randbytes(416)
    sig = o.sign(seed, digest(message))
    for pos in (0, 1, 111, 112, 415):
        m2 = bytearray(message); m2[pos] ^= 0x01
        add(f"flip_message_byte{pos}", bytes(m2), pk, sig)
    add("message_truncated", message[:-1], pk, sig)
    add("message_extended", message + b"\x00", pk, sig)
    for bit in (0, 200):
        p2 = bytearray(pk); p2[bit // 8] ^= 1 << (bit % 8)
        add(f"flip_pk_bit{bit}", message, bytes(p2), sig)
    for bit in (3, 250):
        s2 = bytearray(sig); s2[bit // 8] ^= 1 << (bit % 8)
        add(f"flip_R_bit{bit}", message, pk, bytes(s2))
    for bit in (0, 255):
        s2 = bytearray(sig); s2[32 + bit // 8] ^= 1 << (bit % 8)
        add(f"flip_s_bit{bit}", message, pk, bytes(s2))
    s_int = int.from_bytes(sig[32:], "little")
    add("s_plus_l", message, pk, sig[:32] + (s_int + o.L).to_bytes(32, "little"))
    # signed over the message itself / the full 64-byte hash instead of the digest
    add("signed_raw_message", message, pk, o.sign(seed, message))
    add("signed_full_sha512", message, pk, o.sign(seed, hashlib.sha512(message).digest()))
    # small-order key and R (identity) with an otherwise valid-looking signature
    ident = (1).to_bytes(32, "little")
    add("small_order_pk", message, ident, sig)
    add("small_order_R", message, pk, ident + sig[32:])
    add("all_zero_tx", bytes(100), bytes(32), bytes(64))
    out = os.path.join(HERE, "tx_vectors.json")
    with open(out, "w") as f:
        json.dump({"source": "tests/golden/make_tx_golden.py", "vectors": vecs}, f, indent=0)
    print(f"wrote {len(vecs)} transaction vectors to {out} (libsodium cross-check: {sodium is not None})")


if __name__ == "__main__":
    main()
