"""Pure-Python restatement of the reference's Ed25519 acceptance rules.

Parity status: UNPINNED.  The reference holds no known-answer vectors for this
path and ed25519-dalek cannot be built here; the restatement is cross-checked
against RFC 8032 section 7.1, libsodium and OpenSSL instead.

TEST INFRASTRUCTURE ONLY.  Nothing in the product path (the HIP library under
``hotstuff-digital-signature-benchmarking_amd/``) imports, links or executes
this module.  Only ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py`` may use anything under ``oracle/``, and
only as the checker.

What it restates
----------------
The reference's hot path is ``crypto::Signature::verify`` and
``crypto::Signature::verify_batch`` (reference ``crypto/src/lib.rs:204-223``).
Both are thin glue over the third-party crate ``ed25519-dalek`` (requirement
``"1.0.1"`` with feature ``batch``, ``crypto/Cargo.toml:10``), which sits on
``curve25519-dalek`` 3.x (u64 backend) and ``sha2`` 0.9.  None of that is
vendored under ``/root/reference`` (``Cargo.lock`` is git-ignored,
``.gitignore:17``), and no Rust toolchain exists in this image, so the crate
cannot be built.  This file restates the published algorithm of those crates:

* ``ed25519::Signature::from_bytes`` (ed25519 1.x) - 64-byte R||s, with the
  ``s[31] & 0xE0`` partial check (subsumed by the canonical-s check below).
* ``InternalSignature::try_from`` -> ``check_scalar`` (ed25519-dalek 1.0.1):
  s must be canonical (s < l).
* ``PublicKey::from_bytes`` (ed25519-dalek 1.0.1) ->
  ``CompressedEdwardsY::decompress`` (curve25519-dalek 3.x): y = low 255 bits
  taken mod p (non-canonical y accepted), ``sqrt_ratio_i`` returns the
  non-negative root, negated when the sign bit is set; x = 0 with the sign bit
  set is accepted.
* ``PublicKey::verify_strict`` (ed25519-dalek 1.0.1): reject small-order R or
  A (``is_small_order`` = [8]P == O), k = SHA-512(R_bytes || A_bytes || M)
  mod l, accept iff [k](-A) + [s]B == R as *points* (projective equality).
* ``verify_batch`` (ed25519-dalek 1.0.1, feature ``batch``): any parse error
  is Err; otherwise a random linear combination with 128-bit z_i.  The
  deterministic restatement used here is "all items parse and satisfy the
  cofactorless equation", which always lies in the support of dalek's output
  distribution.

Parity pinning: checked against RFC 8032 section 7.1 test vectors, against
libsodium 1.0.18 (``crypto_sign_verify_detached``) on honest / corrupted /
non-canonical / mixed-order vectors (tests/test_oracle.py), and against the
qualitative outcomes of the reference's own tests
(``crypto/src/tests/crypto_tests.rs:50-115``,
``consensus/src/tests/messages_tests.rs:8-10``).
"""
from __future__ import annotations

import hashlib
from typing import Iterable, List, Optional, Sequence, Tuple

# ---------------------------------------------------------------------------
# Constants (curve25519-dalek 3.x ``constants`` module, restated)
# ---------------------------------------------------------------------------
P = 2**255 - 19
L = 2**252 + 27742317777372353535851937790883648493
D = (-121665 * pow(121666, P - 2, P)) % P
D2 = (2 * D) % P
SQRT_M1 = pow(2, (P - 1) // 4, P)

# Flag bits written per signature (must match include/hsv.h)
STRICT_OK = 0x01   # == dalek PublicKey::verify_strict returns Ok
EQ_OK = 0x02       # parse ok and [s]B == R + [k]A (cofactorless, point equality)
PARSE_OK = 0x04    # s canonical, A decodes, R decodes
SMALL_A = 0x08     # A decodes and [8]A == O
SMALL_R = 0x10     # R decodes and [8]R == O
S_OK = 0x20        # s < l
A_OK = 0x40        # A decodes
R_OK = 0x80        # R decodes


def _inv(x: int) -> int:
    return pow(x, P - 2, P)


def _is_negative(x: int) -> bool:
    """curve25519-dalek ``FieldElement::is_negative``: low bit of canonical bytes."""
    return (x % P) & 1 == 1


def sqrt_ratio_i(u: int, v: int) -> Tuple[bool, int]:
    """curve25519-dalek 3.x ``FieldElement::sqrt_ratio_i``.

    Returns (was_nonzero_square, r) with r the non-negative root.  Note the
    quirk kept from upstream: u == 0 returns (True, 0).
    """
    u %= P
    v %= P
    v3 = v * v % P * v % P
    v7 = v3 * v3 % P * v % P
    r = u * v3 % P * pow(u * v7 % P, (P - 5) // 8, P) % P
    check = v * r % P * r % P
    correct_sign_sqrt = check == u
    flipped_sign_sqrt = check == (-u) % P
    flipped_sign_sqrt_i = check == (-u) * SQRT_M1 % P
    if flipped_sign_sqrt or flipped_sign_sqrt_i:
        r = r * SQRT_M1 % P
    if _is_negative(r):
        r = (-r) % P
    return (correct_sign_sqrt or flipped_sign_sqrt), r


def decompress(b: bytes) -> Optional[Tuple[int, int]]:
    """curve25519-dalek 3.x ``CompressedEdwardsY::decompress`` -> affine (x, y) or None."""
    assert len(b) == 32
    y = (int.from_bytes(b, "little") & ((1 << 255) - 1)) % P   # FieldElement::from_bytes
    yy = y * y % P
    u = (yy - 1) % P
    v = (yy * D + 1) % P
    ok, x = sqrt_ratio_i(u, v)
    if not ok:
        return None
    if b[31] >> 7:
        x = (-x) % P                                          # conditional_negate, -0 == 0
    return x, y


def compress(pt: Tuple[int, int]) -> bytes:
    x, y = pt
    out = bytearray((y % P).to_bytes(32, "little"))
    out[31] |= (x % P & 1) << 7
    return bytes(out)


# Extended twisted Edwards coordinates (X:Y:Z:T), a = -1.
Ext = Tuple[int, int, int, int]
IDENTITY: Ext = (0, 1, 1, 0)


def to_ext(pt: Tuple[int, int]) -> Ext:
    x, y = pt
    return (x % P, y % P, 1, x * y % P)


def to_affine(e: Ext) -> Tuple[int, int]:
    X, Y, Z, _ = e
    zi = _inv(Z)
    return X * zi % P, Y * zi % P


def ext_add(p1: Ext, p2: Ext) -> Ext:
    X1, Y1, Z1, T1 = p1
    X2, Y2, Z2, T2 = p2
    a = (Y1 - X1) * (Y2 - X2) % P
    b = (Y1 + X1) * (Y2 + X2) % P
    c = T1 * D2 % P * T2 % P
    d = Z1 * 2 * Z2 % P
    e, f, g, h = b - a, d - c, d + c, b + a
    return (e * f % P, g * h % P, f * g % P, e * h % P)


def ext_double(p1: Ext) -> Ext:
    return ext_add(p1, p1)


def ext_neg(p1: Ext) -> Ext:
    X, Y, Z, T = p1
    return ((-X) % P, Y, Z, (-T) % P)


def ext_eq(p1: Ext, p2: Ext) -> bool:
    """curve25519-dalek 3.x ``EdwardsPoint::ct_eq``: X1*Z2 == X2*Z1 and Y1*Z2 == Y2*Z1."""
    X1, Y1, Z1, _ = p1
    X2, Y2, Z2, _ = p2
    return (X1 * Z2 - X2 * Z1) % P == 0 and (Y1 * Z2 - Y2 * Z1) % P == 0


def is_identity(p1: Ext) -> bool:
    return ext_eq(p1, IDENTITY)


def scalar_mult(k: int, p1: Ext) -> Ext:
    """[k]P for a non-negative integer k (plain double-and-add, MSB first)."""
    acc = IDENTITY
    for bit in bin(k)[2:] if k > 0 else "":
        acc = ext_double(acc)
        if bit == "1":
            acc = ext_add(acc, p1)
    return acc


def is_small_order(p1: Ext) -> bool:
    """curve25519-dalek ``EdwardsPoint::is_small_order``: [8]P is the identity."""
    return is_identity(ext_double(ext_double(ext_double(p1))))


_BY = 4 * _inv(5) % P
_BX = decompress(_BY.to_bytes(32, "little"))[0]   # non-negative x: standard base point
BASEPOINT: Ext = to_ext((_BX, _BY))


def sha512(data: bytes) -> bytes:
    return hashlib.sha512(data).digest()


def scalar_from_hash(h: bytes) -> int:
    """curve25519-dalek ``Scalar::from_hash`` = from_bytes_mod_order_wide."""
    return int.from_bytes(h, "little") % L


def scalar_is_canonical(s_bytes: bytes) -> bool:
    """ed25519 1.x ``s[31] & 0xE0`` check + dalek ``check_scalar`` => s < l."""
    if s_bytes[31] & 0xE0:
        return False
    return int.from_bytes(s_bytes, "little") < L


# ---------------------------------------------------------------------------
# Verification (dalek 1.0.1 semantics)
# ---------------------------------------------------------------------------
def verify_flags(pk: bytes, sig: bytes, msg: bytes) -> int:
    """Per-signature flag byte (see include/hsv.h); STRICT_OK == verify_strict."""
    assert len(pk) == 32 and len(sig) == 64
    r_bytes, s_bytes = sig[:32], sig[32:]
    flags = 0
    s_ok = scalar_is_canonical(s_bytes)
    a_pt = decompress(pk)
    r_pt = decompress(r_bytes)
    if s_ok:
        flags |= S_OK
    if a_pt is not None:
        flags |= A_OK
        if is_small_order(to_ext(a_pt)):
            flags |= SMALL_A
    if r_pt is not None:
        flags |= R_OK
        if is_small_order(to_ext(r_pt)):
            flags |= SMALL_R
    if not (s_ok and a_pt is not None and r_pt is not None):
        return flags
    flags |= PARSE_OK
    s = int.from_bytes(s_bytes, "little")
    k = scalar_from_hash(sha512(r_bytes + pk + msg))
    # R' = [k](-A) + [s]B   (vartime_double_scalar_mul_basepoint)
    rp = ext_add(scalar_mult(k, ext_neg(to_ext(a_pt))), scalar_mult(s, BASEPOINT))
    if ext_eq(rp, to_ext(r_pt)):
        flags |= EQ_OK
        if not (flags & (SMALL_A | SMALL_R)):
            flags |= STRICT_OK
    return flags


def verify_strict(pk: bytes, sig: bytes, msg: bytes) -> bool:
    """``crypto::Signature::verify`` (crypto/src/lib.rs:204-208)."""
    return bool(verify_flags(pk, sig, msg) & STRICT_OK)


def verify_batch(digest: bytes, votes: Sequence[Tuple[bytes, bytes]]) -> bool:
    """``crypto::Signature::verify_batch`` (crypto/src/lib.rs:210-223), deterministic rule.

    Ok iff every (pk, sig) parses and satisfies the cofactorless equation.
    An empty iterator is Ok (dalek's multiscalar sum over [0]B is the identity).
    """
    for pk, sig in votes:
        f = verify_flags(pk, sig, digest)
        if not (f & PARSE_OK and f & EQ_OK):
            return False
    return True


# ---------------------------------------------------------------------------
# RFC 8032 key generation / signing (dalek Keypair::generate / sign)
# ---------------------------------------------------------------------------
def _expand_seed(seed: bytes) -> Tuple[int, bytes]:
    h = sha512(seed)
    a = bytearray(h[:32])
    a[0] &= 248
    a[31] &= 127
    a[31] |= 64
    return int.from_bytes(a, "little"), h[32:]


def public_key(seed: bytes) -> bytes:
    a, _ = _expand_seed(seed)
    return compress(to_affine(scalar_mult(a, BASEPOINT)))


def sign(seed: bytes, msg: bytes) -> bytes:
    """RFC 8032 deterministic Ed25519 (``Signature::new``, crypto/src/lib.rs:185-191)."""
    a, prefix = _expand_seed(seed)
    pk = compress(to_affine(scalar_mult(a, BASEPOINT)))
    r = int.from_bytes(sha512(prefix + msg), "little") % L
    r_enc = compress(to_affine(scalar_mult(r, BASEPOINT)))
    k = int.from_bytes(sha512(r_enc + pk + msg), "little") % L
    s = (r + k * a) % L
    return r_enc + s.to_bytes(32, "little")


def sign_with_scalar(a: int, prefix: bytes, pk: bytes, msg: bytes) -> bytes:
    """Sign with an explicit secret scalar and public-key bytes (edge-vector builder)."""
    r = int.from_bytes(sha512(prefix + msg), "little") % L
    r_enc = compress(to_affine(scalar_mult(r, BASEPOINT)))
    k = int.from_bytes(sha512(r_enc + pk + msg), "little") % L
    s = (r + k * a) % L
    return r_enc + s.to_bytes(32, "little")


# ---------------------------------------------------------------------------
# Small-order points (the 8-torsion) and their encodings
# ---------------------------------------------------------------------------
def torsion_points() -> List[Ext]:
    """The 8 points of E[8], as multiples of one order-8 point."""
    # order-8 points satisfy x = +-i*y and d*y^4 + 2*y^2 - 1 = 0
    for sign in (1, -1):
        yy = (-1 + sign * _sqrt((1 + D) % P)) * _inv(D) % P
        if yy is None:
            continue
        y = _sqrt(yy)
        if y is None:
            continue
        x = SQRT_M1 * y % P
        t8 = to_ext((x, y))
        pts = [IDENTITY]
        cur = IDENTITY
        for _ in range(7):
            cur = ext_add(cur, t8)
            pts.append(cur)
        if is_identity(ext_add(cur, t8)) and not is_identity(scalar_mult(4, t8)):
            return pts
    raise RuntimeError("no order-8 point found")


def _sqrt(a: int) -> Optional[int]:
    a %= P
    if a == 0:
        return 0
    r = pow(a, (P + 3) // 8, P)
    if r * r % P == a:
        return r
    r = r * SQRT_M1 % P
    if r * r % P == a:
        return r
    return None


def small_order_encodings() -> List[bytes]:
    """Canonical encodings of the 8 small-order points plus their non-canonical aliases.

    Non-canonical aliases: y + p when y + p < 2^255 (only y in [0, 18]), and the
    "negative zero" sign bit on points with x == 0.
    """
    encs = []
    for pt in torsion_points():
        x, y = to_affine(pt)
        enc = compress((x, y))
        encs.append(enc)
        if y + P < 2**255:
            nc = bytearray((y + P).to_bytes(32, "little"))
            nc[31] |= (x & 1) << 7
            encs.append(bytes(nc))
        if x == 0:
            nz = bytearray(enc)
            nz[31] |= 0x80
            encs.append(bytes(nz))
    # de-duplicate, keep order
    seen, out = set(), []
    for e in encs:
        if e not in seen:
            seen.add(e)
            out.append(e)
    return out


def find_undecodable_y(start: int = 2) -> bytes:
    """Smallest y >= start whose encoding does not decompress (u/v non-square)."""
    y = start
    while True:
        enc = y.to_bytes(32, "little")
        if decompress(enc) is None:
            return enc
        y += 1


# ---------------------------------------------------------------------------
# Reference test-fixture recipes
# ---------------------------------------------------------------------------
def chacha20_block(key: bytes, counter: int, nonce8: bytes = b"\x00" * 8) -> bytes:
    """ChaCha20 block (djb variant: 64-bit counter, 64-bit nonce) as used by rand_chacha."""
    def rotl(v, c):
        return ((v << c) & 0xFFFFFFFF) | (v >> (32 - c))

    def qr(s, a, b, c, d):
        s[a] = (s[a] + s[b]) & 0xFFFFFFFF; s[d] = rotl(s[d] ^ s[a], 16)
        s[c] = (s[c] + s[d]) & 0xFFFFFFFF; s[b] = rotl(s[b] ^ s[c], 12)
        s[a] = (s[a] + s[b]) & 0xFFFFFFFF; s[d] = rotl(s[d] ^ s[a], 8)
        s[c] = (s[c] + s[d]) & 0xFFFFFFFF; s[b] = rotl(s[b] ^ s[c], 7)

    const = [0x61707865, 0x3320646E, 0x79622D32, 0x6B206574]
    k = [int.from_bytes(key[i:i + 4], "little") for i in range(0, 32, 4)]
    n = [int.from_bytes(nonce8[i:i + 4], "little") for i in range(0, 8, 4)]
    st = const + k + [counter & 0xFFFFFFFF, counter >> 32] + n
    w = list(st)
    for _ in range(10):
        qr(w, 0, 4, 8, 12); qr(w, 1, 5, 9, 13); qr(w, 2, 6, 10, 14); qr(w, 3, 7, 11, 15)
        qr(w, 0, 5, 10, 15); qr(w, 1, 6, 11, 12); qr(w, 2, 7, 8, 13); qr(w, 3, 4, 9, 14)
    return b"".join(((w[i] + st[i]) & 0xFFFFFFFF).to_bytes(4, "little") for i in range(16))


def reference_key_seeds(seed: bytes = b"\x00" * 32, count: int = 4) -> List[bytes]:
    """Secret seeds of the reference ``keys()`` fixture (crypto/src/tests/crypto_tests.rs:26-29).

    ``StdRng::from_seed(seed)`` in rand 0.7.3 (crypto/Cargo.toml:12) is rand_chacha 0.2's
    ChaCha20Rng (key = seed, counter and nonce zero); dalek ``SecretKey::generate`` fills
    32 bytes from it, so seed i is keystream bytes [32i, 32i+32).  The block function is
    pinned by the RFC 7539 test vectors (tests/test_oracle.py::test_chacha20_block_rfc7539).
    """
    need = 32 * count
    stream = b""
    ctr = 0
    while len(stream) < need:
        stream += chacha20_block(seed, ctr)
        ctr += 1
    return [stream[32 * i: 32 * i + 32] for i in range(count)]


def test_digest(message: bytes) -> bytes:
    """Test-only ``Hash for &[u8]``: SHA-512(msg)[..32] (crypto/src/tests/crypto_tests.rs:8-12)."""
    return sha512(message)[:32]


def qc_digest(block_hash: bytes, round_: int) -> bytes:
    """``QC::digest`` = SHA-512(hash || round_le)[..32] (consensus/src/messages.rs:201-207)."""
    return sha512(block_hash + round_.to_bytes(8, "little"))[:32]


def tc_vote_digest(round_: int, high_qc_round: int) -> bytes:
    """Per-vote TC digest (consensus/src/messages.rs:307-311)."""
    return sha512(round_.to_bytes(8, "little") + high_qc_round.to_bytes(8, "little"))[:32]
