"""Independent Ed25519 verifiers for pinning the oracle (test infrastructure).

Two third-party implementations sit in this image and are loaded through
ctypes; neither shares code with the oracle or the kernels:

* OpenSSL 3.0.2 (`libcrypto.so.3`, `EVP_DigestVerify` on an `EVP_PKEY_ED25519`
  raw public key).  Its `ossl_ed25519_verify` checks s < l, decodes A (y taken
  mod p, "-0" accepted, no small-order rejection), computes
  R' = [s]B - [k]A cofactorless and accepts iff the canonical encoding of R'
  equals the 32 R bytes of the signature.  So it answers the *batch* rule of
  `Signature::verify_batch` (PARSE_OK and EQ_OK,
  `/root/reference/crypto/src/lib.rs:210-223`), except where dalek decodes an R
  that OpenSSL, comparing bytes, can never match: R bytes that are not the
  canonical encoding of their point.
* libsodium 1.0.18 (`crypto_sign_ed25519_verify_detached`), the *strict* rule
  of `Signature::verify` (`lib.rs:204-208`): s < l, small-order
  A and R rejected by blocklist, non-canonical A rejected, R compared by bytes.

`classify_*` name every place where the independent verdict may differ from
the oracle's flag bits; anything else is an unclassified divergence and the
tests fail on it (DESIGN.md section 3 lists the classes).
"""
from __future__ import annotations

import ctypes

import numpy as np

P = 2**255 - 19

# flag bits (include/hsv.h)
STRICT_OK, EQ_OK, PARSE_OK, SMALL_A, SMALL_R, S_OK, A_OK, R_OK = 1, 2, 4, 8, 16, 32, 64, 128

# Divergence classes.  Each holds only with dalek ACCEPTING and the
# independent verifier rejecting, on an item whose point decodes.
OPENSSL_CLASSES = {
    # R's y field is >= p (y + p < 2^255 for y < 19): dalek reduces y mod p and
    # compares points; OpenSSL compares bytes with a canonical re-encoding.
    "R_noncanonical_y",
    # x = 0 (y = 1 or p - 1) with the sign bit set: dalek decodes it as x = 0
    # (curve25519-dalek 3.x accepts "-0"); the canonical encoding has sign 0.
    "R_negative_zero",
}
SODIUM_CLASSES = {
    # Non-canonical A with the strict equation holding.  Only reachable for a
    # small-order A, which dalek's verify_strict rejects too, so the class is
    # expected to stay empty; it is named so a future vector cannot slip by.
    "A_noncanonical",
    # Same for R bytes compared by libsodium against the re-encoding.
    "R_noncanonical",
}


def _load(cands):
    for c in cands:
        try:
            return ctypes.CDLL(c)
        except OSError:
            continue
    return None


class OpenSSL:
    NID_ED25519 = 1087

    def __init__(self):
        lib = _load(("libcrypto.so.3", "/usr/lib/x86_64-linux-gnu/libcrypto.so.3"))
        if lib is None:
            raise OSError("libcrypto.so.3 not found")
        lib.OpenSSL_version.restype = ctypes.c_char_p
        lib.OpenSSL_version.argtypes = [ctypes.c_int]
        lib.EVP_PKEY_new_raw_public_key.restype = ctypes.c_void_p
        lib.EVP_PKEY_new_raw_public_key.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_char_p, ctypes.c_size_t]
        lib.EVP_MD_CTX_new.restype = ctypes.c_void_p
        lib.EVP_MD_CTX_new.argtypes = []
        lib.EVP_DigestVerifyInit.restype = ctypes.c_int
        lib.EVP_DigestVerifyInit.argtypes = [ctypes.c_void_p] * 5
        lib.EVP_DigestVerify.restype = ctypes.c_int
        lib.EVP_DigestVerify.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p,
                                         ctypes.c_size_t]
        lib.EVP_MD_CTX_free.argtypes = [ctypes.c_void_p]
        lib.EVP_PKEY_free.argtypes = [ctypes.c_void_p]
        self.lib = lib
        self.version = lib.OpenSSL_version(0).decode()

    def verify(self, pk: bytes, sig: bytes, msg: bytes) -> bool:
        lib = self.lib
        key = lib.EVP_PKEY_new_raw_public_key(self.NID_ED25519, None, pk, 32)
        if not key:
            return False
        ctx = lib.EVP_MD_CTX_new()
        try:
            if lib.EVP_DigestVerifyInit(ctx, None, None, None, key) != 1:
                raise RuntimeError("EVP_DigestVerifyInit failed")
            return lib.EVP_DigestVerify(ctx, sig, 64, msg, len(msg)) == 1
        finally:
            lib.EVP_MD_CTX_free(ctx)
            lib.EVP_PKEY_free(key)


class Sodium:
    def __init__(self):
        lib = _load(("/opt/conda/lib/libsodium.so.23", "libsodium.so.23"))
        if lib is None or lib.sodium_init() < 0:
            raise OSError("libsodium.so.23 not found")
        lib.sodium_version_string.restype = ctypes.c_char_p
        self.lib = lib
        self.version = lib.sodium_version_string().decode()

    def verify(self, pk: bytes, sig: bytes, msg: bytes) -> bool:
        return self.lib.crypto_sign_ed25519_verify_detached(sig, msg, ctypes.c_ulonglong(len(msg)), pk) == 0


def _y_sign(enc: bytes):
    v = int.from_bytes(enc, "little")
    return v & (2**255 - 1), v >> 255


def r_encoding_class(r: bytes):
    """None if R's 32 bytes are the canonical encoding of their point (or do not
    decode at all), else the OpenSSL class name."""
    y, sign = _y_sign(r)
    if y >= P:
        return "R_noncanonical_y"
    if sign and y in (1, P - 1):
        return "R_negative_zero"
    return None


def classify_openssl(flags: int, sig: bytes, ossl_ok: bool):
    """'agree', a class of OPENSSL_CLASSES, or 'unclassified:<why>'."""
    batch = (flags & (PARSE_OK | EQ_OK)) == (PARSE_OK | EQ_OK)
    if batch == ossl_ok:
        return "agree"
    cls = r_encoding_class(sig[:32])
    if batch and not ossl_ok and cls is not None and flags & R_OK:
        return cls
    return f"unclassified:batch={int(batch)},openssl={int(ossl_ok)},flags=0x{flags:02x}"


def classify_sodium(flags: int, pk: bytes, sig: bytes, sodium_ok: bool):
    strict = bool(flags & STRICT_OK)
    if strict == sodium_ok:
        return "agree"
    if strict and not sodium_ok:
        ya, _ = _y_sign(pk)
        if ya >= P:
            return "A_noncanonical"
        if r_encoding_class(sig[:32]) is not None:
            return "R_noncanonical"
    return f"unclassified:strict={int(strict)},sodium={int(sodium_ok)},flags=0x{flags:02x}"


def run(verifier, pk, sig, msg) -> np.ndarray:
    """Verdicts (bool array) of `verifier` over arrays pk (n,32), sig (n,64),
    msg (n,32) or one shared (32,) digest."""
    pk = np.ascontiguousarray(pk, np.uint8)
    sig = np.ascontiguousarray(sig, np.uint8)
    msg = np.ascontiguousarray(msg, np.uint8)
    n = pk.shape[0]
    out = np.zeros(n, bool)
    shared = msg.ndim == 1
    for i in range(n):
        m = msg.tobytes() if shared else msg[i].tobytes()
        out[i] = verifier.verify(pk[i].tobytes(), sig[i].tobytes(), m)
    return out


def classify_all(flags, pk, sig, ossl=None, sodium=None):
    """Per-record class lists for the verdict arrays given (None skips one)."""
    res = {}
    if ossl is not None:
        res["openssl"] = [classify_openssl(int(f), sig[i].tobytes(), bool(ossl[i])) for i, f in enumerate(flags)]
    if sodium is not None:
        res["sodium"] = [classify_sodium(int(f), pk[i].tobytes(), sig[i].tobytes(), bool(sodium[i]))
                         for i, f in enumerate(flags)]
    return res


def pack_verdicts(v: np.ndarray) -> str:
    return np.packbits(np.asarray(v, bool), bitorder="little").tobytes().hex()


def unpack_verdicts(h: str, n: int) -> np.ndarray:
    return np.unpackbits(np.frombuffer(bytes.fromhex(h), np.uint8), bitorder="little")[:n].astype(bool)


# ---- the record sets the cross-checks run over --------------------------------
def _golden_dir():
    import os
    return os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _records_from_raw(raw):
    return raw[:, :32].copy(), raw[:, 32:96].copy(), raw[:, 96:128].copy(), raw[:, 128].copy()


def datasets(oracle_flags_fn, quick: bool = False):
    """name -> (pk, sig, msg, flags).  Flags of the committed sets are the golden
    ones (Python oracle); those of the synthetic sets come from
    `oracle_flags_fn(pk, sig, msg)` (the C oracle).  quick drops the 2^15 set."""
    import hashlib
    import json
    import os

    g = _golden_dir()
    out = {}
    with open(os.path.join(g, "edge_vectors.json")) as f:
        edge = json.load(f)["vectors"]
    raw = np.fromfile(os.path.join(g, "random_vectors.bin"), dtype=np.uint8).reshape(-1, 129)
    hx = lambda key, w: np.frombuffer(bytes.fromhex("".join(e[key] for e in edge)), np.uint8).reshape(-1, w)
    rpk, rsig, rmsg, rfl = _records_from_raw(raw)
    out["golden"] = (np.concatenate([hx("pk", 32), rpk]), np.concatenate([hx("sig", 64), rsig]),
                     np.concatenate([hx("msg", 32), rmsg]),
                     np.concatenate([np.array([e["flags"] for e in edge], np.uint8), rfl]))
    raw = np.fromfile(os.path.join(g, "lattice_fallback.bin"), dtype=np.uint8).reshape(-1, 129)
    out["lattice_fallback"] = _records_from_raw(raw)

    with open(os.path.join(g, "reference_fixtures.json")) as f:
        fx = json.load(f)["fixtures"]
    recs = []
    for name in sorted(fx):
        v = fx[name]
        if v["op"] == "verify":
            recs.append((v["pk"], v["sig"], v["digest"]))
        else:
            recs.extend((p, s, v["digest"]) for p, s in v["votes"])
    col = lambda j, w: np.frombuffer(bytes.fromhex("".join(r[j] for r in recs)), np.uint8).reshape(-1, w)
    pk, sig, msg = col(0, 32), col(1, 64), col(2, 32)
    out["reference_fixtures"] = (pk, sig, msg, oracle_flags_fn(pk, sig, msg))

    with open(os.path.join(g, "tx_vectors.json")) as f:
        txv = json.load(f)["vectors"]
    txs = [bytes.fromhex(v["tx"]) for v in txv if len(bytes.fromhex(v["tx"])) >= 96]
    pk = np.stack([np.frombuffer(t[-96:-64], np.uint8) for t in txs])
    sig = np.stack([np.frombuffer(t[-64:], np.uint8) for t in txs])
    msg = np.stack([np.frombuffer(hashlib.sha512(t[:-96]).digest()[:32], np.uint8) for t in txs])
    out["tx_golden"] = (pk, sig, msg, oracle_flags_fn(pk, sig, msg))

    from hsverify import synth
    for name, make in (("c3_qc", synth.qc_votes), ("c3_tc", synth.tc_votes)):
        w = make(1000, seed=5, corrupt_frac=0.05)
        msg = w.msg if w.msg.ndim == 2 else np.repeat(w.msg[None], w.n, 0)
        out[name] = (w.pk, w.sig, msg, oracle_flags_fn(w.pk, w.sig, msg))
    if not quick:
        w = synth.independent_triples(1 << 15, seed=99, corrupt_frac=0.2)
        out["random_2p15"] = (w.pk, w.sig, w.msg, oracle_flags_fn(w.pk, w.sig, w.msg))
    return out


def records_digest(pk, sig, msg) -> str:
    import hashlib
    h = hashlib.sha256()
    for a in (pk, sig, msg):
        h.update(np.ascontiguousarray(a, np.uint8).tobytes())
    return h.hexdigest()
