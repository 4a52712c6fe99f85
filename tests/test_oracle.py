"""The oracle pinned: RFC 8032 KATs, golden vectors, libsodium, C restatement.

These run on CPU.  The Python restatement (oracle/ed25519_ref.py) and the C
restatement (oracle/ed25519_oracle.c) are independent implementations of the
ed25519-dalek 1.0.1 rules; both must reproduce every committed golden flag,
and libsodium 1.0.18 must agree with the STRICT_OK bit.
"""
import ctypes
import random

import numpy as np
import pytest

import ed25519_ref as o
from conftest import oracle_flags

# RFC 8032 section 7.1, TEST 1-3 (secret, public, message, signature)
RFC8032 = [
    ("9d61b19deffd5a60ba844af492ec2cc44449c5697b326919703bac031cae7f60",
     "d75a980182b10ab7d54bfed3c964073a0ee172f3daa62325af021a68f707511a", "",
     "e5564300c360ac729086e2cc806e828a84877f1eb8e5d974d873e065224901555fb8821590a33bacc61e39701cf9b46bd25bf5f0595bbe24655141438e7a100b"),
    ("4ccd089b28ff96da9db6c346ec114e0f5b8a319f35aba624da8cf6ed4fb8a6fb",
     "3d4017c3e843895a92b70aa74d1b7ebc9c982ccf2ec4968cc0cd55f12af4660c", "72",
     "92a009a9f0d4cab8720e820b5f642540a2b27b5416503f8fb3762223ebdb69da085ac1e43e15996e458f3613d0f11d8c387b2eaeb4302aeeb00d291612bb0c00"),
    ("c5aa8df43f9f837bedb7442f31dcb7b166d38535076f094b85ce3a2e0b4458f7",
     "fc51cd8e6218a1a38da47ed00230f0580816ed13ba3303ac5deb911548908025", "af82",
     "6291d657deec24024827e69c3abe01a30ce548a284743a445e3680d7db5ac3ac18ff9b538d16f290ae67f760984dc6594a7c15e9716ed28dc027beceea1ec40a"),
]


@pytest.mark.parametrize("sk,pk,msg,sig", RFC8032)
def test_rfc8032_vectors(sk, pk, msg, sig, oracle_lib):
    sk, pk, msg, sig = map(bytes.fromhex, (sk, pk, msg, sig))
    assert o.public_key(sk) == pk
    assert o.sign(sk, msg) == sig
    assert o.verify_strict(pk, sig, msg)
    assert oracle_lib.oracle_verify_flags(pk, sig, msg, len(msg)) & o.STRICT_OK
    bad = bytearray(sig)
    bad[0] ^= 1
    assert not o.verify_strict(pk, bytes(bad), msg)


def test_python_oracle_reproduces_edge_golden(golden):
    n = golden["n_edge"]
    for i in range(n):
        got = o.verify_flags(bytes(golden["pk"][i]), bytes(golden["sig"][i]), bytes(golden["msg"][i]))
        assert got == golden["flags"][i], golden["cases"][i]


def test_python_oracle_reproduces_random_golden_sample(golden):
    rnd = random.Random(7)
    idx = rnd.sample(range(golden["n_edge"], len(golden["flags"])), 150)
    for i in idx:
        got = o.verify_flags(bytes(golden["pk"][i]), bytes(golden["sig"][i]), bytes(golden["msg"][i]))
        assert got == golden["flags"][i]


def test_c_oracle_reproduces_all_golden(golden, oracle_lib):
    got = oracle_flags(oracle_lib, golden["pk"], golden["sig"], golden["msg"])
    bad = np.nonzero(got != golden["flags"])[0]
    assert bad.size == 0, [golden["cases"][i] for i in bad[:10]]


def test_golden_covers_the_edge_catalogue(golden):
    """every case family is present with the expected outcome."""
    f, cases = golden["flags"], golden["cases"]
    byfam = {}
    for c, fl in zip(cases, f):
        byfam.setdefault(c.split("_")[0], []).append(int(fl))
    assert all(x & o.STRICT_OK for x in byfam["honest"])
    assert not any(x & o.STRICT_OK for x in byfam["default"])
    # mixed-order A: both accepted (k kills the torsion) and rejected instances exist
    mixed = [x for c, x in zip(cases, f) if c.startswith("mixed_A")]
    assert any(x & o.STRICT_OK for x in mixed) and any(not x & o.STRICT_OK for x in mixed)
    # small-order R with a valid equation: EQ_OK but not STRICT_OK (batch accepts, strict rejects)
    small_r_eq = [x for c, x in zip(cases, f) if c.startswith("small_R") and x & o.EQ_OK]
    assert small_r_eq and not any(x & o.STRICT_OK for x in small_r_eq)
    # non-canonical s is a parse failure
    assert not any(x & o.S_OK for c, x in zip(cases, f) if c.startswith("s_plus_l") or c == "s_eq_l")
    assert any(x & o.S_OK for c, x in zip(cases, f) if c == "s_eq_l_minus_1")
    # undecodable points
    assert not any(x & o.R_OK for c, x in zip(cases, f) if c.startswith("R_undecodable"))
    assert not any(x & o.A_OK for c, x in zip(cases, f) if c.startswith("A_undecodable"))


def _sodium():
    for cand in ("/opt/conda/lib/libsodium.so.23", "libsodium.so.23"):
        try:
            lib = ctypes.CDLL(cand)
            if lib.sodium_init() >= 0:
                return lib
        except OSError:
            pass
    return None


def test_libsodium_agrees_with_strict_bit(golden):
    lib = _sodium()
    if lib is None:
        pytest.skip("libsodium not present")
    for i in range(len(golden["flags"])):
        pk, sig, msg = bytes(golden["pk"][i]), bytes(golden["sig"][i]), bytes(golden["msg"][i])
        ok = lib.crypto_sign_ed25519_verify_detached(sig, msg, ctypes.c_ulonglong(32), pk) == 0
        assert ok == bool(golden["flags"][i] & o.STRICT_OK), golden["cases"][i]


def test_small_order_y_set_equals_eightfold_identity():
    """The kernel's small-order test (y in a 5-value set) == dalek's [8]P == O."""
    y_set = {0, 1, o.P - 1}
    for pt in o.torsion_points():
        y_set.add(o.to_affine(pt)[1])
    assert len(y_set) == 5
    for enc in o.small_order_encodings():
        pt = o.decompress(enc)
        assert pt is not None
        assert o.is_small_order(o.to_ext(pt)) and pt[1] % o.P in y_set
    rnd = random.Random(11)
    for _ in range(40):
        pt = o.decompress(rnd.randbytes(32))
        if pt is None:
            continue
        assert o.is_small_order(o.to_ext(pt)) == (pt[1] % o.P in y_set)


def test_reference_fixtures_with_oracle(reference_fixtures):
    fx = reference_fixtures["fixtures"]
    assert reference_fixtures["qc_digest"].startswith("f2a4a4b7")
    for name, v in fx.items():
        if v["op"] == "verify":
            got = o.verify_strict(bytes.fromhex(v["pk"]), bytes.fromhex(v["sig"]), bytes.fromhex(v["digest"]))
        else:
            got = o.verify_batch(bytes.fromhex(v["digest"]),
                                 [(bytes.fromhex(p), bytes.fromhex(s)) for p, s in v["votes"]])
        assert got == v["expect_ok"], name


def test_c_oracle_batch_rule(reference_fixtures, oracle_lib):
    for name, v in reference_fixtures["fixtures"].items():
        if v["op"] != "verify_batch" or not v["votes"]:
            continue
        pk = b"".join(bytes.fromhex(p) for p, _ in v["votes"])
        sig = b"".join(bytes.fromhex(s) for _, s in v["votes"])
        got = oracle_lib.oracle_verify_batch(bytes.fromhex(v["digest"]), pk, sig, len(v["votes"]))
        assert bool(got) == v["expect_ok"], name


def test_c_oracle_reproduces_fallback_records(fallback_records, oracle_lib):
    """tests/golden/lattice_fallback.bin (flags from the Python oracle) agrees
    with the C oracle; honest records are accepted, flipped-s / s + l rejected."""
    fb = fallback_records
    got = oracle_flags(oracle_lib, fb["pk"], fb["sig"], fb["msg"])
    assert (got == fb["flags"]).all()
    assert (fb["flags"][0::4] & o.STRICT_OK).all()
