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


# ---- the reference's keys() fixture recipe (crypto/src/tests/crypto_tests.rs:26-29) ----
# rand 0.7.3 (crypto/Cargo.toml:12) StdRng = rand_chacha 0.2 ChaCha20Rng: key =
# the 32-byte seed, 64-bit counter and nonce starting at zero, keystream consumed
# in order by dalek's SecretKey::generate (fill_bytes).  The block function is
# pinned by the published RFC 7539 vectors (A.1 #1/#2: zero key, counters 0/1;
# 2.3.2: key 00..1f, nonce 000000090000004a00000000, counter 1 in the
# 32-bit-counter layout = the djb layout with the first nonce word in the high
# counter half).
@pytest.mark.parametrize("key,counter,nonce8,block", [
    (bytes(32), 0, bytes(8),
     "76b8e0ada0f13d90405d6ae55386bd28bdd219b8a08ded1aa836efcc8b770dc7"
     "da41597c5157488d7724e03fb8d84a376a43b8f41518a11cc387b669b2ee6586"),
    (bytes(32), 1, bytes(8),
     "9f07e7be5551387a98ba977c732d080dcb0f29a048e3656912c6533e32ee7aed"
     "29b721769ce64e43d57133b074d839d531ed1f28510afb45ace10a1f4b794d6f"),
    (bytes(range(32)), 1 + (0x09000000 << 32), bytes.fromhex("0000004a00000000"),
     "10f1e7e4d13b5915500fdd1fa32071c4c7d1f4c733c068030422aa9ac3d46c4e"
     "d2826446079faa0914c2d705d98b02a2b5129cd1de164eb9cbd083e8a2503c4e"),
])
def test_chacha20_block_rfc7539(key, counter, nonce8, block):
    assert o.chacha20_block(key, counter, nonce8).hex() == block


def test_reference_key_seeds_are_the_zero_key_keystream():
    seeds = o.reference_key_seeds()
    assert seeds[0].hex() == "76b8e0ada0f13d90405d6ae55386bd28bdd219b8a08ded1aa836efcc8b770dc7"
    assert b"".join(seeds) == o.chacha20_block(bytes(32), 0) + o.chacha20_block(bytes(32), 1)


def test_reference_fixture_recipe_is_pinned(reference_fixtures):
    assert "unpinned" not in reference_fixtures["key_recipe"]
    pks = {bytes.fromhex(v["pk"]) for v in reference_fixtures["fixtures"].values() if v.get("pk")}
    want = {o.public_key(s) for s in o.reference_key_seeds()}
    assert pks and pks <= want


# ---- fast mod-l reduction used by the C port (Barrett) vs the bit-serial one ----
def test_fast_scalar_reduction_matches_bit_serial(oracle_lib):
    fast, slow = oracle_lib.oracle_sc_reduce64_fast, oracle_lib.oracle_sc_reduce64_slow
    rng = random.Random(7)
    cases = [bytes(64), b"\xff" * 64, o.L.to_bytes(64, "little"), (o.L - 1).to_bytes(64, "little"),
             (o.L * o.L).to_bytes(64, "little"), ((1 << 512) - o.L).to_bytes(64, "little")]
    cases += [rng.getrandbits(512).to_bytes(64, "little") for _ in range(3000)]
    a, b = ctypes.create_string_buffer(32), ctypes.create_string_buffer(32)
    for i, x in enumerate(cases):
        fast(a, x)
        assert int.from_bytes(a.raw, "little") == int.from_bytes(x, "little") % o.L
        if i < 300:
            slow(b, x)
            assert a.raw == b.raw


# ---- C port of ed25519-dalek verify_batch (the QC CPU baseline) ------------------
def _batch_port(oracle_lib):
    f = oracle_lib.oracle_verify_batch_dalek
    f.restype = ctypes.c_int
    f.argtypes = [ctypes.c_char_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint64]
    return f


@pytest.mark.parametrize("committee", [4, 100, 400])   # 3 / 67 / 267 votes: Straus and Pippenger w=6
def test_dalek_batch_port_verdicts(oracle_lib, committee):
    from hsverify import synth
    f = _batch_port(oracle_lib)
    w = synth.qc_votes(committee, seed=committee)
    pk, sig = np.ascontiguousarray(w.pk), np.ascontiguousarray(w.sig)
    for seed in (1, 2):
        assert f(bytes(w.msg), pk.ctypes.data, sig.ctypes.data, w.n, seed) == 1
    for pos in (0, 40, 63):          # R, s and the top byte of s
        bad = sig.copy()
        bad[w.n // 2, pos] ^= 2
        assert f(bytes(w.msg), pk.ctypes.data, bad.ctypes.data, w.n, 3) == 0
    other = bytearray(w.msg)
    other[0] ^= 1
    assert f(bytes(other), pk.ctypes.data, sig.ctypes.data, w.n, 4) == 0
    assert f(bytes(w.msg), pk.ctypes.data, sig.ctypes.data, 0, 5) == 1


def test_dalek_batch_port_agrees_with_deterministic_rule(oracle_lib):
    """Corrupted QCs over every corruption kind (C3 shape at n = 1000, 667
    votes: Pippenger w = 8): the port's verdict equals the build's rule
    (all PARSE_OK and EQ_OK) whenever no failure is pure torsion."""
    from hsverify import synth
    f = _batch_port(oracle_lib)
    for frac, seed in ((0.0, 11), (0.005, 12), (0.05, 13)):
        w = synth.qc_votes(1000, seed=seed, corrupt_frac=frac)
        pk, sig = np.ascontiguousarray(w.pk), np.ascontiguousarray(w.sig)
        flags = oracle_flags(oracle_lib, pk, sig, w.msg)
        rule = int(((flags & (o.PARSE_OK | o.EQ_OK)) == (o.PARSE_OK | o.EQ_OK)).all())
        assert f(bytes(w.msg), pk.ctypes.data, sig.ctypes.data, w.n, seed) == rule
