"""C-ABI library checks that need no GPU: loads, exports, signing, error paths."""
import ctypes
import os
import re

import numpy as np
import pytest

import ed25519_ref as o
from conftest import ROOT


@pytest.fixture(scope="module")
def lib():
    from hsverify import _lib
    return _lib.load(require=True)


def declared_symbols():
    text = open(os.path.join(ROOT, "include", "hsv.h")).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(hsv_[a-z_0-9]+)\s*\(", text)))


def test_header_declares_the_boundary():
    syms = declared_symbols()
    for s in ("hsv_verify", "hsv_verify_strict", "hsv_verify_batch", "hsv_verify_batch_packed",
              "hsv_verify_device", "hsv_verify_device_bits", "hsv_init", "hsv_shutdown", "hsv_sign"):
        assert s in syms


def test_library_exports_every_declared_symbol(lib):
    for s in declared_symbols():
        assert hasattr(lib, s), s


def test_version_and_device_count(lib):
    from hsverify import _lib
    assert "gfx950" in _lib.version()
    assert lib.hsv_device_count() >= 0


def test_public_key_and_sign_match_oracle(lib):
    from hsverify import crypto
    rnd = np.random.default_rng(1)
    for _ in range(8):
        seed = bytes(rnd.integers(0, 256, 32, dtype=np.uint8))
        msg = bytes(rnd.integers(0, 256, 32, dtype=np.uint8))
        assert crypto.public_key_from_seed(seed).data == o.public_key(seed)
        pk, sk = crypto.generate_keypair(lambda n, s=seed: s)
        sig = crypto.Signature.new(crypto.Digest(msg), sk)
        assert sig.flatten() == o.sign(seed, msg)


def test_sign_many_matches_oracle(lib):
    from hsverify import verifier
    rnd = np.random.default_rng(2)
    seeds = rnd.integers(0, 256, (40, 32), dtype=np.uint8)
    msgs = rnd.integers(0, 256, (40, 32), dtype=np.uint8)
    pk, sig = verifier.sign_many(seeds, msgs, nthreads=4)
    for i in range(40):
        assert bytes(pk[i]) == o.public_key(bytes(seeds[i]))
        assert bytes(sig[i]) == o.sign(bytes(seeds[i]), bytes(msgs[i]))


def test_reference_key_fixture_roundtrip(lib):
    """crypto_tests.rs import_export_public_key / import_export_secret_key."""
    from hsverify import crypto
    seed = o.reference_key_seeds()[3]
    pk, sk = crypto.generate_keypair(lambda n: seed)
    assert crypto.PublicKey.decode_base64(pk.encode_base64()) == pk
    assert crypto.SecretKey.decode_base64(sk.encode_base64()) == sk


def test_no_device_fails_loudly(lib):
    """Without a GPU the verifier raises; it never silently rejects or falls back."""
    from hsverify import crypto, _lib
    if lib.hsv_device_count() > 0:
        pytest.skip("a GPU is visible")
    with pytest.raises(_lib.HsvLibraryError):
        crypto.Signature.default().verify(crypto.Digest(bytes(32)), crypto.PublicKey(bytes(32)))
    flags = (ctypes.c_uint8 * 1)()
    assert lib.hsv_verify(bytes(32), bytes(64), bytes(32), 0, 1, flags) == -1


def test_invalid_arguments(lib):
    out = (ctypes.c_uint8 * 4)()
    assert lib.hsv_verify(bytes(32), bytes(64), bytes(32), 7, 1, out) == -3      # bad msg_stride
    assert lib.hsv_verify(None, None, None, 32, 0, None) == 0                     # n == 0 is a no-op
    assert lib.hsv_verify_batch(bytes(32), None, None, 0) == 1                    # empty batch is Ok
    # misaligned device pointers are rejected before any device work
    assert lib.hsv_verify_device(ctypes.c_void_p(8), 32, ctypes.c_void_p(16), 64,
                                 ctypes.c_void_p(32), 32, 1, ctypes.c_void_p(64), None) == -5


def test_synth_workload_shapes(lib):
    from hsverify import synth
    w = synth.independent_triples(256, seed=3, corrupt_frac=0.05)
    assert w.pk.shape == (256, 32) and w.sig.shape == (256, 64) and w.msg.shape == (256, 32)
    assert (~w.honest).sum() == round(256 * 0.05)
    q = synth.qc_votes(100)
    assert q.n == 67 and q.msg.shape == (32,)
    t = synth.tc_votes(1000)
    assert t.n == 667 and t.msg.shape == (667, 32)
