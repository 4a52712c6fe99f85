"""C-ABI library checks that need no GPU: loads, exports, signing, error paths."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

import ed25519_ref as o
from conftest import ROOT


@pytest.fixture(scope="module")
def lib():
    from hsverify import _lib
    return _lib.load(require=True)


def declared_symbols(header=os.path.join(ROOT, "include", "hsv.h")):
    text = open(header).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(hsv_[a-z_0-9]+)\s*\(", text)))


def exported_symbols(path):
    out = subprocess.run(["nm", "-D", "--defined-only", path], capture_output=True, text=True, check=True).stdout
    return sorted(line.split()[-1] for line in out.splitlines() if line.strip())


def test_header_declares_the_boundary():
    syms = declared_symbols()
    for s in ("hsv_verify", "hsv_verify_strict", "hsv_verify_batch", "hsv_verify_batch_packed",
              "hsv_verify_device", "hsv_verify_device_bits", "hsv_init", "hsv_shutdown", "hsv_sign"):
        assert s in syms


def test_library_exports_every_declared_symbol(lib):
    for s in declared_symbols():
        assert hasattr(lib, s), s


def test_product_library_exports_exactly_the_header():
    """libhsv.so's dynamic symbol table is include/hsv.h, nothing more: no test
    hook (fault injection, variant or lattice switches), no internal launch
    entry point, no C++ runtime instantiation (round-3 VERDICT item 6)."""
    from hsverify import _lib
    assert exported_symbols(_lib.LIB_PATH.replace(os.path.basename(_lib.LIB_PATH), "libhsv.so")) == \
        declared_symbols()


# The environment variables the product library reads:
# device binding, slot count, the automatic committee cache, the pack
# threads, the resident latency service (on by default) and its idle time,
# and the workspace pool's kept memory.  Measurement switches live in
# libhsv_test.so's hooks only.
PRODUCT_ENV = {"HSV_DEVICE", "HSV_SLOTS", "HSV_AUTO_COMMITTEE", "HSV_PACK_THREADS", "HSV_QC_RESIDENT",
               "HSV_QC_RESIDENT_IDLE_MS", "HSV_WS_POOL_KEEP_MB", "HSV_TX_FUSED"}


def test_product_library_reads_only_the_documented_environment():
    """Every HSV_* name compiled into libhsv.so (the strings a getenv call
    could read) is on the short allow-list above (round-4 VERDICT item 7: the
    closed experiments' switches -- the streamed host form, the sync and
    pipeline-shape alternatives, the row cut-overs -- are gone from the product
    library), and each allowed one appears in INTEGRATION.md."""
    from hsverify import _lib
    path = _lib.LIB_PATH.replace(os.path.basename(_lib.LIB_PATH), "libhsv.so")
    blob = open(path, "rb").read()
    names = {m.decode() for m in re.findall(rb"(?<![A-Za-z0-9_])HSV_[A-Z0-9_]+(?=\x00)", blob)}
    assert names <= PRODUCT_ENV, sorted(names - PRODUCT_ENV)
    src = os.path.join(ROOT, "hotstuff-digital-signature-benchmarking_amd", "csrc")
    read = set()
    for f in os.listdir(src):
        if f.endswith((".cpp", ".hip", ".h", ".hpp")):
            text = open(os.path.join(src, f)).read()
            read |= set(re.findall(r'(?:getenv|env_int)\("(HSV_[A-Z0-9_]+)"', text))
    assert read <= PRODUCT_ENV, sorted(read - PRODUCT_ENV)
    doc = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    assert all(n in doc for n in PRODUCT_ENV)


def test_test_library_exports_the_header_and_the_hooks():
    from hsverify import _lib
    hooks = declared_symbols(os.path.join(ROOT, "hotstuff-digital-signature-benchmarking_amd", "csrc",
                                          "hsv_test_hooks.h"))
    assert set(hooks) == set(_lib.HOOKS)
    assert exported_symbols(_lib.TEST_LIB_PATH) == sorted(set(declared_symbols()) | set(hooks))


def test_version_and_device_count(lib):
    from hsverify import _lib
    assert "gfx950" in _lib.version()
    assert lib.hsv_device_count() >= 0
    # the header's ABI generation is the library's (0.3.0: d_fault before `stream`)
    hdr = open(os.path.join(ROOT, "include", "hsv.h")).read()
    assert lib.hsv_abi_version() == int(re.search(r"#define HSV_ABI_VERSION (\d+)", hdr).group(1)) == 3
    assert _lib.version().startswith("hsv 0.3.")


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
    assert lib.hsv_verify_device_bits(ctypes.c_void_p(8), 32, ctypes.c_void_p(16), 64, ctypes.c_void_p(32), 32, 1,
                                      ctypes.c_void_p(64), None, None, None) == -5


def test_synth_workload_shapes(lib):
    from hsverify import synth
    w = synth.independent_triples(256, seed=3, corrupt_frac=0.05)
    assert w.pk.shape == (256, 32) and w.sig.shape == (256, 64) and w.msg.shape == (256, 32)
    assert (~w.honest).sum() == round(256 * 0.05)
    q = synth.qc_votes(100)
    assert q.n == 67 and q.msg.shape == (32,)
    t = synth.tc_votes(1000)
    assert t.n == 667 and t.msg.shape == (667, 32)


def test_mixed_order_signer_matches_oracle(lib):
    """hsv_sign_mixed_order (the C3/C4 mixed-order-A corruption): the key is
    [a]B plus an order-8 torsion point, and the oracle decides as SURVEY A.3
    rows 7-8 say -- k = 0 (mod 8): verify_strict Ok (cofactorless equation
    holds, A is not small-order); k != 0 (mod 8): parses but the equation fails."""
    from hsverify import synth
    rnd = np.random.default_rng(9)
    for t in range(4):
        for accept in (True, False):
            seed = bytes(rnd.integers(0, 256, 32, dtype=np.uint8))
            msg = bytes(rnd.integers(0, 256, 32, dtype=np.uint8))
            pk, sig = synth.mixed_order_signature(seed, msg, t, accept)
            pk, sig = bytes(pk), bytes(sig)
            pt = o.decompress(pk)
            assert pt is not None and not o.is_small_order(o.to_ext(pt))
            assert not o.is_identity(o.scalar_mult(o.L, o.to_ext(pt)))       # not in the prime-order subgroup
            assert o.is_identity(o.scalar_mult(8 * o.L, o.to_ext(pt)))
            k = o.scalar_from_hash(o.sha512(sig[:32] + pk + msg))
            assert (k % 8 == 0) == accept
            f = o.verify_flags(pk, sig, msg)
            assert f & o.PARSE_OK and not f & o.SMALL_A
            assert bool(f & o.STRICT_OK) == accept and bool(f & o.EQ_OK) == accept


def test_synth_corruption_mix_has_every_kind(lib):
    """bit-flip in R / s, s + l, wrong digest, undecodable R,
    small-order R / A, mixed-order A -- all present in the 5 % of a C3 quorum,
    and `accept` marks exactly the honest votes and the k = 0 (mod 8)
    mixed-order ones (checked against the Python oracle)."""
    from hsverify import synth
    for make in (synth.qc_votes, synth.tc_votes):
        w = make(1000, seed=5, corrupt_frac=0.05)
        assert set(np.unique(w.kind[w.kind >= 0])) == set(range(len(synth.CORRUPTIONS)))
        msg = w.msg if w.msg.ndim == 2 else np.repeat(w.msg[None], w.n, 0)
        for i in np.nonzero(w.kind >= 0)[0]:
            f = o.verify_flags(bytes(w.pk[i]), bytes(w.sig[i]), bytes(msg[i]))
            assert bool(f & o.STRICT_OK) == bool(w.accept[i]), synth.CORRUPTIONS[w.kind[i]]
