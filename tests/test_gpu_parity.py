"""GPU parity: the HIP path through the C ABI vs the oracle, bit-exact.

Every comparison is on all 8 flag bits (include/hsv.h), not only the verdict.
Sizes: golden fixtures (2193 records), the BASELINE configs C1-C3 exactly,
2^15 random records against the C oracle, and the full C4 size (2^20) through
the device-resident API, checked with size-independent properties plus an
oracle-checked sample.
"""
import asyncio
import os
import threading

import numpy as np
import pytest

import ed25519_ref as o
from conftest import oracle_flags

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def api(hsv):
    from hsverify import crypto, synth, verifier
    return crypto, verifier, synth


def test_golden_every_variant(api, golden):
    """Every variant built into the library (the product's 19 and 21), switched
    through the test library's hook (libhsv_test.so: the same objects)."""
    _, verifier, _ = api
    from hsverify import _testing
    with _testing.test_library():
        default = verifier.get_variant()
        try:
            for v in verifier.variants():
                verifier.set_variant(v)
                got = verifier.verify_flags(golden["pk"], golden["sig"], golden["msg"])
                bad = np.nonzero(got != golden["flags"])[0]
                assert bad.size == 0, (v, [(golden["cases"][i], int(got[i]), int(golden["flags"][i]))
                                           for i in bad[:8]])
        finally:
            verifier.set_variant(default)


def test_golden_row_form_chunks(api, golden):
    """Batches at or below the row form's cut-over (row_max(), 3072 items)
    run the latency kernels: the golden records in chunks of 1000 (above
    kJointMax, 768: hsv_verify_row_kernel, one row per element), of 700 and
    512 (above kQuadMax, 256: hsv_verify_joint_kernel, one item per wave with
    R and A decompressed on the two row pairs and one two-scalar Straus), of
    256 and 200 (hsv_verify_quad_kernel, one point per wave, the formulas'
    four products on the four rows), and ragged small batches (1, 5, 7, 13
    items); every flag bit against the fixtures.  The committee cache is off
    so the generic kernels run."""
    _, verifier, _ = api
    from hsverify import _lib
    lib = _lib.load()
    lib.hsv_set_auto_committee(0)
    try:
        n = len(golden["flags"])
        for chunk in (1000, 700, 512, 256, 200):
            for lo in range(0, n, chunk):
                hi = min(n, lo + chunk)
                got = verifier.verify_flags(golden["pk"][lo:hi], golden["sig"][lo:hi], golden["msg"][lo:hi])
                bad = np.nonzero(got != golden["flags"][lo:hi])[0]
                assert bad.size == 0, [(chunk, golden["cases"][lo + i], int(got[i]), int(golden["flags"][lo + i]))
                                       for i in bad[:8]]
        lo = 0
        for m in (1, 5, 7, 13, 1, 6, 12):
            got = verifier.verify_flags(golden["pk"][lo:lo + m], golden["sig"][lo:lo + m], golden["msg"][lo:lo + m])
            assert (got == golden["flags"][lo:lo + m]).all(), (lo, m)
            lo += 97
    finally:
        lib.hsv_set_auto_committee(1)


def test_golden_pair_form_range(api, golden):
    """Batches between the row form's cut-over (3072) and 2^13 run the pair
    kernel (hsv_verify_pair_fused_kernel): the golden records tiled to 4096
    items, every flag bit.  Committee cache off."""
    _, verifier, _ = api
    from hsverify import _lib
    lib = _lib.load()
    lib.hsv_set_auto_committee(0)
    try:
        idx = np.arange(4096) % len(golden["flags"])
        got = verifier.verify_flags(golden["pk"][idx], golden["sig"][idx], golden["msg"][idx])
        bad = np.nonzero(got != golden["flags"][idx])[0]
        assert bad.size == 0, [(golden["cases"][idx[i]], int(got[i]), int(golden["flags"][idx[i]])) for i in bad[:8]]
    finally:
        lib.hsv_set_auto_committee(1)


@pytest.mark.parametrize("bits", [133, 0])
def test_lattice_fallback_records_every_variant(api, fallback_records, bits):
    """The fixture challenges have no lattice pair below 2^133: with the bound
    lowered to 133 (hsv_set_lattice_bits) they take the full-length path inside
    the half-size kernels (tests/test_kernel_host.py shows the same headers do);
    at the default 138 they stay on the half-size path.  Every variant must
    match the oracle's flags either way.  The automatic committee cache is off
    so the generic kernels run."""
    _, verifier, _ = api
    from hsverify import _testing
    with _testing.test_library() as lib:
        fb = fallback_records
        default = verifier.get_variant()
        prev = _testing.set_lattice_bits(bits)
        lib.hsv_set_auto_committee(0)
        try:
            for v in verifier.variants():
                verifier.set_variant(v)
                got = verifier.verify_flags(fb["pk"], fb["sig"], fb["msg"])
                assert (got == fb["flags"]).all(), (v, np.nonzero(got != fb["flags"])[0][:8])
                # mixed into a wave of ordinary records (the fallback lane diverges)
                idx = np.arange(256) % len(fb["flags"])
                got = verifier.verify_flags(fb["pk"][idx], fb["sig"][idx], fb["msg"][idx])
                assert (got == fb["flags"][idx]).all(), v
                # the joint quad form's range (257 .. 768 items)
                idx = np.arange(600) % len(fb["flags"])
                got = verifier.verify_flags(fb["pk"][idx], fb["sig"][idx], fb["msg"][idx])
                assert (got == fb["flags"][idx]).all(), v
                # the pair form's range (3073 .. 2^13 items)
                idx = np.arange(4096) % len(fb["flags"])
                got = verifier.verify_flags(fb["pk"][idx], fb["sig"][idx], fb["msg"][idx])
                assert (got == fb["flags"][idx]).all(), v
                # past the pair form's cut-over: the point pass deals fallback batches first
                idx = np.arange((1 << 13) + 64) % len(fb["flags"])
                got = verifier.verify_flags(fb["pk"][idx], fb["sig"][idx], fb["msg"][idx])
                assert (got == fb["flags"][idx]).all(), v
        finally:
            verifier.set_variant(default)
            _testing.set_lattice_bits(prev)
            lib.hsv_set_auto_committee(1)


def test_lattice_fallback_records_product_library(api, fallback_records, hsv):
    """The same records on the product library itself (default bound, default
    variant), in the quad, joint, row, pair and point-pass ranges."""
    _, verifier, _ = api
    fb = fallback_records
    hsv.hsv_set_auto_committee(0)
    try:
        for m in (len(fb["flags"]), 256, 600, 1000, 4096, (1 << 13) + 64):
            idx = np.arange(m) % len(fb["flags"])
            got = verifier.verify_flags(fb["pk"][idx], fb["sig"][idx], fb["msg"][idx])
            assert (got == fb["flags"][idx]).all(), m
    finally:
        hsv.hsv_set_auto_committee(1)


def test_host_pipeline_with_fallback_items(api, fallback_records, oracle_lib):
    """Host batches of >= 2^18 items (the chunked copy pipeline: per-chunk
    prepass, then the point pass or, for an item without a short lattice
    pair, the full-length path).  With the bound lowered to 133 every fixture
    record takes the full-length path; they sit at random positions among
    ordinary records."""
    _, verifier, synth = api
    from hsverify import _testing
    fb = fallback_records
    n = (1 << 18) + 100
    w = synth.independent_triples(n, seed=2718, corrupt_frac=0.05)
    pos = np.sort(np.random.default_rng(5).choice(n, 3000, replace=False))
    src = np.arange(pos.size) % len(fb["flags"])
    pk, sig, msg = w.pk.copy(), w.sig.copy(), w.msg.copy()
    pk[pos], sig[pos], msg[pos] = fb["pk"][src], fb["sig"][src], fb["msg"][src]
    with _testing.test_library() as lib:
        lib.hsv_set_auto_committee(0)
        try:
            for bits in (133, 0):
                prev = _testing.set_lattice_bits(bits)
                try:
                    got = verifier.verify_flags(pk, sig, msg)
                finally:
                    _testing.set_lattice_bits(prev)
                assert (got[pos] == fb["flags"][src]).all(), bits
                rest = np.setdiff1d(np.arange(n), pos)
                assert (got[rest][w.accept[rest]] & o.STRICT_OK).all()
                assert not (got[rest][~w.accept[rest]] & o.STRICT_OK).any()
                sample = np.sort(np.random.default_rng(6).choice(rest, 2048, replace=False))
                assert (got[sample] == oracle_flags(oracle_lib, pk[sample], sig[sample], msg[sample])).all()
        finally:
            lib.hsv_set_auto_committee(1)


# ---- the reference's own tests (crypto/src/tests/crypto_tests.rs) ---------
def _keys(crypto):
    return [crypto.generate_keypair(lambda n, s=s: s) for s in o.reference_key_seeds()]


def test_verify_valid_signature(api):
    crypto, _, _ = api
    public_key, secret_key = _keys(crypto).pop()
    digest = crypto.Digest(o.test_digest(b"Hello, world!"))
    signature = crypto.Signature.new(digest, secret_key)
    assert signature.verify(digest, public_key).is_ok()


def test_verify_invalid_signature(api):
    crypto, _, _ = api
    public_key, secret_key = _keys(crypto).pop()
    digest = crypto.Digest(o.test_digest(b"Hello, world!"))
    signature = crypto.Signature.new(digest, secret_key)
    bad = crypto.Digest(o.test_digest(b"Bad message!"))
    assert signature.verify(bad, public_key).is_err()


def test_verify_valid_batch(api):
    crypto, _, _ = api
    digest = crypto.Digest(o.test_digest(b"Hello, world!"))
    keys = _keys(crypto)
    signatures = []
    for _ in range(3):
        public_key, secret_key = keys.pop()
        signatures.append((public_key, crypto.Signature.new(digest, secret_key)))
    assert crypto.Signature.verify_batch(digest, signatures).is_ok()


def test_verify_invalid_batch(api):
    crypto, _, _ = api
    digest = crypto.Digest(o.test_digest(b"Hello, world!"))
    keys = _keys(crypto)
    signatures = []
    for _ in range(2):
        public_key, secret_key = keys.pop()
        signatures.append((public_key, crypto.Signature.new(digest, secret_key)))
    public_key, _ = keys.pop()
    signatures.append((public_key, crypto.Signature.default()))
    assert crypto.Signature.verify_batch(digest, signatures).is_err()


def test_signature_service(api):
    crypto, _, _ = api
    public_key, secret_key = _keys(crypto).pop()
    digest = crypto.Digest(o.test_digest(b"Hello, world!"))

    async def run():
        service = crypto.SignatureService(secret_key)
        try:
            return await service.request_signature(digest)
        finally:
            await service.close()

    loop = asyncio.new_event_loop()
    signature = loop.run_until_complete(run())
    loop.close()
    assert signature.verify(digest, public_key).is_ok()


def test_reference_fixture_file(api, reference_fixtures):
    """Committed fixtures incl. consensus qc() (messages_tests.rs verify_valid_qc)."""
    crypto, _, _ = api
    for name, v in reference_fixtures["fixtures"].items():
        d = crypto.Digest(bytes.fromhex(v["digest"]))
        if v["op"] == "verify":
            sig = bytes.fromhex(v["sig"])
            r = crypto.Signature(sig[:32], sig[32:]).verify(d, crypto.PublicKey(bytes.fromhex(v["pk"])))
        else:
            votes = [(crypto.PublicKey(bytes.fromhex(p)), crypto.Signature(bytes.fromhex(s)[:32], bytes.fromhex(s)[32:]))
                     for p, s in v["votes"]]
            r = crypto.Signature.verify_batch(d, votes)
        assert r.is_ok() == v["expect_ok"], name


# ---- BASELINE configs C1-C3 ---------------------------------------------------
@pytest.mark.parametrize("committee", [4, 100, 1000])
def test_qc_configs(api, oracle_lib, committee):
    crypto, verifier, synth = api
    w = synth.qc_votes(committee, seed=committee)
    votes = [(crypto.PublicKey(bytes(p)), crypto.Signature(bytes(s[:32]), bytes(s[32:]))) for p, s in zip(w.pk, w.sig)]
    d = crypto.Digest(bytes(w.msg))
    assert crypto.Signature.verify_batch(d, votes).is_ok()
    # one bad vote anywhere makes the QC Err
    bad = list(votes)
    i = len(bad) // 2
    s = bytearray(bad[i][1].flatten())
    s[40] ^= 4
    bad[i] = (bad[i][0], crypto.Signature(bytes(s[:32]), bytes(s[32:])))
    assert crypto.Signature.verify_batch(d, bad).is_err()
    # per-vote flags, not only the verdict: clean and corrupted quorums (for C1
    # one vote in three), all 8 bits against the C oracle
    for frac in (0.0, 0.34 if committee == 4 else 0.05):
        wc = synth.qc_votes(committee, seed=committee + 1, corrupt_frac=frac)
        msg = wc.msg if wc.msg.ndim == 2 else np.repeat(wc.msg[None], wc.n, 0)
        got = verifier.verify_flags(wc.pk, wc.sig, msg)
        assert (got == oracle_flags(oracle_lib, wc.pk, wc.sig, msg)).all()
        assert (got[wc.accept] & o.STRICT_OK).all() and not (got[~wc.accept] & o.STRICT_OK).any()


def test_c3_committee_1000_qc_and_tc_bit_exact(api, oracle_lib):
    _, verifier, synth = api
    for make in (synth.qc_votes, synth.tc_votes):
        w = make(1000, seed=5, corrupt_frac=0.05)
        msg = w.msg if w.msg.ndim == 2 else np.repeat(w.msg[None], w.n, 0)
        got = verifier.verify_flags(w.pk, w.sig, msg)
        exp = oracle_flags(oracle_lib, w.pk, w.sig, msg)
        assert (got == exp).all()
        assert (got[w.accept] & o.STRICT_OK).all()
        assert not (got[~w.accept] & o.STRICT_OK).any()
        # every corruption kind SURVEY 8(d) lists is in the vector, mixed-order keys included
        assert set(np.unique(w.kind[w.kind >= 0])) == set(range(len(synth.CORRUPTIONS)))
        assert (got[w.kind == synth.CORRUPTIONS.index("mixed_order_A_ok")] & o.STRICT_OK).all()


def test_random_batch_vs_c_oracle(api, oracle_lib):
    _, verifier, synth = api
    w = synth.independent_triples(1 << 15, seed=99, corrupt_frac=0.2)
    got = verifier.verify_flags(w.pk, w.sig, w.msg)
    exp = oracle_flags(oracle_lib, w.pk, w.sig, w.msg)
    assert (got == exp).all()


def test_random_batches_latency_forms_vs_c_oracle(api, oracle_lib):
    """The same random corrupted triples (every SURVEY 8(d) corruption kind,
    20 %) through each latency kernel's range, cache off: quad form (1, 37,
    256 items), joint form (257, 500, 768) and the row form (769, 2000), every
    flag bit against the C oracle."""
    _, verifier, synth = api
    from hsverify import _lib
    lib = _lib.load()
    lib.hsv_set_auto_committee(0)
    try:
        w = synth.independent_triples(2000, seed=4242, corrupt_frac=0.2)
        exp = oracle_flags(oracle_lib, w.pk, w.sig, w.msg)
        lo = 0
        for m in (1, 37, 256, 257, 500, 768, 769, 2000):
            idx = (np.arange(m) + lo) % w.pk.shape[0]
            lo += 611
            got = verifier.verify_flags(w.pk[idx], w.sig[idx], w.msg[idx])
            bad = np.nonzero(got != exp[idx])[0]
            assert bad.size == 0, (m, [(int(idx[i]), int(got[i]), int(exp[idx][i])) for i in bad[:8]])
    finally:
        lib.hsv_set_auto_committee(1)


# ---- ragged sizes, shared digests, layouts ------------------------------------
@pytest.mark.parametrize("n", [1, 4095, 4096, 4097])
def test_zero_copy_boundary_vs_c_oracle(api, oracle_lib, n):
    """Host batches of <= 2^12 fresh keys are read from pinned memory by the
    kernels (zero-copy); 4097 takes the copy path.  Both must match the oracle."""
    _, verifier, synth = api
    w = synth.independent_triples(n, seed=1000 + n, corrupt_frac=0.2)
    got = verifier.verify_flags(w.pk, w.sig, w.msg)
    exp = oracle_flags(oracle_lib, w.pk, w.sig, w.msg)
    assert (got == exp).all()


@pytest.mark.parametrize("n", [1, 2, 63, 64, 65, 255, 256, 257, 258, 767, 768, 769, 1000])
def test_ragged_sizes(api, golden, n):
    _, verifier, _ = api
    idx = np.arange(n) % len(golden["flags"])
    got = verifier.verify_flags(golden["pk"][idx], golden["sig"][idx], golden["msg"][idx])
    assert (got == golden["flags"][idx]).all()


def test_shared_digest_matches_per_item(api, oracle_lib):
    _, verifier, synth = api
    w = synth.qc_votes(100, seed=3)          # one shared digest
    assert w.msg.shape == (32,)
    for i in range(0, w.n, 7):               # corrupt signatures, keep the digest shared
        w.sig[i, (i * 13) % 64] ^= 1 << (i % 8)
    shared = verifier.verify_flags(w.pk, w.sig, w.msg)
    per_item = verifier.verify_flags(w.pk, w.sig, np.repeat(w.msg[None], w.n, 0))
    assert (shared == per_item).all()
    assert (shared == oracle_flags(oracle_lib, w.pk, w.sig, w.msg)).all()


def test_packed_votes_layout(api, hsv):
    crypto, verifier, synth = api
    w = synth.qc_votes(100, seed=8)
    packed = np.concatenate([w.pk, w.sig], axis=1).tobytes()
    assert hsv.hsv_verify_batch_packed(bytes(w.msg), packed, w.n) == 1
    assert hsv.hsv_verify_batch(bytes(w.msg), w.pk.tobytes(), w.sig.tobytes(), w.n) == 1
    assert hsv.hsv_verify_batch(bytes(w.msg), None, None, 0) == 1


def test_concurrent_host_calls(api, golden):
    _, verifier, _ = api
    results = [None] * 6

    def work(k):
        sl = slice(k * 300, k * 300 + 300)
        results[k] = verifier.verify_flags(golden["pk"][sl], golden["sig"][sl], golden["msg"][sl])

    th = [threading.Thread(target=work, args=(k,)) for k in range(6)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    for k in range(6):
        sl = slice(k * 300, k * 300 + 300)
        assert (results[k] == golden["flags"][sl]).all()


def test_device_api_flags_bits_and_strides(api, golden):
    import torch
    _, verifier, _ = api
    dev = torch.device("cuda:0")
    n = 1000
    idx = np.arange(n) % len(golden["flags"])
    exp = golden["flags"][idx]
    pk = torch.from_numpy(golden["pk"][idx].copy()).to(dev)
    sig = torch.from_numpy(golden["sig"][idx].copy()).to(dev)
    msg = torch.from_numpy(golden["msg"][idx].copy()).to(dev)
    flags = torch.zeros(n, dtype=torch.uint8, device=dev)
    bits = torch.zeros((n + 31) // 32, dtype=torch.int32, device=dev)
    verifier.verify_device(pk, sig, msg, flags, bits)
    torch.cuda.synchronize()
    f = flags.cpu().numpy()
    assert (f == exp).all()
    b = bits.cpu().numpy().view(np.uint32)
    unpacked = np.array([(b[i // 32] >> (i % 32)) & 1 for i in range(n)], np.uint8)
    assert (unpacked == (exp & o.STRICT_OK)).all()
    # packed 128-byte records (pk | sig | msg) read in place through strides
    rec = torch.cat([pk, sig, msg], dim=1).contiguous()
    flags2 = torch.zeros(n, dtype=torch.uint8, device=dev)
    verifier.verify_device(rec[:, 0:32], rec[:, 32:96], rec[:, 96:128], flags2)
    torch.cuda.synchronize()
    assert (flags2.cpu().numpy() == exp).all()


# ---- full C4 size: properties + oracle sample ----------------------------------
def test_c4_full_size_properties(api, oracle_lib):
    import torch
    _, verifier, synth = api
    n = 1 << 20
    w = synth.independent_triples(n, seed=2024, corrupt_frac=0.05)
    dev = torch.device("cuda:0")
    pk, sig, msg = (torch.from_numpy(a).to(dev) for a in (w.pk, w.sig, w.msg))
    flags = torch.zeros(n, dtype=torch.uint8, device=dev)
    verifier.verify_device(pk, sig, msg, flags)
    torch.cuda.synchronize()
    f = flags.cpu().numpy()
    # honest signatures are all accepted; every corruption kind but the
    # accepted mixed-order one (k = 0 mod 8) is rejected
    assert (f[w.accept] & o.STRICT_OK).all()
    assert not (f[~w.accept] & o.STRICT_OK).any()
    kinds = {name: f[w.kind == k] for k, name in enumerate(synth.CORRUPTIONS)}
    assert not (kinds["s_plus_l"] & o.S_OK).any() and not (kinds["s_bit255"] & o.S_OK).any()
    assert not (kinds["undecodable_R"] & o.R_OK).any()
    assert (kinds["small_order_R"] & o.SMALL_R).all() and (kinds["small_order_A"] & o.SMALL_A).all()
    # mixed-order keys: the cofactorless equation decides (Appendix A.3 rows 7-8)
    assert kinds["mixed_order_A_ok"].size and (kinds["mixed_order_A_ok"] & o.STRICT_OK).all()
    assert not (kinds["mixed_order_A_ok"] & o.SMALL_A).any()
    assert kinds["mixed_order_A_bad"].size and (kinds["mixed_order_A_bad"] & o.PARSE_OK).all()
    assert not (kinds["mixed_order_A_bad"] & o.EQ_OK).any()
    # idempotent: a second launch gives identical bytes
    flags2 = torch.zeros_like(flags)
    verifier.verify_device(pk, sig, msg, flags2)
    torch.cuda.synchronize()
    assert torch.equal(flags, flags2)
    # oracle-checked sample across the whole range
    rng = np.random.default_rng(1)
    sample = np.sort(rng.choice(n, 8192, replace=False))
    exp = oracle_flags(oracle_lib, w.pk[sample], w.sig[sample], w.msg[sample])
    assert (f[sample] == exp).all()


def test_host_api_pipelined_chunks_match_device_api(api, oracle_lib):
    """Host batches of >= 2^18 items run the copy pipeline (hsv_capi.cpp
    run_pipelined: launch chunks of 2^16, 3 x 2^16, then the rest, copied in
    pieces of 2^17 items): an uneven last piece, every flag equal to the
    device-resident launch, and an oracle-checked sample."""
    import torch
    _, verifier, synth = api
    n = (1 << 19) + (1 << 18) + 12345
    w = synth.independent_triples(n, seed=77, corrupt_frac=0.05)
    got = verifier.verify_flags(w.pk, w.sig, w.msg)
    dev = torch.device("cuda:0")
    pk, sig, msg = (torch.from_numpy(a).to(dev) for a in (w.pk, w.sig, w.msg))
    flags = torch.zeros(n, dtype=torch.uint8, device=dev)
    verifier.verify_device(pk, sig, msg, flags)
    torch.cuda.synchronize()
    assert (got == flags.cpu().numpy()).all()
    assert (got[w.accept] & o.STRICT_OK).all() and not (got[~w.accept] & o.STRICT_OK).any()
    sample = np.sort(np.random.default_rng(3).choice(n, 4096, replace=False))
    assert (got[sample] == oracle_flags(oracle_lib, w.pk[sample], w.sig[sample], w.msg[sample])).all()


def test_host_api_pipeline_shared_digest_and_packed_votes(api, oracle_lib):
    """The pipelined host path (hsv_capi.cpp run_pipelined: 96-byte records
    and one shared digest staged once) with
    one shared digest (a huge QC) and with packed 96-byte votes
    (hsv_verify_batch_packed's strided records): flags equal the
    device-resident launch and an oracle sample."""
    import torch
    _, verifier, synth = api
    from hsverify import _lib
    lib = _lib.load()
    n = (1 << 18) + 777
    seeds = synth.committee_seeds(n, 3)
    digest = np.frombuffer(synth.qc_digest(bytes(32), 9), np.uint8).copy()
    pk, sig = verifier.sign_many(seeds, np.repeat(digest[None], n, 0))
    sig[5, 40] ^= 1                                   # one forged vote
    got = verifier.verify_flags(pk, sig, digest)       # msg_stride 0, pipelined
    dev = torch.device("cuda:0")
    flags = torch.zeros(n, dtype=torch.uint8, device=dev)
    verifier.verify_device(torch.from_numpy(pk).to(dev), torch.from_numpy(sig).to(dev),
                           torch.from_numpy(digest).to(dev), flags)
    torch.cuda.synchronize()
    assert (got == flags.cpu().numpy()).all()
    assert not got[5] & o.STRICT_OK and (np.delete(got, 5) & o.STRICT_OK).all()
    sample = np.unique(np.concatenate([[5], np.random.default_rng(4).choice(n, 2048, replace=False)]))
    exp = oracle_flags(oracle_lib, pk[sample], sig[sample], np.repeat(digest[None], sample.size, 0))
    assert (got[sample] == exp).all()
    packed = np.concatenate([pk, sig], axis=1)
    lib.hsv_set_auto_committee(0)
    try:
        assert lib.hsv_verify_batch_packed(digest.tobytes(), packed.tobytes(), n) == 0
        packed[5, 32 + 40] ^= 1
        assert lib.hsv_verify_batch_packed(digest.tobytes(), packed.tobytes(), n) == 1
    finally:
        lib.hsv_set_auto_committee(1)


@pytest.mark.parametrize("sched", [[1000, 70000, 3], [1 << 18], [12345, 1 << 17, 5 << 16]])
def test_host_api_pipeline_schedules(api, sched):
    """Any launch schedule of the pipelined host call (hsv_test_pipe_schedule,
    test library: ragged chunks, chunks of several copy pieces, a chunk of one
    item) gives the device-resident launch's flags."""
    import ctypes
    import torch
    from hsverify import _testing
    _, verifier, synth = api
    n = (1 << 18) + 4321
    w = synth.independent_triples(n, seed=78, corrupt_frac=0.05)
    dev = torch.device("cuda:0")
    flags = torch.zeros(n, dtype=torch.uint8, device=dev)
    verifier.verify_device(*(torch.from_numpy(a).to(dev) for a in (w.pk, w.sig, w.msg)), flags)
    torch.cuda.synchronize()
    want = flags.cpu().numpy()
    with _testing.test_library() as lib:
        arr = (ctypes.c_uint64 * len(sched))(*sched)
        assert lib.hsv_test_pipe_schedule(arr, len(sched)) == 0
        try:
            got = verifier.verify_flags(w.pk, w.sig, w.msg)
        finally:
            lib.hsv_test_pipe_schedule(None, 0)
    assert (got == want).all()
