"""Device self-checks: a corrupted workspace is an infrastructure error on
every path, never a verdict (round-2 VERDICT item 1).

The kernels check, for every item whose points decode, that the final
accumulator is a curve point with Z != 0 (ge_is_sane, csrc/hsv_point.hpp),
and every lane of the generic kernels compares a per-launch canary in its
workspace slot after each batch.  The fault injection hook
(hsverify._testing.inject_fault) makes every launch read back corrupted
table entries -- zeroed (what the round-2 forged-vote acceptance came from,
DESIGN.md 6.2), bit-flipped -- or an overwritten canary.  Each case runs
once, deterministically; the hook is reset afterwards and the same calls then
verify correctly again.

The hooks live in libhsv_test.so only (the product library exports exactly
include/hsv.h); `_testing.test_library()` runs a test's calls on that
instance, and injection is scoped to the calling thread's launches.

The CPU side of the same checks is tests/test_kernel_host.py (host-built
kernel headers with the same injection).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

FAULT = -7  # HSV_ERR_DEVICE_FAULT


@pytest.fixture(scope="module")
def env(hsv):
    from hsverify import _lib, _testing, crypto, synth, verifier
    return _lib, _testing, crypto, synth, verifier


@pytest.fixture
def tlib(env):
    """Every hsverify call of the test goes to libhsv_test.so."""
    with env[1].test_library() as lib:
        yield lib


@pytest.fixture
def generic(tlib):
    """The automatic committee cache off, so the generic kernels run."""
    tlib.hsv_set_auto_committee(0)
    yield
    tlib.hsv_set_auto_committee(1)


@pytest.mark.parametrize("mode", [1, 2, 3])
def test_generic_paths_report_faults(env, tlib, generic, mode):
    _lib, _testing, crypto, synth, verifier = env
    lib = tlib
    w = synth.qc_votes(100, seed=5)                                # 67 votes, quad-form latency kernel
    joint = synth.independent_triples(600, seed=19, corrupt_frac=0.0)  # joint quad form (257..768)
    row = synth.independent_triples(1000, seed=20, corrupt_frac=0.0)   # row form (769..3072)
    mid = synth.independent_triples(4096, seed=8, corrupt_frac=0.0)  # pair latency kernel (3073..8192)
    big = synth.independent_triples((1 << 13) + 64, seed=6, corrupt_frac=0.0)  # point-pass kernels
    packed = np.concatenate([w.pk, w.sig], axis=1).copy()
    want_small = verifier.verify_flags(w.pk, w.sig, w.msg)
    want_mid = verifier.verify_flags(mid.pk, mid.sig, mid.msg)
    want_big = verifier.verify_flags(big.pk, big.sig, big.msg)
    assert (want_small & 1).all() and (want_mid & 1).all() and (want_big & 1).all()
    assert (verifier.verify_flags(joint.pk, joint.sig, joint.msg) & 1).all()
    assert (verifier.verify_flags(row.pk, row.sig, row.msg) & 1).all()
    with _testing.injected_fault(mode):
        for pk, sig, msg in ((w.pk, w.sig, w.msg), (joint.pk, joint.sig, joint.msg), (row.pk, row.sig, row.msg),
                             (mid.pk, mid.sig, mid.msg), (big.pk, big.sig, big.msg)):
            with pytest.raises(_lib.HsvLibraryError, match="HSV_ERR_DEVICE_FAULT"):
                verifier.verify_flags(pk, sig, msg)
        assert lib.hsv_verify_batch_packed(w.msg.tobytes(), packed.tobytes(), w.n) == FAULT
        assert lib.hsv_verify_strict(w.msg.tobytes(), w.pk[0].tobytes(), w.sig[0].tobytes()) == FAULT
        assert "self-check" in _lib.last_error()
        # the reference-shaped mirror raises instead of answering Ok or Err
        votes = [(crypto.PublicKey(bytes(p)), crypto.Signature(bytes(s[:32]), bytes(s[32:])))
                 for p, s in zip(w.pk, w.sig)]
        with pytest.raises(_lib.HsvLibraryError):
            crypto.Signature.verify_batch(crypto.Digest(w.msg.tobytes()), votes)
    # injection off: the same calls verify again, nothing stale in the slots
    assert (verifier.verify_flags(w.pk, w.sig, w.msg) == want_small).all()
    assert (verifier.verify_flags(mid.pk, mid.sig, mid.msg) == want_mid).all()
    assert (verifier.verify_flags(big.pk, big.sig, big.msg) == want_big).all()
    assert lib.hsv_verify_batch_packed(w.msg.tobytes(), packed.tobytes(), w.n) == 1


@pytest.mark.parametrize("mode", [1, 2, 3])
def test_device_api_records_faults(env, tlib, mode):
    import torch
    _lib, _testing, _, synth, verifier = env
    w = synth.independent_triples((1 << 14) + 5, seed=7, corrupt_frac=0.05)
    dev = torch.device("cuda:0")
    pk = torch.from_numpy(w.pk).to(dev)
    sig = torch.from_numpy(w.sig).to(dev)
    msg = torch.from_numpy(w.msg).to(dev)
    flags = torch.zeros(w.n, dtype=torch.uint8, device=dev)
    verifier.device_faults(-1, clear=True)
    verifier.verify_device(pk, sig, msg, flags)
    torch.cuda.synchronize()
    assert verifier.device_faults() == 0
    want = flags.cpu().numpy().copy()
    with _testing.injected_fault(mode):
        verifier.verify_device(pk, sig, msg, flags)
        torch.cuda.synchronize()
    bits = verifier.device_faults(-1, clear=False)
    assert bits == (2 if mode == 2 else 1), bits
    with pytest.raises(_lib.HsvLibraryError, match="HSV_ERR_DEVICE_FAULT"):
        verifier.check_device_faults()
    assert verifier.device_faults() == 0  # check_device_faults cleared it
    verifier.verify_device(pk, sig, msg, flags)
    torch.cuda.synchronize()
    assert verifier.device_faults() == 0
    assert (flags.cpu().numpy() == want).all()


@pytest.mark.parametrize("mode", [1, 3])
def test_committee_and_transaction_paths_report_faults(env, tlib, generic, mode):
    _lib, _testing, _, synth, verifier = env
    from hsverify import committee, mempool
    w = synth.qc_votes(100, seed=9)
    with committee.Committee(w.pk) as cm:
        idx = np.arange(w.n, dtype=np.uint32)
        want = cm.verify_flags(idx, w.sig, w.msg)
        assert (want & 1).all()
        with _testing.injected_fault(mode):
            with pytest.raises(_lib.HsvLibraryError, match="HSV_ERR_DEVICE_FAULT"):
                cm.verify_flags(idx, w.sig, w.msg)
        assert (cm.verify_flags(idx, w.sig, w.msg) == want).all()
    t = synth.transactions(300, tx_size=200, seed=4, corrupt_frac=0.0)
    txs = [bytes(r) for r in t.txs]
    assert (mempool.verify_transactions(txs) & 1).all()
    with _testing.injected_fault(mode):
        with pytest.raises(_lib.HsvLibraryError, match="HSV_ERR_DEVICE_FAULT"):
            mempool.verify_transactions(txs)


def test_auto_committee_path_reports_faults(env, tlib, mode=1):
    """The drop-in verify_batch with the committee cache warm: the cached path
    faults (its view is dropped and the fault counted), the generic path it
    falls back to faults too, and the call returns the infrastructure error."""
    _lib, _testing, _, synth, verifier = env
    lib = tlib
    lib.hsv_set_auto_committee(1)
    w = synth.qc_votes(100, seed=11)
    packed = np.concatenate([w.pk, w.sig], axis=1).copy()
    for _ in range(3):
        assert lib.hsv_verify_batch_packed(w.msg.tobytes(), packed.tobytes(), w.n) == 1
    assert lib.hsv_auto_committee_wait(20000) == 1
    assert lib.hsv_verify_batch_packed(w.msg.tobytes(), packed.tobytes(), w.n) == 1
    assert lib.hsv_auto_committee_size() >= w.n
    faults = lib.hsv_auto_committee_faults()
    with _testing.injected_fault(mode):
        assert lib.hsv_verify_batch_packed(w.msg.tobytes(), packed.tobytes(), w.n) == FAULT
        assert lib.hsv_verify_strict(w.msg.tobytes(), w.pk[0].tobytes(), w.sig[0].tobytes()) == FAULT
    assert lib.hsv_auto_committee_faults() == faults + 1
    assert lib.hsv_auto_committee_size() == 0  # the cache is no longer trusted
    assert lib.hsv_verify_batch_packed(w.msg.tobytes(), packed.tobytes(), w.n) == 1


def test_auto_committee_corrupted_tables_are_dropped_and_relearnt(env, tlib):
    """only the cached tables are corrupted (zeroed in
    HBM, no injection).  The cached path's self-check fails; the call is
    answered by the generic kernels with the right verdicts, the fault is
    counted, the cache is dropped -- so later QCs do not pay the faulting
    kernel first -- and relearnt from the next batches."""
    _lib, _testing, _, synth, verifier = env
    lib = tlib
    lib.hsv_set_auto_committee(0)
    lib.hsv_set_auto_committee(1)
    w = synth.qc_votes(100, seed=12)
    bad = synth.qc_votes(100, seed=12, corrupt_frac=0.05)
    keep = ~np.isin(bad.kind, [synth.CORRUPTIONS.index(k) for k in synth.KEY_KINDS])
    packed = np.concatenate([w.pk, w.sig], axis=1).tobytes()
    packed_bad = np.concatenate([bad.pk[keep], bad.sig[keep]], axis=1).tobytes()
    d = w.msg.tobytes()
    for _ in range(3):
        assert lib.hsv_verify_batch_packed(d, packed, w.n) == 1
    assert lib.hsv_auto_committee_wait(20000) == 1
    assert lib.hsv_auto_committee_size() >= w.n
    faults = lib.hsv_auto_committee_faults()
    assert _testing.corrupt_auto_committee() >= w.n
    assert lib.hsv_verify_batch_packed(d, packed, w.n) == 1          # generic kernels answered
    assert lib.hsv_auto_committee_faults() == faults + 1
    assert lib.hsv_auto_committee_size() == 0
    assert lib.hsv_verify_batch_packed(bad.msg.tobytes(), packed_bad, int(keep.sum())) == 0
    # relearnt: two sightings queue the keys, the background build publishes them
    for _ in range(3):
        assert lib.hsv_verify_batch_packed(d, packed, w.n) == 1
    assert lib.hsv_auto_committee_wait(20000) == 1
    assert lib.hsv_auto_committee_size() >= w.n
    assert lib.hsv_verify_batch_packed(d, packed, w.n) == 1
    assert lib.hsv_verify_batch_packed(bad.msg.tobytes(), packed_bad, int(keep.sum())) == 0
    assert lib.hsv_auto_committee_faults() == faults + 1


def test_committee_path_canary_mode_is_not_a_fault(env, tlib, generic):
    """The committee kernels keep no workspace, so the canary injection (mode 2)
    has nothing to overwrite: the call verifies normally."""
    _lib, _testing, _, synth, verifier = env
    from hsverify import committee
    w = synth.qc_votes(100, seed=13, corrupt_frac=0.05)
    with committee.Committee(w.pk) as cm:
        idx = np.arange(w.n, dtype=np.uint32)
        want = cm.verify_flags(idx, w.sig, w.msg)
        with _testing.injected_fault(2):
            assert (cm.verify_flags(idx, w.sig, w.msg) == want).all()


@pytest.mark.parametrize("mode", [1, 2, 3])
def test_large_transaction_batch_reports_faults(env, tlib, mode):
    """More than 2^13 transactions: the fused launch (records, prepass and
    point pass in one kernel, hsv_launch_verify_tx), canary included (ADVICE
    round 3)."""
    _lib, _testing, _, synth, verifier = env
    from hsverify import mempool
    t = synth.transactions((1 << 13) + 64, tx_size=160, seed=14, corrupt_frac=0.0)
    want = mempool.verify_transactions_fixed(t.txs)
    assert (want & 1).all()
    with _testing.injected_fault(mode):
        with pytest.raises(_lib.HsvLibraryError, match="HSV_ERR_DEVICE_FAULT"):
            mempool.verify_transactions_fixed(t.txs)
    assert (mempool.verify_transactions_fixed(t.txs) == want).all()


@pytest.mark.parametrize("mode", [1, 2])
def test_pipelined_host_call_reports_faults(env, tlib, generic, mode):
    """A host batch of >= 2 pipeline chunks (2^18 items) runs run_pipelined,
    whose fault words sit after all the flags and are written from two compute
    streams."""
    _lib, _testing, _, synth, verifier = env
    w = synth.independent_triples((1 << 18) + 64, seed=15, corrupt_frac=0.0)
    with _testing.injected_fault(mode):
        with pytest.raises(_lib.HsvLibraryError, match="HSV_ERR_DEVICE_FAULT"):
            verifier.verify_flags(w.pk, w.sig, w.msg)
    got = verifier.verify_flags(w.pk, w.sig, w.msg)
    assert (got & 1).all()


def test_concurrent_device_calls_own_their_fault_words(env, tlib):
    """Round-3 VERDICT item 2: two device calls in flight on two streams, only
    one injected.  Each call's own fault words report only its own fault; the
    per-device word's read-and-clear is one atomic exchange, so a fault
    recorded while a reader clears is never lost."""
    import torch
    _lib, _testing, _, synth, verifier = env
    from hsverify import committee, mempool
    w = synth.independent_triples((1 << 14) + 5, seed=16, corrupt_frac=0.05)
    dev = torch.device("cuda:0")
    pk, sig, msg = (torch.from_numpy(a).to(dev) for a in (w.pk, w.sig, w.msg))
    s1, s2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    f1 = torch.zeros(w.n, dtype=torch.uint8, device=dev)
    f2 = torch.zeros(w.n, dtype=torch.uint8, device=dev)
    for mode in (1, 2):
        w1 = torch.full((2,), -1, dtype=torch.int32, device=dev)  # the library zeroes them
        w2 = torch.full((2,), -1, dtype=torch.int32, device=dev)
        torch.cuda.synchronize()
        with _testing.injected_fault(mode):
            verifier.verify_device(pk, sig, msg, f1, stream=s1.cuda_stream, fault=w1)
        verifier.verify_device(pk, sig, msg, f2, stream=s2.cuda_stream, fault=w2)
        torch.cuda.synchronize()
        assert verifier.fault_bits(w1) == (2 if mode == 2 else 1)
        assert verifier.fault_bits(w2) == 0
    want = verifier.verify_flags(w.pk, w.sig, w.msg)
    assert (f2.cpu().numpy() == want).all()
    # committee and transaction device calls take their own words too
    q = synth.qc_votes(100, seed=17)
    with committee.Committee(q.pk) as cm:
        idx = torch.arange(q.n, dtype=torch.int32, device=dev)
        qs = torch.from_numpy(q.sig).to(dev)
        qm = torch.from_numpy(np.repeat(q.msg[None], q.n, 0)).to(dev)
        qf = torch.zeros(q.n, dtype=torch.uint8, device=dev)
        wq = torch.full((2,), -1, dtype=torch.int32, device=dev)
        with _testing.injected_fault(1):
            cm.verify_device(idx, qs, qm, qf, stream=s1.cuda_stream, fault=wq)
        torch.cuda.synchronize()
        assert verifier.fault_bits(wq) == 1
    t = synth.transactions(300, tx_size=200, seed=18, corrupt_frac=0.0)
    txs = torch.from_numpy(np.ascontiguousarray(t.txs)).to(dev).view(-1)
    tf = torch.zeros(t.n, dtype=torch.uint8, device=dev)
    wt = torch.full((2,), -1, dtype=torch.int32, device=dev)
    mempool.verify_transactions_device(txs, tx_size=200, n=t.n, flags=tf, stream=s2.cuda_stream, fault=wt)
    torch.cuda.synchronize()
    assert verifier.fault_bits(wt) == 0 and (tf.cpu().numpy() & 1).all()
    # the per-device word (calls without words of their own): a read-and-clear
    # racing an injected launch either returns its fault or leaves it for the
    # next read
    verifier.device_faults(-1, clear=True)
    with _testing.injected_fault(1):
        verifier.verify_device(pk, sig, msg, f1, stream=s1.cuda_stream)
    first = verifier.device_faults(-1, clear=True)   # while the launch may still run
    torch.cuda.synchronize()
    second = verifier.device_faults(-1, clear=True)
    assert (first | second) == 1
    assert verifier.device_faults(-1, clear=True) == 0


def test_unpublished_transaction_batch_is_a_device_fault(env, tlib):
    """The fused transaction launch hands record batches to point batches
    through per-batch ready words.  With one batch never
    published (INJECT_NO_PUBLISH), the bounded waits end (0.5 s of the wall
    clock each): the launch finishes within seconds, its fault words report
    it, no transaction of that batch is accepted, the host API returns
    HSV_ERR_DEVICE_FAULT -- and without the hook the same call verifies."""
    import time
    import torch
    _lib, _testing, _, synth, verifier = env
    from hsverify import mempool
    t = synth.transactions((1 << 13) + 512, tx_size=200, seed=21, corrupt_frac=0.0)
    dev = torch.device("cuda:0")
    d = torch.from_numpy(np.ascontiguousarray(t.txs)).to(dev).view(-1)
    flags = torch.zeros(t.n, dtype=torch.uint8, device=dev)
    words = torch.full((2,), -1, dtype=torch.int32, device=dev)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    with _testing.injected_fault(_testing.INJECT_NO_PUBLISH):
        mempool.verify_transactions_device(d, tx_size=200, n=t.n, flags=flags, fault=words)
    torch.cuda.synchronize()
    assert time.perf_counter() - t0 < 20.0
    assert verifier.fault_bits(words) & 1
    got = flags.cpu().numpy()
    assert not (got[:64] & 1).any()  # batch 0: never verified, never accepted
    with _testing.injected_fault(_testing.INJECT_NO_PUBLISH):
        with pytest.raises(_lib.HsvLibraryError, match="HSV_ERR_DEVICE_FAULT"):
            mempool.verify_transactions_fixed(t.txs)
    assert (mempool.verify_transactions_fixed(t.txs) & 1).all()
