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
def generic(env):
    """The automatic committee cache off, so the generic kernels run."""
    lib = env[0].load()
    lib.hsv_set_auto_committee(0)
    yield
    lib.hsv_set_auto_committee(1)


@pytest.mark.parametrize("mode", [1, 2, 3])
def test_generic_paths_report_faults(env, generic, mode):
    _lib, _testing, crypto, synth, verifier = env
    lib = _lib.load()
    w = synth.qc_votes(100, seed=5)                                # 67 votes, row-form latency kernel
    mid = synth.independent_triples(4096, seed=8, corrupt_frac=0.0)  # pair latency kernel (3073..8192)
    big = synth.independent_triples((1 << 13) + 64, seed=6, corrupt_frac=0.0)  # point-pass kernels
    packed = np.concatenate([w.pk, w.sig], axis=1).copy()
    want_small = verifier.verify_flags(w.pk, w.sig, w.msg)
    want_mid = verifier.verify_flags(mid.pk, mid.sig, mid.msg)
    want_big = verifier.verify_flags(big.pk, big.sig, big.msg)
    assert (want_small & 1).all() and (want_mid & 1).all() and (want_big & 1).all()
    with _testing.injected_fault(mode):
        for pk, sig, msg in ((w.pk, w.sig, w.msg), (mid.pk, mid.sig, mid.msg), (big.pk, big.sig, big.msg)):
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
def test_device_api_records_faults(env, mode):
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
def test_committee_and_transaction_paths_report_faults(env, generic, mode):
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


def test_auto_committee_path_reports_faults(env, mode=1):
    """The drop-in verify_batch with the committee cache warm: the cached path
    faults, the generic path it falls back to faults too, and the call returns
    the infrastructure error."""
    _lib, _testing, _, synth, verifier = env
    lib = _lib.load()
    lib.hsv_set_auto_committee(1)
    w = synth.qc_votes(100, seed=11)
    packed = np.concatenate([w.pk, w.sig], axis=1).copy()
    for _ in range(3):
        assert lib.hsv_verify_batch_packed(w.msg.tobytes(), packed.tobytes(), w.n) == 1
    assert lib.hsv_auto_committee_wait(20000) == 1
    assert lib.hsv_verify_batch_packed(w.msg.tobytes(), packed.tobytes(), w.n) == 1
    assert lib.hsv_auto_committee_size() >= w.n
    with _testing.injected_fault(mode):
        assert lib.hsv_verify_batch_packed(w.msg.tobytes(), packed.tobytes(), w.n) == FAULT
        assert lib.hsv_verify_strict(w.msg.tobytes(), w.pk[0].tobytes(), w.sig[0].tobytes()) == FAULT
    assert lib.hsv_verify_batch_packed(w.msg.tobytes(), packed.tobytes(), w.n) == 1
