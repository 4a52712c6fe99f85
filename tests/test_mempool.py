"""Mempool transaction verification.

The reference's transaction check (mempool/src/batch_maker.rs:79-85,
consensus/src/core.rs:121-127): tx = message || pk || sig, accepted iff
Signature::verify(Digest(SHA-512(message)[..32]), pk).  CPU tests pin the C
oracle against the committed golden vectors (tests/golden/make_tx_golden.py,
expected flags from oracle/ed25519_ref.py, cross-checked with libsodium) and
the host-side argument checks; GPU tests compare the HIP path (record kernel +
verification kernels, through the C ABI) with the oracle bit-exactly.
"""
import os

import numpy as np
import pytest

import ed25519_ref as o
from conftest import oracle_tx_flags


def _pack(txs):
    from hsverify import mempool
    return mempool.pack(txs)


# ---- CPU ------------------------------------------------------------------
def test_oracle_matches_tx_golden(oracle_lib, tx_golden):
    buf, offsets = _pack(tx_golden["txs"])
    got = oracle_tx_flags(oracle_lib, buf, offsets)
    bad = np.nonzero(got != tx_golden["flags"])[0]
    assert bad.size == 0, [(tx_golden["cases"][i], int(got[i])) for i in bad]


def test_tx_golden_semantics(tx_golden):
    """Honest transactions accepted, every corruption rejected (the verdict the
    reference's BatchMaker filters on)."""
    for case, f in zip(tx_golden["cases"], tx_golden["flags"]):
        assert bool(f & o.STRICT_OK) == case.startswith("honest"), case


def test_oracle_fixed_size_layout(oracle_lib):
    from hsverify import synth  # noqa: F401  (import check only; signing needs libhsv)
    txs = [t for t in _fixed_txs(8, 512)]
    buf = np.frombuffer(b"".join(txs), np.uint8)
    got = oracle_tx_flags(oracle_lib, buf, tx_size=512, n=len(txs))
    assert (got & o.STRICT_OK).all()


def _fixed_txs(n, size, seed=3):
    rnd = np.random.default_rng(seed)
    out = []
    for i in range(n):
        s = bytes(rnd.integers(0, 256, 32, dtype=np.uint8))
        m = bytes(rnd.integers(0, 256, size - 96, dtype=np.uint8))
        import hashlib
        d = hashlib.sha512(m).digest()[:32]
        out.append(m + o.public_key(s) + o.sign(s, d))
    return out


def test_short_transaction_is_an_argument_error(hsv_lib_cpu):
    """A transaction under 96 bytes makes the reference's slice panic; the host
    API refuses it before touching a device (so this runs without a GPU)."""
    from hsverify import _lib, mempool
    with pytest.raises(_lib.HsvLibraryError):
        mempool.verify_transactions([bytes(200), bytes(95)])
    with pytest.raises(_lib.HsvLibraryError):
        mempool.verify_transactions_fixed(np.zeros((4, 90), np.uint8))
    assert mempool.verify_transactions([]).size == 0


@pytest.fixture(scope="module")
def hsv_lib_cpu():
    from hsverify import _lib
    return _lib.load(require=True)


# ---- GPU ------------------------------------------------------------------
@pytest.mark.gpu
def test_tx_golden_ragged_host_api(hsv, tx_golden):
    from hsverify import mempool
    got = mempool.verify_transactions(tx_golden["txs"])
    bad = np.nonzero(got != tx_golden["flags"])[0]
    assert bad.size == 0, [(tx_golden["cases"][i], int(got[i]), int(tx_golden["flags"][i])) for i in bad]


@pytest.mark.gpu
def test_tx_golden_every_variant(hsv, tx_golden):
    from hsverify import _testing, mempool, verifier
    with _testing.test_library():
        default = verifier.get_variant()
        try:
            for v in verifier.variants():
                verifier.set_variant(v)
                got = mempool.verify_transactions(tx_golden["txs"])
                assert (got == tx_golden["flags"]).all(), (v, np.nonzero(got != tx_golden["flags"])[0][:8])
        finally:
            verifier.set_variant(default)


@pytest.mark.gpu
def test_tx_reference_call_shapes(hsv, tx_golden):
    """BatchMaker keeps the passing transactions; Core::make_vote needs all."""
    from hsverify import mempool
    txs = tx_golden["txs"]
    honest = [t for t, c in zip(txs, tx_golden["cases"]) if c.startswith("honest")]
    assert mempool.filter_transactions(txs) == honest
    assert mempool.verify_batch_transactions(honest)
    assert not mempool.verify_batch_transactions(txs)
    assert mempool.verify_batch_transactions([])


@pytest.mark.gpu
@pytest.mark.parametrize("size", [96, 97, 207, 208, 512, 1024])
def test_tx_fixed_size_vs_oracle(hsv, oracle_lib, size):
    from hsverify import mempool, synth
    w = synth.transactions(1000, tx_size=size, seed=size, corrupt_frac=0.05)
    got = mempool.verify_transactions_fixed(w.txs)
    exp = oracle_tx_flags(oracle_lib, w.txs.reshape(-1), tx_size=size, n=w.n)
    assert (got == exp).all(), np.nonzero(got != exp)[0][:8]
    assert (got[w.accept] & o.STRICT_OK).all() and not (got[~w.accept] & o.STRICT_OK).any()


@pytest.mark.gpu
def test_tx_ragged_random_vs_oracle(hsv, oracle_lib):
    """Random lengths 96..1200 bytes, so every start alignment and block count
    occurs inside one wave."""
    import hashlib
    from hsverify import mempool, verifier
    rnd = np.random.default_rng(11)
    n = 3000
    lens = rnd.integers(0, 1100, n)
    msgs = [rnd.integers(0, 256, int(m), dtype=np.uint8).tobytes() for m in lens]
    seeds = rnd.integers(0, 256, (n, 32), dtype=np.uint8)
    dig = np.stack([np.frombuffer(hashlib.sha512(m).digest()[:32], np.uint8) for m in msgs])
    pk, sig = verifier.sign_many(seeds, dig)
    sig[::17, 40] ^= 1                     # some bad signatures
    txs = [m + pk[i].tobytes() + sig[i].tobytes() for i, m in enumerate(msgs)]
    txs[5] = b"\x01" + txs[5]              # message changed -> digest changed
    buf, offsets = mempool.pack(txs)
    got = mempool.verify_transactions(txs)
    exp = oracle_tx_flags(oracle_lib, buf, offsets)
    assert (got == exp).all(), np.nonzero(got != exp)[0][:8]
    assert not (got[5] & o.STRICT_OK) and not (got[::17] & o.STRICT_OK).any()


@pytest.mark.gpu
def test_tx_device_api_unaligned_offsets_bits_and_short(hsv, oracle_lib):
    """Device-resident ragged transactions at an odd base address, STRICT_OK bit
    packing, and a short (< 96 B) transaction that must get flags 0."""
    import hashlib
    import torch
    from hsverify import mempool, verifier
    rnd = np.random.default_rng(12)
    n = 777
    lens = rnd.integers(0, 700, n)
    msgs = [rnd.integers(0, 256, int(m), dtype=np.uint8).tobytes() for m in lens]
    seeds = rnd.integers(0, 256, (n, 32), dtype=np.uint8)
    dig = np.stack([np.frombuffer(hashlib.sha512(m).digest()[:32], np.uint8) for m in msgs])
    pk, sig = verifier.sign_many(seeds, dig)
    sig[::9, 1] ^= 4
    txs = [m + pk[i].tobytes() + sig[i].tobytes() for i, m in enumerate(msgs)]
    txs[100] = txs[100][:60]               # short transaction
    buf, offsets = mempool.pack(txs)
    exp = oracle_tx_flags(oracle_lib, buf, offsets)
    assert exp[100] == 0
    dev = torch.device("cuda:0")
    backing = torch.zeros(buf.size + 64, dtype=torch.uint8, device=dev)
    d_txs = backing[3:3 + buf.size]
    d_txs.copy_(torch.from_numpy(buf))
    d_off = torch.from_numpy(offsets.view(np.int64)).to(dev)
    flags = torch.zeros(n, dtype=torch.uint8, device=dev)
    bits = torch.zeros((n + 31) // 32, dtype=torch.int32, device=dev)
    mempool.verify_transactions_device(d_txs, d_off, n=n, flags=flags, strict_bits=bits)
    torch.cuda.synchronize()
    got = flags.cpu().numpy()
    assert (got == exp).all(), np.nonzero(got != exp)[0][:8]
    b = bits.cpu().numpy().view(np.uint32)
    unpacked = np.array([(b[i // 32] >> (i % 32)) & 1 for i in range(n)], np.uint8)
    assert (unpacked == (exp & o.STRICT_OK)).all()


@pytest.mark.gpu
def test_tx_device_fixed_2p16_vs_oracle(hsv, oracle_lib):
    """The reference benchmark's 512-byte transactions, 2^16 on the device API,
    bit-exact against the C oracle, and idempotent."""
    import torch
    from hsverify import mempool, synth
    w = synth.transactions(1 << 16, tx_size=512, seed=7)
    dev = torch.device("cuda:0")
    d = torch.from_numpy(w.txs.reshape(-1)).to(dev)
    flags = torch.zeros(w.n, dtype=torch.uint8, device=dev)
    mempool.verify_transactions_device(d, None, tx_size=512, n=w.n, flags=flags)
    torch.cuda.synchronize()
    got = flags.cpu().numpy()
    exp = oracle_tx_flags(oracle_lib, w.txs.reshape(-1), tx_size=512, n=w.n)
    assert (got == exp).all(), np.nonzero(got != exp)[0][:8]
    flags2 = torch.zeros_like(flags)
    mempool.verify_transactions_device(d, None, tx_size=512, n=w.n, flags=flags2)
    torch.cuda.synchronize()
    assert torch.equal(flags, flags2)


def _ragged_txs(seed, n, max_msg):
    import hashlib
    from hsverify import verifier
    rnd = np.random.default_rng(seed)
    lens = rnd.integers(0, max_msg, n)
    msgs = [rnd.integers(0, 256, int(m), dtype=np.uint8).tobytes() for m in lens]
    seeds = rnd.integers(0, 256, (n, 32), dtype=np.uint8)
    dig = np.stack([np.frombuffer(hashlib.sha512(m).digest()[:32], np.uint8) for m in msgs])
    pk, sig = verifier.sign_many(seeds, dig)
    sig[::13, 7] ^= 2                      # bad R
    sig[5::29, 40] ^= 1                    # bad s
    return [m + pk[i].tobytes() + sig[i].tobytes() for i, m in enumerate(msgs)]


@pytest.mark.gpu
@pytest.mark.parametrize("bits", [0, 128])
def test_tx_fused_launch_ragged_unaligned_vs_oracle(hsv, oracle_lib, bits):
    """Above 2^13 transactions the device path is ONE launch: record batches,
    then point batches behind per-batch ready words, then the fallback list
    (hsv_verify_tx_fused_kernel).  Ragged lengths at an odd base
    address, short transactions, flags and STRICT_OK bits, against the C
    oracle; with the lattice bound lowered to 128 (test library) items without
    a short pair go down the fallback list the launch runs last.  Run twice:
    the outputs must not depend on which wave published which batch."""
    import torch
    from hsverify import _testing, mempool
    n = 12000
    txs = _ragged_txs(31 + bits, n, 700)
    for i in (100, 8191, 11999):
        txs[i] = txs[i][:50]               # short transactions: flags 0
    buf, offsets = mempool.pack(txs)
    exp = oracle_tx_flags(oracle_lib, buf, offsets)
    assert exp[100] == 0 and exp[11999] == 0 and (exp & o.STRICT_OK).sum() > n // 2
    dev = torch.device("cuda:0")
    backing = torch.zeros(buf.size + 64, dtype=torch.uint8, device=dev)
    d_txs = backing[5:5 + buf.size]
    d_txs.copy_(torch.from_numpy(buf))
    d_off = torch.from_numpy(offsets.view(np.int64)).to(dev)
    with _testing.test_library():
        prev = _testing.set_lattice_bits(bits)
        try:
            for _ in range(2):
                flags = torch.zeros(n, dtype=torch.uint8, device=dev)
                bits_out = torch.zeros((n + 31) // 32, dtype=torch.int32, device=dev)
                fault = torch.zeros(2, dtype=torch.int32, device=dev)
                mempool.verify_transactions_device(d_txs, d_off, n=n, flags=flags, strict_bits=bits_out, fault=fault)
                torch.cuda.synchronize()
                got = flags.cpu().numpy()
                assert (got == exp).all(), np.nonzero(got != exp)[0][:8]
                b = bits_out.cpu().numpy().view(np.uint32)
                unpacked = (b[np.arange(n) // 32] >> (np.arange(n) % 32)) & 1
                assert (unpacked == (exp & o.STRICT_OK)).all()
                assert not fault.cpu().numpy().any()
        finally:
            _testing.set_lattice_bits(prev)


@pytest.mark.gpu
def test_tx_fused_and_two_launch_forms_agree():
    """HSV_TX_FUSED=0 (record kernel + point pass, the round-5 form) and the
    fused launch give the same flags on 2^15 fixed-size transactions with
    corruptions (a child process per form: the switch is read once)."""
    import subprocess
    import sys
    from conftest import ROOT
    child = r"""
import sys, numpy as np, torch
sys.path.insert(0, %r); sys.path.insert(0, %r + "/hotstuff-digital-signature-benchmarking_amd")
from hsverify import mempool, synth
w = synth.transactions(1 << 15, tx_size=333, seed=77, corrupt_frac=0.05)
d = torch.from_numpy(w.txs.reshape(-1)).to("cuda:0")
f = torch.zeros(w.n, dtype=torch.uint8, device="cuda:0")
mempool.verify_transactions_device(d, None, tx_size=333, n=w.n, flags=f)
torch.cuda.synchronize()
sys.stdout.buffer.write(f.cpu().numpy().tobytes())
""" % (ROOT, ROOT)
    outs = []
    for fused in ("1", "0"):
        env = dict(os.environ, HSV_TX_FUSED=fused)
        r = subprocess.run([sys.executable, "-c", child], capture_output=True, timeout=180, env=env)
        assert r.returncode == 0, r.stderr.decode()[-2000:]
        outs.append(np.frombuffer(r.stdout, np.uint8))
    assert outs[0].size == 1 << 15 and (outs[0] == outs[1]).all()
    assert (outs[0] & o.STRICT_OK).sum() > (1 << 14)
