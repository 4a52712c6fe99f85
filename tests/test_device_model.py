"""The boundary's device model (include/hsv.h, hsv_init) on the GPU.

* hsv_init(d) binds host-buffer calls to device d; hsv_init(-1) selects every
  device (large host batches sharded by contiguous range).
* The multi-device shard / thread / gather path of run_host runs with
  virtual shards mapped onto the one GPU of the box (hsv_set_virtual_shards),
  compared with the unsharded result and the C oracle.
* Slot pools: concurrent host calls from many threads stay exact.
* Committees survive hsv_shutdown (the B table is rebuilt on use); the
  automatic cache ignores batches above its 8192-key capacity.
The reference runs several nodes per process on a multi-thread runtime
(node/src/main.rs:16, consensus/src/tests/consensus_tests.rs:10-56), which is
what the binding and the slot pools serve.
"""
import threading

import numpy as np
import pytest

import ed25519_ref as o
from conftest import oracle_flags

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def mods(hsv):
    from hsverify import _lib, committee, synth, verifier
    return _lib, committee, synth, verifier


def test_init_binds_and_reports_device(mods, hsv):
    _lib, _, synth, verifier = mods
    ndev = hsv.hsv_device_count()
    try:
        assert verifier.bind_device(0) == 1
        assert hsv.hsv_bound_device() == 0
        w = synth.qc_votes(100, seed=12)
        assert (verifier.verify_flags(w.pk, w.sig, w.msg) & o.STRICT_OK).all()
        assert hsv.hsv_init(ndev) < 0                      # out of range: an error, binding unchanged
        assert hsv.hsv_bound_device() == 0
        assert hsv.hsv_init(-2) < 0
        assert verifier.bind_device(-1) == ndev
        assert hsv.hsv_bound_device() == -1
        assert (verifier.verify_flags(w.pk, w.sig, w.msg) & o.STRICT_OK).all()
    finally:
        hsv.hsv_init(-1)


@pytest.mark.parametrize("shards", [2, 3, 5, 8])
def test_virtual_shards_gather_matches_unsharded_and_oracle(mods, oracle_lib, shards):
    """run_host's multi-device path: contiguous shards, each on the persistent
    shard worker of its index (pinned to its GPU's NUMA node, run_sharded) with
    a slot and the device's pack pool, flags written into the caller's buffer
    at the shard offsets; k = 8 as on an 8-GPU node (more shards than slots:
    they queue for the device's four slots)."""
    _, _, synth, verifier = mods
    from hsverify import _testing
    n = (1 << 16) + 12345
    w = synth.independent_triples(n, seed=500 + shards, corrupt_frac=0.05)
    with _testing.test_library():
        verifier.set_virtual_shards(0)
        whole = verifier.verify_flags(w.pk, w.sig, w.msg)
        try:
            verifier.set_virtual_shards(shards)
            sharded = verifier.verify_flags(w.pk, w.sig, w.msg)
        finally:
            verifier.set_virtual_shards(0)
    assert (sharded == whole).all()
    assert (whole[w.accept] & o.STRICT_OK).all() and not (whole[~w.accept] & o.STRICT_OK).any()
    # oracle sample around every shard boundary
    cuts = [n * d // shards for d in range(1, shards)]
    idx = np.unique(np.concatenate([np.arange(max(0, c - 40), min(n, c + 40)) for c in cuts] + [np.arange(64)]))
    assert (sharded[idx] == oracle_flags(oracle_lib, w.pk[idx], w.sig[idx], w.msg[idx])).all()


def test_virtual_shards_transactions(mods, oracle_lib):
    from hsverify import mempool
    _, _, synth, verifier = mods
    from hsverify import _testing
    n = (1 << 16) + 77
    w = synth.transactions(n, tx_size=200, seed=31)
    with _testing.test_library():
        whole = mempool.verify_transactions_fixed(w.txs)
        try:
            verifier.set_virtual_shards(4)
            sharded = mempool.verify_transactions_fixed(w.txs)
        finally:
            verifier.set_virtual_shards(0)
    assert (sharded == whole).all()
    assert (whole[w.accept] & o.STRICT_OK).all() and not (whole[~w.accept] & o.STRICT_OK).any()


def test_many_concurrent_small_calls(mods, golden):
    """More threads than slots: QC-sized and single-vote calls interleave."""
    _, _, _, verifier = mods
    errors = []

    def work(k):
        try:
            rng = np.random.default_rng(k)
            for _ in range(6):
                m = int(rng.integers(1, 700))
                sl = rng.integers(0, len(golden["flags"]), m)
                got = verifier.verify_flags(golden["pk"][sl], golden["sig"][sl], golden["msg"][sl])
                if not (got == golden["flags"][sl]).all():
                    errors.append(k)
        except Exception as e:  # pragma: no cover - reported below
            errors.append(repr(e))

    th = [threading.Thread(target=work, args=(k,)) for k in range(12)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errors


def test_device_batches_on_concurrent_streams(mods, golden):
    """bench.py's form: consecutive device batches alternating over three
    streams, with a mid-size batch (two-pass kernels) and a small one (latency
    form) in flight together; each launch takes its workspace from the
    library's pool on its own stream.  Every output equals the one-stream
    result and the golden flags."""
    import torch
    _, _, synth, verifier = mods
    dev = torch.device("cuda", 0)
    n = (1 << 15) + 333
    w = synth.independent_triples(n, seed=77, corrupt_frac=0.05)
    pk, sig, msg = (torch.from_numpy(x).to(dev) for x in (w.pk, w.sig, w.msg))
    g = golden
    gpk, gsig, gmsg = (torch.from_numpy(np.ascontiguousarray(g[k])).to(dev) for k in ("pk", "sig", "msg"))
    ref = torch.zeros(n, dtype=torch.uint8, device=dev)
    verifier.verify_device(pk, sig, msg, ref)
    torch.cuda.synchronize(dev)
    streams = [torch.cuda.Stream(dev) for _ in range(3)]
    outs = [torch.zeros(n, dtype=torch.uint8, device=dev) for _ in range(6)]
    gouts = [torch.zeros(len(g["flags"]), dtype=torch.uint8, device=dev) for _ in range(6)]
    for i in range(6):
        s = streams[i % 3].cuda_stream
        verifier.verify_device(pk, sig, msg, outs[i], stream=s)
        verifier.verify_device(gpk, gsig, gmsg, gouts[i], stream=s)
    torch.cuda.synchronize(dev)
    for i in range(6):
        assert torch.equal(outs[i], ref), i
        assert (gouts[i].cpu().numpy() == g["flags"]).all(), i
    f = ref.cpu().numpy()
    assert (f[w.accept] & o.STRICT_OK).all() and not (f[~w.accept] & o.STRICT_OK).any()


def test_distinct_batches_on_concurrent_streams(mods):
    """Concurrent launches on different streams over DIFFERENT inputs (the
    form above uses one input set, which cannot show two launches sharing a
    workspace): three large batches and their flags, alternating over two
    streams, two rounds, each output equal to its batch's one-stream result."""
    import torch
    _, _, synth, verifier = mods
    dev = torch.device("cuda", 0)
    n = (1 << 16) + 77
    sets, refs = [], []
    for k in range(3):
        w = synth.independent_triples(n, seed=300 + k, corrupt_frac=0.2)
        t = tuple(torch.from_numpy(x).to(dev) for x in (w.pk, w.sig, w.msg))
        r = torch.zeros(n, dtype=torch.uint8, device=dev)
        verifier.verify_device(*t, r)
        torch.cuda.synchronize(dev)
        sets.append(t)
        refs.append(r)
    streams = [torch.cuda.Stream(dev) for _ in range(2)]
    outs = [torch.zeros(n, dtype=torch.uint8, device=dev) for _ in range(6)]
    for i in range(6):
        verifier.verify_device(*sets[i % 3], outs[i], stream=streams[i % 2].cuda_stream)
    torch.cuda.synchronize(dev)
    for i in range(6):
        assert torch.equal(outs[i], refs[i % 3]), (i, int((outs[i] != refs[i % 3]).sum()))


@pytest.mark.parametrize("n", [(1 << 16) + 77, 3000, 600, 200])
def test_batches_behind_cross_stream_event_chains(mods, n):
    """A pipeline whose streams order their work through events recorded on
    each other (the mempool split form of tools/mempool_split_probe.py: a
    producer stream waits for the batch that used its buffer, the consumer
    streams wait for the producer): two launches in flight on two streams must
    never share a workspace block.  Round 5 found them doing so through the
    pool's event-dependency reuse (profiles/r05ar_mempool_split.txt); every
    output must equal its batch's one-stream result.  Sizes: the two-pass
    kernels, the row, joint and quad latency forms."""
    import torch
    _, _, synth, verifier = mods
    dev = torch.device("cuda", 0)
    sets, refs = [], []
    for k in range(3):
        w = synth.independent_triples(n, seed=310 + k, corrupt_frac=0.2)
        t = tuple(torch.from_numpy(x).to(dev) for x in (w.pk, w.sig, w.msg))
        r = torch.zeros(n, dtype=torch.uint8, device=dev)
        verifier.verify_device(*t, r)
        torch.cuda.synchronize(dev)
        sets.append(t)
        refs.append(r)
    prod = torch.cuda.Stream(dev)
    cons = [torch.cuda.Stream(dev) for _ in range(2)]
    bufs = [torch.zeros(n, 128, dtype=torch.uint8, device=dev) for _ in range(3)]
    steps = 10
    outs = [torch.zeros(n, dtype=torch.uint8, device=dev) for _ in range(steps)]
    done = []
    verifier.device_faults(-1, clear=True)
    for k in range(steps):
        if k >= 3:
            prod.wait_event(done[k - 3])
        with torch.cuda.stream(prod):
            bufs[k % 3].add_(1)  # the producer's work on the batch's buffer
        ev = torch.cuda.Event()
        ev.record(prod)
        c = cons[k % 2]
        c.wait_event(ev)
        verifier.verify_device(*sets[k % 3], outs[k], stream=c.cuda_stream)
        ev2 = torch.cuda.Event()
        ev2.record(c)
        done.append(ev2)
    torch.cuda.synchronize(dev)
    bad = [int((outs[k] != refs[k % 3]).sum()) for k in range(steps)]
    faults = verifier.device_faults(-1, clear=True)
    assert not any(bad) and faults == 0, (bad, faults)


def test_transaction_batches_behind_cross_stream_event_chains(mods):
    """The same event-ordered pipeline through the transaction device call
    (records + the fused prepass above 2^13 items, workspaces from the pool):
    every batch's flags equal its one-stream result, with no fault."""
    import torch
    from hsverify import mempool
    _, _, synth, verifier = mods
    dev = torch.device("cuda", 0)
    n, size = (1 << 14) + 5, 200
    sets, refs = [], []
    for k in range(3):
        t = synth.transactions(n, tx_size=size, seed=320 + k, corrupt_frac=0.2)
        d = torch.from_numpy(np.ascontiguousarray(t.txs)).to(dev).view(-1)
        r = torch.zeros(n, dtype=torch.uint8, device=dev)
        mempool.verify_transactions_device(d, tx_size=size, n=n, flags=r)
        torch.cuda.synchronize(dev)
        sets.append(d)
        refs.append(r)
    prod = torch.cuda.Stream(dev)
    cons = [torch.cuda.Stream(dev) for _ in range(2)]
    bufs = [torch.zeros(n, 128, dtype=torch.uint8, device=dev) for _ in range(3)]
    steps = 10
    outs = [torch.zeros(n, dtype=torch.uint8, device=dev) for _ in range(steps)]
    done = []
    verifier.device_faults(-1, clear=True)
    for k in range(steps):
        if k >= 3:
            prod.wait_event(done[k - 3])
        with torch.cuda.stream(prod):
            bufs[k % 3].add_(1)
        ev = torch.cuda.Event()
        ev.record(prod)
        c = cons[k % 2]
        c.wait_event(ev)
        mempool.verify_transactions_device(sets[k % 3], tx_size=size, n=n, flags=outs[k], stream=c.cuda_stream)
        ev2 = torch.cuda.Event()
        ev2.record(c)
        done.append(ev2)
    torch.cuda.synchronize(dev)
    bad = [int((outs[k] != refs[k % 3]).sum()) for k in range(steps)]
    faults = verifier.device_faults(-1, clear=True)
    assert not any(bad) and faults == 0, (bad, faults)


def test_committee_survives_shutdown(mods, hsv, golden):
    _, committee, _, _ = mods
    keys = golden["pk"][:8]
    with committee.Committee(keys) as c:
        hsv.hsv_shutdown()                       # frees the B tables and staging slots
        got = c.verify_flags(np.arange(8, dtype=np.uint32), golden["sig"][:8], golden["msg"][:8])
        assert (got == golden["flags"][:8]).all()


def test_auto_cache_ignores_batches_above_capacity(mods, hsv):
    """A recurring 8193-vote batch is never cached (the cache holds 8192 keys at
    most) and its verdict is the generic one."""
    _, _, synth, verifier = mods
    hsv.hsv_set_auto_committee(0)
    hsv.hsv_set_auto_committee(1)
    try:
        n = 8193
        seeds = synth.committee_seeds(n, 3)
        digest = np.frombuffer(bytes(range(32)), np.uint8)
        pk, sig = verifier.sign_many(seeds, np.repeat(digest[None], n, 0))
        packed = np.concatenate([pk, sig], 1).tobytes()
        for _ in range(3):
            assert hsv.hsv_verify_batch_packed(bytes(digest), packed, n) == 1
        assert hsv.hsv_auto_committee_wait(30000) == 1
        assert hsv.hsv_auto_committee_size() == 0
        bad = bytearray(packed)
        bad[96 * 4000 + 40] ^= 1
        assert hsv.hsv_verify_batch_packed(bytes(digest), bytes(bad), n) == 0
    finally:
        hsv.hsv_set_auto_committee(0)
        hsv.hsv_set_auto_committee(1)


def test_auto_cache_counts_a_key_once_per_batch(mods, hsv):
    """A key repeated inside one batch (a duplicated vote) is not 'recurring'."""
    _, _, synth, _ = mods
    hsv.hsv_set_auto_committee(0)
    hsv.hsv_set_auto_committee(1)
    try:
        w = synth.qc_votes(4, seed=77)
        votes = np.concatenate([w.pk, w.sig], 1)
        dup = np.concatenate([votes, votes], 0).tobytes()   # every key twice in one batch
        assert hsv.hsv_verify_batch_packed(bytes(w.msg), dup, 2 * w.n) == 1
        assert hsv.hsv_auto_committee_wait(30000) == 1
        assert hsv.hsv_auto_committee_size() == 0
        assert hsv.hsv_verify_batch_packed(bytes(w.msg), dup, 2 * w.n) == 1   # second batch: now recurring
        assert hsv.hsv_auto_committee_wait(30000) == 1
        assert hsv.hsv_auto_committee_size() == w.n
        assert hsv.hsv_verify_batch_packed(bytes(w.msg), dup, 2 * w.n) == 1   # through the cache
    finally:
        hsv.hsv_set_auto_committee(0)
        hsv.hsv_set_auto_committee(1)
