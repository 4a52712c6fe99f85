"""N > 1 path on CPU: world_size-2 gloo, contiguous shards, STRICT bitmask gather.

The per-rank verifier here is the C oracle (CPU); on MI355X the same
hsverify.dist code runs with the GPU verifier (bench.py)."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from conftest import ORACLE, PKG


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, n, q):
    import sys
    for p in (PKG, ORACLE, os.path.dirname(__file__)):
        sys.path.insert(0, p)
    import ctypes
    import torch.distributed as dist
    from hsverify import dist as hd, synth
    from conftest import oracle_flags

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        lib = ctypes.CDLL(os.path.join(ORACLE, "_build", "libhsv_oracle.so"))
        lib.oracle_verify_many.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_size_t] * 2 + [ctypes.c_void_p, ctypes.c_int]
        w = synth.independent_triples(n, seed=77, corrupt_frac=0.1, nthreads=2)  # same global batch on every rank
        lo, hi = hd.shard_range(n, rank, world)
        strict = hd.verify_sharded(w.pk, w.sig, w.msg, lambda p, s, m: oracle_flags(lib, p, s, m, nthreads=2))
        q.put((rank, lo, hi, strict.tolist(), w.honest.tolist()))
    finally:
        dist.destroy_process_group()


def test_shard_range_partitions():
    from hsverify import dist as hd
    for n in (0, 1, 7, 1000, 1 << 20):
        for world in (1, 2, 3, 8):
            ranges = [hd.shard_range(n, r, world) for r in range(world)]
            assert ranges[0][0] == 0 and ranges[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(ranges, ranges[1:]))


def test_bit_packing_roundtrip():
    from hsverify import dist as hd
    rng = np.random.default_rng(0)
    for n in (1, 31, 32, 33, 1000):
        flags = rng.integers(0, 256, n).astype(np.uint8)
        words = hd.pack_strict_bits(flags)
        assert words.size == (n + 31) // 32
        assert (hd.unpack_strict_bits(words, n) == (flags & 1).astype(bool)).all()
        # kernel layout: bit i of word i // 32
        i = n - 1
        assert bool((words[i // 32] >> (i % 32)) & 1) == bool(flags[i] & 1)


def test_world_size_2_gloo_gather_matches_single_process(oracle_lib, tmp_path):
    from conftest import oracle_flags
    from hsverify import synth
    n, world = 301, 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    w = synth.independent_triples(n, seed=77, corrupt_frac=0.1, nthreads=2)
    expect = (oracle_flags(oracle_lib, w.pk, w.sig, w.msg) & 1).astype(bool)
    for rank, lo, hi, strict, honest in sorted(res):
        assert (np.array(strict) == expect).all()          # every rank holds the global vector
        assert (np.array(strict)[np.array(honest)]).all()  # honest items accepted
    (r0, r1) = sorted(res)
    assert r0[1] == 0 and r0[2] == r1[1] and r1[2] == n   # contiguous disjoint shards
