"""Multi-GPU sharding of independent verifications.

One process per GPU.  Rank r owns the contiguous range shard_range(n, r, world)
of the global batch and verifies it on its own device with no data-path
collective.  The only exchange is the final host gather of the per-signature
STRICT_OK bitmask (n/8 bytes in total), done here with torch.distributed
all_gather over whatever process group the caller initialised (gloo on CPU,
nccl = RCCL on MI355X; the bitmask is tiny, so the backend does not matter).
"""
from __future__ import annotations

import numpy as np


def shard_range(n: int, rank: int, world: int) -> tuple:
    """Contiguous [lo, hi) of n items for rank r of world (sizes differ by <= 1)."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("bad rank/world")
    return n * rank // world, n * (rank + 1) // world


def pack_strict_bits(flags: np.ndarray) -> np.ndarray:
    """Per-item flag bytes -> STRICT_OK bitmask, bit i of word i//32 (little-endian)."""
    bits = (np.asarray(flags, np.uint8) & 1).astype(np.uint8)
    pad = (-bits.size) % 32
    if pad:
        bits = np.concatenate([bits, np.zeros(pad, np.uint8)])
    return np.packbits(bits, bitorder="little").view("<u4")


def unpack_strict_bits(words: np.ndarray, n: int) -> np.ndarray:
    b = np.unpackbits(np.ascontiguousarray(words, "<u4").view(np.uint8), bitorder="little")
    return b[:n].astype(bool)


def gather_strict(flags_local: np.ndarray, n_global: int, group=None) -> np.ndarray:
    """All-gather every rank's STRICT_OK bits into the global boolean vector."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    words = pack_strict_bits(flags_local)
    sizes = [shard_range(n_global, r, world) for r in range(world)]
    maxw = max((hi - lo + 31) // 32 for lo, hi in sizes)
    buf = torch.zeros(maxw, dtype=torch.int32)
    buf[: words.size] = torch.from_numpy(words.view(np.int32).copy())
    out = [torch.zeros(maxw, dtype=torch.int32) for _ in range(world)]
    dist.all_gather(out, buf, group=group)
    parts = []
    for r, (lo, hi) in enumerate(sizes):
        parts.append(unpack_strict_bits(out[r].numpy().view("<u4"), hi - lo))
    return np.concatenate(parts)


def verify_sharded(pk, sig, msg, verify_local, group=None) -> np.ndarray:
    """Each rank verifies its contiguous shard with ``verify_local(pk, sig, msg)``
    (the GPU path on MI355X) and all ranks receive the global STRICT_OK vector."""
    import torch.distributed as dist

    world, rank = dist.get_world_size(group), dist.get_rank(group)
    n = pk.shape[0]
    lo, hi = shard_range(n, rank, world)
    m = msg if msg.ndim == 1 else msg[lo:hi]
    flags = verify_local(pk[lo:hi], sig[lo:hi], m)
    return gather_strict(flags, n, group)
