"""Synthetic workloads for the BASELINE.json configs (no network, no datasets).

C1  QC, 4-node committee: 3 votes over one digest
C2  QC, n = 100: 67 votes over one digest
C3  n = 1000: QC of 667 votes + TC of 667 timeouts, 5 % corrupted
C4  2^20 independent (pk, digest, sig) triples, 5 % corrupted
C5  2^24 triples sharded across GPUs (each rank builds its own shard)

Keys are derived from seeded 32-byte secrets; messages are 32-byte digests
shaped like the reference's (QC digest = SHA-512(hash || round_le)[..32],
consensus/src/messages.rs:201-207; TC vote digest = SHA-512(round_le ||
high_qc_round_le)[..32], messages.rs:307-311).  Corruptions are spread evenly
over the kinds SURVEY 8(d) lists for C3/C4, mixed-order keys included
(A' = [a]B + T8 from hsv_sign_mixed_order, in both variants: k = 0 mod 8,
which verify_strict ACCEPTS, and k != 0 mod 8, which it rejects).  The key of
a mixed-order vote replaces the signer's key, i.e. it is that committee
member's (malformed) key.  `accept` holds the expected verify_strict result.
"""
from __future__ import annotations

import hashlib
from dataclasses import dataclass, field

import numpy as np

from .verifier import sign_many

L = 2**252 + 27742317777372353535851937790883648493

# encodings of the 8 small-order points plus non-canonical aliases (13 in all)
SMALL_ORDER_ENCODINGS = [bytes.fromhex(h) for h in (
    "0100000000000000000000000000000000000000000000000000000000000000",
    "eeffffffffffffffffffffffffffffffffffffffffffffffffffffffffffff7f",
    "0100000000000000000000000000000000000000000000000000000000000080",
    "26e8958fc2b227b045c3f489f2ef98f0d5dfac05d3c63339b13802886d53fc05",
    "0000000000000000000000000000000000000000000000000000000000000000",
    "edffffffffffffffffffffffffffffffffffffffffffffffffffffffffffff7f",
    "c7176a703d4dd84fba3c0b760d10670f2a2053fa2c39ccc64ec7fd7792ac037a",
    "ecffffffffffffffffffffffffffffffffffffffffffffffffffffffffffff7f",
    "ecffffffffffffffffffffffffffffffffffffffffffffffffffffffffffffff",
    "c7176a703d4dd84fba3c0b760d10670f2a2053fa2c39ccc64ec7fd7792ac03fa",
    "0000000000000000000000000000000000000000000000000000000000000080",
    "edffffffffffffffffffffffffffffffffffffffffffffffffffffffffffffff",
    "26e8958fc2b227b045c3f489f2ef98f0d5dfac05d3c63339b13802886d53fc85",
)]
# y = 2: (y^2 - 1) / (d y^2 + 1) is not a square -> does not decompress
UNDECODABLE = bytes.fromhex("0200000000000000000000000000000000000000000000000000000000000000")

CORRUPTIONS = ("flip_R", "flip_s", "s_plus_l", "wrong_digest", "undecodable_R", "small_order_R",
               "small_order_A", "s_bit255", "mixed_order_A_ok", "mixed_order_A_bad")
# kinds whose verify_strict result is still Ok (the cofactorless equation holds)
ACCEPTED_KINDS = ("mixed_order_A_ok",)
# kinds that replace the signer's key
KEY_KINDS = ("small_order_A", "mixed_order_A_ok", "mixed_order_A_bad")


@dataclass
class Workload:
    pk: np.ndarray        # (n, 32) uint8
    sig: np.ndarray       # (n, 64) uint8
    msg: np.ndarray       # (n, 32) uint8, or (32,) for one shared digest
    honest: np.ndarray    # (n,) bool: untouched honest signature
    kind: np.ndarray = field(default=None)  # (n,) int8: -1 honest, else CORRUPTIONS index
    seeds: np.ndarray = field(default=None)  # (n, 32) uint8: the signers' secret seeds
    accept: np.ndarray = field(default=None)  # (n,) bool: expected verify_strict Ok

    def __post_init__(self):
        if self.accept is None:
            self.accept = self.honest.copy()

    @property
    def n(self) -> int:
        return self.pk.shape[0]


def mixed_order_signature(seed: bytes, msg: bytes, torsion: int, accept: bool):
    """(pk', sig) for the mixed-order key A' = [a]B + [2 torsion + 1]T8 of
    `seed`, over msg, with k = 0 (mod 8) (accept) or not (hsv_sign_mixed_order)."""
    import ctypes
    from . import _lib
    pk = ctypes.create_string_buffer(32)
    sig = ctypes.create_string_buffer(64)
    _lib.check(_lib.load().hsv_sign_mixed_order(bytes(seed), bytes(msg), len(msg), int(torsion), 1 if accept else 0,
                                                pk, sig), "hsv_sign_mixed_order")
    return np.frombuffer(pk.raw, np.uint8), np.frombuffer(sig.raw, np.uint8)


def qc_digest(block_hash: bytes, round_: int) -> bytes:
    return hashlib.sha512(block_hash + int(round_).to_bytes(8, "little")).digest()[:32]


def tc_vote_digest(round_: int, high_qc_round: int) -> bytes:
    return hashlib.sha512(int(round_).to_bytes(8, "little") + int(high_qc_round).to_bytes(8, "little")).digest()[:32]


def corrupt(w: Workload, frac: float, rng: np.random.Generator) -> None:
    """Corrupt round(frac * n) items in place, kinds spread evenly (seeded)."""
    n = w.n
    m = int(round(n * frac))
    if m == 0:
        return
    idx = rng.choice(n, size=m, replace=False)
    shared = w.msg.ndim == 1
    if shared and m:
        w.msg = np.repeat(w.msg[None, :], n, axis=0)
    for j, i in enumerate(idx):
        kind = j % len(CORRUPTIONS)
        name = CORRUPTIONS[kind]
        w.kind[i] = kind
        w.honest[i] = False
        w.accept[i] = name in ACCEPTED_KINDS
        if name.startswith("mixed_order_A"):
            if w.seeds is None:
                raise ValueError("mixed-order corruption needs the workload's signer seeds")
            pk, sg = mixed_order_signature(bytes(w.seeds[i]), bytes(w.msg[i]), int(rng.integers(0, 4)),
                                           name == "mixed_order_A_ok")
            w.pk[i] = pk
            w.sig[i] = sg
        elif name == "flip_R":
            b = int(rng.integers(0, 255))
            w.sig[i, b // 8] ^= np.uint8(1 << (b % 8))
        elif name == "flip_s":
            b = int(rng.integers(0, 253))
            w.sig[i, 32 + b // 8] ^= np.uint8(1 << (b % 8))
        elif name == "s_plus_l":
            s = int.from_bytes(bytes(w.sig[i, 32:]), "little") + L
            w.sig[i, 32:] = np.frombuffer((s % 2**256).to_bytes(32, "little"), np.uint8)
        elif name == "wrong_digest":
            b = int(rng.integers(0, 256))
            w.msg[i, b // 8] ^= np.uint8(1 << (b % 8))
        elif name == "undecodable_R":
            w.sig[i, :32] = np.frombuffer(UNDECODABLE, np.uint8)
        elif name == "small_order_R":
            w.sig[i, :32] = np.frombuffer(SMALL_ORDER_ENCODINGS[int(rng.integers(0, 13))], np.uint8)
        elif name == "small_order_A":
            w.pk[i] = np.frombuffer(SMALL_ORDER_ENCODINGS[int(rng.integers(0, 13))], np.uint8)
        elif name == "s_bit255":
            w.sig[i, 63] |= np.uint8(0x80)


def independent_triples(n: int, seed: int, corrupt_frac: float = 0.05, nthreads: int = 0) -> Workload:
    """C4 / C5 shard: n independent keys, digests and signatures."""
    rng = np.random.default_rng(seed)
    seeds = rng.integers(0, 256, size=(n, 32), dtype=np.uint8)
    msgs = rng.integers(0, 256, size=(n, 32), dtype=np.uint8)
    pk, sig = sign_many(seeds, msgs, nthreads)
    w = Workload(pk, sig, msgs, np.ones(n, bool), np.full(n, -1, np.int8), seeds=seeds)
    corrupt(w, corrupt_frac, rng)
    return w


def committee_seeds(n: int, seed: int = 0) -> np.ndarray:
    rng = np.random.default_rng(1_000_003 + seed)
    return rng.integers(0, 256, size=(n, 32), dtype=np.uint8)


def qc_votes(committee: int, seed: int = 0, corrupt_frac: float = 0.0, round_: int = 1) -> Workload:
    """A QC of 2f+1 = 2*committee//3 + 1 votes over one digest (C1/C2/C3)."""
    quorum = 2 * committee // 3 + 1
    seeds = committee_seeds(committee, seed)[:quorum]
    digest = qc_digest(hashlib.sha512(b"block" + seed.to_bytes(4, "little")).digest()[:32], round_)
    msgs = np.repeat(np.frombuffer(digest, np.uint8)[None, :], quorum, axis=0)
    pk, sig = sign_many(seeds, msgs)
    w = Workload(pk, sig, np.frombuffer(digest, np.uint8).copy(), np.ones(quorum, bool),
                 np.full(quorum, -1, np.int8), seeds=seeds)
    corrupt(w, corrupt_frac, np.random.default_rng(seed + 17))
    return w


def tc_votes(committee: int, seed: int = 0, corrupt_frac: float = 0.0, round_: int = 1000) -> Workload:
    """A TC of 2f+1 timeouts, per-vote digests over high_qc_round in [round-10, round-1] (C3)."""
    quorum = 2 * committee // 3 + 1
    seeds = committee_seeds(committee, seed)[:quorum]
    rng = np.random.default_rng(seed + 29)
    hqc = rng.integers(round_ - 10, round_, size=quorum)
    msgs = np.stack([np.frombuffer(tc_vote_digest(round_, int(h)), np.uint8) for h in hqc])
    pk, sig = sign_many(seeds, msgs)
    w = Workload(pk, sig, msgs, np.ones(quorum, bool), np.full(quorum, -1, np.int8), seeds=seeds)
    corrupt(w, corrupt_frac, rng)
    return w


@dataclass
class TxWorkload:
    txs: np.ndarray       # (n, tx_size) uint8: message || pk || sig
    honest: np.ndarray    # (n,) bool
    kind: np.ndarray      # (n,) int8: -1 honest, else CORRUPTIONS index
    accept: np.ndarray = field(default=None)  # (n,) bool: expected verify(..).is_ok()

    @property
    def n(self) -> int:
        return self.txs.shape[0]


def transactions(n: int, tx_size: int = 512, seed: int = 0, corrupt_frac: float = 0.05,
                 nthreads: int = 0) -> TxWorkload:
    """Mempool workload: n client transactions of tx_size
    bytes (the reference benchmark's default is 512, benchmark/fabfile.py),
    each message || pk || Signature::new(Digest(SHA-512(message)[..32]))
    (mempool/src/batch_maker.rs:79-85).  Corruptions as `corrupt`; the
    "wrong_digest" kind flips a message byte instead."""
    if tx_size < 96:
        raise ValueError("a transaction carries pk and signature: tx_size >= 96")
    mlen = tx_size - 96
    rng = np.random.default_rng(seed)
    seeds = rng.integers(0, 256, size=(n, 32), dtype=np.uint8)
    msgs = rng.integers(0, 256, size=(n, mlen), dtype=np.uint8)
    digests = np.empty((n, 32), np.uint8)
    for i in range(n):
        digests[i] = np.frombuffer(hashlib.sha512(msgs[i].tobytes()).digest()[:32], np.uint8)
    pk, sig = sign_many(seeds, digests, nthreads)
    w = Workload(pk, sig, digests, np.ones(n, bool), np.full(n, -1, np.int8), seeds=seeds)
    corrupt(w, corrupt_frac, rng)
    bad_msg = np.nonzero(w.kind == CORRUPTIONS.index("wrong_digest"))[0]
    if mlen:
        for i in bad_msg:
            b = int(rng.integers(0, mlen * 8))
            msgs[i, b // 8] ^= np.uint8(1 << (b % 8))
    else:  # no message bytes to flip: corrupt the signature's s instead
        for i in bad_msg:
            w.sig[i, 32] ^= np.uint8(1)
    txs = np.concatenate([msgs, w.pk, w.sig], axis=1)
    return TxWorkload(np.ascontiguousarray(txs), w.honest, w.kind, w.accept)
