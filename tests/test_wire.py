"""Wire formats: QC / TC verified from bincode bytes.

Encoding follows bincode 1.3's documented default encoding of the reference's
serde derives (hsverify/wire.py).  No Rust toolchain exists here and the
reference holds no serialized certificates, so the byte layout is a
restatement of the spec, not pinned by a reference fixture ("parity
unpinned" for the framing); the signature verdicts are pinned by the C oracle.
CPU tests cover the parser's error paths (they fail before any device call);
GPU tests verify certificates end to end.
"""
import base64
import hashlib
import struct

import numpy as np
import pytest

import ed25519_ref as o
from conftest import oracle_flags


@pytest.fixture(scope="module")
def lib():
    from hsverify import _lib
    return _lib.load(require=True)


def _qc_parts(n=3, seed=1, round_=7):
    block_hash = hashlib.sha512(b"block%d" % seed).digest()[:32]
    digest = hashlib.sha512(block_hash + struct.pack("<Q", round_)).digest()[:32]
    rnd = np.random.default_rng(seed)
    votes = []
    for _ in range(n):
        s = bytes(rnd.integers(0, 256, 32, dtype=np.uint8))
        votes.append((o.public_key(s), o.sign(s, digest)))
    return block_hash, round_, votes


# ---- CPU ------------------------------------------------------------------
def test_encoding_layout():
    from hsverify import wire
    block_hash, round_, votes = _qc_parts()
    buf = wire.encode_qc(block_hash, round_, votes)
    assert len(buf) == 32 + 8 + 8 + 3 * (8 + 44 + 64)
    assert buf[:32] == block_hash and struct.unpack("<QQ", buf[32:48]) == (round_, 3)
    assert struct.unpack("<Q", buf[48:56]) == (44,)
    assert base64.b64decode(buf[56:100]) == votes[0][0]
    tc = wire.encode_tc(9, [(votes[0][0], votes[0][1], 8)])
    assert len(tc) == 16 + 8 + 44 + 64 + 8 and tc[-8:] == struct.pack("<Q", 8)


@pytest.mark.parametrize("mutate", ["truncate_header", "truncate_vote", "bad_char", "short_key", "trailing_bits",
                                    "trailing_bytes", "huge_count", "bad_padding"])
def test_malformed_qc_is_a_parse_error(lib, mutate):
    from hsverify import _lib, wire
    block_hash, round_, votes = _qc_parts()
    buf = bytearray(wire.encode_qc(block_hash, round_, votes))
    key0 = 56  # first base64 character of vote 0
    if mutate == "truncate_header":
        buf = buf[:40]
    elif mutate == "truncate_vote":
        buf = buf[:-1]
    elif mutate == "bad_char":
        buf[key0 + 5] = ord("*")
    elif mutate == "short_key":   # 40 chars decode to 30 bytes (< 32: the reference's slice fails)
        enc = base64.b64encode(votes[0][0][:30])
        buf = bytearray(block_hash + struct.pack("<QQ", round_, 1) + struct.pack("<Q", len(enc)) + enc + votes[0][1])
    elif mutate == "trailing_bits":  # last symbol carries non-zero unused bits
        c = buf[key0 + 42]
        alphabet = b"ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/"
        buf[key0 + 42] = alphabet[(alphabet.index(c) ^ 1)]
    elif mutate == "trailing_bytes":
        buf += b"\x00"
    elif mutate == "huge_count":
        buf[40:48] = struct.pack("<Q", 1 << 60)
    elif mutate == "bad_padding":   # '=' inside the string
        buf[key0 + 10] = ord("=")
    with pytest.raises(_lib.HsvLibraryError, match="HSV_ERR_PARSE"):
        wire.qc_verify(bytes(buf))


def test_malformed_tc_is_a_parse_error(lib):
    from hsverify import _lib, wire
    _, _, votes = _qc_parts(1)
    buf = wire.encode_tc(5, [(votes[0][0], votes[0][1], 4)])
    for bad in (buf[:-3], buf + b"\x01", buf[:8]):
        with pytest.raises(_lib.HsvLibraryError, match="HSV_ERR_PARSE"):
            wire.tc_verify(bad)


# ---- GPU ------------------------------------------------------------------
@pytest.mark.gpu
def test_qc_bincode_c1_shape(hsv):
    """C1: a 4-node committee's QC of 3 votes; a corrupted vote makes it Err."""
    from hsverify import wire
    block_hash, round_, votes = _qc_parts(3, seed=4, round_=1)
    ok, pks = wire.qc_verify(wire.encode_qc(block_hash, round_, votes))
    assert ok and [bytes(p) for p in pks] == [v[0] for v in votes]
    bad = list(votes)
    s = bytearray(bad[1][1]); s[40] ^= 2
    bad[1] = (bad[1][0], bytes(s))
    assert not wire.qc_verify(wire.encode_qc(block_hash, round_, bad))[0]
    # wrong round -> different qc.digest() -> Err
    assert not wire.qc_verify(wire.encode_qc(block_hash, round_ + 1, votes))[0]
    # the genesis QC (no votes) verifies, as verify_batch over nothing does
    assert wire.qc_verify(wire.encode_qc(bytes(32), 0, []))[0]


@pytest.mark.gpu
def test_qc_bincode_c3_quorum(hsv):
    from hsverify import synth, wire
    w = synth.qc_votes(1000, seed=3)
    block_hash = hashlib.sha512(b"block" + (3).to_bytes(4, "little")).digest()[:32]
    votes = [(bytes(p), bytes(s)) for p, s in zip(w.pk, w.sig)]
    ok, pks = wire.qc_verify(wire.encode_qc(block_hash, 1, votes))
    assert ok and pks.shape == (667, 32)


@pytest.mark.gpu
def test_tc_bincode_vs_oracle(hsv, oracle_lib):
    """C3 TC: 667 timeouts, per-vote digests, 5 % corrupted: per-vote flags
    bit-exact against the C oracle; the verdict is Ok iff all are STRICT_OK."""
    from hsverify import synth, wire
    round_ = 1000
    rng = np.random.default_rng(31)
    w = synth.tc_votes(1000, seed=31, corrupt_frac=0.05, round_=round_)
    # recover each vote's high_qc_round from its (uncorrupted) digest
    table = {synth.tc_vote_digest(round_, h): h for h in range(round_ - 10, round_)}
    hqc = []
    for i in range(w.n):
        d = bytes(w.msg[i])
        hqc.append(table.get(d, int(rng.integers(round_ - 10, round_))))  # wrong_digest items: any round
    votes = [(bytes(p), bytes(s), h) for p, s, h in zip(w.pk, w.sig, hqc)]
    ok, flags = wire.tc_verify(wire.encode_tc(round_, votes))
    digests = np.stack([np.frombuffer(synth.tc_vote_digest(round_, h), np.uint8) for h in hqc])
    exp = oracle_flags(oracle_lib, w.pk, w.sig, digests)
    assert (flags == exp).all(), np.nonzero(flags != exp)[0][:8]
    assert not ok and not (exp & o.STRICT_OK).all()
    honest = [v for v, f in zip(votes, exp) if f & o.STRICT_OK]
    ok2, flags2 = wire.tc_verify(wire.encode_tc(round_, honest))
    assert ok2 and (flags2 & o.STRICT_OK).all()
