"""Config C5 (BASELINE.json configs[4]: 2^24 triples) and the chunked device API.

hsv_verify_device_bits splits a batch into launches of 2^22 items
(hsv_host.h kChunk) and offsets the STRICT_OK bit words by base / 32 per
chunk.  These tests run more than one chunk:

* 2^22 + 4097 items (two chunks, a ragged tail) with flags and bits, against
  the same items verified as two separate calls (each within one chunk) and
  against a 16 384-item oracle sample straddling the chunk boundary;
* 2^24 items (C5's global batch on one GPU, four chunks): honest all
  accepted, every corruption kind rejected with its flag pattern, bits equal
  to the flags, and idempotence.  The 2^24 input tiles a 2^16-item seeded
  base set (C5's shape: QC-independent triples, consensus/src/messages.rs
  Digest-sized messages), so the oracle cost stays bounded; the kernels do
  not see the repetition (every item is an independent lane).
"""
import numpy as np
import pytest

import ed25519_ref as o
from conftest import oracle_flags

pytestmark = pytest.mark.gpu

CHUNK = 1 << 22


def _unpack(bits, n):
    b = bits.view(np.uint32)
    return ((b[np.arange(n) // 32] >> (np.arange(n) % 32).astype(np.uint32)) & 1).astype(np.uint8)


@pytest.fixture(scope="module")
def mods(hsv):
    from hsverify import synth, verifier
    return synth, verifier


def test_two_chunks_ragged_tail_with_bits(mods, oracle_lib):
    import torch
    synth, verifier = mods
    n = CHUNK + 4097
    base = synth.independent_triples(1 << 16, seed=4242, corrupt_frac=0.05)
    rep = np.arange(n) % base.n
    # perturb the digests of the tiled copies so neighbouring chunks differ
    msg = base.msg[rep].copy()
    msg[:, 0] ^= (np.arange(n) // base.n).astype(np.uint8)
    pk, sig = base.pk[rep], base.sig[rep]
    dev = torch.device("cuda:0")
    t_pk, t_sig, t_msg = (torch.from_numpy(np.ascontiguousarray(a)).to(dev) for a in (pk, sig, msg))
    flags = torch.zeros(n, dtype=torch.uint8, device=dev)
    bits = torch.zeros((n + 31) // 32, dtype=torch.int32, device=dev)
    verifier.verify_device(t_pk, t_sig, t_msg, flags, bits)
    # the same items as two single-chunk calls
    f1 = torch.zeros(CHUNK, dtype=torch.uint8, device=dev)
    b1 = torch.zeros(CHUNK // 32, dtype=torch.int32, device=dev)
    f2 = torch.zeros(n - CHUNK, dtype=torch.uint8, device=dev)
    b2 = torch.zeros((n - CHUNK + 31) // 32, dtype=torch.int32, device=dev)
    verifier.verify_device(t_pk[:CHUNK], t_sig[:CHUNK], t_msg[:CHUNK], f1, b1)
    verifier.verify_device(t_pk[CHUNK:], t_sig[CHUNK:], t_msg[CHUNK:], f2, b2)
    torch.cuda.synchronize()
    f = flags.cpu().numpy()
    assert (f == np.concatenate([f1.cpu().numpy(), f2.cpu().numpy()])).all()
    assert (bits.cpu().numpy() == np.concatenate([b1.cpu().numpy(), b2.cpu().numpy()])).all()
    assert (_unpack(bits.cpu().numpy(), n) == (f & o.STRICT_OK)).all()
    # oracle sample: 8192 on each side of the chunk boundary, plus the tail end
    idx = np.unique(np.concatenate([np.arange(CHUNK - 8192, CHUNK + 4097), np.arange(n - 64, n)]))
    idx = np.concatenate([idx, np.sort(np.random.default_rng(5).choice(CHUNK - 8192, 16384 - idx.size, replace=False))])
    exp = oracle_flags(oracle_lib, pk[idx], sig[idx], msg[idx])
    assert (f[idx] == exp).all()
    # copy 0 keeps its digests: its honest items verify and its corrupted ones do
    # not (a perturbed copy can undo a wrong_digest corruption, so only copy 0)
    h0 = base.accept
    assert (f[:base.n][h0] & o.STRICT_OK).all() and not (f[:base.n][~h0] & o.STRICT_OK).any()


def test_c5_2p24_properties(mods, oracle_lib):
    import torch
    synth, verifier = mods
    n = 1 << 24
    base = synth.independent_triples(1 << 16, seed=0xC5, corrupt_frac=0.05)
    reps = n // base.n
    dev = torch.device("cuda:0")
    t_pk = torch.from_numpy(base.pk).to(dev).repeat(reps, 1)
    t_sig = torch.from_numpy(base.sig).to(dev).repeat(reps, 1)
    t_msg = torch.from_numpy(base.msg).to(dev).repeat(reps, 1)
    flags = torch.zeros(n, dtype=torch.uint8, device=dev)
    bits = torch.zeros(n // 32, dtype=torch.int32, device=dev)
    verifier.verify_device(t_pk, t_sig, t_msg, flags, bits)
    torch.cuda.synchronize()
    f = flags.cpu().numpy()
    # every copy of the base set gives the same bytes (four launches, 256 copies)
    per_copy = f.reshape(reps, base.n)
    assert (per_copy == per_copy[0][None, :]).all()
    exp = oracle_flags(oracle_lib, base.pk, base.sig, base.msg)
    assert (per_copy[0] == exp).all()
    assert (_unpack(bits.cpu().numpy(), n) == (f & o.STRICT_OK)).all()
    honest = np.tile(base.accept, reps)
    assert (f[honest] & o.STRICT_OK).all() and not (f[~honest] & o.STRICT_OK).any()
    kinds = {name: per_copy[0][base.kind == k] for k, name in enumerate(synth.CORRUPTIONS)}
    assert not (kinds["s_plus_l"] & o.S_OK).any() and not (kinds["s_bit255"] & o.S_OK).any()
    assert not (kinds["undecodable_R"] & o.R_OK).any()
    assert (kinds["small_order_R"] & o.SMALL_R).all() and (kinds["small_order_A"] & o.SMALL_A).all()
    # mixed-order keys: the cofactorless equation decides (Appendix A.3 rows 7-8)
    assert kinds["mixed_order_A_ok"].size and (kinds["mixed_order_A_ok"] & o.STRICT_OK).all()
    assert not (kinds["mixed_order_A_ok"] & o.SMALL_A).any()
    assert kinds["mixed_order_A_bad"].size and (kinds["mixed_order_A_bad"] & o.PARSE_OK).all()
    assert not (kinds["mixed_order_A_bad"] & o.EQ_OK).any()
    # idempotent
    flags2 = torch.zeros_like(flags)
    verifier.verify_device(t_pk, t_sig, t_msg, flags2)
    torch.cuda.synchronize()
    assert torch.equal(flags, flags2)
