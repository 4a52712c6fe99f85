#!/usr/bin/env python3
"""Generate the committed golden vectors for the Ed25519 verification hot path.

Outputs (all messages are 32-byte consensus digests, as on the hot path):
  edge_vectors.json       SURVEY.md Appendix A.3 edge catalogue, labelled
  reference_fixtures.json the reference's own crypto/consensus test shapes
  random_vectors.bin      bulk honest + corrupted records, 129 B each:
                          pk(32) | sig(64) | msg(32) | flags(1)

Expected flags come from oracle/ed25519_ref.py (restatement of ed25519-dalek
1.0.1 / curve25519-dalek 3.x).  Every STRICT_OK bit is cross-checked against
libsodium 1.0.18 crypto_sign_verify_detached when the library is present
(it is in this image at /opt/conda/lib/libsodium.so.23); the generator aborts
on any disagreement.

Run from the repo root:  python tests/golden/make_golden.py
"""
import ctypes
import hashlib
import json
import os
import random
import struct
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.abspath(os.path.join(HERE, "..", ".."))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import ed25519_ref as o  # noqa: E402

N_RANDOM = int(os.environ.get("HSV_GOLDEN_N", "2048"))


def load_sodium():
    for cand in ("/opt/conda/lib/libsodium.so.23", "libsodium.so.23", "libsodium.so"):
        try:
            lib = ctypes.CDLL(cand)
            if lib.sodium_init() < 0:
                continue
            return lib
        except OSError:
            continue
    return None


def sodium_verify(lib, pk, sig, msg):
    return lib.crypto_sign_ed25519_verify_detached(sig, msg, ctypes.c_ulonglong(len(msg)), pk) == 0


def seed_bytes(i, tag=b"hsv-golden"):
    return hashlib.sha512(tag + struct.pack("<Q", i)).digest()[:32]


def expand(seed):
    h = o.sha512(seed)
    a = bytearray(h[:32])
    a[0] &= 248
    a[31] &= 127
    a[31] |= 64
    return int.from_bytes(a, "little"), h[32:]


def enc_point(e):
    return o.compress(o.to_affine(e))


def main():
    rnd = random.Random(20250204)
    sodium = load_sodium()
    edge = []

    def add_edge(case, pk, sig, msg):
        f = o.verify_flags(pk, sig, msg)
        edge.append({"case": case, "pk": pk.hex(), "sig": sig.hex(), "msg": msg.hex(), "flags": f})

    torsion = o.torsion_points()
    small_encs = o.small_order_encodings()
    undecodable = o.find_undecodable_y()
    # a second undecodable encoding with the sign bit set
    undecodable_neg = bytearray(undecodable)
    undecodable_neg[31] |= 0x80
    undecodable_neg = bytes(undecodable_neg)

    # 1 / 10: honest signatures
    for i in range(8):
        seed = seed_bytes(i)
        msg = rnd.randbytes(32)
        add_edge("honest", o.public_key(seed), o.sign(seed, msg), msg)
    seed = seed_bytes(100)
    pk = o.public_key(seed)
    msg = rnd.randbytes(32)
    sig = o.sign(seed, msg)
    a, prefix = expand(seed)
    # 2: corruptions
    add_edge("wrong_digest", pk, sig, rnd.randbytes(32))
    for bit in (0, 77, 200, 254, 255):
        s2 = bytearray(sig); s2[bit // 8] ^= 1 << (bit % 8)
        add_edge(f"flip_R_bit{bit}", pk, bytes(s2), msg)
    for bit in (0, 100, 251, 252, 253, 255):
        s2 = bytearray(sig); s2[32 + bit // 8] ^= 1 << (bit % 8)
        add_edge(f"flip_s_bit{bit}", pk, bytes(s2), msg)
    for bit in (0, 130, 254, 255):
        p2 = bytearray(pk); p2[bit // 8] ^= 1 << (bit % 8)
        add_edge(f"flip_A_bit{bit}", bytes(p2), sig, msg)
    for bit in (0, 255):
        m2 = bytearray(msg); m2[bit // 8] ^= 1 << (bit % 8)
        add_edge(f"flip_M_bit{bit}", pk, sig, bytes(m2))
    # 3: non-canonical s
    s_int = int.from_bytes(sig[32:], "little")
    # find a signature whose s + l still has bits 253..255 clear
    for j in range(64):
        m_j = rnd.randbytes(32)
        sig_j = o.sign(seed, m_j)
        sj = int.from_bytes(sig_j[32:], "little")
        if sj + o.L < 2**253:
            add_edge("s_plus_l_top_clear", pk, sig_j[:32] + (sj + o.L).to_bytes(32, "little"), m_j)
            break
    if s_int + o.L < 2**256:
        add_edge("s_plus_l", pk, sig[:32] + (s_int + o.L).to_bytes(32, "little"), msg)
    add_edge("s_bit255_set", pk, sig[:32] + (s_int | (1 << 255)).to_bytes(32, "little"), msg)
    add_edge("s_eq_l", pk, sig[:32] + o.L.to_bytes(32, "little"), msg)
    add_edge("s_eq_l_minus_1", pk, sig[:32] + (o.L - 1).to_bytes(32, "little"), msg)
    add_edge("s_max", pk, sig[:32] + b"\xff" * 32, msg)
    # 4: undecodable R / A
    add_edge("R_undecodable", pk, undecodable + sig[32:], msg)
    add_edge("R_undecodable_signbit", pk, undecodable_neg + sig[32:], msg)
    add_edge("A_undecodable", undecodable, sig, msg)
    add_edge("A_undecodable_signbit", undecodable_neg, sig, msg)
    # 5: small-order A (all 13 encodings incl. non-canonical), R = [r]B, s = r
    for idx, enc in enumerate(small_encs):
        r = rnd.randrange(1, o.L)
        r_enc = enc_point(o.scalar_mult(r, o.BASEPOINT))
        add_edge(f"small_A_{idx}_s_eq_r", enc, r_enc + r.to_bytes(32, "little"), rnd.randbytes(32))
        # and a random signature against the small-order key
        add_edge(f"small_A_{idx}_random_sig", enc, sig, msg)
    # 6: small-order R with a valid equation: R = identity encodings, s = k*a
    for idx, enc in enumerate(small_encs):
        m_j = rnd.randbytes(32)
        k = o.scalar_from_hash(o.sha512(enc + pk + m_j))
        s_val = (k * a) % o.L
        add_edge(f"small_R_{idx}_s_eq_ka", pk, enc + s_val.to_bytes(32, "little"), m_j)
        add_edge(f"small_R_{idx}_random_s", pk, enc + sig[32:], msg)
    # identity R and identity A with s = 0: equation holds (batch accepts), strict rejects
    for idx, enc in enumerate(small_encs):
        pt = o.decompress(enc)
        if pt is not None and o.is_identity(o.to_ext(pt)):
            add_edge(f"identity_R_{idx}_identity_A_s0", enc, enc + bytes(32), rnd.randbytes(32))
    # 7 / 8: mixed-order A = [a]B + T, grind the message for k = 0 mod ord(T)
    for t_idx in range(1, 8):
        T = torsion[t_idx]
        A_mixed = o.ext_add(o.scalar_mult(a, o.BASEPOINT), T)
        a_enc = enc_point(A_mixed)
        got_acc = got_rej = 0
        for _ in range(200):
            m_j = rnd.randbytes(32)
            s_j = o.sign_with_scalar(a, prefix + m_j[:4], a_enc, m_j)
            f = o.verify_flags(a_enc, s_j, m_j)
            if f & o.STRICT_OK and got_acc < 2:
                add_edge(f"mixed_A_T{t_idx}_k_kills_torsion", a_enc, s_j, m_j)
                got_acc += 1
            elif not f & o.STRICT_OK and got_rej < 2:
                add_edge(f"mixed_A_T{t_idx}_torsion_survives", a_enc, s_j, m_j)
                got_rej += 1
            if got_acc >= 2 and got_rej >= 2:
                break
    # mixed-order R = [r]B + T with s = r + k a: holds iff T = O -> reject (eq fails)
    for t_idx in (1, 4):
        m_j = rnd.randbytes(32)
        r = rnd.randrange(1, o.L)
        R_mixed = o.ext_add(o.scalar_mult(r, o.BASEPOINT), torsion[t_idx])
        r_enc = enc_point(R_mixed)
        k = o.scalar_from_hash(o.sha512(r_enc + pk + m_j))
        add_edge(f"mixed_R_T{t_idx}", pk, r_enc + ((r + k * a) % o.L).to_bytes(32, "little"), m_j)
    # small-order R with mixed-order A where the torsion cancels: R = T2, A = [a]B + T2, k odd
    T2 = torsion[4]
    assert o.is_identity(o.ext_double(T2)) and not o.is_identity(T2)
    A_m2 = enc_point(o.ext_add(o.scalar_mult(a, o.BASEPOINT), T2))
    t2_enc = enc_point(T2)
    for _ in range(50):
        m_j = rnd.randbytes(32)
        k = o.scalar_from_hash(o.sha512(t2_enc + A_m2 + m_j))
        if k & 1:
            add_edge("small_R_T2_mixed_A_T2_cancel", A_m2, t2_enc + ((k * a) % o.L).to_bytes(32, "little"), m_j)
            break
    # non-canonical encodings of large-order points (y + p, y in [2, 18])
    for y in range(2, 19):
        pt = o.decompress(y.to_bytes(32, "little"))
        if pt is None:
            continue
        enc = bytearray((y + o.P).to_bytes(32, "little"))
        enc[31] |= (pt[0] & 1) << 7
        enc = bytes(enc)
        add_edge(f"noncanonical_A_y{y}", enc, sig, msg)
        add_edge(f"noncanonical_R_y{y}", pk, enc + sig[32:], msg)
    # 9: Signature::default() (64 zero bytes)
    add_edge("default_signature", pk, bytes(64), msg)
    add_edge("all_zero_everything", bytes(32), bytes(64), bytes(32))
    add_edge("all_ff_everything", b"\xff" * 32, b"\xff" * 64, b"\xff" * 32)

    # libsodium cross-check of the strict bit
    if sodium is not None:
        for e in edge:
            pk_, sig_, msg_ = (bytes.fromhex(e[k]) for k in ("pk", "sig", "msg"))
            ls = sodium_verify(sodium, pk_, sig_, msg_)
            if ls != bool(e["flags"] & o.STRICT_OK):
                raise SystemExit(f"libsodium disagrees on {e['case']}: sodium={ls} flags={e['flags']:#x}")
    with open(os.path.join(HERE, "edge_vectors.json"), "w") as f:
        json.dump({"generator": "tests/golden/make_golden.py", "oracle": "oracle/ed25519_ref.py",
                   "libsodium_crosscheck": sodium is not None, "vectors": edge}, f, indent=1)
    print("edge vectors:", len(edge))

    # --- reference test fixtures (crypto_tests.rs, messages_tests.rs) -----------
    seeds = o.reference_key_seeds()
    pks = [o.public_key(s) for s in seeds]
    hello = o.test_digest(b"Hello, world!")
    bad = o.test_digest(b"Bad message!")
    fx = {}
    # verify_valid_signature / verify_invalid_signature: keys().pop() == keys[3]
    sig3 = o.sign(seeds[3], hello)
    fx["verify_valid_signature"] = {"op": "verify", "digest": hello.hex(), "pk": pks[3].hex(),
                                    "sig": sig3.hex(), "expect_ok": True}
    fx["verify_invalid_signature"] = {"op": "verify", "digest": bad.hex(), "pk": pks[3].hex(),
                                      "sig": sig3.hex(), "expect_ok": False}
    # verify_valid_batch: 3 signatures from keys[3], keys[2], keys[1] over one digest
    votes = [(pks[i].hex(), o.sign(seeds[i], hello).hex()) for i in (3, 2, 1)]
    fx["verify_valid_batch"] = {"op": "verify_batch", "digest": hello.hex(), "votes": votes,
                                "expect_ok": True}
    # verify_invalid_batch: 2 valid + (keys[1], Signature::default())
    votes_bad = [(pks[i].hex(), o.sign(seeds[i], hello).hex()) for i in (3, 2)]
    votes_bad.append((pks[1].hex(), bytes(64).hex()))
    fx["verify_invalid_batch"] = {"op": "verify_batch", "digest": hello.hex(), "votes": votes_bad,
                                  "expect_ok": False}
    # consensus qc() fixture: hash = 0^32, round = 1, votes from keys[3], [2], [1]
    qd = o.qc_digest(bytes(32), 1)
    qvotes = [(pks[i].hex(), o.sign(seeds[i], qd).hex()) for i in (3, 2, 1)]
    fx["verify_valid_qc"] = {"op": "verify_batch", "digest": qd.hex(), "votes": qvotes, "expect_ok": True}
    fx["empty_batch"] = {"op": "verify_batch", "digest": qd.hex(), "votes": [], "expect_ok": True}
    for name, v in fx.items():
        if v["op"] == "verify":
            got = o.verify_strict(bytes.fromhex(v["pk"]), bytes.fromhex(v["sig"]), bytes.fromhex(v["digest"]))
        else:
            got = o.verify_batch(bytes.fromhex(v["digest"]),
                                 [(bytes.fromhex(p), bytes.fromhex(s)) for p, s in v["votes"]])
        assert got == v["expect_ok"], name
    with open(os.path.join(HERE, "reference_fixtures.json"), "w") as f:
        json.dump({"generator": "tests/golden/make_golden.py",
                   "key_recipe": "StdRng::from_seed([0;32]) (rand 0.7.3 = rand_chacha 0.2 ChaCha20Rng) keystream, 32 B per key; ChaCha20 block pinned by RFC 7539 A.1/2.3.2 (tests/test_oracle.py)",
                   "qc_digest": qd.hex(), "fixtures": fx}, f, indent=1)
    print("reference fixtures:", len(fx), "qc digest", qd.hex())

    # --- bulk random records ------------------------------------------------------
    recs = bytearray()
    kinds = ["honest"] * 8 + ["flip_R", "flip_s", "s_plus_l", "wrong_digest", "R_undecodable",
                              "small_R", "small_A", "mixed_A", "flip_A"]
    n_bad_sodium = 0
    for i in range(N_RANDOM):
        seed = seed_bytes(10_000 + i)
        msg = rnd.randbytes(32)
        kind = kinds[rnd.randrange(len(kinds))]
        if kind == "mixed_A":
            aa, pre = expand(seed)
            pk = enc_point(o.ext_add(o.scalar_mult(aa, o.BASEPOINT), torsion[rnd.randrange(1, 8)]))
            sig = o.sign_with_scalar(aa, pre, pk, msg)
        else:
            pk = o.public_key(seed)
            sig = o.sign(seed, msg)
        if kind == "flip_R":
            b = rnd.randrange(256); s2 = bytearray(sig); s2[b // 8] ^= 1 << (b % 8); sig = bytes(s2)
        elif kind == "flip_s":
            b = rnd.randrange(256); s2 = bytearray(sig); s2[32 + b // 8] ^= 1 << (b % 8); sig = bytes(s2)
        elif kind == "flip_A":
            b = rnd.randrange(256); p2 = bytearray(pk); p2[b // 8] ^= 1 << (b % 8); pk = bytes(p2)
        elif kind == "s_plus_l":
            sv = int.from_bytes(sig[32:], "little") + o.L
            sig = sig[:32] + (sv % 2**256).to_bytes(32, "little")
        elif kind == "wrong_digest":
            msg = rnd.randbytes(32)
        elif kind == "R_undecodable":
            sig = undecodable + sig[32:]
        elif kind == "small_R":
            sig = small_encs[rnd.randrange(len(small_encs))] + sig[32:]
        elif kind == "small_A":
            pk = small_encs[rnd.randrange(len(small_encs))]
        f = o.verify_flags(pk, sig, msg)
        if sodium is not None and sodium_verify(sodium, pk, sig, msg) != bool(f & o.STRICT_OK):
            n_bad_sodium += 1
        recs += pk + sig + msg + bytes([f])
    if n_bad_sodium:
        raise SystemExit(f"libsodium disagrees on {n_bad_sodium} random records")
    with open(os.path.join(HERE, "random_vectors.bin"), "wb") as f:
        f.write(bytes(recs))
    acc = sum(1 for i in range(N_RANDOM) if recs[129 * i + 128] & o.STRICT_OK)
    print("random records:", N_RANDOM, "strict accepted:", acc,
          "sha256", hashlib.sha256(bytes(recs)).hexdigest())


if __name__ == "__main__":
    main()
