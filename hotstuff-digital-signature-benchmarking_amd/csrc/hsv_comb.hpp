// Committee key cache: fixed-base comb tables.
//
// Consensus verifies signatures of a fixed committee (consensus/src/config.rs
// Committee; QC/TC votes are looked up by stake(name), messages.rs:186).  For
// such keys the variable-base product [k](-A) becomes a fixed-base one: with
//   T_P[j][m] = [m * 2^(8j)] P,   j in [0, 32), m in [1, 128]   (affine Niels)
// and the signed radix-2^8 digits k_j of k (k + C8, C8 = sum 128 * 256^j),
//   [k]P = sum_j T_P[j][k_j]        (T[j][-m] = -T[j][m], T[j][0] = O)
// exactly, for any curve point P including torsion (signed-digit recoding is
// an identity on the integer k).  Verification then needs 32 + 32 mixed
// additions (P = -A and P = B) and no doublings, no A decompression, no
// per-signature table build.  Flags are identical to verify_one's.
//
// Table layout: entry (j, m) at word ((j * 128) + m - 1) * 24 of a key's
// table; 24 words = y+x, y-x, 2dxy, each a canonical 8-word encoding.
// A key's table is 32 * 128 * 96 B = 384 KiB.
#pragma once
#include "hsv_point.hpp"
#include "hsv_scalar.hpp"
#include "hsv_sha512.hpp"
#include "hsv_verify_core.hpp"

namespace hsv {

constexpr int kCombPos = 32;
constexpr int kCombEnt = 128;
constexpr int kCombEntryWords = 24;
constexpr uint64_t kCombTableWords = (uint64_t)kCombPos * kCombEnt * kCombEntryWords;  // per key

// key flag byte stored next to each committee key
enum : uint32_t { kKeyAOk = 0x1, kKeySmallA = 0x2 };

// Fill entries m = 1..128 of one position from base = [2^(8j)]P:
// out[(m-1)*24 ...] = affine Niels of [m]base.  tmp: 128 * 8 words scratch
// (prefix products of Z for one batched inversion).
HSV_INL void comb_build_position(const ge_ext &base, uint32_t *out, uint32_t *tmp) {
  const ge_cached bc = ge_to_cached(base);
  ge_ext acc = base;
  fe pp = fe_small(1);
  HSV_NOUNROLL
  for (int m = 1; m <= kCombEnt; ++m) {
    if (m > 1) acc = ge_add_cached<true>(acc, bc);
    uint32_t *e = out + (m - 1) * kCombEntryWords;
    fe_pack(acc.X, e);
    fe_pack(acc.Y, e + 8);
    fe_pack(acc.Z, e + 16);
    pp = fe_mul(pp, acc.Z);
    fe_pack(pp, tmp + (m - 1) * 8);
  }
  fe inv = fe_invert(pp);  // 1 / (Z_1 ... Z_128)
  HSV_NOUNROLL
  for (int m = kCombEnt; m >= 1; --m) {
    uint32_t *e = out + (m - 1) * kCombEntryWords;
    const fe X = fe_from_words_masked(e), Y = fe_from_words_masked(e + 8), Z = fe_from_words_masked(e + 16);
    fe zinv = inv;
    if (m > 1) {
      zinv = fe_mul(inv, fe_from_words_masked(tmp + (m - 2) * 8));
      inv = fe_mul(inv, Z);
    }
    const fe x = fe_mul(X, zinv), y = fe_mul(Y, zinv);
    fe_pack(fe_add(y, x), e);
    fe_pack(fe_sub(y, x), e + 8);
    fe_pack(fe_mul(fe_mul(x, y), fe_d2()), e + 16);
  }
}

// Wide comb of B for the generic kernels: 16-bit signed digits, so [b]B for
// b < 2^256 is 16 mixed additions instead of 32.
//   T16[j][m] = [m * 2^(16j)] B,   j in [0, 16), m in [1, 32768]
// Entry (j, m) at word ((j * 32768) + m - 1) * 24 (same 24-word format),
// 16 * 32768 * 96 B = 48 MiB per device: MALL-resident, one 96-byte read per
// addition.  Built on the GPU in chunks of 128 consecutive multiples, one
// chunk per lane (hsv_comb16_build_kernel).
constexpr int kComb16Pos = 16;
constexpr int kComb16Ent = 1 << 15;
constexpr int kComb16Chunk = 128;
constexpr int kComb16ChunksPerPos = kComb16Ent / kComb16Chunk;  // 256
constexpr uint64_t kComb16TableWords = (uint64_t)kComb16Pos * kComb16Ent * kCombEntryWords;

// Fill kComb16Chunk entries [start + m * base] (m = 1..128) of a run of the
// table: projective sums first, then one batched inversion.
HSV_INL void comb_build_run(const ge_ext &start, const ge_ext &base, uint32_t *out, uint32_t *tmp) {
  const ge_cached bc = ge_to_cached(base);
  ge_ext acc = start;
  fe pp = fe_small(1);
  HSV_NOUNROLL
  for (int m = 1; m <= kComb16Chunk; ++m) {
    acc = ge_add_cached<true>(acc, bc);
    uint32_t *e = out + (m - 1) * kCombEntryWords;
    fe_pack(acc.X, e);
    fe_pack(acc.Y, e + 8);
    fe_pack(acc.Z, e + 16);
    pp = fe_mul(pp, acc.Z);
    fe_pack(pp, tmp + (m - 1) * 8);
  }
  fe inv = fe_invert(pp);
  HSV_NOUNROLL
  for (int m = kComb16Chunk; m >= 1; --m) {
    uint32_t *e = out + (m - 1) * kCombEntryWords;
    const fe X = fe_from_words_masked(e), Y = fe_from_words_masked(e + 8), Z = fe_from_words_masked(e + 16);
    fe zinv = inv;
    if (m > 1) {
      zinv = fe_mul(inv, fe_from_words_masked(tmp + (m - 2) * 8));
      inv = fe_mul(inv, Z);
    }
    const fe x = fe_mul(X, zinv), y = fe_mul(Y, zinv);
    fe_pack(fe_add(y, x), e);
    fe_pack(fe_sub(y, x), e + 8);
    fe_pack(fe_mul(fe_mul(x, y), fe_d2()), e + 16);
  }
}

// One chunk (position j, chunk c) of the wide B table: entries
// m = 128c + 1 .. 128c + 128 of position j.  bx, by: affine B.
HSV_INL void comb16_build_chunk(const fe &bx, const fe &by, int j, uint32_t c, uint32_t *table, uint32_t *tmp) {
  ge_ext base;
  base.X = bx;
  base.Y = by;
  base.Z = fe_small(1);
  base.T = fe_mul(bx, by);
  HSV_NOUNROLL
  for (int i = 0; i < 16 * j; ++i) base = ge_dbl<true>(base);  // [2^(16j)]B
  ge_ext step = base;
  HSV_NOUNROLL
  for (int i = 0; i < 7; ++i) step = ge_dbl<true>(step);  // [128 * 2^(16j)]B
  const ge_cached sc128 = ge_to_cached(step);
  ge_ext start = ge_identity();
  HSV_NOUNROLL
  for (int b = 7; b >= 0; --b) {  // start = [128c] base
    start = ge_dbl<true>(start);
    if ((c >> b) & 1u) start = ge_add_cached<true>(start, sc128);
  }
  comb_build_run(start, base,
                 table + ((uint64_t)j * kComb16Ent + (uint64_t)c * kComb16Chunk) * kCombEntryWords, tmp);
}

// [2^(8j)] P for a decompressed affine P (negated when neg), extended coords.
HSV_INL ge_ext comb_position_base(const fe &x, const fe &y, uint32_t neg, int j) {
  ge_ext p;
  p.X = fe_carry(fe_select(x, fe_neg(x), neg));
  p.Y = y;
  p.Z = fe_small(1);
  p.T = fe_mul(p.X, p.Y);
  HSV_NOUNROLL
  for (int i = 0; i < 8 * j; ++i) p = ge_dbl<true>(p);
  return p;
}

// Loader over one position's 128 entries in memory (global or host).
struct CombPosTab {
  const uint32_t *base;
  HSV_MEMBER ge_niels load(uint32_t idx) const {
    const uint32_t *e = base + idx * kCombEntryWords;
    uint32_t w[24];
#if defined(__HIP_DEVICE_COMPILE__)
    const uint4 *q = reinterpret_cast<const uint4 *>(e);
    HSV_UNROLL
    for (int i = 0; i < 6; ++i) {
      const uint4 v = q[i];
      w[4 * i] = v.x; w[4 * i + 1] = v.y; w[4 * i + 2] = v.z; w[4 * i + 3] = v.w;
    }
#else
    for (int i = 0; i < 24; ++i) w[i] = e[i];
#endif
    ge_niels n;
    n.ypx = fe_from_words_masked(w);
    n.ymx = fe_from_words_masked(w + 8);
    n.xy2d = fe_from_words_masked(w + 16);
    return n;
  }
};

// Fault injection (tests only): what a corrupted key-table entry reads back as.
HSV_INL ge_niels niels_injected(const ge_niels &n, uint32_t inject) {
  ge_niels r = n;
  if (inject == kInjectZeroTables) {
    r.ypx = fe_small(0);
    r.ymx = fe_small(0);
    r.xy2d = fe_small(0);
  } else if (inject == kInjectFlipTables) {
    r.ypx.v[0] ^= 1u;
  }
  return r;
}

// Verification against a cached committee key.  ta: the key's table of -A,
// tb: the table of B, pk: the key's original 32 bytes (hashed as-is),
// key_flags: kKeyAOk / kKeySmallA computed when the table was built.
// Returns the same flag byte as verify_one for (pk, sig, msg), plus kFault
// (fault_bit).  inject: fault injection (tests), applied to the first key entry.
HSV_INL uint32_t verify_one_comb(const uint32_t pk[8], uint32_t key_flags, const uint32_t sig[16],
                                 const uint32_t msg[8], const uint32_t *ta, const uint32_t *tb,
                                 uint32_t inject = kInjectNone) {
  const uint32_t s_ok = sc_is_canonical(sig + 8);
  uint32_t h[16];
  sha512_96(sig, pk, msg, h);
  const sc k = sc_reduce512(h);

  // signed radix-2^8 digits of k and s (32 each), consumed from the bottom
  uint32_t kr[9], sr[9];
  recode_add<9, 8, kCombPos>(k.v, 8, kr);
  recode_add<9, 8, kCombPos>(sig + 8, 8, sr);

  ge_ext q = ge_identity();
  HSV_NOUNROLL
  for (int j = 0; j < kCombPos; ++j) {
    const uint32_t ca = kr[0] & 0xffu, cb = sr[0] & 0xffu;
    HSV_UNROLL
    for (int i = 0; i < 8; ++i) {
      kr[i] = (kr[i] >> 8) | (kr[i + 1] << 24);
      sr[i] = (sr[i] >> 8) | (sr[i + 1] << 24);
    }
    kr[8] >>= 8;
    sr[8] >>= 8;
    const CombPosTab tpa{ta + (uint64_t)j * kCombEnt * kCombEntryWords};
    const CombPosTab tpb{tb + (uint64_t)j * kCombEnt * kCombEntryWords};
    ge_niels na = select_niels<8>(tpa, ca);
    if (inject != kInjectNone && j == 0) na = niels_injected(na, inject);
    q = ge_add_niels<true>(q, na);
    q = ge_add_niels<true>(q, select_niels<8>(tpb, cb));
  }

  fe rx, ry;
  const uint32_t r_ok = ge_decompress(sig, rx, ry);
  const uint32_t small_r = r_ok & y_is_small_order(ry);
  const uint32_t same = ge_eq_affine(q, rx, ry);
  const uint32_t a_ok = (key_flags & kKeyAOk) ? 1u : 0u;
  const uint32_t small_a = a_ok & ((key_flags & kKeySmallA) ? 1u : 0u);

  const uint32_t parse_ok = s_ok & a_ok & r_ok;
  const uint32_t eq_ok = parse_ok & same;
  const uint32_t strict_ok = eq_ok & (small_a ^ 1u) & (small_r ^ 1u);
  return (strict_ok ? kStrictOk : 0u) | (eq_ok ? kEqOk : 0u) | (parse_ok ? kParseOk : 0u) |
         (small_a ? kSmallA : 0u) | (small_r ? kSmallR : 0u) | (s_ok ? kSOk : 0u) |
         (a_ok ? kAOk : 0u) | (r_ok ? kROk : 0u) | fault_bit(a_ok, r_ok, q);
}

}  // namespace hsv
