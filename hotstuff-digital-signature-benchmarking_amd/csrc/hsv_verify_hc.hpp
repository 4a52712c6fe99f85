// Half-size scalars + fixed-base comb for B (the default generic kernel).
//
// Same verification equation as verify_one_half (hsv_verify_core.hpp):
//   EQ_OK  <=>  [c1](-R) + [|c0|](-sign(c0) A) + [b]B == O,
//   (c0, c1) = lattice_reduce(k),  b = (c1 s) mod l,
// evaluated in two phases so the hot loop stays small:
//   1. Straus over the two ~128-bit scalars c1, |c0| (< 2^138): NW windows of WA bits,
//      WA doublings + 2 cached additions per window, entries of the per-lane
//      tables [0..2^(WA-1)](-R), [0..2^(WA-1)](-sign(c0) A) read from memory
//      (VT, one 128-byte line per entry) a window ahead of their use;
//   2. [b]B from the comb table T_B[j][m] = [m 2^(8j)]B (hsv_comb.hpp, built
//      once per device, L2-resident): 32 mixed additions, no doublings.
// Each phase has one copy of its point formula (runtime with_t flag), so the
// window loop is ~3k instructions instead of ~10k and stays in the shared
// instruction cache.  A lane whose lattice reduction fails (~2^-22.6) takes
// verify_one_full_comb: the same two phases with the full-length k.
#pragma once
#include "hsv_comb.hpp"
#include "hsv_lattice.hpp"
#include "hsv_verify_core.hpp"

namespace hsv {

// q += [s]B for a scalar s < 2^256 (8 words) via a comb table of B: CB = 8,
// the 384 KiB table (32 signed radix-2^8 digits), or CB = 16, the 48 MiB
// wide table (16 signed radix-2^16 digits); digits consumed from the bottom.
// (s >= 2^256 - C is only reached for non-canonical s, whose flags do not
// depend on the equation.)
template <int CB>
HSV_INL ge_ext comb_add_b(ge_ext q, const uint32_t s[8], const uint32_t *tb) {
  static_assert(CB == 8 || CB == 16, "comb digit width");
#ifdef HSV_TIMING_STUB_COMB  // tools/phase_probe.py only
  return q;
#endif
  constexpr int NP = 256 / CB;
  constexpr int ENT = 1 << (CB - 1);
  uint32_t sr[9];
  recode_add<9, CB, NP>(s, 8, sr);
  HSV_NOUNROLL
  for (int j = 0; j < NP; ++j) {
    const uint32_t cb = sr[0] & ((1u << CB) - 1u);
    HSV_UNROLL
    for (int i = 0; i < 8; ++i) sr[i] = (sr[i] >> CB) | (sr[i + 1] << (32 - CB));
    sr[8] >>= CB;
    const CombPosTab tpb{tb + (uint64_t)j * ENT * kCombEntryWords};
    q = ge_add_niels<true>(q, select_niels<CB>(tpb, cb));
  }
  return q;
}

HSV_INL uint32_t flags_byte(uint32_t s_ok, uint32_t a_ok, uint32_t r_ok, uint32_t small_a, uint32_t small_r,
                            uint32_t same) {
  const uint32_t parse_ok = s_ok & a_ok & r_ok;
  const uint32_t eq_ok = parse_ok & same;
  const uint32_t strict_ok = eq_ok & (small_a ^ 1u) & (small_r ^ 1u);
  return (strict_ok ? kStrictOk : 0u) | (eq_ok ? kEqOk : 0u) | (parse_ok ? kParseOk : 0u) |
         (small_a ? kSmallA : 0u) | (small_r ? kSmallR : 0u) | (s_ok ? kSOk : 0u) |
         (a_ok ? kAOk : 0u) | (r_ok ? kROk : 0u);
}

// Straus over NV (1 or 2) variable bases from VT tables 0..NV-1, scalars given
// as recoded digit registers d[v] (L limbs, top window at the top bit).
// Returns the accumulator with T valid (the comb phase follows).
// flip_last: negate every digit of the last scalar (its table holds the
// negated base).
// Leading windows whose digits are zero in every lane of the wave only add
// the identity to the identity and are skipped (wave-uniform: the window
// count is the wave's largest scalar).  The lattice outputs of a 64-lane
// wave fit 131 bits in ~88% of waves, which drops the top window and its
// four doublings (tools/lattice_bits.py).
template <class T>
HSV_INL bool wave_any(T c) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __ballot(c != 0) != 0;
#else
  return c != 0;
#endif
}

template <int WA, int NW, int L, int NV, bool PREFETCH, class VT>
HSV_INL ge_ext straus_vt(uint32_t d[NV][L], VT &vt, uint32_t flip_last = 0) {
  constexpr int TS = 1 << (WA - 1);
  ge_ext q = ge_identity();
#ifdef HSV_TIMING_STUB_STRAUS  // tools/phase_probe.py only: wrong results, timing share of the window loop
  return q;
#endif
  int top = NW - 1;
  HSV_NOUNROLL
  while (top > 0) {
    uint32_t nz = 0;
    HSV_UNROLL
    for (int v = 0; v < NV; ++v) nz |= (d[v][L - 1] >> (32 - WA)) ^ (uint32_t)TS;
    if (wave_any(nz)) break;
    HSV_UNROLL
    for (int v = 0; v < NV; ++v) limbs_shl<L>(d[v], WA);
    --top;
  }
  HSV_NOUNROLL
  for (int i = top; i >= 0; --i) {
    uint32_t m[NV], neg[NV];
    HSV_UNROLL
    for (int v = 0; v < NV; ++v) {
      m[v] = digit_mag<TS>(d[v][L - 1] >> (32 - WA), neg[v]);
      if (v == NV - 1) neg[v] ^= flip_last;
      limbs_shl<L>(d[v], WA);
    }
    if constexpr (PREFETCH) {
      // both entries in flight during the doublings (2 x 32 registers)
      uint32_t w[NV][32];
      HSV_UNROLL
      for (int v = 0; v < NV; ++v) vt.get(v, m[v], w[v]);
      if (i != top) {
        HSV_NOUNROLL
        for (int j = 0; j < WA; ++j) q = ge_dbl_rt(q, j == WA - 1);
      }
      uint32_t cur[32], cneg = neg[0];
      HSV_UNROLL
      for (int x = 0; x < 32; ++x) cur[x] = w[0][x];
      HSV_NOUNROLL
      for (int v = 0; v < NV; ++v) {
        q = ge_add_cached_rt(q, ge_cached_cneg(cached_unpack(cur), cneg), v + 1 < NV || i == 0);
        if (NV > 1) {
          HSV_UNROLL
          for (int x = 0; x < 32; ++x) cur[x] = w[NV - 1][x];
          cneg = neg[NV - 1];
        }
      }
    } else {
      // entries loaded right before their addition (fewer live registers;
      // latency left to the other waves of the SIMD)
      if (i != top) {
        HSV_NOUNROLL
        for (int j = 0; j < WA; ++j) q = ge_dbl_rt(q, j == WA - 1);
      }
      uint32_t mv = m[0], cneg = neg[0];
      HSV_NOUNROLL
      for (int v = 0; v < NV; ++v) {
        uint32_t cur[32];
        vt.get(v, mv, cur);
        q = ge_add_cached_rt(q, ge_cached_cneg(cached_unpack(cur), cneg), v + 1 < NV || i == 0);
        mv = m[NV - 1];
        cneg = neg[NV - 1];
      }
    }
  }
  return q;
}

// Full-length path (fallback): [k](-A) by Straus with table 0, [s]B by comb,
// compared with R as points (dalek's check, verify_one's flags).
template <int WA, bool PREFETCH = true, int CB = 8, class VT>
HSV_INL uint32_t verify_one_full_comb(const uint32_t pk[8], const uint32_t sig[16], const uint32_t msg[8],
                                      const uint32_t *tb, VT &vt) {
  using G = Windows<WA, WA>;
  const uint32_t s_ok = sc_is_canonical(sig + 8);
  uint32_t h[16];
  sha512_96(sig, pk, msg, h);
  const sc k = sc_reduce512(h);
  fe ax, ay;
  const uint32_t a_ok = ge_decompress(pk, ax, ay);
  const uint32_t small_a = a_ok & y_is_small_order(ay);
  vt_build<G::TS>(vt, 0, fe_carry(fe_neg(ax)), ay);
  uint32_t d[1][8];
  recode_add<8, WA, G::NA>(k.v, 8, d[0]);
  limbs_shl_const<8, 256 - G::KBITS>(d[0]);
  ge_ext q = straus_vt<WA, G::NA, 8, 1, PREFETCH>(d, vt);
  q = comb_add_b<CB>(q, sig + 8, tb);
  fe rx, ry;
  const uint32_t r_ok = ge_decompress(sig, rx, ry);
  const uint32_t small_r = r_ok & y_is_small_order(ry);
  return flags_byte(s_ok, a_ok, r_ok, small_a, small_r, ge_eq_affine(q, rx, ry)) | fault_bit(a_ok, r_ok, q);
}

template <int WA>
struct HalfCombWindows {
  static constexpr int NW = (kLatCombBits + 1 + WA) / WA;  // c + C_WA < 2^(NW*WA) for c < 2^138
  static constexpr int BITS = NW * WA;
  static_assert(BITS <= 160 && BITS >= kLatCombBits + 2, "scalar bound vs loop length");
};

template <int WA, bool PREFETCH = true, int CB = 8, class VT>
HSV_INL uint32_t verify_one_half_comb(const uint32_t pk[8], const uint32_t sig[16], const uint32_t msg[8],
                                      const uint32_t *tb, VT &vt, bool &fallback, int lat_bits = kLatCombBits) {
  using G = HalfCombWindows<WA>;
  constexpr int TS = 1 << (WA - 1);
  const uint32_t s_ok = sc_is_canonical(sig + 8);
  uint32_t h[16];
  sha512_96(sig, pk, msg, h);
  const sc k = sc_reduce512(h);

  // tables first (R and A are dead afterwards), the lattice reduction after
  // them, so its outputs are not live across the two root chains
  uint32_t a_ok, small_a, r_ok, small_r;
  {
    fe x, y;
    r_ok = ge_decompress(sig, x, y);
    small_r = r_ok & y_is_small_order(y);
    vt_build<TS>(vt, 0, fe_carry(fe_neg(x)), y);
  }
  {
    fe x, y;
    a_ok = ge_decompress(pk, x, y);
    small_a = a_ok & y_is_small_order(y);
    vt_build<TS>(vt, 1, fe_carry(fe_neg(x)), y);  // -A; the sign of c0 flips the digits
  }
  const LatOut lat = lattice_reduce(k, lat_bits);
  fallback = !lat.ok;
  uint32_t d[2][5];
  recode_top5<WA, G::NW>(lat.c1, d[0]);
  recode_top5<WA, G::NW>(lat.c0, d[1]);
  ge_ext q = straus_vt<WA, G::NW, 5, 2, PREFETCH>(d, vt, lat.c0_neg);
  const sc b = sc_mul_small(lat.c1, sig + 8);
  q = comb_add_b<CB>(q, b.v, tb);
  const uint32_t same = ge_is_neutral(q);  // Q == O
  return flags_byte(s_ok, a_ok, r_ok, small_a, small_r, same) | fault_bit(a_ok, r_ok, q);
}

// ---- two-pass form: scalar prepass + point pass ---------------------------
// The prepass (one lane per item) does everything that depends only on the
// scalars: s < l, SHA-512, k mod l, the lattice reduction, the recoded
// digits of c1 and |c0| and b = (c1 s) mod l, and writes them to a
// structure-of-arrays record (word j of item i at rec[j * stride + i]).
// Items without a short pair are flagged there and listed, so the point pass
// can deal them out first: their full-length work then overlaps the bulk of
// the batch instead of trailing it.
constexpr int kPrepWords = 19;  // d(c1)[5] | d(|c0|)[5] | b[8] | meta
enum : uint32_t { kPrepSOk = 1u, kPrepC0Neg = 2u, kPrepFallback = 4u };

// How prep_scalars stores its record words: plain stores here; the fused
// transaction launch (hsv_mempool.hip) passes write-through stores, because
// other workgroups of the same launch read the records.
struct PutPlain {
  static HSV_MEMBER void u32(uint32_t *p, uint32_t v) { *p = v; }
};

// lat_bits: the lattice bound (kLatCombBits; lower values only to exercise the
// full-length path in tests, hsvi_set_lattice_bits).
template <int WA, class Put = PutPlain>
HSV_INL bool prep_scalars(const uint32_t pk[8], const uint32_t sig[16], const uint32_t msg[8], uint32_t *rec,
                          uint64_t stride, int lat_bits = kLatCombBits) {
  using G = HalfCombWindows<WA>;
  const uint32_t s_ok = sc_is_canonical(sig + 8);
  uint32_t h[16];
  sha512_96(sig, pk, msg, h);
  const sc k = sc_reduce512(h);
  const LatOut lat = lattice_reduce(k, lat_bits);
  uint32_t d[5];
  recode_top5<WA, G::NW>(lat.c1, d);
  HSV_UNROLL
  for (int i = 0; i < 5; ++i) Put::u32(rec + i * stride, d[i]);
  recode_top5<WA, G::NW>(lat.c0, d);
  HSV_UNROLL
  for (int i = 0; i < 5; ++i) Put::u32(rec + (5 + i) * stride, d[i]);
  const sc b = sc_mul_small(lat.c1, sig + 8);
  HSV_UNROLL
  for (int i = 0; i < 8; ++i) Put::u32(rec + (10 + i) * stride, b.v[i]);
  Put::u32(rec + 18 * stride,
           (s_ok ? kPrepSOk : 0u) | (lat.c0_neg ? kPrepC0Neg : 0u) | (lat.ok ? 0u : kPrepFallback));
  return !lat.ok;
}

// Point pass of a prepped item: the half-size equation of
// verify_one_half_comb with the scalars read back from the record.
// `rb` is R (the first 32 bytes of the signature).
// HSV_PHASE_CLOCKS (tools/phase_clock_probe.py only): wall-clock stamps at the
// phase boundaries of the point pass, clk[1..3] after decompression, tables
// and the window loop.
#ifdef HSV_PHASE_CLOCKS
#define HSV_CLK(j)                       \
  do {                                   \
    if (clk) clk[j] = wall_clock64();    \
  } while (0)
#else
#define HSV_CLK(j) \
  do {             \
  } while (0)
#endif

template <int WA, int CB, class VT>
HSV_INL uint32_t verify_one_prepped(const uint32_t pk[8], const uint32_t rb[8], const uint32_t *rec,
                                    uint64_t stride, const uint32_t meta, const uint32_t *tb, VT &vt,
                                    uint64_t *clk = nullptr) {
  using G = HalfCombWindows<WA>;
  constexpr int TS = 1 << (WA - 1);
  uint32_t a_ok, small_a, r_ok, small_r;
  {
    fe xr, yr, xa, ya;
    ge_decompress2(rb, pk, xr, yr, xa, ya, r_ok, a_ok);  // both root chains at once
    small_r = r_ok & y_is_small_order(yr);
    small_a = a_ok & y_is_small_order(ya);
    HSV_CLK(1);
    vt_build<TS>(vt, 0, fe_carry(fe_neg(xr)), yr);
    vt_build<TS>(vt, 1, fe_carry(fe_neg(xa)), ya);
    HSV_CLK(2);
  }
  uint32_t d[2][5];
  HSV_UNROLL
  for (int i = 0; i < 5; ++i) {
    d[0][i] = rec[i * stride];
    d[1][i] = rec[(5 + i) * stride];
  }
  ge_ext q = straus_vt<WA, G::NW, 5, 2, false>(d, vt, (meta & kPrepC0Neg) ? 1u : 0u);
  HSV_CLK(3);
  uint32_t b[8];
  HSV_UNROLL
  for (int i = 0; i < 8; ++i) b[i] = rec[(10 + i) * stride];
  q = comb_add_b<CB>(q, b, tb);
  const uint32_t same = ge_is_neutral(q);
  return flags_byte(meta & kPrepSOk, a_ok, r_ok, small_a, small_r, same) | fault_bit(a_ok, r_ok, q);
}

}  // namespace hsv
