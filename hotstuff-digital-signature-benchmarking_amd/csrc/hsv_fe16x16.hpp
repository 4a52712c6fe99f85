// GF(2^255 - 19) spread over a row of 16 lanes (device only): the latency
// form of a field element for a lone wave.
//
// A lone wave issues one VALU instruction per 4 clocks (8 for v_mad_u64_u32)
// however many of its lanes are active, so a product on one lane costs its
// whole instruction count: ~97 instructions and ~620 clocks for a squaring in
// radix 2^25.5 (hsv_fe26x10.hpp, profiles/r02w_ubench_fe_lone_wave.txt).
// Here lane k of a 16-lane DPP row holds limb k of a radix-2^16 element
// (2^256 = 38 mod p), and a product runs the 16 columns side by side:
//
//   step i = 0..15:  acc_k += f_i * g'_k,   g'_k = g_{(k-i) mod 16}, times 38
//                    once the limb has wrapped past lane 15 (2^256 = 38)
//   f_i  reaches every lane of the row by DPP row_newbcast:i,
//   g'   moves one lane up per step by DPP row_ror:1 folded into the
//        v_mul_u32_u24 that scales the wrapped limb (38 on lane 0, 1 elsewhere);
//   two carry passes (lane k's carry to lane k + 1, lane 15's times 38 to
//   lane 0) leave limbs <= 2^16.05 (the bound is a fixed point of the
//   passes; operands may also be unreduced sums with limbs < 2^18, whose
//   product comes out <= 2^16.1: tools/lanesplit_model.py checks every
//   instruction's bound over worst-case inputs, tests/test_lanesplit.py).
//
// 16 v_mad_u64_u32 + 16 broadcasts + 15 rotations + 8 carry instructions:
// ~55 instructions and ~290 clocks per product or squaring on a lone wave.
// Four rows of a wave hold four independent elements.
//
// Bounds (limbs <= M = 2^16.05 in, out):
//   g' <= 38 M < 2^21.3 (the u24 multiply needs < 2^24);
//   acc_0 <= M^2 (15 * 38 + 1) < 2^41.3;
//   pass 1 carry <= 2^25.3 (lane 15's: <= 16 M^2 / 2^16, times 38 < 2^25.4);
//   pass 2 carry <= 2^9.3, lane 15's times 38 <= 2^11.1.
#pragma once
#include "hsv_point.hpp"

#if defined(__HIPCC__)
namespace hsv {

// lane constants of the row form, computed once per kernel
struct RowLane {
  uint32_t k;     // limb index = lane & 15
  uint32_t win;   // 38 on lane 0 (a limb arriving from lane 15 wraps), else 1
  uint32_t wout;  // 38 on lane 15 (its carry wraps to lane 0), else 1
  __device__ __forceinline__ RowLane() {
    k = __lane_id() & 15u;
    win = k == 0u ? 38u : 1u;
    wout = k == 15u ? 38u : 1u;
  }
};

// DPP within a row of 16 lanes
template <int I>
__device__ __forceinline__ uint32_t row_bcast(uint32_t x) {  // lane I of the row, to every lane of it
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x150 + I, 0xf, 0xf, true);
}
__device__ __forceinline__ uint32_t row_ror1(uint32_t x) {  // lane k <- lane (k - 1) mod 16
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x121, 0xf, 0xf, true);
}
__device__ __forceinline__ uint32_t row_shl1(uint32_t x) {  // lane k <- lane k + 1 (lane 15 <- 0)
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x101, 0xf, 0xf, true);
}

template <int I>
__device__ __forceinline__ fe fe_row_bcast(const fe &a) {
  fe r;
  HSV_UNROLL
  for (int l = 0; l < kFeLimbs; ++l) r.v[l] = row_bcast<I>(a.v[l]);
  return r;
}

// a on row lane 0 (and 3..15), b on lane 1, c on lane 2
__device__ __forceinline__ fe fe_row_pick3(const fe &a, const fe &b, const fe &c) {
  fe r;
  const uint64_t m1 = 0x0002000200020002ull, m2 = 0x0004000400040004ull;
  HSV_UNROLL
  for (int l = 0; l < kFeLimbs; ++l) {
    uint32_t x;
    asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(x) : "v"(a.v[l]), "v"(b.v[l]), "s"(m1));
    asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(r.v[l]) : "v"(x), "v"(c.v[l]), "s"(m2));
  }
  return r;
}

template <int I>
__device__ __forceinline__ void fl_mul_step(uint64_t &acc, uint32_t &gr, uint32_t f, const RowLane &L) {
  if constexpr (I > 0) gr = __umul24(row_ror1(gr), L.win);
  acc += (uint64_t)row_bcast<I>(f) * gr;
  if constexpr (I < 15) fl_mul_step<I + 1>(acc, gr, f, L);
}

// f * g, limbs <= 2^16.05 in and out
__device__ __forceinline__ uint32_t fl_mul(uint32_t f, uint32_t g, const RowLane &L) {
  HSV_SCHED_FENCE();
  uint64_t acc = 0;
  uint32_t gr = g;
  fl_mul_step<0>(acc, gr, f, L);
  // pass 1: the carry may exceed 2^24, so lane 15's factor 38 is a full multiply
  uint32_t lo = (uint32_t)acc & 0xffffu;
  uint32_t t = __builtin_amdgcn_alignbit((uint32_t)(acc >> 32), (uint32_t)acc, 16);
  uint32_t x = lo + row_ror1(t * L.wout);
  // pass 2
  lo = x & 0xffffu;
  t = x >> 16;
  x = lo + row_ror1(__umul24(t, L.wout));
  HSV_SCHED_FENCE();
  return x;
}

__device__ __forceinline__ uint32_t fl_sq(uint32_t f, const RowLane &L) { return fl_mul(f, f, L); }

// ---- two rows per element ---------------------------------------------------
// Rows 2j and 2j+1 hold the same element; a product splits its 16 steps
// between them (the even row steps 0..7, the odd row steps 8..15, starting
// from g turned by 8 lanes with the wrapped half times 38 and from f turned by
// 8 so that row_newbcast:i yields f_(i+8)), and v_permlane16_swap adds the two
// rows' column sums, so both rows end with the whole product.  8 steps instead
// of 16 on the critical path.
struct RowLane2 : RowLane {
  uint32_t w8;  // 38 on lanes 0..7 of an odd row (their turned limbs wrapped), else 1
  __device__ __forceinline__ RowLane2() : RowLane() { w8 = ((__lane_id() >> 4) & 1u) && k < 8u ? 38u : 1u; }
};

// x on even rows, x turned by 8 lanes on odd rows: one DPP move whose row
// mask (0xa) leaves the even rows' old value
__device__ __forceinline__ uint32_t row_odd_ror8(uint32_t x) {
  return (uint32_t)__builtin_amdgcn_update_dpp((int)x, (int)x, 0x128, 0xa, 0xf, false);
}

template <int I>
__device__ __forceinline__ void fl2_mul_step(uint64_t &acc, uint32_t &gr, uint32_t f, const RowLane &L) {
  if constexpr (I > 0) gr = __umul24(row_ror1(gr), L.win);
  acc += (uint64_t)row_bcast<I>(f) * gr;
  if constexpr (I < 7) fl2_mul_step<I + 1>(acc, gr, f, L);
}

__device__ __forceinline__ uint32_t fl2_mul(uint32_t f, uint32_t g, const RowLane2 &L) {
  HSV_SCHED_FENCE();
  uint64_t acc = 0;
  uint32_t gr = __umul24(row_odd_ror8(g), L.w8);
  fl2_mul_step<0>(acc, gr, row_odd_ror8(f), L);
  // each row's half column sums split at bit 16, then the two rows' halves
  // added across the pair (lane 15's column has no wrapped terms, so the
  // summed carry times 38 stays below 2^32 as in fl_mul)
  const uint32_t lo_h = (uint32_t)acc & 0xffffu;
  const uint32_t t_h = __builtin_amdgcn_alignbit((uint32_t)(acc >> 32), (uint32_t)acc, 16);
  const auto ls = __builtin_amdgcn_permlane16_swap(lo_h, lo_h, false, false);
  const auto ts = __builtin_amdgcn_permlane16_swap(t_h, t_h, false, false);
  uint32_t x = (ls[0] + ls[1]) + row_ror1((ts[0] + ts[1]) * L.wout);
  uint32_t lo16 = x & 0xffffu;
  uint32_t t = x >> 16;
  x = lo16 + row_ror1(__umul24(t, L.wout));
  HSV_SCHED_FENCE();
  return x;
}

// the two-row form behind the same names, so fl_pow22523 and
// ge_decompress_row take either lane layout
__device__ __forceinline__ uint32_t fl_mul(uint32_t f, uint32_t g, const RowLane2 &L) { return fl2_mul(f, g, L); }
__device__ __forceinline__ uint32_t fl_sq(uint32_t f, const RowLane2 &L) { return fl2_mul(f, f, L); }

template <class Lane>
__device__ __forceinline__ uint32_t fl_sqn(uint32_t f, int n, const Lane &L) {
  HSV_NOUNROLL
  for (int i = 0; i < n; ++i) f = fl_sq(f, L);
  return f;
}

// (Round 4's compact form of this chain -- one squaring body and one product
// body looped over a 12-step program -- shortened the R waves at C3 but made
// the drop-in call 2.2-2.5 us slower, profiles/r04t_qc_ab_compact.txt; it was
// removed in round 5 and is in git history at 5c186e7.)

// z^((p-5)/8) = z^(2^252 - 3), the chain of fe_pow22523 (hsv_field.hpp)
template <class Lane>
__device__ __forceinline__ uint32_t fl_pow22523(uint32_t z, const Lane &L) {
  uint32_t t0 = fl_sq(z, L);                 // 2
  uint32_t t1 = fl_sq(fl_sq(t0, L), L);      // 8
  t1 = fl_mul(z, t1, L);                     // 9
  t0 = fl_mul(t0, t1, L);                    // 11
  t0 = fl_sq(t0, L);                         // 22
  t0 = fl_mul(t1, t0, L);                    // 31 = 2^5 - 1
  t1 = fl_sqn(t0, 5, L);
  t0 = fl_mul(t1, t0, L);                    // 2^10 - 1
  t1 = fl_sqn(t0, 10, L);
  t1 = fl_mul(t1, t0, L);                    // 2^20 - 1
  uint32_t t2 = fl_sqn(t1, 20, L);
  t1 = fl_mul(t2, t1, L);                    // 2^40 - 1
  t1 = fl_sqn(t1, 10, L);
  t0 = fl_mul(t1, t0, L);                    // 2^50 - 1
  t1 = fl_sqn(t0, 50, L);
  t1 = fl_mul(t1, t0, L);                    // 2^100 - 1
  t2 = fl_sqn(t1, 100, L);
  t1 = fl_mul(t2, t1, L);                    // 2^200 - 1
  t1 = fl_sqn(t1, 50, L);
  t0 = fl_mul(t1, t0, L);                    // 2^250 - 1
  t0 = fl_sqn(t0, 2, L);                     // 2^252 - 4
  return fl_mul(t0, z, L);                   // 2^252 - 3
}

// Limb k of 8 little-endian words held identically by every lane of the row:
// word k/2 by selects on lane masks (the row pattern repeats every 16 lanes),
// no indexed register access.
__device__ __forceinline__ uint32_t row_limb_of_words(const uint32_t w[8], const RowLane &L) {
  uint32_t x = w[0];
  HSV_UNROLL
  for (int j = 1; j < 8; ++j) {
    const uint64_t m = 0x0003000300030003ull << (2 * j);
    asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(x) : "v"(x), "v"(w[j]), "s"(m));
  }
  return (L.k & 1u) ? x >> 16 : x & 0xffffu;
}

// The element held identically by every lane of the row (class R, ten
// limbs) -> this lane's radix-2^16 limb of its canonical value.
__device__ __forceinline__ uint32_t fl_from_fe(const fe &a, const RowLane &L) {
  uint32_t w[8];
  fe_pack(a, w);
  return row_limb_of_words(w, L);
}

// this row's element (limbs <= 2^16.05) -> ten limbs (class R, value < 2^255,
// possibly >= p) in every lane of the row.  nc |= 1 when the carry passes did
// not converge (a lane still holds bits above its limb width after the cap):
// the bounds model (tools/lanesplit_model.py) never needs more than 17
// passes, so that is an out-of-model input -- the callers OR it into the
// launch's self-check word, so it becomes HSV_ERR_DEVICE_FAULT, never a verdict.
__device__ __forceinline__ fe fl_to_fe(uint32_t x, const RowLane &L, uint32_t &nc) {
  // exact limbs: 16 bits each, 15 for limb 15, whose carry (weight 2^255)
  // wraps to lane 0 times 19; repeated until no lane of the wave carries
  const uint32_t sh = L.k == 15u ? 15u : 16u;
  const uint32_t mask = (1u << sh) - 1u;
  const uint32_t w19 = L.k == 15u ? 19u : 1u;
  // at most 17 passes carry anything (a carry can ripple once round the row);
  // the cap keeps the loop finite whatever the limbs hold
  for (int pass = 0; pass < 20; ++pass) {
    const uint32_t t = x >> sh;
    x = (x & mask) + row_ror1(__umul24(t, w19));
    if (!__ballot(t != 0u)) break;
  }
  if (__ballot((x >> sh) != 0u)) nc = 1u;
  // words: lane 2j holds limbs 2j | 2j+1, then each word to every lane
  const uint32_t pair = x | (row_shl1(x) << 16);
  uint32_t w[8];
  w[0] = row_bcast<0>(pair);
  w[1] = row_bcast<2>(pair);
  w[2] = row_bcast<4>(pair);
  w[3] = row_bcast<6>(pair);
  w[4] = row_bcast<8>(pair);
  w[5] = row_bcast<10>(pair);
  w[6] = row_bcast<12>(pair);
  w[7] = row_bcast<14>(pair);
  return fe_from_words_masked(w);
}

__device__ __forceinline__ fe fl_to_fe(uint32_t x, const RowLane &L) {
  uint32_t nc = 0;
  return fl_to_fe(x, L, nc);
}

// ---- checks of a point held identically by every lane of a row ----
// ge_is_sane (hsv_point.hpp) in three rounds instead of seven operations:
// X^2 | Y^2 | Z^2, then (Y^2 - X^2) Z^2 | X^2 Y^2 | Z^4, then d X^2 Y^2.
// Z != 0 comes back separately for the equation check.
__device__ __forceinline__ uint32_t ge_is_sane_row(const ge_ext &p, uint32_t &z_nonzero) {
  const fe s1 = fe_sq(fe_row_pick3(p.X, p.Y, p.Z));
  const fe xx = fe_row_bcast<0>(s1), yy = fe_row_bcast<1>(s1), zz = fe_row_bcast<2>(s1);
  const fe s2 = fe_mul(fe_row_pick3(fe_sub(yy, xx), xx, zz), fe_row_pick3(zz, yy, zz));
  const fe lhs = fe_row_bcast<0>(s2), xy = fe_row_bcast<1>(s2), z4 = fe_row_bcast<2>(s2);
  const fe dxy = fe_mul(xy, fe_d());
  z_nonzero = fe_is_zero(p.Z) ^ 1u;
  return fe_eq(lhs, fe_add(z4, dxy)) & z_nonzero;
}

// ge_eq_affine (Q == (x, y), Z != 0 known): x Z == X on row lane 0 and
// y Z == Y on lane 1, one product each
__device__ __forceinline__ uint32_t ge_eq_affine_row(const ge_ext &p, const fe &x, const fe &y, uint32_t z_nonzero) {
  const fe t = fe_mul(fe_row_pick3(x, y, y), p.Z);
  const uint32_t e = fe_eq(t, fe_row_pick3(p.X, p.Y, p.Y));
  return row_bcast<0>(e) & row_bcast<1>(e) & z_nonzero;
}

// CompressedEdwardsY::decompress (ge_decompress, hsv_point.hpp) for one
// encoding per row, every lane of the row holding it: the products of
// sqrt_ratio_i -- y^2, d y^2, v^3, v^7, u v^7, the root chain, u v^3 (.)
// and v r^2 -- in the row form; the sign rules on ten limbs with their
// independent operations on separate lanes of the row (one product, then one
// comparison per lane).  Every lane of the row returns the same (x, y),
// flag and small-order bit as ge_decompress and y_is_small_order.
// nc |= 1: a carry normalisation did not converge (fl_to_fe).
template <class Lane>
__device__ __forceinline__ uint32_t ge_decompress_row(const uint32_t enc[8], fe &x, fe &y, uint32_t &small,
                                                      uint32_t &nc, const Lane &L) {
  y = fe_from_words_masked(enc);
  uint32_t yl = row_limb_of_words(enc, L);
  if (L.k == 15u) yl &= 0x7fffu;  // bit 255 is the sign of x
  const uint32_t yy = fl_sq(yl, L);
  // u = y^2 - 1 as y^2 + (p - 1), limbs < 2^17.1 (a product operand may be < 2^18)
  const uint32_t ul = yy + (L.k == 0u ? 0xffecu : L.k == 15u ? 0x7fffu : 0xffffu);
  const uint32_t v = fl_mul(yy, fl_from_fe(fe_d(), L), L) + (L.k == 0u ? 1u : 0u);
  const uint32_t v3 = fl_mul(fl_sq(v, L), v, L);
  const uint32_t v7 = fl_mul(fl_sq(v3, L), v, L);
  const uint32_t rl = fl_mul(fl_mul(ul, v3, L), fl_pow22523(fl_mul(ul, v7, L), L), L);
  const fe check = fl_to_fe(fl_mul(v, fl_sq(rl, L), L), L, nc);
  const fe u = fl_to_fe(ul, L, nc), r = fl_to_fe(rl, L, nc);
  // fe_sqrt_ratio_fix_chk: lane 0 -u sqrt(-1), lane 1 r sqrt(-1); then lane 0
  // check == u, lane 1 check == -u, lane 2 check == -u sqrt(-1)
  const fe neg_u = fe_neg(u);
  const fe t = fe_mul(fe_row_pick3(neg_u, r, r), fe_sqrtm1());
  const uint32_t e = fe_eq(check, fe_row_pick3(u, neg_u, fe_row_bcast<0>(t)));
  const uint32_t correct = row_bcast<0>(e), flipped = row_bcast<1>(e), flipped_i = row_bcast<2>(e);
  const fe rr = fe_select(r, fe_row_bcast<1>(t), flipped | flipped_i);
  // the non-negative root, then x's sign bit (-0 == 0 is accepted): one
  // negation decided by both, canonical; y canonical beside it on lane 1
  const uint32_t flip = fe_is_negative(rr) ^ (enc[7] >> 31);
  const fe c = fe_canon(fe_row_pick3(fe_select(rr, fe_neg(rr), flip), y, y));
  x = fe_row_bcast<0>(c);
  small = y_is_small_order_canon(fe_row_bcast<1>(c));
  return correct | flipped;
}

}  // namespace hsv
#endif
