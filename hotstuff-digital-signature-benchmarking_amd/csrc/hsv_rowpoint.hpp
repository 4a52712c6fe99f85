// Edwards25519 point arithmetic in the row form (hsv_fe16x16.hpp): one
// point per 16-lane DPP row, lane k holding limb k of each coordinate (or one
// point per pair of rows, Lane = RowLane2, with the products split between
// them).  The
// formulas are hsv_point.hpp's (HWCD, complete for a = -1), operation for
// operation, so the row kernels compute exactly what the one-lane kernels do.
//
// Operand bounds (limbs; tools/lanesplit_model.py replays these sequences on
// worst-case limbs, tests/test_lanesplit.py):
//   * a product's output is <= 2^16.3 when its operands are < 2^18.75 (the
//     model's largest over these formulas: 2^16.23);
//   * a - b is a + 4p - b (4p = 2^257 - 76 as limbs 0x1ffb4, 0x1fffe, ...,
//     each >= 2^17 - 76): b must be a product output;
//   * every product operand is a product output, a sum of two of them, or
//     one difference (< 2^18.4), below the 2^18.75 the rotated operand of
//     fl_mul allows (its limb times 38 feeds v_mul_u32_u24);
//   * the doubling's F (2 Z^2 + X^2 - Y^2) gets one carry pass, as in
//     ge_dbl_rt (fe_carry).
#pragma once
#include "hsv_fe16x16.hpp"
#include "hsv_verify_hc.hpp"

#if defined(__HIPCC__)
namespace hsv {

struct rp_ext {
  uint32_t X, Y, Z, T;
};
struct rp_cached {
  uint32_t YpX, YmX, Z2, T2d;
};

__device__ __forceinline__ uint32_t fl_small(uint32_t v, const RowLane &L) { return L.k == 0u ? v : 0u; }
__device__ __forceinline__ uint32_t fl_4p(const RowLane &L) { return L.k == 0u ? 0x1ffb4u : 0x1fffeu; }
// a - b (b a product output)
__device__ __forceinline__ uint32_t fl_sub(uint32_t a, uint32_t b, const RowLane &L) { return a + fl_4p(L) - b; }
// one carry pass (limbs < 2^24 in, <= 2^16 + 38 * 2^8 out)
__device__ __forceinline__ uint32_t fl_carry(uint32_t x, const RowLane &L) {
  return (x & 0xffffu) + row_ror1(__umul24(x >> 16, L.wout));
}

__device__ __forceinline__ rp_ext rp_identity(const RowLane &L) {
  return rp_ext{0u, fl_small(1, L), fl_small(1, L), 0u};
}

// X3 = E F, Y3 = G H, Z3 = F G, T3 = E H (ge_finish_rt); without T, T is 0
template <class Lane>
__device__ __forceinline__ rp_ext rp_finish(uint32_t E, uint32_t F, uint32_t G, uint32_t H, bool with_t,
                                            const Lane &L) {
  rp_ext r;
  r.X = fl_mul(E, F, L);
  r.Y = fl_mul(G, H, L);
  r.Z = fl_mul(F, G, L);
  r.T = with_t ? fl_mul(E, H, L) : 0u;
  return r;
}

// 2P (ge_dbl_rt)
template <class Lane>
__device__ __forceinline__ rp_ext rp_dbl(const rp_ext &p, bool with_t, const Lane &L) {
  const uint32_t A = fl_sq(p.X, L), B = fl_sq(p.Y, L), C = fl_sq(p.Z, L), S = fl_sq(p.X + p.Y, L);
  const uint32_t H = A + B;
  const uint32_t E = fl_sub(H, S, L);
  const uint32_t G = fl_sub(A, B, L);
  const uint32_t F = fl_carry(C + C + G, L);
  return rp_finish(E, F, G, H, with_t, L);
}

// P + Q, Q cached (ge_add_cached_rt)
template <class Lane>
__device__ __forceinline__ rp_ext rp_add_cached(const rp_ext &p, const rp_cached &q, bool with_t, const Lane &L) {
  const uint32_t A = fl_mul(fl_sub(p.Y, p.X, L), q.YmX, L);
  const uint32_t B = fl_mul(p.Y + p.X, q.YpX, L);
  const uint32_t C = fl_mul(p.T, q.T2d, L);
  const uint32_t D = fl_mul(p.Z, q.Z2, L);
  return rp_finish(fl_sub(B, A, L), fl_sub(D, C, L), D + C, B + A, with_t, L);
}

// P + Q, Q affine Niels (y + x, y - x, 2dxy) (ge_add_niels)
template <class Lane>
__device__ __forceinline__ rp_ext rp_add_niels(const rp_ext &p, uint32_t ypx, uint32_t ymx, uint32_t xy2d,
                                               bool with_t, const Lane &L) {
  const uint32_t A = fl_mul(fl_sub(p.Y, p.X, L), ymx, L);
  const uint32_t B = fl_mul(p.Y + p.X, ypx, L);
  const uint32_t C = fl_mul(p.T, xy2d, L);
  const uint32_t D = p.Z + p.Z;
  return rp_finish(fl_sub(B, A, L), fl_sub(D, C, L), D + C, B + A, with_t, L);
}

template <class Lane>
__device__ __forceinline__ rp_cached rp_to_cached(const rp_ext &p, uint32_t d2, const Lane &L) {
  return rp_cached{p.Y + p.X, fl_sub(p.Y, p.X, L), p.Z + p.Z, fl_mul(p.T, d2, L)};
}

// The point of the partner row (lane ^ 16: rows 0 <-> 1, 2 <-> 3), or of the
// partner row pair (lane ^ 32) in the two-row form
__device__ __forceinline__ rp_ext rp_swap_rows(const rp_ext &p, int mask = 16) {
  return rp_ext{(uint32_t)__shfl_xor((int)p.X, mask, 64), (uint32_t)__shfl_xor((int)p.Y, mask, 64),
                (uint32_t)__shfl_xor((int)p.Z, mask, 64), (uint32_t)__shfl_xor((int)p.T, mask, 64)};
}

// ---- the per-row variable-base table in LDS --------------------------------
// Entries m = 0..TS of [m](-P), cached form, at tab[(m * 4 + c) * 16 + k]
// (c: YpX, YmX, Z2, T2d); entry 0 is the identity.  Built as
// [m](-P) = [m-1](-P) + (-P) with -P in affine Niels form, as vt_build.
// inject (tests): entries 1.. stored as zeros, or with one bit flipped when
// flip_this_table (the pair kernel's table 0, R).
template <int TS, class Lane>
__device__ __forceinline__ void row_table_build(uint32_t *tab, const fe &x, const fe &y, const Lane &L,
                                                uint32_t inject, bool flip_this_table) {
  const uint32_t nx = fl_from_fe(fe_carry(fe_neg(x)), L);  // -x
  const uint32_t yl = fl_from_fe(y, L);
  const uint32_t d2 = fl_from_fe(fe_d2(), L);
  const uint32_t t1 = fl_mul(nx, yl, L);
  const uint32_t ypx = yl + nx, ymx = fl_sub(yl, nx, L), xy2d = fl_mul(t1, d2, L);
  auto put = [&](int m, uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
    if (m > 0 && inject == kInjectZeroTables) a = b = c = d = 0u;
    if (m > 0 && inject == kInjectFlipTables && flip_this_table && L.k == 0u) a ^= 1u;
    tab[(m * 4 + 0) * 16 + L.k] = a;
    tab[(m * 4 + 1) * 16 + L.k] = b;
    tab[(m * 4 + 2) * 16 + L.k] = c;
    tab[(m * 4 + 3) * 16 + L.k] = d;
  };
  put(0, fl_small(1, L), fl_small(1, L), fl_small(2, L), 0u);
  put(1, ypx, ymx, fl_small(2, L), xy2d);
  rp_ext p{nx, yl, fl_small(1, L), t1};
  HSV_NOUNROLL
  for (int m = 2; m <= TS; ++m) {
    p = rp_add_niels(p, ypx, ymx, xy2d, true, L);
    const rp_cached c = rp_to_cached(p, d2, L);
    put(m, c.YpX, c.YmX, c.Z2, c.T2d);
  }
}

// entry m of the row's table, negated when neg (swap Y+X / Y-X, -2dT)
__device__ __forceinline__ rp_cached row_table_entry(const uint32_t *tab, uint32_t m, uint32_t neg,
                                                     const RowLane &L) {
  const uint32_t *e = tab + m * 64u + L.k;
  const uint32_t a = e[0], b = e[16], z2 = e[32], t = e[48];
  return rp_cached{neg ? b : a, neg ? a : b, z2, neg ? fl_sub(0u, t, L) : t};
}

// One-scalar Straus over the row's table: the digit registers d (5 words,
// top window at the top bits, as recode_top5) of NW windows of WA bits;
// flip negates every digit.  Leading windows whose digits are zero in every
// row of the wave are skipped (wave-uniform).  T is valid on return.
template <int WA, int NW, class Lane>
__device__ __forceinline__ rp_ext row_straus(uint32_t d[5], const uint32_t *tab, uint32_t flip, const Lane &L) {
  constexpr int TS = 1 << (WA - 1);
  rp_ext q = rp_identity(L);
  int top = NW - 1;
  HSV_NOUNROLL
  while (top > 0) {
    if (__ballot(((d[4] >> (32 - WA)) ^ (uint32_t)TS) != 0u)) break;
    limbs_shl<5>(d, WA);
    --top;
  }
  HSV_NOUNROLL
  for (int i = top; i >= 0; --i) {
    uint32_t neg;
    const uint32_t m = digit_mag<TS>(d[4] >> (32 - WA), neg);
    limbs_shl<5>(d, WA);
    if (i != top) {
      HSV_NOUNROLL
      for (int j = 0; j < WA; ++j) q = rp_dbl(q, j == WA - 1, L);
    }
    q = rp_add_cached(q, row_table_entry(tab, m, neg ^ flip, L), i == 0, L);
  }
  return q;
}

// q + the comb digits of half h of s (comb_add_b_half): positions
// [h NP/2, (h+1) NP/2) of the CB-bit comb table tb; each lane reads its 16-bit
// limb of the entry's three packed coordinates.
template <int CB, class Lane>
__device__ __forceinline__ rp_ext row_comb_half(rp_ext q, const uint32_t s[8], const uint32_t *tb, uint32_t h,
                                                const Lane &L) {
  constexpr int NP = 256 / CB, HALF = NP / 2;
  constexpr int ENT = 1 << (CB - 1);
  uint32_t sr[9];
  recode_add<9, CB, NP>(s, 8, sr);
  HSV_UNROLL
  for (int i = 0; i < 4; ++i) sr[i] = h ? sr[i + 4] : sr[i];
  const uint32_t wsel = L.k >> 1, hs = (L.k & 1u) * 16u;
  HSV_NOUNROLL
  for (int j = 0; j < HALF; ++j) {
    const uint32_t cb = sr[0] & ((1u << CB) - 1u);
    HSV_UNROLL
    for (int i = 0; i < 3; ++i) sr[i] = (sr[i] >> CB) | (sr[i + 1] << (32 - CB));
    sr[3] >>= CB;
    const int32_t dg = (int32_t)cb - (1 << (CB - 1));
    const uint32_t neg = dg < 0, mag = (uint32_t)(neg ? -dg : dg);
    const uint32_t idx = mag == 0u ? 0u : mag - 1u;
    const uint32_t *e = tb + ((uint64_t)(j + (int)h * HALF) * ENT + idx) * kCombEntryWords;
    uint32_t a = (e[wsel] >> hs) & 0xffffu, b = (e[8 + wsel] >> hs) & 0xffffu, c = (e[16 + wsel] >> hs) & 0xffffu;
    if (mag == 0u) {
      a = fl_small(1, L);
      b = fl_small(1, L);
      c = 0u;
    }
    q = rp_add_niels(q, neg ? b : a, neg ? a : b, neg ? fl_sub(0u, c, L) : c, true, L);
  }
  return q;
}

// ---- one point per wave, the formulas' four products on the four rows ----
// The HWCD formulas above are two rounds of four independent products each:
// a doubling squares X, Y, Z and X + Y, then forms E F, G H, F G, E H; an
// addition multiplies (Y - X, Y + X, T, Z) by the other point's four
// components, then forms the same four products.  Here every row of a wave
// holds the whole point (row-form limbs, lane k of each row holding limb k of
// X, Y, Z and T) and row r computes product r of each round with fl_mul on
// RowLane -- four products in the time of one -- then three permlane swaps
// give every row all four results.  Against RowLane2, which splits each
// product of the same sequence over two rows, a doubling issues ~135
// instructions instead of ~330.  The values are those of rp_dbl /
// rp_add_cached / rp_add_niels operation for operation (the Niels addition's D
// = 2 Z is computed as Z * 2 on row 3), so tools/lanesplit_model.py's bounds
// carry over.
struct QuadLane : RowLane {
  uint32_t r;  // row of the wave: which product of a round this lane's row computes
  __device__ __forceinline__ QuadLane() : RowLane() { r = (__lane_id() >> 4) & 3u; }
};

struct qp_ext {
  uint32_t X, Y, Z, T;
};

// a0 on row 0, a1 on row 1, a2 on row 2, a3 on row 3
__device__ __forceinline__ uint32_t qsel(uint32_t a0, uint32_t a1, uint32_t a2, uint32_t a3) {
  uint32_t x;
  asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(x) : "v"(a0), "v"(a1), "s"(0x00000000ffff0000ull));
  asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(x) : "v"(x), "v"(a2), "s"(0x0000ffff00000000ull));
  asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(x) : "v"(x), "v"(a3), "s"(0xffff000000000000ull));
  return x;
}

// rows 0..3's values of v, on every row: v_permlane16_swap leaves the even
// row's value of each row pair in result 0 and the odd row's in result 1, on
// both rows of the pair; v_permlane32_swap does the same for the two halves
__device__ __forceinline__ void qgather(uint32_t v, uint32_t &v0, uint32_t &v1, uint32_t &v2, uint32_t &v3) {
  const auto p = __builtin_amdgcn_permlane16_swap(v, v, false, false);
  const auto q0 = __builtin_amdgcn_permlane32_swap(p[0], p[0], false, false);
  const auto q1 = __builtin_amdgcn_permlane32_swap(p[1], p[1], false, false);
  v0 = q0[0];
  v1 = q1[0];
  v2 = q0[1];
  v3 = q1[1];
}

// round 2 of every formula: X3 = E F, Y3 = G H, Z3 = F G, T3 = E H
__device__ __forceinline__ qp_ext q_finish(uint32_t E, uint32_t F, uint32_t G, uint32_t H, const QuadLane &L) {
  const uint32_t t = fl_mul(qsel(E, G, F, E), qsel(F, H, G, H), L);
  qp_ext r;
  qgather(t, r.X, r.Y, r.Z, r.T);
  return r;
}

// 2P (rp_dbl, T always formed)
__device__ __forceinline__ qp_ext q_dbl(const qp_ext &p, const QuadLane &L) {
  const uint32_t s = fl_sq(qsel(p.X, p.Y, p.Z, p.X + p.Y), L);
  uint32_t A, B, C, S;
  qgather(s, A, B, C, S);
  const uint32_t H = A + B;
  return q_finish(fl_sub(H, S, L), fl_carry(C + C + fl_sub(A, B, L), L), fl_sub(A, B, L), H, L);
}

// P + Q given Q's operand for this row: row 0 (y - x)', row 1 (y + x)', row 2
// the T factor (2dT, or 2dxy for a Niels entry), row 3 the Z factor (2Z, or 2
// for a Niels entry) -- rp_add_cached / rp_add_niels
__device__ __forceinline__ qp_ext q_add_op(const qp_ext &p, uint32_t op, const QuadLane &L) {
  const uint32_t s = fl_mul(qsel(fl_sub(p.Y, p.X, L), p.Y + p.X, p.T, p.Z), op, L);
  uint32_t A, B, C, D;
  qgather(s, A, B, C, D);
  return q_finish(fl_sub(B, A, L), fl_sub(D, C, L), D + C, B + A, L);
}

// this row's component of P's cached form (rp_to_cached): row 0 Y + X,
// row 1 Y - X, row 2 2Z, row 3 2dT
__device__ __forceinline__ uint32_t q_cached_component(const qp_ext &p, uint32_t d2, const QuadLane &L) {
  const uint32_t t2d = fl_mul(p.T, d2, L);
  return qsel(p.Y + p.X, fl_sub(p.Y, p.X, L), p.Z + p.Z, t2d);
}

// this row's operand for adding a point handed over in cached form (c[r * 16
// + k] = component r, q_cached_component's layout): row 0 YmX, row 1 YpX, row
// 2 T2d, row 3 Z2
__device__ __forceinline__ uint32_t q_op_of_cached(const uint32_t *c, const QuadLane &L) {
  return c[(L.r ^ 1u) * 16u + L.k];  // components 0 <-> 1, 2 <-> 3
}

// this row's operand for adding a cached entry (components c = 0 YpX, 1 YmX,
// 2 Z2, 3 T2d of cmp_of(c)), negated when neg (swap YpX / YmX, -2dT)
__device__ __forceinline__ uint32_t q_cached_col(uint32_t r, uint32_t neg) {
  // row 0 wants YmX (YpX when negated), row 1 YpX (YmX), row 2 T2d, row 3 Z2
  return r < 2u ? (r ^ (neg ? 0u : 1u)) : (r == 2u ? 3u : 2u);
}

// The wave's variable-base table in LDS, entries m = 0..TS of [m](-P) in
// cached form at tab[(m * 4 + c) * 16 + k] (row_table_build's layout): built
// as [m](-P) = [m-1](-P) + (-P), -P as an affine Niels operand.
template <int TS>
__device__ __forceinline__ void quad_table_build(uint32_t *tab, const fe &x, const fe &y, const QuadLane &L,
                                                 uint32_t inject, bool flip_this_table) {
  const uint32_t nx = fl_from_fe(fe_carry(fe_neg(x)), L);  // -x
  const uint32_t yl = fl_from_fe(y, L);
  const uint32_t d2 = fl_from_fe(fe_d2(), L);
  const uint32_t t1 = fl_mul(nx, yl, L);
  const uint32_t ypx = yl + nx, ymx = fl_sub(yl, nx, L), xy2d = fl_mul(t1, d2, L);
  auto put = [&](int m, uint32_t v) {  // this row's component c = r of entry m
    if (m > 0 && inject == kInjectZeroTables) v = 0u;
    if (m > 0 && inject == kInjectFlipTables && flip_this_table && L.k == 0u && L.r == 0u) v ^= 1u;
    tab[(m * 4 + (int)L.r) * 16 + L.k] = v;
  };
  put(0, qsel(fl_small(1, L), fl_small(1, L), fl_small(2, L), 0u));
  put(1, qsel(ypx, ymx, fl_small(2, L), xy2d));
  const uint32_t op = qsel(ymx, ypx, xy2d, fl_small(2, L));  // -P as a Niels operand
  qp_ext p{nx, yl, fl_small(1, L), t1};
  HSV_NOUNROLL
  for (int m = 2; m <= TS; ++m) {
    p = q_add_op(p, op, L);
    put(m, q_cached_component(p, d2, L));
  }
}

// One-scalar Straus over the wave's table (row_straus).  T is valid on return.
// LO > 0: windows LO-1..0 are only doubled through, their digits left to a
// helper wave (quad_straus_low): the sum is [c - c_lo](-P), c_lo the signed
// value of the low LO windows, so a helper's [c_lo](-P) completes it.
template <int WA, int NW, int LO = 0>
__device__ __forceinline__ qp_ext quad_straus(uint32_t d[5], const uint32_t *tab, uint32_t flip, const QuadLane &L) {
  constexpr int TS = 1 << (WA - 1);
  qp_ext q{0u, fl_small(1, L), fl_small(1, L), 0u};
  int top = NW - 1;
  HSV_NOUNROLL
  while (top > 0) {
    if (__ballot(((d[4] >> (32 - WA)) ^ (uint32_t)TS) != 0u)) break;
    limbs_shl<5>(d, WA);
    --top;
  }
  HSV_NOUNROLL
  for (int i = top; i >= 0; --i) {
    uint32_t neg;
    const uint32_t m = digit_mag<TS>(d[4] >> (32 - WA), neg);
    limbs_shl<5>(d, WA);
    neg ^= flip;
    uint32_t op = 0u;
    if (i >= LO) {
      op = tab[(m * 4u + q_cached_col(L.r, neg)) * 16u + L.k];
      if (neg && L.r == 2u) op = fl_sub(0u, op, L);
    }
    if (i != top) {
      HSV_NOUNROLL
      for (int j = 0; j < WA; ++j) q = q_dbl(q, L);
    }
    if (i >= LO) q = q_add_op(q, op, L);
  }
  return q;
}

// The helper's part of a split Straus: [c_lo](-P) over the low LO windows of
// the same digits (the main wave runs quad_straus<WA, NW, LO>).
template <int WA, int NW, int LO>
__device__ __forceinline__ qp_ext quad_straus_low(uint32_t d[5], const uint32_t *tab, uint32_t flip,
                                                  const QuadLane &L) {
  static_assert(LO > 0 && LO < NW, "split window");
  HSV_UNROLL
  for (int i = 0; i < NW - LO; ++i) limbs_shl<5>(d, WA);
  return quad_straus<WA, LO, 0>(d, tab, flip, L);
}

// The two-scalar Straus of one wave holding both tables (the joint form):
// [c1](-R) + [c0](-A) with shared doublings, digits d1 over tab_r and d0 over
// tab_a (the sign of c0 flips the A digits), as straus_vt over two tables.
// LO > 0: the low LO windows are only doubled through (quad_straus, and
// quad_straus2_low for the helper's part).
template <int WA, int NW, int LO = 0>
__device__ __forceinline__ qp_ext quad_straus2(uint32_t d1[5], uint32_t d0[5], const uint32_t *tab_r,
                                               const uint32_t *tab_a, uint32_t flip_a, const QuadLane &L) {
  constexpr int TS = 1 << (WA - 1);
  qp_ext q{0u, fl_small(1, L), fl_small(1, L), 0u};
  int top = NW - 1;
  HSV_NOUNROLL
  while (top > 0) {
    if (__ballot((((d1[4] >> (32 - WA)) ^ (uint32_t)TS) | ((d0[4] >> (32 - WA)) ^ (uint32_t)TS)) != 0u)) break;
    limbs_shl<5>(d1, WA);
    limbs_shl<5>(d0, WA);
    --top;
  }
  HSV_NOUNROLL
  for (int i = top; i >= 0; --i) {
    uint32_t n1, n0;
    const uint32_t m1 = digit_mag<TS>(d1[4] >> (32 - WA), n1);
    const uint32_t m0 = digit_mag<TS>(d0[4] >> (32 - WA), n0);
    limbs_shl<5>(d1, WA);
    limbs_shl<5>(d0, WA);
    n0 ^= flip_a;
    uint32_t op1 = 0u, op0 = 0u;
    if (i >= LO) {
      op1 = tab_r[(m1 * 4u + q_cached_col(L.r, n1)) * 16u + L.k];
      op0 = tab_a[(m0 * 4u + q_cached_col(L.r, n0)) * 16u + L.k];
      if (n1 && L.r == 2u) op1 = fl_sub(0u, op1, L);
      if (n0 && L.r == 2u) op0 = fl_sub(0u, op0, L);
    }
    if (i != top) {
      HSV_NOUNROLL
      for (int j = 0; j < WA; ++j) q = q_dbl(q, L);
    }
    if (i >= LO) {
      q = q_add_op(q, op1, L);
      q = q_add_op(q, op0, L);
    }
  }
  return q;
}

// The helper's part of a split two-scalar Straus: the low LO windows of both
// digit strings (the main wave runs quad_straus2<WA, NW, LO>).
template <int WA, int NW, int LO>
__device__ __forceinline__ qp_ext quad_straus2_low(uint32_t d1[5], uint32_t d0[5], const uint32_t *tab_r,
                                                   const uint32_t *tab_a, uint32_t flip_a, const QuadLane &L) {
  static_assert(LO > 0 && LO < NW, "split window");
  HSV_UNROLL
  for (int i = 0; i < NW - LO; ++i) {
    limbs_shl<5>(d1, WA);
    limbs_shl<5>(d0, WA);
  }
  return quad_straus2<WA, LO, 0>(d1, d0, tab_r, tab_a, flip_a, L);
}

// q + the comb digits of half h of s (row_comb_half), each row reading only
// the coordinate its product needs; the half's entries are loaded up front so
// their latency overlaps the additions
template <int CB>
__device__ __forceinline__ qp_ext quad_comb_half(qp_ext q, const uint32_t s[8], const uint32_t *tb, uint32_t h,
                                                 const QuadLane &L) {
  constexpr int NP = 256 / CB, HALF = NP / 2;
  constexpr int ENT = 1 << (CB - 1);
  uint32_t sr[9];
  recode_add<9, CB, NP>(s, 8, sr);
  HSV_UNROLL
  for (int i = 0; i < 4; ++i) sr[i] = h ? sr[i + 4] : sr[i];
  const uint32_t wsel = L.k >> 1, hs = (L.k & 1u) * 16u;
  uint32_t op[HALF];
  HSV_UNROLL
  for (int j = 0; j < HALF; ++j) {
    const uint32_t cb = sr[0] & ((1u << CB) - 1u);
    HSV_UNROLL
    for (int i = 0; i < 3; ++i) sr[i] = (sr[i] >> CB) | (sr[i + 1] << (32 - CB));
    sr[3] >>= CB;
    const int32_t dg = (int32_t)cb - (1 << (CB - 1));
    const uint32_t neg = dg < 0, mag = (uint32_t)(neg ? -dg : dg);
    const uint32_t idx = mag == 0u ? 0u : mag - 1u;
    const uint32_t *e = tb + ((uint64_t)(j + (int)h * HALF) * ENT + idx) * kCombEntryWords;
    // row 0: y - x (y + x when negated), row 1: y + x (y - x), row 2: 2dxy (negated), row 3: 2
    const uint32_t coord = L.r == 2u ? 16u : (L.r ^ (neg ? 1u : 0u)) == 0u ? 8u : 0u;
    uint32_t v = L.r == 3u ? 0u : (e[coord + wsel] >> hs) & 0xffffu;
    if (mag == 0u) v = L.r == 2u ? 0u : fl_small(1, L);
    if (L.r == 3u) v = fl_small(2, L);
    if (neg && L.r == 2u && mag != 0u) v = fl_sub(0u, v, L);
    op[j] = v;
  }
  HSV_UNROLL
  for (int j = 0; j < HALF; ++j) q = q_add_op(q, op[j], L);
  return q;
}

}  // namespace hsv
#endif
