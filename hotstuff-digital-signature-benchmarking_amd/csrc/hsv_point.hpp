// Edwards25519 group operations for the verification kernels.
//
// Curve: -x^2 + y^2 = 1 + d x^2 y^2 over GF(2^255-19).
// Representations:
//   ge_ext    (X:Y:Z:T), x = X/Z, y = Y/Z, T = XY/Z           (accumulator)
//   ge_cached (Y+X, Y-X, 2Z, 2dT)                            (variable-base table)
//   ge_niels  (y+x, y-x, 2dxy), affine                       (fixed-base B table)
// Formulas: Hisil-Wong-Carter-Dawson 2008 ("dbl-2008-hwcd", "add-2008-hwcd-3"),
// both complete for a = -1 because d is a non-square, so the identity and
// torsion points need no special cases (no divergence between lanes).
//
// Restated from curve25519-dalek 3.x:
//   CompressedEdwardsY::decompress  -> ge_decompress
//   EdwardsPoint::ct_eq (X1 Z2 == X2 Z1 && Y1 Z2 == Y2 Z1) -> ge_eq_affine
//   EdwardsPoint::is_small_order ([8]P == O) -> y_is_small_order (equivalent:
//   P is in E[8] iff its canonical y is one of the five y values of E[8]).
#pragma once
#include "hsv_field.hpp"

namespace hsv {

struct ge_ext {
  fe X, Y, Z, T;
};
struct ge_cached {
  fe YpX, YmX, Z2, T2d;
};
struct ge_niels {
  fe ypx, ymx, xy2d;
};

HSV_INL ge_ext ge_identity() {
  ge_ext r;
  r.X = fe_small(0);
  r.Y = fe_small(1);
  r.Z = fe_small(1);
  r.T = fe_small(0);
  return r;
}

HSV_INL ge_cached ge_cached_identity() {
  ge_cached r;
  r.YpX = fe_small(1);
  r.YmX = fe_small(1);
  r.Z2 = fe_small(2);
  r.T2d = fe_small(0);
  return r;
}

HSV_INL ge_cached ge_to_cached(const ge_ext &p) {
  ge_cached r;
  r.YpX = fe_add(p.Y, p.X);
  r.YmX = fe_sub(p.Y, p.X);
  r.Z2 = fe_add(p.Z, p.Z);
  r.T2d = fe_mul(p.T, fe_d2());
  return r;
}

// The four output products of every formula below, from E, F, G, H:
//   X3 = E F,  Y3 = G H,  Z3 = G F,  T3 = E H,
// each operand prescaled once (E, G as f; F, H as g) and the products taken
// in interleaved pairs (fe_mul2_p).  Without T, r.T is left holding Z3.
HSV_INL ge_ext ge_finish_rt(const fe &E, const fe &F, const fe &G, const fe &H, bool with_t) {
  const fe_f Ef = fe_prep_f(E), Gf = fe_prep_f(G);
  const fe_g Fg = fe_prep_g(F), Hg = fe_prep_g(H);
  ge_ext r;
  fe_mul2_p(Ef, Fg, Gf, Hg, r.X, r.Y);
  if (with_t) {
    fe_mul2_p(Gf, Fg, Ef, Hg, r.Z, r.T);
  } else {
    r.Z = fe_mul_p(Gf, Fg);
    r.T = r.Z;
  }
  return r;
}

// 2P.  with_t = false skips T3 (saves one multiply when the next op is a doubling).
// Operand classes (hsv_fe26x10.hpp): X, Y, Z in R.  H, C in S2, G in D,
// E = H - S in 4R (used only as the unscaled f operand), F carried to R.
// The four squarings run as two interleaved pairs.
HSV_INL ge_ext ge_dbl_rt(const ge_ext &p, bool with_t) {
  fe A, B, C, S;
  fe_sq2(p.X, p.Y, A, B);
  fe_sq2(p.Z, fe_add(p.X, p.Y), C, S);
  C = fe_add(C, C);
  const fe H = fe_add(A, B);
  const fe E = fe_sub(H, S);
  const fe G = fe_sub(A, B);
  const fe F = fe_carry(fe_add(C, G));
  return ge_finish_rt(E, F, G, H, with_t);
}

template <bool with_t>
HSV_INL ge_ext ge_dbl(const ge_ext &p) {
  ge_ext r = ge_dbl_rt(p, with_t);
  if (!with_t) r.T = fe_small(0);
  return r;
}

// P + Q with Q cached.  P in R; Q.YpX / Q.YmX in S2 / D (swapped when
// negated), Q.Z2 in S2, Q.T2d in R (2R when negated).  E, F in D; G, H in S2.
HSV_INL ge_ext ge_add_cached_rt(const ge_ext &p, const ge_cached &q, bool with_t) {
  fe A, B, C, D;
  fe_mul2(fe_sub(p.Y, p.X), q.YmX, fe_add(p.Y, p.X), q.YpX, A, B);
  fe_mul2(p.T, q.T2d, p.Z, q.Z2, C, D);
  return ge_finish_rt(fe_sub(B, A), fe_sub(D, C), fe_add(D, C), fe_add(B, A), with_t);
}

template <bool with_t>
HSV_INL ge_ext ge_add_cached(const ge_ext &p, const ge_cached &q) {
  ge_ext r = ge_add_cached_rt(p, q, with_t);
  if (!with_t) r.T = fe_small(0);
  return r;
}

// P + Q with Q affine Niels (Z2 = 1).
template <bool with_t>
HSV_INL ge_ext ge_add_niels(const ge_ext &p, const ge_niels &q) {
  fe A, B;
  fe_mul2(fe_sub(p.Y, p.X), q.ymx, fe_add(p.Y, p.X), q.ypx, A, B);
  const fe C = fe_mul(p.T, q.xy2d);
  const fe D = fe_carry(fe_add(p.Z, p.Z));  // minuend and subtrahend below: keep it in R
  ge_ext r = ge_finish_rt(fe_sub(B, A), fe_sub(D, C), fe_add(D, C), fe_add(B, A), with_t);
  if (!with_t) r.T = fe_small(0);
  return r;
}

// -Q for a cached point: swap Y+X / Y-X, negate 2dT.
HSV_INL ge_cached ge_cached_cneg(const ge_cached &q, uint32_t neg) {
  ge_cached r;
  r.YpX = fe_select(q.YpX, q.YmX, neg);
  r.YmX = fe_select(q.YmX, q.YpX, neg);
  r.Z2 = q.Z2;
  r.T2d = fe_select(q.T2d, fe_neg(q.T2d), neg);
  return r;
}

HSV_INL ge_niels ge_niels_cneg(const ge_niels &q, uint32_t neg) {
  ge_niels r;
  r.ypx = fe_select(q.ypx, q.ymx, neg);
  r.ymx = fe_select(q.ymx, q.ypx, neg);
  r.xy2d = fe_select(q.xy2d, fe_neg(q.xy2d), neg);
  return r;
}

// Tail of sqrt_ratio_i once the candidate root r = u v^3 (u v^7)^((p-5)/8)
// is known: fix up by sqrt(-1), pick the non-negative root.
// check = v r^2, computed by the caller (the lane-split R decompression has it
// from its own products)
HSV_INL uint32_t fe_sqrt_ratio_fix_chk(const fe &u, const fe &check, fe r, fe &r_out) {
  fe neg_u = fe_neg(u);
  uint32_t correct = fe_eq(check, u);
  uint32_t flipped = fe_eq(check, neg_u);
  uint32_t flipped_i = fe_eq(check, fe_mul(neg_u, fe_sqrtm1()));
  fe r_prime = fe_mul(r, fe_sqrtm1());
  r = fe_select(r, r_prime, flipped | flipped_i);
  const uint32_t neg = fe_is_negative(r);
  r_out = fe_canon(fe_select(r, fe_neg(r), neg));
  return correct | flipped;
}

HSV_INL uint32_t fe_sqrt_ratio_fix(const fe &u, const fe &v, fe r, fe &r_out) {
  return fe_sqrt_ratio_fix_chk(u, fe_mul(v, fe_sq(r)), r, r_out);
}

// curve25519-dalek FieldElement::sqrt_ratio_i: returns was_nonzero_square
// (true also for u == 0) and the non-negative root r.
HSV_INL uint32_t fe_sqrt_ratio_i(const fe &u, const fe &v, fe &r_out) {
  fe v3 = fe_mul(fe_sq(v), v);
  fe v7 = fe_mul(fe_sq(v3), v);
  fe r = fe_mul(fe_mul(u, v3), fe_pow22523(fe_mul(u, v7)));
  return fe_sqrt_ratio_fix(u, v, r, r_out);
}

// CompressedEdwardsY::decompress.  enc = 32 bytes as 8 little-endian words.
// Returns 1 on success with the affine point (x, y); y keeps the (possibly
// non-canonical) masked input value (class R), x is canonical.
HSV_INL uint32_t ge_decompress(const uint32_t enc[8], fe &x, fe &y) {
  y = fe_from_words_masked(enc);
  fe yy = fe_sq(y);
  fe u = fe_carry(fe_sub(yy, fe_small(1)));  // negated inside sqrt_ratio_i: keep in R
  fe v = fe_add(fe_mul(yy, fe_d()), fe_small(1));
  uint32_t ok = fe_sqrt_ratio_i(u, v, x);
  uint32_t sign = enc[7] >> 31;
  x = fe_canon(fe_select(x, fe_neg(x), sign));  // -0 == 0 is accepted (no rejection)
  return ok;
}

// Two decompressions (R and A of one signature) with their root chains run
// as interleaved pairs (fe_pow22523_2); results as two ge_decompress calls.
HSV_INL void ge_decompress2(const uint32_t ea[8], const uint32_t eb[8], fe &xa, fe &ya, fe &xb, fe &yb,
                            uint32_t &oka, uint32_t &okb) {
  ya = fe_from_words_masked(ea);
  yb = fe_from_words_masked(eb);
  fe yya, yyb;
  fe_sq2(ya, yb, yya, yyb);
  const fe ua = fe_carry(fe_sub(yya, fe_small(1))), ub = fe_carry(fe_sub(yyb, fe_small(1)));
  fe va, vb;
  fe_mul2(yya, fe_d(), yyb, fe_d(), va, vb);
  va = fe_add(va, fe_small(1));
  vb = fe_add(vb, fe_small(1));
  fe sa, sb, v3a, v3b, v7a, v7b;
  fe_sq2(va, vb, sa, sb);
  fe_mul2(sa, va, sb, vb, v3a, v3b);  // v^3
  fe_sq2(v3a, v3b, sa, sb);
  fe_mul2(sa, va, sb, vb, v7a, v7b);  // v^7
  fe wa, wb;
  fe_mul2(ua, v7a, ub, v7b, wa, wb);
  fe pa, pb;
  fe_pow22523_2(wa, wb, pa, pb);
  fe ta, tb;
  fe_mul2(ua, v3a, ub, v3b, ta, tb);
  fe ra, rb;
  fe_mul2(ta, pa, tb, pb, ra, rb);
  oka = fe_sqrt_ratio_fix(ua, va, ra, xa);
  okb = fe_sqrt_ratio_fix(ub, vb, rb, xb);
  xa = fe_canon(fe_select(xa, fe_neg(xa), ea[7] >> 31));
  xb = fe_canon(fe_select(xb, fe_neg(xb), eb[7] >> 31));
}

// [8]P == O  <=>  canonical y in {0, 1, p-1, y8, p-y8}  (the y values of E[8]);
// y_is_small_order_canon takes y already canonical (limbs exact, < p)
HSV_INL uint32_t y_is_small_order_words(const uint32_t c[8]);
HSV_INL uint32_t y_is_small_order(const fe &y) {
  uint32_t c[8];
  fe_pack(y, c);
  return y_is_small_order_words(c);
}
HSV_INL uint32_t y_is_small_order_canon(const fe &y) {
#if HSV_FE_RADIX != 26
  return y_is_small_order(y);
#else
  uint32_t c[8];
  HSV_UNROLL
  for (int j = 0; j < 8; ++j) c[j] = 0;
  HSV_UNROLL
  for (int i = 0; i < 10; ++i) {  // fe_pack without its fe_canon
    const int off = fe26_off(i), wi = off >> 5, sh = off & 31;
    c[wi] |= y.v[i] << sh;
    if (sh + fe26_bits(i) > 32 && wi + 1 < 8) c[wi + 1] |= y.v[i] >> (32 - sh);
  }
  return y_is_small_order_words(c);
#endif
}
HSV_INL uint32_t y_is_small_order_words(const uint32_t c[8]) {
  const uint32_t y8[8] = {0x706a17c7u, 0x4fd84d3du, 0x760b3cbau, 0x0f67100du,
                          0xfa53202au, 0xc6cc392cu, 0x77fdc74eu, 0x7a03ac92u};
  const uint32_t py8[8] = {0x8f95e826u, 0xb027b2c2u, 0x89f4c345u, 0xf098eff2u,
                           0x05acdfd5u, 0x3933c6d3u, 0x880238b1u, 0x05fc536du};
  uint32_t hi = 0;  // OR of words 1..7
  HSV_UNROLL
  for (int i = 1; i < 8; ++i) hi |= c[i];
  const uint32_t is0 = (hi == 0) & (c[0] == 0u);
  const uint32_t is1 = (hi == 0) & (c[0] == 1u);
  uint32_t pm1 = (c[0] == 0xffffffecu) & (c[7] == 0x7fffffffu);
  uint32_t e8 = 1u, ep8 = 1u;
  HSV_UNROLL
  for (int i = 0; i < 8; ++i) {
    if (i >= 1 && i <= 6) pm1 &= (c[i] == 0xffffffffu);
    e8 &= (c[i] == y8[i]);
    ep8 &= (c[i] == py8[i]);
  }
  return is0 | is1 | pm1 | e8 | ep8;
}

// Projective point == affine point (x, y): X == x Z and Y == y Z, with Z != 0.
// No point has Z == 0; a (0 : 0 : 0 : 0) accumulator only comes from zeroed
// table memory and would satisfy both equations, so it fails closed here.
#ifdef HSV_NEUTRAL_NO_Z_CHECK  // A/B diagnosis builds only: the round-2 checks without Z != 0
#define HSV_Z_NONZERO(z) 1u
#else
#define HSV_Z_NONZERO(z) (fe_is_zero(z) ^ 1u)
#endif
HSV_INL uint32_t ge_eq_affine(const ge_ext &p, const fe &x, const fe &y) {
  return fe_eq(p.X, fe_mul(x, p.Z)) & fe_eq(p.Y, fe_mul(y, p.Z)) & HSV_Z_NONZERO(p.Z);
}

// Q == O: X == 0 and Y == Z != 0 (same fail-closed rule as ge_eq_affine).
HSV_INL uint32_t ge_is_neutral(const ge_ext &q) { return fe_is_zero(q.X) & fe_eq(q.Y, q.Z) & HSV_Z_NONZERO(q.Z); }

// Device self-check of a final accumulator: 1 iff (X : Y : Z) is a point of
// the curve, (Y^2 - X^2) Z^2 == Z^4 + d X^2 Y^2 with Z != 0 (T not needed).
// Every formula above is exact and complete, so sums and multiples of curve
// points are curve points: a final Q that fails this was computed from
// something other than what the kernel wrote or was given (table memory,
// workspace, comb tables or registers corrupted).  All-zero entries give
// (0 : 0 : 0 : 0), which satisfies the equation but not Z != 0; a garbage
// entry gives an off-curve sum.  7 field operations per verification.
HSV_INL uint32_t ge_is_sane(const ge_ext &p) {
  fe xx, yy, zz, lhs, xy, z4, dxy;
  fe_sq2(p.X, p.Y, xx, yy);
  zz = fe_sq(p.Z);
  fe_mul2(fe_sub(yy, xx), zz, xx, yy, lhs, xy);
  fe_mul2(zz, zz, xy, fe_d(), z4, dxy);
  return fe_eq(lhs, fe_add(z4, dxy)) & (fe_is_zero(p.Z) ^ 1u);
}

// Compress (x, y) = (X/Z, Y/Z) -> 32 bytes as 8 words (host-side signing).
HSV_INL void ge_compress(const ge_ext &p, uint32_t out[8]) {
  const fe zi = fe_invert(p.Z);
  const uint32_t xneg = fe_is_negative(fe_mul(p.X, zi));
  fe_pack(fe_mul(p.Y, zi), out);
  out[7] |= xneg << 31;
}

}  // namespace hsv
