// Half-size scalars for the verification equation (lattice reduction in
// dimension 2; cf. Pornin, "Optimized lattice basis reduction in dimension 2,
// and fast Schnorr and EdDSA signature verification", 2020), adapted so the
// result is EXACTLY dalek's cofactorless check, torsion included.
//
// The Ed25519 group E(F_p) is cyclic of order N = 8l.  For the challenge k we
// find (c0, c1) in the lattice  { (x, y) : x == y k (mod N) }  with c1 odd and
// |c0|, |c1| around 2^128.  Then [c1] is a bijection of E (gcd(c1, 8l) = 1:
// c1 odd, 0 < c1 < l) and [x]P depends only on x mod N, so
//    e = [s]B - R - [k]A = O   <=>   [c1]e = [(c1 s) mod l]B - [c1]R - [c0]A = O.
// The right-hand side needs ~135 doublings instead of ~252.
//
// Reduction: Euclid on (N, k) with cofactors t (r == t k mod N, exact integer
// arithmetic; quotients estimated in double precision and never over-
// estimated, so every step is an exact unimodular update).  It stops at the
// first remainder below 2^128, where |t| <= N / 2^128 < 2^128.  If that t is
// even, the odd partner is the previous vector reduced against it (one
// Gauss step).  Vectors longer than max_bits are reported as !ok and the
// caller falls back to the full-length path (probability ~2^-13.5 per lane at
// 133 bits, ~2^-22.6 at the comb path's 138).
#pragma once
#include <math.h>

#include "hsv_scalar.hpp"

namespace hsv {

constexpr int kLatMaxBits = 133;  // |c0|, |c1| < 2^133 (recoding over 135 bits needs < 2^133.78)
// Bound of the comb-path kernels (hsv_verify_hc.hpp: 35 windows of 4 bits,
// c + C < 2^140 for c < 2^138.9).  A pair with max(|c0|, |c1|) >= 2^138 needs
// a shortest vector below ~2^117 with an even cofactor: about 2^-22.6 of the
// challenges, against ~2^-13.5 at 133 bits, so a 2^20 batch almost never holds
// a full-length item (each one costs its SIMD a second batch of work at the
// end of the persistent grid).
constexpr int kLatCombBits = 138;

struct LatOut {
  uint32_t c0[5];  // |c0|, little-endian
  uint32_t c1[5];  // c1 > 0, odd
  uint32_t c0_neg; // c0 < 0
  uint32_t ok;
};

#if defined(__HIP_DEVICE_COMPILE__)
HSV_INL bool hsv_any(bool p) { return __any(p); }
#else
HSV_INL bool hsv_any(bool p) { return p; }
#endif

// value of an N-limb unsigned integer as a double (top 96 bits, then rounded)
template <int N>
HSV_INL double mp_to_double(const uint32_t x[N]) {
  uint32_t a = 0, b = 0, c = 0;
  int h = 0;
  HSV_UNROLL
  for (int i = 0; i < N; ++i) {
    if (x[i] != 0) {
      h = i;
      a = x[i];
      b = i >= 1 ? x[i - 1] : 0u;
      c = i >= 2 ? x[i - 2] : 0u;
    }
  }
  const double d = ((double)a * 4294967296.0 + (double)b) * 4294967296.0 + (double)c;
  return ldexp(d, 32 * (h - 2));
}

// signed two's-complement N-limb value as a double
template <int N>
HSV_INL double mps_to_double(const uint32_t x[N]) {
  const bool neg = (x[N - 1] >> 31) != 0;
  uint32_t m[N];
  uint64_t c = 1;
  HSV_UNROLL
  for (int i = 0; i < N; ++i) {
    c += (uint64_t)(uint32_t)~x[i];
    m[i] = neg ? (uint32_t)c : x[i];
    c >>= 32;
  }
  const double d = mp_to_double<N>(m);
  return neg ? -d : d;
}

// r = a - q*b  (q < 2^64), N limbs, modulo 2^(32N)
template <int N>
HSV_INL void mp_sub_mulq(uint32_t r[N], const uint32_t a[N], const uint32_t b[N], uint64_t q) {
  const uint32_t ql = (uint32_t)q, qh = (uint32_t)(q >> 32);
  uint32_t p[N];
  uint64_t c = 0;
  HSV_UNROLL
  for (int i = 0; i < N; ++i) {
    c = (uint64_t)b[i] * ql + (c >> 32);
    p[i] = (uint32_t)c;
  }
  c = 0;
  HSV_UNROLL
  for (int i = 1; i < N; ++i) {
    c = (uint64_t)b[i - 1] * qh + p[i] + (c >> 32);
    p[i] = (uint32_t)c;
  }
  int64_t t = 0;
  HSV_UNROLL
  for (int i = 0; i < N; ++i) {
    t += (int64_t)a[i] - (int64_t)p[i];
    r[i] = (uint32_t)t;
    t >>= 32;
  }
}

// a < b (unsigned)
template <int N>
HSV_INL bool mp_lt(const uint32_t a[N], const uint32_t b[N]) {
  int64_t t = 0;
  HSV_UNROLL
  for (int i = 0; i < N; ++i) {
    t += (int64_t)a[i] - (int64_t)b[i];
    t >>= 32;
  }
  return t != 0;
}

// |x| < 2^bits for a signed two's-complement N-limb value; writes |x| to mag (5 limbs)
template <int N>
HSV_INL bool mps_abs_fits(const uint32_t x[N], int bits, uint32_t mag[5], uint32_t &neg) {
  neg = x[N - 1] >> 31;
  uint32_t m[N];
  uint64_t c = 1;
  HSV_UNROLL
  for (int i = 0; i < N; ++i) {
    c += (uint64_t)(uint32_t)~x[i];
    m[i] = neg ? (uint32_t)c : x[i];
    c >>= 32;
  }
  bool fits = true;
  HSV_UNROLL
  for (int i = 0; i < N; ++i) {
    const int lo = 32 * i;
    if (lo >= bits) fits = fits && (m[i] == 0);
    else if (lo + 32 > bits) fits = fits && ((m[i] >> (bits - lo)) == 0);
  }
  HSV_UNROLL
  for (int i = 0; i < 5; ++i) mag[i] = i < N ? m[i] : 0u;
  return fits;
}


// One (possibly partial) Euclid step on the full numbers: q = an under-
// estimate of floor(a / b) (never over: the quotient comes from doubles and is
// scaled down by 1 - 2^-40), r = a - q b; (a, b) <- (b, r) when r < b, else
// a <- r (the next step continues the division).  Cofactors follow.
HSV_INL void lat_exact_step(uint32_t a[8], uint32_t b[8], uint32_t ta[6], uint32_t tb[6], bool active) {
  const double qd = mp_to_double<8>(a) / mp_to_double<8>(b);
  double qf = floor(qd * (1.0 - 0x1p-40));
  qf = qf < 1.0 ? 1.0 : (qf > 0x1p50 ? 0x1p50 : qf);
  const uint64_t q = active ? (uint64_t)qf : 0u;
  uint32_t r[8], tr[6];
  mp_sub_mulq<8>(r, a, b, q);
  mp_sub_mulq<6>(tr, ta, tb, q);
  const bool swap = active && mp_lt<8>(r, b);
  HSV_UNROLL
  for (int i = 0; i < 8; ++i) {
    const uint32_t nb = swap ? r[i] : b[i];
    a[i] = swap ? b[i] : (active ? r[i] : a[i]);
    b[i] = nb;
  }
  HSV_UNROLL
  for (int i = 0; i < 6; ++i) {
    const uint32_t ntb = swap ? tr[i] : tb[i];
    ta[i] = swap ? tb[i] : (active ? tr[i] : ta[i]);
    tb[i] = ntb;
  }
}

// Euclid until b < 2^128, one exact step per iteration (reference form).
HSV_INL void lat_euclid_to_128(uint32_t a[8], uint32_t b[8], uint32_t ta[6], uint32_t tb[6]) {
  HSV_NOUNROLL
  for (int it = 0; it < 512; ++it) {
    const bool active = (b[4] | b[5] | b[6] | b[7]) != 0;
    if (!hsv_any(active)) break;
    lat_exact_step(a, b, ta, tb, active);
  }
}

// out = s * (|A| x - |B| y)  mod 2^(32N), s = -1 when A < 0 (or A == 0 < B),
// else +1.
// |A|, |B| < 2^31; x, y as N little-endian limbs (two's complement for the
// cofactors).  For a Euclid cofactor matrix A and B have opposite signs (or
// one is 0), so A x + B y = s (|A| x - |B| y).
template <int N>
HSV_INL void lat_combine(uint32_t out[N], const uint32_t x[N], const uint32_t y[N], int64_t A, int64_t B) {
  const uint32_t ma = (uint32_t)(A < 0 ? -A : A), mb = (uint32_t)(B < 0 ? -B : B);
  int64_t c = 0;
  HSV_UNROLL
  for (int i = 0; i < N; ++i) {
    const int64_t t = (int64_t)((uint64_t)ma * x[i]) - (int64_t)((uint64_t)mb * y[i]) + c;
    out[i] = (uint32_t)t;
    c = t >> 32;
  }
  if (A < 0 || (A == 0 && B > 0)) {
    uint64_t cc = 1;
    HSV_UNROLL
    for (int i = 0; i < N; ++i) {
      cc += (uint64_t)(uint32_t)~out[i];
      out[i] = (uint32_t)cc;
      cc >>= 32;
    }
  }
}

// floor(n / d) estimate for integers 0 <= n < 2^53, 1 <= d < 2^53 held in
// doubles: hardware reciprocal, then one exact remainder correction.  The
// caller's step conditions reject any step whose quotient is not the true one,
// so an estimate that is still off only ends the single-precision run early.
HSV_INL double lat_floor_div(double n, double d) {
#if defined(__HIP_DEVICE_COMPILE__)
  double q = floor(n * __builtin_amdgcn_rcp(d));
#elif defined(HSV_LAT_HOST_RCP_ERR)  // host tests only: a reciprocal off by a relative error
  double q = floor(n * ((1.0 / d) * (1.0 + HSV_LAT_HOST_RCP_ERR)));
#else
  double q = floor(n / d);
#endif
  const double r = fma(-q, d, n);
  q += (r >= d) ? 1.0 : (r < 0.0 ? -1.0 : 0.0);
  return q;
}

// bits [s, s + 52) of an 8-limb number, as an exact double (0 <= s <= 204)
HSV_INL double lat_digits52(const uint32_t x[8], int s) {
  const int w = s >> 5, sh = s & 31;
  uint32_t l0 = 0, l1 = 0, l2 = 0;
  HSV_UNROLL
  for (int i = 0; i < 8; ++i) {
    l0 = (i == w) ? x[i] : l0;
    l1 = (i == w + 1) ? x[i] : l1;
    l2 = (i == w + 2) ? x[i] : l2;
  }
  uint64_t v = (((uint64_t)l1 << 32) | l0) >> sh;
  if (sh) v |= (uint64_t)l2 << (64 - sh);
  return (double)(v & ((1ull << 52) - 1));
}

HSV_INL int lat_bitlen8(const uint32_t x[8]) {
  int h = 0;
  HSV_UNROLL
  for (int i = 0; i < 8; ++i)
    if (x[i] != 0) h = 32 * i + 32 - __builtin_clz(x[i]);
  return h;
}

// Lehmer's algorithm (Knuth 4.5.2, Algorithm L) on 52-bit leading digits held
// in doubles, stopping exactly at the first remainder below 2^128 like
// lat_euclid_to_128.  Each round runs single-precision Euclid steps on the
// leading digits while the two quotient bounds agree, the cofactors stay
// below 2^31 and the new remainder is provably >= 2^128, then applies the
// 2x2 cofactor matrix to (a, b) and (ta, tb); a round that can take no step
// takes one exact full-precision step instead.  All lanes of a wave iterate
// together; finished lanes are masked.
HSV_INL void lat_lehmer_to_128(uint32_t a[8], uint32_t b[8], uint32_t ta[6], uint32_t tb[6]) {
  HSV_NOUNROLL
  for (int round = 0; round < 256; ++round) {
    const bool active = (b[4] | b[5] | b[6] | b[7]) != 0;
    if (!hsv_any(active)) break;
    const int h = lat_bitlen8(a);
    const int s = active ? h - 52 : 0;  // h >= 129 while active
    double x = lat_digits52(a, s), y = lat_digits52(b, s);
    const double thr = ldexp(1.0, 128 - s);
    double A = 1.0, B = 0.0, C = 0.0, D = 1.0;
    bool go = active;
    HSV_NOUNROLL
    for (int j = 0; j < 64; ++j) {
      if (!hsv_any(go)) break;
      // The true current pair is r0 = x + A al + B be, r1 = y + C al + D be
      // (al, be in [0, 1): the digits cut off below 2^s); row entries have
      // opposite signs, so over the box r2 = ny + nC al + nD be is smallest
      // near ny + min(nC, nD) and r1 - r2 near (y - ny) + min(C - nC, D - nD).
      // q is the true quotient iff 0 <= r2 < r1 for every (al, be): checked
      // below, together with r2 >= 2^128 (never step past the first remainder
      // under 2^128).  One division per step.
      bool ok = go && y >= 1.0;
      const double q = ok ? lat_floor_div(x, y) : 0.0;
      const double nC = fma(-q, C, A), nD = fma(-q, D, B), ny = fma(-q, y, x);
      ok = ok && q >= 1.0 && q < 0x1p30 && fabs(nC) < 0x1p31 && fabs(nD) < 0x1p31 &&
           ny + fmin(nC, nD) >= thr && (y - ny) + fmin(C - nC, D - nD) >= 1.0;
      if (ok) {
        A = C; B = D; C = nC; D = nD;
        x = y; y = ny;
      }
      go = ok;
    }
    const bool matrix = active && B != 0.0;
    if (hsv_any(matrix)) {
      uint32_t na[8], nb[8], nta[6], ntb[6];
      const int64_t iA = (int64_t)A, iB = (int64_t)B, iC = (int64_t)C, iD = (int64_t)D;
      lat_combine<8>(na, a, b, iA, iB);
      lat_combine<8>(nb, a, b, iC, iD);
      lat_combine<6>(nta, ta, tb, iA, iB);
      lat_combine<6>(ntb, ta, tb, iC, iD);
      HSV_UNROLL
      for (int i = 0; i < 8; ++i) {
        a[i] = matrix ? na[i] : a[i];
        b[i] = matrix ? nb[i] : b[i];
      }
      HSV_UNROLL
      for (int i = 0; i < 6; ++i) {
        ta[i] = matrix ? nta[i] : ta[i];
        tb[i] = matrix ? ntb[i] : tb[i];
      }
    }
    const bool exact = active && B == 0.0;
    if (hsv_any(exact)) lat_exact_step(a, b, ta, tb, exact);
  }
}

// ---- lean Lehmer (default since round 2) -----------------------------------
// The same Euclid sequence as lat_lehmer_to_128, in a form with a small outer
// round.  Two facts of the Euclid cofactor sequence make it sign-free:
//  - remainders are >= 0 and the 2x2 matrix rows have entries of opposite
//    signs, so  A a + B b = | |A| a - |B| b |  (one product chain each side,
//    the sign of the difference picks the orientation);
//  - the cofactors t alternate in sign, so  A ta + B tb  adds two terms of the
//    same sign:  |ta'| = |A| |ta| + |B| |tb|.
// The cofactors are kept as magnitudes below 2^128 (|t| <= N / a and a >= 2^128
// while a lane is active: 4 limbs) with `par` = 1 when tb < 0 (ta has the
// other sign); the signed form is rebuilt once at the end.  A lane that is not
// active keeps the identity matrix, so the update needs no selects.
// The inner loop also takes the step that crosses 2^128 when its quotient is
// provably exact, and stops after it, so the last division of a lane needs no
// full-precision step.

// out = | m1 x - m2 y |  (x, y 8 limbs, m1, m2 < 2^31, the result < 2^256)
HSV_INL void lat_absdiff8(uint32_t out[8], const uint32_t x[8], const uint32_t y[8], uint32_t m1, uint32_t m2) {
  uint32_t p[9], q[9];
  uint64_t c = 0, e = 0;
  HSV_UNROLL
  for (int i = 0; i < 8; ++i) {
    c = (uint64_t)x[i] * m1 + (c >> 32);
    e = (uint64_t)y[i] * m2 + (e >> 32);
    p[i] = (uint32_t)c;
    q[i] = (uint32_t)e;
  }
  p[8] = (uint32_t)(c >> 32);
  q[8] = (uint32_t)(e >> 32);
  uint32_t d[8];
  uint32_t br = 0;
  HSV_UNROLL
  for (int i = 0; i < 9; ++i) {
    const uint64_t t = (uint64_t)p[i] - q[i] - br;
    if (i < 8) d[i] = (uint32_t)t;
    br = (uint32_t)(t >> 63);
  }
  const uint32_t m = 0u - br;  // all ones when m1 x < m2 y
  uint64_t cc = br;
  HSV_UNROLL
  for (int i = 0; i < 8; ++i) {
    cc += (uint64_t)(d[i] ^ m);
    out[i] = (uint32_t)cc;
    cc >>= 32;
  }
}

// out = m1 x + m2 y  (4 limbs, modulo 2^128; m1, m2 < 2^31)
HSV_INL void lat_addmul4(uint32_t out[4], const uint32_t x[4], const uint32_t y[4], uint32_t m1, uint32_t m2) {
  uint64_t c = 0, e = 0;
  HSV_UNROLL
  for (int i = 0; i < 4; ++i) {
    c = (uint64_t)x[i] * m1 + (c >> 32);
    e = (uint64_t)y[i] * m2 + (uint32_t)c + (e >> 32);
    out[i] = (uint32_t)e;
  }
}

// One exact (possibly partial) division step on lanes with `on`, magnitudes
// form of lat_exact_step:  q <= floor(a / b),  r = a - q b,  |t| = |ta| + q |tb|;
// (a, b) <- (b, r) and par flips when r < b, else a <- r.
HSV_INL void lat_exact_step_mag(uint32_t a[8], uint32_t b[8], uint32_t ua[4], uint32_t ub[4], uint32_t &par,
                                bool on) {
  const double qd = mp_to_double<8>(a) / mp_to_double<8>(b);
  double qf = floor(qd * (1.0 - 0x1p-40));
  qf = qf < 1.0 ? 1.0 : (qf > 0x1p50 ? 0x1p50 : qf);
  const uint64_t q = on ? (uint64_t)qf : 0u;
  uint32_t r[8], t[4];
  mp_sub_mulq<8>(r, a, b, q);
  {
    const uint32_t ql = (uint32_t)q, qh = (uint32_t)(q >> 32);
    uint64_t c = 0, e = 0;
    HSV_UNROLL
    for (int i = 0; i < 4; ++i) {
      c = (uint64_t)ub[i] * ql + ua[i] + (c >> 32);
      const uint32_t lo = (uint32_t)c;
      e = (i >= 1 ? (uint64_t)ub[i - 1] * qh : 0u) + lo + (e >> 32);
      t[i] = (uint32_t)e;
    }
  }
  const bool swap = on && mp_lt<8>(r, b);
  HSV_UNROLL
  for (int i = 0; i < 8; ++i) {
    const uint32_t nb = swap ? r[i] : b[i];
    a[i] = swap ? b[i] : (on ? r[i] : a[i]);
    b[i] = nb;
  }
  HSV_UNROLL
  for (int i = 0; i < 4; ++i) {
    const uint32_t nub = swap ? t[i] : ub[i];
    ua[i] = swap ? ub[i] : (on ? t[i] : ua[i]);
    ub[i] = nub;
  }
  par ^= swap ? 1u : 0u;
}

HSV_INL void lat_lehmer_lean_to_128(uint32_t a[8], uint32_t b[8], uint32_t ta[6], uint32_t tb[6]) {
  uint32_t ua[4] = {0u, 0u, 0u, 0u}, ub[4] = {1u, 0u, 0u, 0u}, par = 0;
  HSV_NOUNROLL
  for (int round = 0; round < 256; ++round) {
    const bool active = (b[4] | b[5] | b[6] | b[7]) != 0;
    if (!hsv_any(active)) break;
    const int h = lat_bitlen8(a);
    const int s = active ? h - 52 : 0;  // h >= 129 while active
    double x = lat_digits52(a, s), y = lat_digits52(b, s);
    const double thr = ldexp(1.0, 128 - s);
    double A = 1.0, B = 0.0, C = 0.0, D = 1.0;
    bool go = active;
    // At most kLatRoundSteps steps per round: a lane that could go on resumes
    // in the next round (any prefix of exact steps is a valid state).  Rounds
    // are wave-synchronous, so the inner loop runs the wave's longest round;
    // the cap trims that tail (121 -> 99 inner iterations per wave in a
    // Python simulation of this loop over random challenges, rounds unchanged
    // at 6.1).
    constexpr int kLatRoundSteps = 17;
    HSV_NOUNROLL
    for (int j = 0; j < kLatRoundSteps; ++j) {
      if (!hsv_any(go)) break;
      // true pair: r0 = x + A al + B be, r1 = y + C al + D be, al, be in [0, 1)
      // (lat_lehmer_to_128); q is exact iff 0 <= r2 < r1 over the box.  The
      // step is taken when q is exact; the round goes on only while r2 is
      // provably >= 2^128.  |nD| < 2^31 also bounds q and |nC|: in a Euclid
      // cofactor matrix |D| >= |C| and |D| >= 1, so |nD| >= |nC| and |nD| >= q.
      bool ok = go && y >= 1.0;
      const double q = ok ? lat_floor_div(x, y) : 0.0;
      const double nC = fma(-q, C, A), nD = fma(-q, D, B), ny = fma(-q, y, x);
      const double lo = ny + fmin(nC, nD);
      ok = ok && q >= 1.0 && fabs(nD) < 0x1p31 && lo >= 0.0 && (y - ny) + fmin(C - nC, D - nD) >= 1.0;
      if (ok) {
        A = C; B = D; C = nC; D = nD;
        x = y; y = ny;
      }
      go = ok && lo >= thr;
    }
    {  // identity on lanes that took no step
      const uint32_t mA = (uint32_t)fabs(A), mB = (uint32_t)fabs(B), mC = (uint32_t)fabs(C), mD = (uint32_t)fabs(D);
      uint32_t na[8], nb[8], nua[4], nub[4];
      lat_absdiff8(na, a, b, mA, mB);
      lat_absdiff8(nb, a, b, mC, mD);
      lat_addmul4(nua, ua, ub, mA, mB);
      lat_addmul4(nub, ua, ub, mC, mD);
      HSV_UNROLL
      for (int i = 0; i < 8; ++i) {
        a[i] = na[i];
        b[i] = nb[i];
      }
      HSV_UNROLL
      for (int i = 0; i < 4; ++i) {
        ua[i] = nua[i];
        ub[i] = nub[i];
      }
      par ^= D < 0.0 ? 1u : 0u;  // sign(D) = (-1)^(steps taken)
    }
    const bool exact = active && B == 0.0;
    if (hsv_any(exact)) lat_exact_step_mag(a, b, ua, ub, par, exact);
  }
  // signed cofactors: tb = (-1)^par |tb|, ta = -(-1)^par |ta|
  const uint32_t ma = par ? 0u : ~0u, mb = par ? ~0u : 0u;
  uint64_t ca = ma & 1u, cb = mb & 1u;
  HSV_UNROLL
  for (int i = 0; i < 6; ++i) {
    ca += (uint64_t)((i < 4 ? ua[i] : 0u) ^ ma);
    cb += (uint64_t)((i < 4 ? ub[i] : 0u) ^ mb);
    ta[i] = (uint32_t)ca;
    tb[i] = (uint32_t)cb;
    ca >>= 32;
    cb >>= 32;
  }
}

// c0s == c1 k (mod 8l), c0s = (c0_neg ? -c0 : c0)?  Checked as
// F = c1 k - c0s + 8l * 2^140 (>= 0):  F == 0 mod 8  and  F == 0 mod l.
// The reduction maintains the congruence by construction; this check makes
// a wrong pair cost only the full-length path, never a wrong flag.
HSV_INL bool lat_congruent(const sc &k, const LatOut &o) {
  uint32_t f[16];
  HSV_UNROLL
  for (int i = 0; i < 16; ++i) f[i] = 0;
  HSV_UNROLL
  for (int i = 0; i < 5; ++i) {  // c1 * k
    uint64_t c = 0;
    HSV_UNROLL
    for (int j = 0; j < 8; ++j) {
      c = (uint64_t)o.c1[i] * k.v[j] + f[i + j] + (c >> 32);
      f[i + j] = (uint32_t)c;
    }
    f[i + 8] = (uint32_t)(c >> 32);
  }
  {  // + 8l * 2^140 = l << 143: limbs 4.. of (l << 15)
    uint32_t l[8];
    sc_l(l);
    uint64_t c = 0;
    HSV_UNROLL
    for (int i = 0; i < 9; ++i) {
      const uint32_t li = (i < 8 ? (l[i] << 15) : 0u) | (i >= 1 ? (l[i - 1] >> 17) : 0u);
      c += (uint64_t)f[4 + i] + li;
      f[4 + i] = (uint32_t)c;
      c >>= 32;
    }
    HSV_UNROLL
    for (int i = 13; i < 16; ++i) {
      c += f[i];
      f[i] = (uint32_t)c;
      c >>= 32;
    }
  }
  {  // -/+ c0
    int64_t c = 0;
    HSV_UNROLL
    for (int i = 0; i < 16; ++i) {
      const int64_t ci = i < 5 ? (int64_t)o.c0[i] : 0;
      c += (int64_t)f[i] + (o.c0_neg ? ci : -ci);
      f[i] = (uint32_t)c;
      c >>= 32;
    }
  }
  const sc r = sc_reduce512(f);
  uint32_t nz = f[0] & 7u;
  HSV_UNROLL
  for (int i = 0; i < 8; ++i) nz |= r.v[i];
  return nz == 0;
}

// max_bits: the largest accepted bit length of |c0| and |c1| (<= 159).
HSV_INL LatOut lattice_reduce(const sc &k, int max_bits = kLatMaxBits) {
#ifdef HSV_TIMING_STUB_LATTICE  // tools/phase_probe.py only: wrong results, timing share of the reduction
  {
    LatOut o;
    for (int i = 0; i < 5; ++i) { o.c0[i] = i < 4 ? k.v[i] : 0u; o.c1[i] = i < 4 ? k.v[4 + i] : 0u; }
    o.c1[0] |= 1u;
    o.c0_neg = 0;
    o.ok = 1;
    return o;
  }
#endif
  // a = N = 8l, ta = 0;  b = k, tb = 1.   Invariant: a == ta*k, b == tb*k (mod N)
  uint32_t a[8], b[8], ta[6], tb[6];
  {
    uint32_t l[8];
    sc_l(l);
    uint32_t c = 0;
    HSV_UNROLL
    for (int i = 0; i < 8; ++i) {
      a[i] = (l[i] << 3) | c;
      c = l[i] >> 29;
      b[i] = k.v[i];
    }
  }
  HSV_UNROLL
  for (int i = 0; i < 6; ++i) {
    ta[i] = 0;
    tb[i] = i == 0 ? 1u : 0u;
  }
#if defined(HSV_LATTICE_LEHMER1)  // round-1 Lehmer form (the host cross-check)
  lat_lehmer_to_128(a, b, ta, tb);
#else
  lat_lehmer_lean_to_128(a, b, ta, tb);
#endif
  LatOut o;
  o.ok = 0;
  o.c0_neg = 0;
  // candidate 1: (b, tb) when tb is odd:  c0 = b, c1 = tb
  // candidate 2: (a, ta) - qv (b, tb), qv = round(<v,u>/<u,u>)  (ta odd when tb even)
  const bool tb_odd = (tb[0] & 1u) != 0;
  uint32_t c0[9], c1[6];
  {
    const double db = mp_to_double<8>(b), da = mp_to_double<8>(a);
    const double dtb = mps_to_double<6>(tb), dta = mps_to_double<6>(ta);
    const double den = db * db + dtb * dtb;
    double qv = den > 0.0 ? rint((da * db + dta * dtb) / den) : 0.0;
    const bool qv_ok = qv >= -0x1p50 && qv <= 0x1p50;
    qv = qv_ok ? qv : 0.0;
    // v - qv*u with qv >= 0, or v - |qv|*(-u) with qv < 0 (two's complement)
    const bool qneg = qv < 0.0;
    const uint64_t q = (uint64_t)(qneg ? -qv : qv);
    uint32_t a9[9], b9[9], r9[9], tr[6], tbn[6];
    {
      uint64_t cb = 1, ct = 1;
      HSV_UNROLL
      for (int i = 0; i < 9; ++i) {
        a9[i] = i < 8 ? a[i] : 0u;
        const uint32_t bi = i < 8 ? b[i] : 0u;
        cb += (uint64_t)(uint32_t)~bi;
        b9[i] = qneg ? (uint32_t)cb : bi;
        cb >>= 32;
      }
      HSV_UNROLL
      for (int i = 0; i < 6; ++i) {
        ct += (uint64_t)(uint32_t)~tb[i];
        tbn[i] = qneg ? (uint32_t)ct : tb[i];
        ct >>= 32;
      }
    }
    mp_sub_mulq<9>(r9, a9, b9, q);
    mp_sub_mulq<6>(tr, ta, tbn, q);
    if (qneg) {  // candidate 1 needs the un-negated u
      uint64_t cb = 1;
      HSV_UNROLL
      for (int i = 0; i < 9; ++i) {
        cb += (uint64_t)(uint32_t)~b9[i];
        b9[i] = (uint32_t)cb;
        cb >>= 32;
      }
    }
    HSV_UNROLL
    for (int i = 0; i < 9; ++i) c0[i] = tb_odd ? b9[i] : r9[i];
    HSV_UNROLL
    for (int i = 0; i < 6; ++i) c1[i] = tb_odd ? tb[i] : tr[i];
    if (!tb_odd && !qv_ok) c1[0] &= ~1u;  // force the "not ok" path below (even c1)
  }
  // normalise c1 > 0 (negate the whole vector), then bound-check
  uint32_t n1;
  uint32_t c1mag[5], c0mag[5];
  const bool f1 = mps_abs_fits<6>(c1, max_bits, c1mag, n1);
  uint32_t n0;
  const bool f0 = mps_abs_fits<9>(c0, max_bits, c0mag, n0);
  const bool odd = (c1[0] & 1u) != 0;
  bool nz = false;
  HSV_UNROLL
  for (int i = 0; i < 5; ++i) nz = nz || (c1mag[i] != 0);
  o.ok = (f0 && f1 && odd && nz) ? 1u : 0u;
  o.c0_neg = n0 ^ n1;  // sign of c0 after making c1 positive
  HSV_UNROLL
  for (int i = 0; i < 5; ++i) {
    o.c0[i] = c0mag[i];
    o.c1[i] = c1mag[i];
  }
  o.ok = (o.ok && lat_congruent(k, o)) ? 1u : 0u;
  return o;
}

// (c1 * s) mod l for c1 < 2^160 (5 limbs) and s < 2^256
HSV_INL sc sc_mul_small(const uint32_t c1[5], const uint32_t s[8]) {
  uint32_t t[16];
  HSV_UNROLL
  for (int i = 0; i < 16; ++i) t[i] = 0;
  HSV_UNROLL
  for (int i = 0; i < 5; ++i) {
    uint64_t c = 0;
    HSV_UNROLL
    for (int j = 0; j < 8; ++j) {
      c = (uint64_t)c1[i] * s[j] + t[i + j] + (c >> 32);
      t[i + j] = (uint32_t)c;
    }
    t[i + 8] = (uint32_t)(c >> 32);
  }
  return sc_reduce512(t);
}

}  // namespace hsv
