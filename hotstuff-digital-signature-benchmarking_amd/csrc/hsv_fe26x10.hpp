// GF(2^255 - 19), representation B: 10 limbs in radix 2^25.5.
//
// Limb i holds bits [off(i), off(i) + bits(i)) with bits = 26, 25, 26, 25, ...
// and off = 0, 26, 51, 77, 102, 128, 153, 179, 204, 230 (25.5 * 10 = 255).
//
// Multiplication: column k of f*g is  sum_i f_i * G(k-i)  where the partner
// limb is pre-scaled so the mod-p fold happens inside the product:
//   * 19 when i + j >= 10   (2^255 == 19),
//   * 2  when i and j are both odd (off(i) + off(j) = off(i+j) + 1).
// Each column is a chain of 10 v_mad_u64_u32 accumulating in place into a
// 64-bit register pair -- no carries inside the product, no extra adds.  One
// carry chain per multiply (ref10 order, two interleaved chains) normalises
// the 10 column sums.  Squaring uses the 55 distinct products.
//
// Operand classes (limb-wise upper bounds, R = 2^26 for even limbs / 2^25 for
// odd limbs):
//   R   output of mul / sq / carry / canon / from_words   (<= 1.004 R)
//   S2  fe_add(R, R)                                      (<= 2.01 R)
//   D   fe_sub(R-or-S2 minuend, R subtrahend) = a + 2p - b (<= 3.01 R, 4.01 R for an S2 minuend)
// Rules (checked on the host with -DHSV_CHECK_BOUNDS):
//   fe_sub(a, b)  b must be <= 2p limb-wise (class R)
//   fe_mul(f, g)  g <= 3.368 R (19*g must fit 32 bits); column sums < 2^64,
//                 which holds whenever class(f) * class(g) < 32
//   fe_sq(f)      f <= 3.368 R
//   fe_carry(x)   any x with limbs < 2^31 -> class R
// Included by hsv_field.hpp when HSV_FE_RADIX == 26 (the default).
#pragma once

#if defined(HSV_CHECK_BOUNDS) && !defined(__HIP_DEVICE_COMPILE__)
#include <cstdio>
#include <cstdlib>
#define HSV_BOUND(cond, what)                                           \
  do {                                                                  \
    if (!(cond)) {                                                      \
      std::fprintf(stderr, "hsv bound violated: %s (%s:%d)\n", what,    \
                   __FILE__, __LINE__);                                 \
      std::abort();                                                     \
    }                                                                   \
  } while (0)
#else
#define HSV_BOUND(cond, what) ((void)0)
#endif

namespace hsv {

struct fe {
  uint32_t v[10];
};

constexpr int kFeLimbs = 10;

HSV_INL constexpr int fe26_bits(int i) { return (i & 1) ? 25 : 26; }
HSV_INL constexpr int fe26_off(int i) { return (i * 51 + 1) / 2; }
HSV_INL constexpr uint32_t fe26_mask(int i) { return (i & 1) ? 0x1ffffffu : 0x3ffffffu; }
// limbs of 2p: 2 * (2^26 - 19), 2 * (2^25 - 1), 2 * (2^26 - 1), ...
HSV_INL constexpr uint32_t fe26_2p(int i) { return i == 0 ? 0x7ffffdau : ((i & 1) ? 0x3fffffeu : 0x7fffffeu); }
// largest limb value g may hold in fe_mul (so that 19 * g fits 32 bits)
HSV_INL constexpr uint32_t fe26_gmax(int i) { return (i & 1) ? 113025455u : 226050910u; }

// 2x as v_add_u32 (x + x): the compiler's canonical form is a left shift,
// and v_lshlrev_b32 issues at the VOP3 rate on gfx950 while v_add_u32 is a
// full-rate op (tools/ubench_isa.hip, profiles/r02_ubench_isa.txt)
HSV_INL uint32_t fe26_x2(uint32_t x) {
#if defined(__HIP_DEVICE_COMPILE__)
  uint32_t r;
  asm("v_add_u32_e32 %0, %1, %1" : "=v"(r) : "v"(x));
  return r;
#else
  return x * 2u;
#endif
}

HSV_INL fe fe_small(uint32_t x) {
  fe r;
  r.v[0] = x;
  HSV_UNROLL
  for (int i = 1; i < 10; ++i) r.v[i] = 0;
  return r;
}

// 8 little-endian words -> element; bit 255 masked (FieldElement::from_bytes).
// The value may be >= p (non-canonical y is accepted and reduced implicitly).
HSV_INL fe fe_from_words_masked(const uint32_t w[8]) {
  fe r;
  HSV_UNROLL
  for (int i = 0; i < 10; ++i) {
    const int off = fe26_off(i), wi = off >> 5, sh = off & 31;
    const uint32_t lo = w[wi];
    const uint32_t hi = (wi + 1 < 8) ? w[wi + 1] : 0u;
    const uint32_t x = sh ? ((lo >> sh) | (hi << ((32 - sh) & 31))) : lo;
    r.v[i] = x & fe26_mask(i);
  }
  return r;
}

HSV_INL fe fe_add(const fe &a, const fe &b) {
  fe r;
  HSV_UNROLL
  for (int i = 0; i < 10; ++i) {
    HSV_BOUND((uint64_t)a.v[i] + b.v[i] < (1ull << 32), "fe_add overflow");
    r.v[i] = a.v[i] + b.v[i];
  }
  return r;
}

// a - b computed as a + 2p - b; b must be class R (<= 2p limb-wise).
HSV_INL fe fe_sub(const fe &a, const fe &b) {
  fe r;
  HSV_UNROLL
  for (int i = 0; i < 10; ++i) {
    HSV_BOUND(b.v[i] <= fe26_2p(i), "fe_sub subtrahend not reduced");
    HSV_BOUND((uint64_t)a.v[i] + fe26_2p(i) < (1ull << 32), "fe_sub overflow");
    r.v[i] = a.v[i] + fe26_2p(i) - b.v[i];
  }
  return r;
}

HSV_INL fe fe_neg(const fe &a) { return fe_sub(fe_small(0), a); }

// --- carries ------------------------------------------------------------
template <int I>
HSV_INL void fe26_carry_step(uint32_t h[10]) {
  const uint32_t c = h[I] >> fe26_bits(I);
  h[I] &= fe26_mask(I);
  h[I + 1] += c;
}

HSV_INL void fe26_carry_wrap(uint32_t h[10]) {
  const uint32_t c = h[9] >> 25;
  h[9] &= 0x1ffffffu;
  h[0] += c * 19u;
}

// Any limbs < 2^31 -> class R (ref10 order: two interleaved chains).
HSV_INL fe fe_carry(const fe &a) {
  uint32_t h[10];
  HSV_UNROLL
  for (int i = 0; i < 10; ++i) h[i] = a.v[i];
  fe26_carry_step<0>(h);
  fe26_carry_step<4>(h);
  fe26_carry_step<1>(h);
  fe26_carry_step<5>(h);
  fe26_carry_step<2>(h);
  fe26_carry_step<6>(h);
  fe26_carry_step<3>(h);
  fe26_carry_step<7>(h);
  fe26_carry_step<4>(h);
  fe26_carry_step<8>(h);
  fe26_carry_wrap(h);
  fe26_carry_step<0>(h);
  fe r;
  HSV_UNROLL
  for (int i = 0; i < 10; ++i) r.v[i] = h[i];
  return r;
}

// 64-bit column sums -> class R.
template <int I>
HSV_INL void fe26_carry64_step(uint64_t h[10]) {
  const uint64_t c = h[I] >> fe26_bits(I);
  h[I] &= fe26_mask(I);
  h[I + 1] += c;
}

HSV_INL fe fe26_carry64(uint64_t h[10]) {
  fe26_carry64_step<0>(h);
  fe26_carry64_step<4>(h);
  fe26_carry64_step<1>(h);
  fe26_carry64_step<5>(h);
  fe26_carry64_step<2>(h);
  fe26_carry64_step<6>(h);
  fe26_carry64_step<3>(h);
  fe26_carry64_step<7>(h);
  fe26_carry64_step<4>(h);
  fe26_carry64_step<8>(h);
  {
    const uint64_t c = h[9] >> 25;
    h[9] &= 0x1ffffffu;
    h[0] += c * 19u;
  }
  fe26_carry64_step<0>(h);
  fe r;
  HSV_UNROLL
  for (int i = 0; i < 10; ++i) r.v[i] = (uint32_t)h[i];
  return r;
}

#if defined(HSV_CHECK_BOUNDS) && !defined(__HIP_DEVICE_COMPILE__)
// exact column sums in 128-bit arithmetic: each must stay below 2^64
HSV_INL void fe26_check_columns(const fe &f, const fe &g) {
  for (int k = 0; k < 10; ++k) {
    unsigned __int128 acc = 0;
    for (int i = 0; i < 10; ++i) {
      int j = k - i;
      unsigned m = 1;
      if (j < 0) { j += 10; m *= 19; }
      if ((i & 1) && (j & 1)) m *= 2;
      acc += (unsigned __int128)f.v[i] * g.v[j] * m;
    }
    HSV_BOUND(((acc + ((unsigned __int128)1 << 40)) >> 64) == 0, "fe_mul column overflow (incl. carry-in)");
  }
}
#endif

// acc + sum_i a[i] * b[i] as ONE chain of v_mad_u64_u32 starting from acc.
// On the device the chain is a single asm statement: the compiler would
// otherwise split a column into parallel partial sums (and move the carry-in
// to the end), paying a 64-bit add per split; a dependent chain issues as
// fast as independent ones on gfx950 (tools/ubench_chain.hip).  The carry-out
// carry-out SGPR pair of the instruction is dead (see below).
template <int N, bool ZERO = false>
HSV_INL uint64_t fe26_chain(const uint32_t *a, const uint32_t *b, uint64_t acc) {
#if defined(__HIP_DEVICE_COMPILE__)
  static_assert(N == 5 || N == 6 || N == 10, "chain length");
  // Operand i of the chain is (a[i], b[i]) = (%(2i+1), %(2i+2)).  The
  // instruction's carry-out SGPR pair is dead: it goes to VCC, declared
  // clobbered (an SGPR output operand makes the compiler pad every chain
  // with an s_nop).  A ZERO chain starts from the inline constant 0 instead
  // of a cleared register pair (early-clobber output: the inputs are read
  // after the first instruction writes it).
#define HSV_MC(x, y, c) "v_mad_u64_u32 %0, vcc, %" #x ", %" #y ", " c "\n\t"
#define HSV_C0 (ZERO ? "0" : "%0")
#define HSV_P(i) "v"(a[i]), "v"(b[i])
#define HSV_BODY5 HSV_MC(3, 4, "%0") HSV_MC(5, 6, "%0") HSV_MC(7, 8, "%0") HSV_MC(9, 10, "%0")
#define HSV_BODY6 HSV_BODY5 HSV_MC(11, 12, "%0")
#define HSV_BODY10 HSV_BODY6 HSV_MC(13, 14, "%0") HSV_MC(15, 16, "%0") HSV_MC(17, 18, "%0") HSV_MC(19, 20, "%0")
#define HSV_IN5 HSV_P(0), HSV_P(1), HSV_P(2), HSV_P(3), HSV_P(4)
#define HSV_IN6 HSV_IN5, HSV_P(5)
#define HSV_IN10 HSV_IN6, HSV_P(6), HSV_P(7), HSV_P(8), HSV_P(9)
  if constexpr (ZERO) {
    static_assert(N != 5, "zero-start chains are columns 0 (6 or 10 products)");
    if constexpr (N == 6) asm(HSV_MC(1, 2, "0") HSV_BODY6 : "=&v"(acc) : HSV_IN6 : "vcc");
    else asm(HSV_MC(1, 2, "0") HSV_BODY10 : "=&v"(acc) : HSV_IN10 : "vcc");
  } else {
    if constexpr (N == 5) asm(HSV_MC(1, 2, "%0") HSV_BODY5 : "+v"(acc) : HSV_IN5 : "vcc");
    else if constexpr (N == 6) asm(HSV_MC(1, 2, "%0") HSV_BODY6 : "+v"(acc) : HSV_IN6 : "vcc");
    else asm(HSV_MC(1, 2, "%0") HSV_BODY10 : "+v"(acc) : HSV_IN10 : "vcc");
  }
#undef HSV_MC
#undef HSV_C0
#undef HSV_P
#undef HSV_BODY5
#undef HSV_BODY6
#undef HSV_BODY10
#undef HSV_IN5
#undef HSV_IN6
#undef HSV_IN10
  return acc;
#else
  if (ZERO) acc = 0;
  for (int i = 0; i < N; ++i) acc += (uint64_t)a[i] * b[i];
  return acc;
#endif
}

// Columns are produced in order 0..9; the carry out of column k is the
// initial accumulator of column k+1 (v_mad_u64_u32 adds it for free), so the
// carry chain costs one 64-bit shift and one mask per limb and no 64-bit adds.
// The final carry (weight 2^255) wraps into limbs 0/1 times 19.
// -DHSV_FE26_PARALLEL_CARRY selects the earlier form (independent column
// sums, then a ref10-order carry pass).
HSV_INL void fe26_wrap_carry(fe &r, uint64_t acc) {
  const uint64_t t = (uint64_t)r.v[0] + acc * 19u;
  r.v[0] = (uint32_t)t & 0x3ffffffu;
  r.v[1] += (uint32_t)(t >> 26);
}

// column K of f*g (10 products, with the 19x / 2x folds) added to acc; column
// 0 starts from zero
template <int K>
HSV_INL uint64_t fe26_mul_column(const uint32_t *f, const uint32_t *f2, const uint32_t *g, const uint32_t *g19,
                                 uint64_t acc) {
  uint32_t ca[10], cb[10];
  HSV_UNROLL
  for (int i = 0; i < 10; ++i) {
    int j = K - i;
    const bool wrap = j < 0;
    if (wrap) j += 10;
    ca[i] = ((i & 1) && (j & 1)) ? f2[i] : f[i];
    cb[i] = wrap ? g19[j] : g[j];
  }
  return K == 0 ? fe26_chain<10, true>(ca, cb, 0) : fe26_chain<10>(ca, cb, acc);
}

// operand prescaling of fe_mul: 19 g (every limb), 2 f (odd limbs)
HSV_INL void fe26_mul_prescale(const fe &f, const fe &g, uint32_t f2[10], uint32_t g19[10]) {
#if defined(HSV_CHECK_BOUNDS) && !defined(__HIP_DEVICE_COMPILE__)
  for (int i = 0; i < 10; ++i) HSV_BOUND(g.v[i] <= fe26_gmax(i), "fe_mul g operand too large");
  fe26_check_columns(f, g);
#endif
  HSV_UNROLL
  for (int i = 0; i < 10; ++i) {
    g19[i] = g.v[i] * 19u;
    f2[i] = (i & 1) ? fe26_x2(f.v[i]) : f.v[i];
  }
}

HSV_INL fe fe_mul(const fe &f, const fe &g) {
  HSV_SCHED_FENCE();
  uint32_t g19[10], f2[10];
  fe26_mul_prescale(f, g, f2, g19);
#ifdef HSV_FE26_PARALLEL_CARRY
  uint64_t h[10];
  HSV_UNROLL
  for (int k = 0; k < 10; ++k) {
    uint64_t acc = 0;
    HSV_UNROLL
    for (int i = 0; i < 10; ++i) {
      int j = k - i;
      const bool wrap = j < 0;
      if (wrap) j += 10;
      const uint32_t a = ((i & 1) && (j & 1)) ? f2[i] : f.v[i];
      const uint32_t b = wrap ? g19[j] : g.v[j];
      acc += (uint64_t)a * b;
    }
    h[k] = acc;
  }
  fe r = fe26_carry64(h);
#else
  fe r;
  uint64_t acc = 0;
#define HSV_MULC(K)                                         \
  acc = fe26_mul_column<K>(f.v, f2, g.v, g19, acc);         \
  r.v[K] = (uint32_t)acc & fe26_mask(K);                    \
  acc >>= fe26_bits(K);
  HSV_MULC(0) HSV_MULC(1) HSV_MULC(2) HSV_MULC(3) HSV_MULC(4)
  HSV_MULC(5) HSV_MULC(6) HSV_MULC(7) HSV_MULC(8) HSV_MULC(9)
#undef HSV_MULC
  fe26_wrap_carry(r, acc);
#endif
  HSV_SCHED_FENCE();
  return r;
}

// Two independent products r = f g, s = h k, interleaved column by column:
// two dependency chains per wave instead of one.  A lone chain leaves the
// SIMD's v_mad_u64_u32 issue short of its rate at the point pass's 3 waves per
// SIMD (tools/ubench_fe.hip), and the instruction after each chain no longer
// reads that chain's result (no s_nop pad behind the inline asm).
HSV_INL void fe_mul2(const fe &f, const fe &g, const fe &h, const fe &k, fe &r, fe &s) {
  HSV_SCHED_FENCE();
  uint32_t g19[10], f2[10], k19[10], h2[10];
  fe26_mul_prescale(f, g, f2, g19);
  fe26_mul_prescale(h, k, h2, k19);
  uint64_t a0 = 0, a1 = 0;
#define HSV_MULC2(K)                                        \
  a0 = fe26_mul_column<K>(f.v, f2, g.v, g19, a0);           \
  a1 = fe26_mul_column<K>(h.v, h2, k.v, k19, a1);           \
  r.v[K] = (uint32_t)a0 & fe26_mask(K);                     \
  a0 >>= fe26_bits(K);                                      \
  s.v[K] = (uint32_t)a1 & fe26_mask(K);                     \
  a1 >>= fe26_bits(K);
  HSV_MULC2(0) HSV_MULC2(1) HSV_MULC2(2) HSV_MULC2(3) HSV_MULC2(4)
  HSV_MULC2(5) HSV_MULC2(6) HSV_MULC2(7) HSV_MULC2(8) HSV_MULC2(9)
#undef HSV_MULC2
  fe26_wrap_carry(r, a0);
  fe26_wrap_carry(s, a1);
  HSV_SCHED_FENCE();
}

// Prepared operands: the prescaling of fe_mul done once for an operand that
// several products share (the point formulas' E, F, G, H).
//   fe_f: f with odd limbs doubled;  fe_g: g with every limb times 19.
struct fe_f {
  fe v;
  uint32_t x2[10];
};
struct fe_g {
  fe v;
  uint32_t x19[10];
};

HSV_INL fe_f fe_prep_f(const fe &f) {
  fe_f r;
  r.v = f;
  HSV_UNROLL
  for (int i = 0; i < 10; ++i) r.x2[i] = (i & 1) ? fe26_x2(f.v[i]) : f.v[i];
  return r;
}

HSV_INL fe_g fe_prep_g(const fe &g) {
#if defined(HSV_CHECK_BOUNDS) && !defined(__HIP_DEVICE_COMPILE__)
  for (int i = 0; i < 10; ++i) HSV_BOUND(g.v[i] <= fe26_gmax(i), "fe_mul g operand too large");
#endif
  fe_g r;
  r.v = g;
  HSV_UNROLL
  for (int i = 0; i < 10; ++i) r.x19[i] = g.v[i] * 19u;
  return r;
}

// f g from prepared operands (sequential carry, as fe_mul)
HSV_INL fe fe_mul_p(const fe_f &f, const fe_g &g) {
  HSV_SCHED_FENCE();
#if defined(HSV_CHECK_BOUNDS) && !defined(__HIP_DEVICE_COMPILE__)
  fe26_check_columns(f.v, g.v);
#endif
  fe r;
  uint64_t acc = 0;
#define HSV_MULC(K)                                         \
  acc = fe26_mul_column<K>(f.v.v, f.x2, g.v.v, g.x19, acc); \
  r.v[K] = (uint32_t)acc & fe26_mask(K);                    \
  acc >>= fe26_bits(K);
  HSV_MULC(0) HSV_MULC(1) HSV_MULC(2) HSV_MULC(3) HSV_MULC(4)
  HSV_MULC(5) HSV_MULC(6) HSV_MULC(7) HSV_MULC(8) HSV_MULC(9)
#undef HSV_MULC
  fe26_wrap_carry(r, acc);
  HSV_SCHED_FENCE();
  return r;
}

// r = f g and s = h k from prepared operands, interleaved (fe_mul2)
HSV_INL void fe_mul2_p(const fe_f &f, const fe_g &g, const fe_f &h, const fe_g &k, fe &r, fe &s) {
  HSV_SCHED_FENCE();
#if defined(HSV_CHECK_BOUNDS) && !defined(__HIP_DEVICE_COMPILE__)
  fe26_check_columns(f.v, g.v);
  fe26_check_columns(h.v, k.v);
#endif
  uint64_t a0 = 0, a1 = 0;
#define HSV_MULC2(K)                                        \
  a0 = fe26_mul_column<K>(f.v.v, f.x2, g.v.v, g.x19, a0);   \
  a1 = fe26_mul_column<K>(h.v.v, h.x2, k.v.v, k.x19, a1);   \
  r.v[K] = (uint32_t)a0 & fe26_mask(K);                     \
  a0 >>= fe26_bits(K);                                      \
  s.v[K] = (uint32_t)a1 & fe26_mask(K);                     \
  a1 >>= fe26_bits(K);
  HSV_MULC2(0) HSV_MULC2(1) HSV_MULC2(2) HSV_MULC2(3) HSV_MULC2(4)
  HSV_MULC2(5) HSV_MULC2(6) HSV_MULC2(7) HSV_MULC2(8) HSV_MULC2(9)
#undef HSV_MULC2
  fe26_wrap_carry(r, a0);
  fe26_wrap_carry(s, a1);
  HSV_SCHED_FENCE();
}

// operands of the product f_i f_j (i <= j) in a squaring, with its factor
// (2 for i != j, 2 for odd i and j, 19 for a wrap past limb 9) folded in
HSV_INL void fe26_sq_operands(int i, int j, const uint32_t *f, const uint32_t *f2, const uint32_t *f19,
                              const uint32_t *f38, uint32_t &a, uint32_t &b) {
  const bool odd = (i & 1) && (j & 1);
  const bool wrap = i + j >= 10;
  const int m = (i != j ? 2 : 1) * (odd ? 2 : 1) * (wrap ? 19 : 1);
  if (m == 1) { a = f[i]; b = f[j]; }
  else if (m == 2) { a = f2[i]; b = f[j]; }
  else if (m == 4) { a = f2[i]; b = f2[j]; }
  else if (m == 19) { a = f[i]; b = f19[j]; }
  else if (m == 38) {
    if (i == j) { a = f[i]; b = f38[j]; }
    else { a = f2[i]; b = f19[j]; }
  } else { a = f2[i]; b = f38[j]; }  // m == 76
}

// column K of a squaring (6 products for even K, 5 for odd K) added to acc
template <int K>
HSV_INL uint64_t fe26_sq_column(const uint32_t *f, const uint32_t *f2, const uint32_t *f19, const uint32_t *f38,
                                uint64_t acc) {
  constexpr bool ZERO = K == 0;
  constexpr int N = (K % 2 == 0) ? 6 : 5;
  uint32_t ca[N], cb[N];
  int n = 0;
  HSV_UNROLL
  for (int i = 0; i < 10; ++i) {
    HSV_UNROLL
    for (int j = i; j < 10; ++j) {
      if ((i + j) % 10 != K) continue;
      fe26_sq_operands(i, j, f, f2, f19, f38, ca[n], cb[n]);
      ++n;
    }
  }
  return fe26_chain<N, ZERO>(ca, cb, acc);
}

HSV_INL void fe26_sq_prescale(const fe &f, uint32_t f2[10], uint32_t f19[10], uint32_t f38[10]) {
#if defined(HSV_CHECK_BOUNDS) && !defined(__HIP_DEVICE_COMPILE__)
  for (int i = 0; i < 10; ++i) HSV_BOUND(f.v[i] <= fe26_gmax(i), "fe_sq operand too large");
  fe26_check_columns(f, f);
#endif
  HSV_UNROLL
  for (int i = 0; i < 10; ++i) {
    f2[i] = fe26_x2(f.v[i]);
    // 19x only where a product wraps past limb 9 (j >= 5 in f_i f_j, i <= j);
    // 38x only for odd j >= 5, as 19x + 19x (one VOP3 multiply per limb)
    f19[i] = i >= 5 ? f.v[i] * 19u : 0u;
    f38[i] = (i >= 5 && (i & 1)) ? fe26_x2(f19[i]) : 0u;
  }
}

HSV_INL fe fe_sq(const fe &f) {
  HSV_SCHED_FENCE();
  uint32_t f2[10], f19[10], f38[10];
  fe26_sq_prescale(f, f2, f19, f38);
#ifdef HSV_FE26_PARALLEL_CARRY
  uint64_t h[10];
  HSV_UNROLL
  for (int k = 0; k < 10; ++k) {
    uint64_t acc = 0;
    HSV_UNROLL
    for (int i = 0; i < 10; ++i) {
      HSV_UNROLL
      for (int j = i; j < 10; ++j) {
        if ((i + j) % 10 != k) continue;
        uint32_t a, b;
        fe26_sq_operands(i, j, f.v, f2, f19, f38, a, b);
        acc += (uint64_t)a * b;
      }
    }
    h[k] = acc;
  }
  fe r = fe26_carry64(h);
#else
  fe r;
  uint64_t acc = 0;
#define HSV_SQC(K)                                 \
  acc = fe26_sq_column<K>(f.v, f2, f19, f38, acc); \
  r.v[K] = (uint32_t)acc & fe26_mask(K);           \
  acc >>= fe26_bits(K);
  HSV_SQC(0) HSV_SQC(1) HSV_SQC(2) HSV_SQC(3) HSV_SQC(4)
  HSV_SQC(5) HSV_SQC(6) HSV_SQC(7) HSV_SQC(8) HSV_SQC(9)
#undef HSV_SQC
  fe26_wrap_carry(r, acc);
#endif
  HSV_SCHED_FENCE();
  return r;
}

// Two independent squarings ra = a^2, rb = b^2 interleaved (see fe_mul2).
HSV_INL void fe_sq2(const fe &a, const fe &b, fe &ra, fe &rb) {
  HSV_SCHED_FENCE();
  uint32_t a2[10], a19[10], a38[10], b2[10], b19[10], b38[10];
  fe26_sq_prescale(a, a2, a19, a38);
  fe26_sq_prescale(b, b2, b19, b38);
  uint64_t x0 = 0, x1 = 0;
#define HSV_SQC2(K)                                  \
  x0 = fe26_sq_column<K>(a.v, a2, a19, a38, x0);     \
  x1 = fe26_sq_column<K>(b.v, b2, b19, b38, x1);     \
  ra.v[K] = (uint32_t)x0 & fe26_mask(K);             \
  x0 >>= fe26_bits(K);                               \
  rb.v[K] = (uint32_t)x1 & fe26_mask(K);             \
  x1 >>= fe26_bits(K);
  HSV_SQC2(0) HSV_SQC2(1) HSV_SQC2(2) HSV_SQC2(3) HSV_SQC2(4)
  HSV_SQC2(5) HSV_SQC2(6) HSV_SQC2(7) HSV_SQC2(8) HSV_SQC2(9)
#undef HSV_SQC2
  fe26_wrap_carry(ra, x0);
  fe26_wrap_carry(rb, x1);
  HSV_SCHED_FENCE();
}

// Unique representative in [0, p), limbs exact.
HSV_INL fe fe_canon(const fe &a) {
  uint32_t h[10];
  HSV_UNROLL
  for (int i = 0; i < 10; ++i) h[i] = a.v[i];
  // three sequential passes: limbs exact, value < 2^255
  HSV_UNROLL
  for (int pass = 0; pass < 3; ++pass) {
    fe26_carry_step<0>(h);
    fe26_carry_step<1>(h);
    fe26_carry_step<2>(h);
    fe26_carry_step<3>(h);
    fe26_carry_step<4>(h);
    fe26_carry_step<5>(h);
    fe26_carry_step<6>(h);
    fe26_carry_step<7>(h);
    fe26_carry_step<8>(h);
    fe26_carry_wrap(h);
  }
  // q = [h >= p] = [h + 19 >= 2^255]
  uint32_t q = (h[0] + 19u) >> 26;
  HSV_UNROLL
  for (int i = 1; i < 10; ++i) q = (h[i] + q) >> fe26_bits(i);
  h[0] += 19u * q;
  fe26_carry_step<0>(h);
  fe26_carry_step<1>(h);
  fe26_carry_step<2>(h);
  fe26_carry_step<3>(h);
  fe26_carry_step<4>(h);
  fe26_carry_step<5>(h);
  fe26_carry_step<6>(h);
  fe26_carry_step<7>(h);
  fe26_carry_step<8>(h);
  h[9] &= 0x1ffffffu;  // drops 2^255 (subtracting p = 2^255 - 19 after the +19q)
  fe r;
  HSV_UNROLL
  for (int i = 0; i < 10; ++i) r.v[i] = h[i];
  return r;
}

// canonical encoding as 8 little-endian words
HSV_INL void fe_pack(const fe &a, uint32_t w[8]) {
  const fe c = fe_canon(a);
  HSV_UNROLL
  for (int j = 0; j < 8; ++j) w[j] = 0;
  HSV_UNROLL
  for (int i = 0; i < 10; ++i) {
    const int off = fe26_off(i), wi = off >> 5, sh = off & 31;
    w[wi] |= c.v[i] << sh;
    if (sh + fe26_bits(i) > 32 && wi + 1 < 8) w[wi + 1] |= c.v[i] >> (32 - sh);
  }
}

// Loose 256-bit encoding for values kept in memory only to be read back into
// arithmetic (the per-lane point tables): one sequential carry pass instead of
// fe_canon, so the value is exact but not necessarily < p.  After the pass
// limbs 0 and 2..9 fit their widths and limb 1 fits 26 bits (it takes the one
// carry out of the wrapped limb 0), so the widths 26,26,26,25,26,25,26,25,26,25
// fill exactly 256 bits.  Input: limbs < 2^31.
HSV_INL constexpr int fe26_loose_bits(int i) { return i < 3 ? 26 : fe26_bits(i); }
HSV_INL constexpr int fe26_loose_off(int i) { return i == 0 ? 0 : fe26_loose_off(i - 1) + fe26_loose_bits(i - 1); }

HSV_INL void fe_pack_loose(const fe &a, uint32_t w[8]) {
  uint32_t h[10];
  HSV_UNROLL
  for (int i = 0; i < 10; ++i) h[i] = a.v[i];
  fe26_carry_step<0>(h);
  fe26_carry_step<1>(h);
  fe26_carry_step<2>(h);
  fe26_carry_step<3>(h);
  fe26_carry_step<4>(h);
  fe26_carry_step<5>(h);
  fe26_carry_step<6>(h);
  fe26_carry_step<7>(h);
  fe26_carry_step<8>(h);
  fe26_carry_wrap(h);
  fe26_carry_step<0>(h);
  HSV_BOUND(h[1] < (1u << 26), "fe_pack_loose limb 1");
  HSV_UNROLL
  for (int j = 0; j < 8; ++j) w[j] = 0;
  HSV_UNROLL
  for (int i = 0; i < 10; ++i) {
    const int off = fe26_loose_off(i), wi = off >> 5, sh = off & 31;
    w[wi] |= h[i] << sh;
    if (sh + fe26_loose_bits(i) > 32) w[wi + 1] |= h[i] >> (32 - sh);
  }
}

HSV_INL fe fe_unpack_loose(const uint32_t w[8]) {
  fe r;
  HSV_UNROLL
  for (int i = 0; i < 10; ++i) {
    const int off = fe26_loose_off(i), wi = off >> 5, sh = off & 31;
    const uint32_t lo = w[wi];
    const uint32_t hi = (wi + 1 < 8) ? w[wi + 1] : 0u;
    const uint32_t x = sh ? ((lo >> sh) | (hi << ((32 - sh) & 31))) : lo;
    r.v[i] = x & ((1u << fe26_loose_bits(i)) - 1u);
  }
  return r;
}

HSV_INL uint32_t fe_canon_low_bit(const fe &a) { return fe_canon(a).v[0] & 1u; }

HSV_INL uint32_t fe_is_zero(const fe &a) {
  const fe c = fe_canon(a);
  uint32_t acc = 0;
  HSV_UNROLL
  for (int i = 0; i < 10; ++i) acc |= c.v[i];
  return acc == 0;
}

HSV_INL uint32_t fe_eq(const fe &a, const fe &b) {
  const fe x = fe_canon(a), y = fe_canon(b);
  uint32_t acc = 0;
  HSV_UNROLL
  for (int i = 0; i < 10; ++i) acc |= x.v[i] ^ y.v[i];
  return acc == 0;
}

// Per-lane select.  On the device the lane mask is an explicit SGPR pair
// (ballot) read by v_cndmask_b32_e64: the compiler's VCC form
// (v_cndmask_b32_e32) issues ~5x slower on gfx950 when several read VCC in a
// row (tools/ubench_isa.hip, profiles/r02_ubench_isa.txt).
HSV_INL fe fe_select(const fe &a, const fe &b, uint32_t take_b) {
  fe r;
#if defined(__HIP_DEVICE_COMPILE__)
  const uint64_t m = __ballot(take_b != 0u);
  HSV_UNROLL
  for (int i = 0; i < 10; ++i) asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(r.v[i]) : "v"(a.v[i]), "v"(b.v[i]), "s"(m));
#else
  HSV_UNROLL
  for (int i = 0; i < 10; ++i) r.v[i] = take_b ? b.v[i] : a.v[i];
#endif
  return r;
}

}  // namespace hsv
