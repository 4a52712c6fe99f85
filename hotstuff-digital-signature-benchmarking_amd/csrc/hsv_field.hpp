// GF(2^255 - 19) arithmetic for the Ed25519 verification kernels.
//
// Representation: 8 little-endian 32-bit limbs, value in [0, 2^256) and
// congruent mod p (a "weakly reduced" element).  2^256 == 38 (mod p), so every
// carry out of limb 7 folds back into limb 0 multiplied by 38.  Only
// fe_canon() produces the unique representative in [0, p).
//
// Multiplication is 8x8 operand scanning on v_mad_u64_u32 (32x32+64 -> 64):
// each partial product a_i*b_j + t_{i+j} + carry fits in 64 bits exactly.
// The same code is compiled for the host (g++) so tests can check it on CPU;
// the product library only ever runs it on the GPU.
//
// Semantics restated from curve25519-dalek 3.x FieldElement (u64 backend):
// from_bytes masks bit 255 and accepts y >= p (reduced implicitly),
// is_negative is the low bit of the canonical encoding, ct_eq compares
// canonical encodings.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define HSV_INL __host__ __device__ __forceinline__
#else
#define HSV_INL static inline __attribute__((always_inline))
#endif

#if defined(__HIP_DEVICE_COMPILE__)
#define HSV_UNROLL _Pragma("unroll")
#define HSV_NOUNROLL _Pragma("nounroll")
// Keep the scheduler from interleaving independent field multiplies: one
// multiply alone has ample ILP, several interleaved multiply the live registers.
#ifndef HSV_NO_SCHED_FENCE
#define HSV_SCHED_FENCE() __builtin_amdgcn_sched_barrier(0)
#else
#define HSV_SCHED_FENCE()
#endif
#else
#define HSV_UNROLL _Pragma("GCC unroll 16")
#define HSV_NOUNROLL
#define HSV_SCHED_FENCE()
#endif

namespace hsv {

struct fe {
  uint32_t v[8];
};

HSV_INL fe fe_const(uint32_t a0, uint32_t a1, uint32_t a2, uint32_t a3, uint32_t a4, uint32_t a5,
                    uint32_t a6, uint32_t a7) {
  fe r;
  r.v[0] = a0; r.v[1] = a1; r.v[2] = a2; r.v[3] = a3;
  r.v[4] = a4; r.v[5] = a5; r.v[6] = a6; r.v[7] = a7;
  return r;
}

HSV_INL fe fe_small(uint32_t x) { return fe_const(x, 0, 0, 0, 0, 0, 0, 0); }

// p = 2^255 - 19
HSV_INL fe fe_p() {
  return fe_const(0xffffffedu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu,
                  0xffffffffu, 0x7fffffffu);
}

// d = -121665/121666
HSV_INL fe fe_d() {
  return fe_const(0x135978a3u, 0x75eb4dcau, 0x4141d8abu, 0x00700a4du, 0x7779e898u, 0x8cc74079u,
                  0x2b6ffe73u, 0x52036ceeu);
}

// 2d
HSV_INL fe fe_d2() {
  return fe_const(0x26b2f159u, 0xebd69b94u, 0x8283b156u, 0x00e0149au, 0xeef3d130u, 0x198e80f2u,
                  0x56dffce7u, 0x2406d9dcu);
}

// sqrt(-1) = 2^((p-1)/4)
HSV_INL fe fe_sqrtm1() {
  return fe_const(0x4a0ea0b0u, 0xc4ee1b27u, 0xad2fe478u, 0x2f431806u, 0x3dfbd7a7u, 0x2b4d0099u,
                  0x4fc1df0bu, 0x2b832480u);
}

// Fold a carry c (0 <= c < 2^32/38) out of bit 256 back into the low limbs.
HSV_INL void fe_fold_carry(fe &r, uint32_t c) {
  uint64_t t = (uint64_t)r.v[0] + (uint64_t)c * 38u;
  r.v[0] = (uint32_t)t;
  t >>= 32;
  HSV_UNROLL
  for (int i = 1; i < 8; ++i) {
    t += r.v[i];
    r.v[i] = (uint32_t)t;
    t >>= 32;
  }
  // A second wrap leaves a value < 38 in limb 0, so this add cannot carry.
  r.v[0] += (uint32_t)t * 38u;
}

HSV_INL fe fe_add(const fe &a, const fe &b) {
  fe r;
  uint64_t t = 0;
  HSV_UNROLL
  for (int i = 0; i < 8; ++i) {
    t += (uint64_t)a.v[i] + b.v[i];
    r.v[i] = (uint32_t)t;
    t >>= 32;
  }
  fe_fold_carry(r, (uint32_t)t);
  return r;
}

HSV_INL fe fe_sub(const fe &a, const fe &b) {
  fe r;
  int64_t t = 0;
  HSV_UNROLL
  for (int i = 0; i < 8; ++i) {
    t += (int64_t)a.v[i] - (int64_t)b.v[i];
    r.v[i] = (uint32_t)t;
    t >>= 32;  // arithmetic: 0 or -1
  }
  // borrow out of bit 256: value wrapped by +2^256 == +38, subtract 38
  uint32_t borrow = (uint32_t)(-t);
  int64_t u = (int64_t)r.v[0] - (int64_t)(borrow * 38u);
  r.v[0] = (uint32_t)u;
  u >>= 32;
  HSV_UNROLL
  for (int i = 1; i < 8; ++i) {
    u += r.v[i];
    r.v[i] = (uint32_t)u;
    u >>= 32;
  }
  // A second borrow leaves a value >= 2^256 - 38 in limb 0's range: no further borrow.
  r.v[0] -= (uint32_t)(-u) * 38u;
  return r;
}

HSV_INL fe fe_neg(const fe &a) { return fe_sub(fe_small(0), a); }

// r = lo + 38*hi for a 512-bit product t[16], result weakly reduced.
HSV_INL fe fe_reduce_wide(const uint32_t t[16]) {
  fe r;
  uint64_t c = 0;
  HSV_UNROLL
  for (int i = 0; i < 8; ++i) {
    c = (uint64_t)t[8 + i] * 38u + t[i] + (c >> 32);
    r.v[i] = (uint32_t)c;
  }
  fe_fold_carry(r, (uint32_t)(c >> 32));
  return r;
}

HSV_INL fe fe_mul(const fe &a, const fe &b) {
  HSV_SCHED_FENCE();
  uint32_t t[16];
  uint64_t c = 0;
  HSV_UNROLL
  for (int j = 0; j < 8; ++j) {
    c = (uint64_t)a.v[0] * b.v[j] + (c >> 32);
    t[j] = (uint32_t)c;
  }
  t[8] = (uint32_t)(c >> 32);
  HSV_UNROLL
  for (int i = 1; i < 8; ++i) {
    c = 0;
    HSV_UNROLL
    for (int j = 0; j < 8; ++j) {
      c = (uint64_t)a.v[i] * b.v[j] + t[i + j] + (c >> 32);
      t[i + j] = (uint32_t)c;
    }
    t[i + 8] = (uint32_t)(c >> 32);
  }
  fe r = fe_reduce_wide(t);
  HSV_SCHED_FENCE();
  return r;
}

HSV_INL fe fe_sq(const fe &a) {
  HSV_SCHED_FENCE();
  uint32_t t[16];
  // off-diagonal products a_i*a_j, i < j
  t[0] = 0;
  uint64_t c = 0;
  HSV_UNROLL
  for (int j = 1; j < 8; ++j) {
    c = (uint64_t)a.v[0] * a.v[j] + (c >> 32);
    t[j] = (uint32_t)c;
  }
  t[8] = (uint32_t)(c >> 32);
  HSV_UNROLL
  for (int i = 1; i < 7; ++i) {
    c = 0;
    HSV_UNROLL
    for (int j = i + 1; j < 8; ++j) {
      c = (uint64_t)a.v[i] * a.v[j] + t[i + j] + (c >> 32);
      t[i + j] = (uint32_t)c;
    }
    t[i + 8] = (uint32_t)(c >> 32);
  }
  t[15] = 0;
  // double the off-diagonal sum (it is < 2^511, so the shift cannot overflow)
  HSV_UNROLL
  for (int i = 15; i > 0; --i) t[i] = (t[i] << 1) | (t[i - 1] >> 31);
  t[0] = t[0] << 1;
  // add the diagonal squares
  c = 0;
  HSV_UNROLL
  for (int i = 0; i < 8; ++i) {
    c = (uint64_t)a.v[i] * a.v[i] + t[2 * i] + (c >> 32);
    t[2 * i] = (uint32_t)c;
    c = (uint64_t)t[2 * i + 1] + (c >> 32);
    t[2 * i + 1] = (uint32_t)c;
  }
  fe r = fe_reduce_wide(t);
  HSV_SCHED_FENCE();
  return r;
}

// Unique representative in [0, p).
HSV_INL fe fe_canon(const fe &a) {
  fe r = a;
  // fold bit 255 twice: value < 2^255 afterwards
  HSV_UNROLL
  for (int pass = 0; pass < 2; ++pass) {
    uint32_t top = r.v[7] >> 31;
    r.v[7] &= 0x7fffffffu;
    uint64_t t = (uint64_t)r.v[0] + top * 19u;
    r.v[0] = (uint32_t)t;
    t >>= 32;
    HSV_UNROLL
    for (int i = 1; i < 8; ++i) {
      t += r.v[i];
      r.v[i] = (uint32_t)t;
      t >>= 32;
    }
  }
  // now r < 2^255 = p + 19: subtract p iff r + 19 >= 2^255
  fe s;
  uint64_t t = (uint64_t)r.v[0] + 19u;
  s.v[0] = (uint32_t)t;
  t >>= 32;
  HSV_UNROLL
  for (int i = 1; i < 8; ++i) {
    t += r.v[i];
    s.v[i] = (uint32_t)t;
    t >>= 32;
  }
  uint32_t ge = s.v[7] >> 31;
  s.v[7] &= 0x7fffffffu;
  HSV_UNROLL
  for (int i = 0; i < 8; ++i) r.v[i] = ge ? s.v[i] : r.v[i];
  return r;
}

HSV_INL uint32_t fe_is_zero(const fe &a) {
  fe c = fe_canon(a);
  uint32_t acc = 0;
  HSV_UNROLL
  for (int i = 0; i < 8; ++i) acc |= c.v[i];
  return acc == 0;
}

HSV_INL uint32_t fe_eq(const fe &a, const fe &b) { return fe_is_zero(fe_sub(a, b)); }

HSV_INL uint32_t fe_eq_canon_const(const fe &canon_a, const fe &b_const) {
  uint32_t acc = 0;
  HSV_UNROLL
  for (int i = 0; i < 8; ++i) acc |= canon_a.v[i] ^ b_const.v[i];
  return acc == 0;
}

HSV_INL uint32_t fe_is_negative(const fe &a) { return fe_canon(a).v[0] & 1u; }

HSV_INL fe fe_select(const fe &a, const fe &b, uint32_t take_b) {
  fe r;
  HSV_UNROLL
  for (int i = 0; i < 8; ++i) r.v[i] = take_b ? b.v[i] : a.v[i];
  return r;
}

HSV_INL fe fe_sqn(fe a, int n) {
  HSV_NOUNROLL
  for (int i = 0; i < n; ++i) a = fe_sq(a);
  return a;
}

// z^((p-5)/8) = z^(2^252 - 3)
HSV_INL fe fe_pow22523(const fe &z) {
  fe t0 = fe_sq(z);                    // 2
  fe t1 = fe_sq(fe_sq(t0));            // 8
  t1 = fe_mul(z, t1);                  // 9
  t0 = fe_mul(t0, t1);                 // 11
  t0 = fe_sq(t0);                      // 22
  t0 = fe_mul(t1, t0);                 // 31 = 2^5 - 1
  t1 = fe_sqn(t0, 5);
  t0 = fe_mul(t1, t0);                 // 2^10 - 1
  t1 = fe_sqn(t0, 10);
  t1 = fe_mul(t1, t0);                 // 2^20 - 1
  fe t2 = fe_sqn(t1, 20);
  t1 = fe_mul(t2, t1);                 // 2^40 - 1
  t1 = fe_sqn(t1, 10);
  t0 = fe_mul(t1, t0);                 // 2^50 - 1
  t1 = fe_sqn(t0, 50);
  t1 = fe_mul(t1, t0);                 // 2^100 - 1
  t2 = fe_sqn(t1, 100);
  t1 = fe_mul(t2, t1);                 // 2^200 - 1
  t1 = fe_sqn(t1, 50);
  t0 = fe_mul(t1, t0);                 // 2^250 - 1
  t0 = fe_sqn(t0, 2);                  // 2^252 - 4
  return fe_mul(t0, z);                // 2^252 - 3
}

// z^(p-2) = z^(2^255 - 21): inversion (host-side signing / encoding only)
HSV_INL fe fe_invert(const fe &z) {
  fe t0 = fe_sq(z);                    // 2
  fe t1 = fe_sq(fe_sq(t0));            // 8
  t1 = fe_mul(z, t1);                  // 9
  t0 = fe_mul(t0, t1);                 // 11
  fe t2 = fe_sq(t0);                   // 22
  t1 = fe_mul(t1, t2);                 // 31
  t2 = fe_sqn(t1, 5);
  t1 = fe_mul(t2, t1);                 // 2^10 - 1
  t2 = fe_sqn(t1, 10);
  t2 = fe_mul(t2, t1);                 // 2^20 - 1
  fe t3 = fe_sqn(t2, 20);
  t2 = fe_mul(t3, t2);                 // 2^40 - 1
  t2 = fe_sqn(t2, 10);
  t1 = fe_mul(t2, t1);                 // 2^50 - 1
  t2 = fe_sqn(t1, 50);
  t2 = fe_mul(t2, t1);                 // 2^100 - 1
  t3 = fe_sqn(t2, 100);
  t2 = fe_mul(t3, t2);                 // 2^200 - 1
  t2 = fe_sqn(t2, 50);
  t1 = fe_mul(t2, t1);                 // 2^250 - 1
  t1 = fe_sqn(t1, 5);                  // 2^255 - 32
  return fe_mul(t1, t0);               // 2^255 - 21
}

// 32 little-endian bytes -> field element with bit 255 masked (FieldElement::from_bytes)
HSV_INL fe fe_from_words_masked(const uint32_t w[8]) {
  fe r;
  HSV_UNROLL
  for (int i = 0; i < 8; ++i) r.v[i] = w[i];
  r.v[7] &= 0x7fffffffu;
  return r;
}

}  // namespace hsv
