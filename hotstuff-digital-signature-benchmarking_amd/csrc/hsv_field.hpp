// GF(2^255 - 19) arithmetic for the Ed25519 verification kernels.
//
// Two interchangeable representations behind one API (selected at compile
// time by HSV_FE_RADIX):
//   26 (default)  hsv_fe26x10.hpp: 10 limbs of 26/25 bits (radix 2^25.5);
//                 column sums accumulate in place on v_mad_u64_u32 with the
//                 mod-p fold pre-applied (19x / 2x operand scaling).
//   32            hsv_fe32x8.hpp: 8 limbs of 32 bits, operand scanning -- a
//                 measured alternative kept for the host test build only
//                 (tests/native/, built with -I tests/native).
// API: fe, fe_small, fe_from_words_masked, fe_pack (canonical 8 words),
// fe_add, fe_sub, fe_neg, fe_mul, fe_sq, fe_carry, fe_canon, fe_is_zero,
// fe_select, fe_d / fe_d2 / fe_sqrtm1, plus the generic chains below.
// Operand-bound discipline (matters for radix 26, free for radix 32) is
// documented in hsv_fe26x10.hpp; point formulas insert fe_carry() where
// a value must be normalised.
//
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
#define HSV_MEMBER __host__ __device__ __forceinline__
#else
#define HSV_INL static inline  // host test builds: let the compiler decide
#define HSV_MEMBER inline
#endif

#if defined(__HIP_DEVICE_COMPILE__)
#define HSV_UNROLL _Pragma("unroll")
#define HSV_NOUNROLL _Pragma("nounroll")
// Keep the scheduler from interleaving independent field multiplies: one
// multiply alone has ample ILP, several interleaved multiply the live registers.
#define HSV_SCHED_FENCE() __builtin_amdgcn_sched_barrier(0)
#else
#define HSV_UNROLL _Pragma("GCC unroll 16")
#define HSV_NOUNROLL
#define HSV_SCHED_FENCE()
#endif

#ifndef HSV_FE_RADIX
#define HSV_FE_RADIX 26
#endif

#if HSV_FE_RADIX == 32
#include "hsv_fe32x8.hpp"
#elif HSV_FE_RADIX == 26
#include "hsv_fe26x10.hpp"
#else
#error "HSV_FE_RADIX must be 26 or 32"
#endif

namespace hsv {

HSV_INL fe fe_d() {
  const uint32_t w[8] = {0x135978a3u, 0x75eb4dcau, 0x4141d8abu, 0x00700a4du,
                         0x7779e898u, 0x8cc74079u, 0x2b6ffe73u, 0x52036ceeu};
  return fe_from_words_masked(w);
}

HSV_INL fe fe_d2() {
  const uint32_t w[8] = {0x26b2f159u, 0xebd69b94u, 0x8283b156u, 0x00e0149au,
                         0xeef3d130u, 0x198e80f2u, 0x56dffce7u, 0x2406d9dcu};
  return fe_from_words_masked(w);
}

HSV_INL fe fe_sqrtm1() {
  const uint32_t w[8] = {0x4a0ea0b0u, 0xc4ee1b27u, 0xad2fe478u, 0x2f431806u,
                         0x3dfbd7a7u, 0x2b4d0099u, 0x4fc1df0bu, 0x2b832480u};
  return fe_from_words_masked(w);
}

// canonical encoding == 8 constant words
HSV_INL uint32_t fe_eq_words(const fe &a, const uint32_t w[8]) {
  uint32_t c[8];
  fe_pack(a, c);
  uint32_t acc = 0;
  HSV_UNROLL
  for (int i = 0; i < 8; ++i) acc |= c[i] ^ w[i];
  return acc == 0;
}

HSV_INL uint32_t fe_is_negative(const fe &a) { return fe_canon_low_bit(a); }

HSV_INL fe fe_sqn(fe a, int n) {
  HSV_NOUNROLL
  for (int i = 0; i < n; ++i) a = fe_sq(a);
  return a;
}

// z^((p-5)/8) = z^(2^252 - 3)
HSV_INL fe fe_pow22523(const fe &z) {
#ifdef HSV_TIMING_STUB_SQRT  // tools/phase_probe.py only: wrong results, timing share of the root chain
  return z;
#endif
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

// Paired forms for two independent inputs (two root chains per lane run as
// interleaved pairs of squarings / products: fe_sq2, fe_mul2).
HSV_INL void fe_sqn2(fe &a, fe &b, int n) {
  if (n & 1) {
    fe x, y;
    fe_sq2(a, b, x, y);
    a = x;
    b = y;
  }
  // two steps per trip: the values return to (a, b) without register copies
  HSV_NOUNROLL
  for (int i = 0; i < n / 2; ++i) {
    fe x, y;
    fe_sq2(a, b, x, y);
    fe_sq2(x, y, a, b);
  }
}

HSV_INL void fe_mul2_inplace(fe &a, const fe &ga, fe &b, const fe &gb) {
  fe x, y;
  fe_mul2(a, ga, b, gb, x, y);
  a = x;
  b = y;
}

// (z^((p-5)/8), w^((p-5)/8)), the chain of fe_pow22523 on both inputs
HSV_INL void fe_pow22523_2(const fe &z, const fe &w, fe &rz, fe &rw) {
#ifdef HSV_TIMING_STUB_SQRT
  rz = z;
  rw = w;
  return;
#endif
  fe t0z, t0w, t1z, t1w, t2z, t2w;
  fe_sq2(z, w, t0z, t0w);                                    // 2
  t1z = t0z;
  t1w = t0w;
  fe_sqn2(t1z, t1w, 2);                                      // 8
  fe_mul2_inplace(t1z, z, t1w, w);                           // 9
  fe_mul2_inplace(t0z, t1z, t0w, t1w);                       // 11
  fe_sqn2(t0z, t0w, 1);                                      // 22
  fe_mul2_inplace(t0z, t1z, t0w, t1w);                       // 31 = 2^5 - 1
  t1z = t0z;
  t1w = t0w;
  fe_sqn2(t1z, t1w, 5);
  fe_mul2_inplace(t0z, t1z, t0w, t1w);                       // 2^10 - 1
  t1z = t0z;
  t1w = t0w;
  fe_sqn2(t1z, t1w, 10);
  fe_mul2_inplace(t1z, t0z, t1w, t0w);                       // 2^20 - 1
  t2z = t1z;
  t2w = t1w;
  fe_sqn2(t2z, t2w, 20);
  fe_mul2_inplace(t1z, t2z, t1w, t2w);                       // 2^40 - 1
  fe_sqn2(t1z, t1w, 10);
  fe_mul2_inplace(t0z, t1z, t0w, t1w);                       // 2^50 - 1
  t1z = t0z;
  t1w = t0w;
  fe_sqn2(t1z, t1w, 50);
  fe_mul2_inplace(t1z, t0z, t1w, t0w);                       // 2^100 - 1
  t2z = t1z;
  t2w = t1w;
  fe_sqn2(t2z, t2w, 100);
  fe_mul2_inplace(t1z, t2z, t1w, t2w);                       // 2^200 - 1
  fe_sqn2(t1z, t1w, 50);
  fe_mul2_inplace(t0z, t1z, t0w, t1w);                       // 2^250 - 1
  fe_sqn2(t0z, t0w, 2);                                      // 2^252 - 4
  fe_mul2(t0z, z, t0w, w, rz, rw);                           // 2^252 - 3
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

}  // namespace hsv
