// Scalars modulo the Ed25519 group order
//   l = 2^252 + 27742317777372353535851937790883648493
// as 8 little-endian 32-bit limbs.
//
// Restated semantics (curve25519-dalek 3.x Scalar, ed25519-dalek 1.0.1):
//  * check_scalar / Scalar::from_canonical_bytes: s is accepted iff s < l
//    (the ed25519 1.x `s[31] & 0xE0` pre-check is implied by s < l < 2^253).
//  * Scalar::from_hash: SHA-512 output read as a 512-bit little-endian integer,
//    reduced mod l (from_bytes_mod_order_wide).  Here: Barrett reduction,
//    b = 2^32, k = 8, mu = floor(2^512 / l) (Handbook of Applied Cryptography 14.42).
//  * Signed fixed-window recoding used by the verification loop: adding
//    C_w = sum_i 2^(w-1) * 2^(w*i) to a scalar makes every w-bit chunk c_i of the
//    sum encode the signed digit c_i - 2^(w-1) in [-2^(w-1), 2^(w-1)).
#pragma once
#include "hsv_field.hpp"

namespace hsv {

struct sc {
  uint32_t v[8];
};

HSV_INL void sc_l(uint32_t l[8]) {
  l[0] = 0x5cf5d3edu; l[1] = 0x5812631au; l[2] = 0xa2f79cd6u; l[3] = 0x14def9deu;
  l[4] = 0u; l[5] = 0u; l[6] = 0u; l[7] = 0x10000000u;
}

// s < l ?  (s given as 8 little-endian limbs)
HSV_INL uint32_t sc_is_canonical(const uint32_t s[8]) {
  uint32_t l[8];
  sc_l(l);
  // compute s - l; s < l iff the subtraction borrows
  int64_t t = 0;
  HSV_UNROLL
  for (int i = 0; i < 8; ++i) {
    t += (int64_t)s[i] - (int64_t)l[i];
    t >>= 32;
  }
  return t != 0;
}

// r = x mod l, x a 512-bit little-endian integer (16 limbs).
HSV_INL sc sc_reduce512(const uint32_t x[16]) {
  const uint32_t mu[9] = {0x0a2c131bu, 0xed9ce5a3u, 0x086329a7u, 0x2106215du, 0xffffffebu,
                          0xffffffffu, 0xffffffffu, 0xffffffffu, 0x0000000fu};
  uint32_t l[8];
  sc_l(l);
  // q1 = x >> 224 (9 limbs); q2 = q1 * mu (18 limbs); q3 = q2 >> 288 (limbs 9..17)
  uint32_t q2[18];
  HSV_UNROLL
  for (int i = 0; i < 18; ++i) q2[i] = 0;
  HSV_UNROLL
  for (int i = 0; i < 9; ++i) {
    uint64_t c = 0;
    HSV_UNROLL
    for (int j = 0; j < 9; ++j) {
      c = (uint64_t)x[7 + i] * mu[j] + q2[i + j] + (c >> 32);
      q2[i + j] = (uint32_t)c;
    }
    q2[i + 9] = (uint32_t)(c >> 32);
  }
  // r2 = (q3 * l) mod 2^288 (9 limbs)
  uint32_t r2[9];
  HSV_UNROLL
  for (int i = 0; i < 9; ++i) r2[i] = 0;
  HSV_UNROLL
  for (int i = 0; i < 9; ++i) {
    uint64_t c = 0;
    HSV_UNROLL
    for (int j = 0; j < 8; ++j) {
      if (i + j < 9) {
        c = (uint64_t)q2[9 + i] * l[j] + r2[i + j] + (c >> 32);
        r2[i + j] = (uint32_t)c;
      }
    }
    if (i == 0) r2[8] = (uint32_t)(c >> 32);
  }
  // r = (x mod 2^288) - r2  (mod 2^288); 0 <= r < 3l
  uint32_t r[9];
  int64_t t = 0;
  HSV_UNROLL
  for (int i = 0; i < 9; ++i) {
    t += (int64_t)x[i] - (int64_t)r2[i];
    r[i] = (uint32_t)t;
    t >>= 32;
  }
  // at most two conditional subtractions of l
  HSV_UNROLL
  for (int pass = 0; pass < 2; ++pass) {
    uint32_t d[9];
    int64_t u = 0;
    HSV_UNROLL
    for (int i = 0; i < 9; ++i) {
      u += (int64_t)r[i] - (int64_t)(i < 8 ? l[i] : 0u);
      d[i] = (uint32_t)u;
      u >>= 32;
    }
    uint32_t keep = (u != 0);  // borrow => r < l
    HSV_UNROLL
    for (int i = 0; i < 9; ++i) r[i] = keep ? r[i] : d[i];
  }
  sc out;
  HSV_UNROLL
  for (int i = 0; i < 8; ++i) out.v[i] = r[i];
  return out;
}

// (a * b + c) mod l   -- host-side signing (S = r + k*a)
HSV_INL sc sc_muladd(const sc &a, const sc &b, const sc &c) {
  uint32_t t[16];
  HSV_UNROLL
  for (int i = 0; i < 16; ++i) t[i] = 0;
  HSV_UNROLL
  for (int i = 0; i < 8; ++i) {
    uint64_t cy = 0;
    HSV_UNROLL
    for (int j = 0; j < 8; ++j) {
      cy = (uint64_t)a.v[i] * b.v[j] + t[i + j] + (cy >> 32);
      t[i + j] = (uint32_t)cy;
    }
    t[i + 8] = (uint32_t)(cy >> 32);
  }
  uint64_t cy = 0;
  HSV_UNROLL
  for (int i = 0; i < 16; ++i) {
    cy += (uint64_t)t[i] + (i < 8 ? c.v[i] : 0u);
    t[i] = (uint32_t)cy;
    cy >>= 32;
  }
  return sc_reduce512(t);
}

}  // namespace hsv
