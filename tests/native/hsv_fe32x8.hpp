// GF(2^255 - 19), representation A: 8 little-endian 32-bit limbs (radix 2^32).
//
// Value in [0, 2^256), congruent mod p ("weakly reduced"): every result of
// add / sub / mul / sq is weakly reduced, so operations compose freely and
// fe_carry is the identity.  2^256 == 38 (mod p): carries out of limb 7 fold
// back into limb 0 times 38.  Multiplication is 8x8 operand scanning on
// v_mad_u64_u32 (each a_i*b_j + t_{i+j} + carry fits 64 bits).
// Included by hsv_field.hpp when HSV_FE_RADIX == 32.
#pragma once

namespace hsv {

struct fe {
  uint32_t v[8];
};

constexpr int kFeLimbs = 8;

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

// prepared operands and paired forms (the radix-26 field prescales operands
// once and interleaves the two products; here they are plain products)
struct fe_f {
  fe v;
};
struct fe_g {
  fe v;
};
HSV_INL fe_f fe_prep_f(const fe &f) { return fe_f{f}; }
HSV_INL fe_g fe_prep_g(const fe &g) { return fe_g{g}; }
HSV_INL fe fe_mul_p(const fe_f &f, const fe_g &g) { return fe_mul(f.v, g.v); }
HSV_INL void fe_mul2_p(const fe_f &f, const fe_g &g, const fe_f &h, const fe_g &k, fe &r, fe &s) {
  r = fe_mul(f.v, g.v);
  s = fe_mul(h.v, k.v);
}
HSV_INL void fe_mul2(const fe &f, const fe &g, const fe &h, const fe &k, fe &r, fe &s) {
  r = fe_mul(f, g);
  s = fe_mul(h, k);
}
HSV_INL void fe_sq2(const fe &a, const fe &b, fe &ra, fe &rb) {
  ra = fe_sq(a);
  rb = fe_sq(b);
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

HSV_INL fe fe_select(const fe &a, const fe &b, uint32_t take_b) {
  fe r;
  HSV_UNROLL
  for (int i = 0; i < 8; ++i) r.v[i] = take_b ? b.v[i] : a.v[i];
  return r;
}

HSV_INL fe fe_carry(const fe &a) { return a; }

// 8 little-endian words -> element (bit 255 masked: FieldElement::from_bytes)
HSV_INL fe fe_from_words_masked(const uint32_t w[8]) {
  fe r;
  HSV_UNROLL
  for (int i = 0; i < 8; ++i) r.v[i] = w[i];
  r.v[7] &= 0x7fffffffu;
  return r;
}

// canonical encoding (value in [0, p)) as 8 little-endian words
HSV_INL void fe_pack(const fe &a, uint32_t w[8]) {
  const fe c = fe_canon(a);
  HSV_UNROLL
  for (int i = 0; i < 8; ++i) w[i] = c.v[i];
}

HSV_INL uint32_t fe_canon_low_bit(const fe &a) { return fe_canon(a).v[0] & 1u; }

// memory encoding of table entries (the radix-26 field has a cheaper loose form)
HSV_INL void fe_pack_loose(const fe &a, uint32_t w[8]) { fe_pack(a, w); }
HSV_INL fe fe_unpack_loose(const uint32_t w[8]) { return fe_from_words_masked(w); }

}  // namespace hsv
