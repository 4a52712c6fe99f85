/*
 * ed25519_oracle.c -- C restatement of the reference's Ed25519 verification
 * rules (ed25519-dalek 1.0.1 on curve25519-dalek 3.x, u64 backend).
 *
 * Parity status: UNPINNED (the reference holds no known-answer vectors for
 * this path and ed25519-dalek cannot be built here); cross-checked against
 * RFC 8032 section 7.1, libsodium and OpenSSL.
 *
 * TEST INFRASTRUCTURE ONLY.  Used by tests/ as a fast checker (cross-checked
 * against oracle/ed25519_ref.py and the golden vectors) and by bench.py's
 * cpu_baseline leg as the "port" CPU baseline.  The product library never
 * links or calls it.
 *
 * Algorithm (restated from the published upstream crates; none of it is
 * vendored in /root/reference, whose hot path is crypto/src/lib.rs:204-223):
 *   FieldElement51      5 x 51-bit limbs, u128 products, 19-folding
 *   decompress          CompressedEdwardsY::decompress (sqrt_ratio_i; bit 255
 *                       masked; non-canonical y accepted; -0 accepted)
 *   check_scalar        s < l
 *   verify_strict       small-order rejection of A and R ([8]P == O),
 *                       k = SHA-512(R || A || M) mod l,
 *                       R' = vartime_double_scalar_mul_basepoint(k, -A, s)
 *                       (width-5 NAF for A, width-8 NAF table for B), R' == R
 *                       as projective points.
 *   verify_batch        (oracle_verify_batch_dalek) random linear combination,
 *                       one multiscalar multiplication (Straus / Pippenger),
 *                       the reference's QC path; timed as the QC CPU baseline.
 * Flag bits match include/hsv.h.
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef unsigned __int128 u128;
typedef struct { uint64_t v[5]; } fe51;

#define MASK51 ((1ull << 51) - 1)

static inline uint64_t load64(const uint8_t *b) {
  uint64_t r = 0;
  for (int i = 7; i >= 0; --i) r = (r << 8) | b[i];
  return r;
}

static void fe_frombytes(fe51 *h, const uint8_t s[32]) {
  h->v[0] = load64(s) & MASK51;
  h->v[1] = (load64(s + 6) >> 3) & MASK51;
  h->v[2] = (load64(s + 12) >> 6) & MASK51;
  h->v[3] = (load64(s + 19) >> 1) & MASK51;
  h->v[4] = (load64(s + 24) >> 12) & MASK51;  /* drops bit 255 */
}

static void fe_reduce(fe51 *h) {
  uint64_t c0 = h->v[0] >> 51, c1 = h->v[1] >> 51, c2 = h->v[2] >> 51, c3 = h->v[3] >> 51,
           c4 = h->v[4] >> 51;
  h->v[0] = (h->v[0] & MASK51) + c4 * 19;
  h->v[1] = (h->v[1] & MASK51) + c0;
  h->v[2] = (h->v[2] & MASK51) + c1;
  h->v[3] = (h->v[3] & MASK51) + c2;
  h->v[4] = (h->v[4] & MASK51) + c3;
}

static void fe_tobytes(uint8_t s[32], const fe51 *f) {
  fe51 h = *f;
  fe_reduce(&h);
  /* compute q = floor((h + 19) / 2^255) */
  uint64_t q = (h.v[0] + 19) >> 51;
  q = (h.v[1] + q) >> 51;
  q = (h.v[2] + q) >> 51;
  q = (h.v[3] + q) >> 51;
  q = (h.v[4] + q) >> 51;
  h.v[0] += 19 * q;
  h.v[1] += h.v[0] >> 51; h.v[0] &= MASK51;
  h.v[2] += h.v[1] >> 51; h.v[1] &= MASK51;
  h.v[3] += h.v[2] >> 51; h.v[2] &= MASK51;
  h.v[4] += h.v[3] >> 51; h.v[3] &= MASK51;
  h.v[4] &= MASK51;
  uint8_t out[32];
  uint64_t w0 = h.v[0] | (h.v[1] << 51);
  uint64_t w1 = (h.v[1] >> 13) | (h.v[2] << 38);
  uint64_t w2 = (h.v[2] >> 26) | (h.v[3] << 25);
  uint64_t w3 = (h.v[3] >> 39) | (h.v[4] << 12);
  for (int i = 0; i < 8; ++i) {
    out[i] = (uint8_t)(w0 >> (8 * i));
    out[8 + i] = (uint8_t)(w1 >> (8 * i));
    out[16 + i] = (uint8_t)(w2 >> (8 * i));
    out[24 + i] = (uint8_t)(w3 >> (8 * i));
  }
  memcpy(s, out, 32);
}

static inline void fe_add(fe51 *h, const fe51 *f, const fe51 *g) {
  for (int i = 0; i < 5; ++i) h->v[i] = f->v[i] + g->v[i];
  fe_reduce(h);
}

/* f - g computed as f + 16p - g (limbs of g must be < 16 * 2^51), then reduced */
static inline void fe_sub(fe51 *h, const fe51 *f, const fe51 *g) {
  h->v[0] = (f->v[0] + 36028797018963664ull) - g->v[0];
  h->v[1] = (f->v[1] + 36028797018963952ull) - g->v[1];
  h->v[2] = (f->v[2] + 36028797018963952ull) - g->v[2];
  h->v[3] = (f->v[3] + 36028797018963952ull) - g->v[3];
  h->v[4] = (f->v[4] + 36028797018963952ull) - g->v[4];
  fe_reduce(h);
}

static inline void fe_neg(fe51 *h, const fe51 *f) {
  fe51 z = {{0, 0, 0, 0, 0}};
  fe_sub(h, &z, f);
}

static void fe_mul(fe51 *h, const fe51 *f, const fe51 *g) {
  const uint64_t *a = f->v, *b = g->v;
  uint64_t b1_19 = b[1] * 19, b2_19 = b[2] * 19, b3_19 = b[3] * 19, b4_19 = b[4] * 19;
  u128 c0 = (u128)a[0] * b[0] + (u128)a[4] * b1_19 + (u128)a[3] * b2_19 + (u128)a[2] * b3_19 + (u128)a[1] * b4_19;
  u128 c1 = (u128)a[1] * b[0] + (u128)a[0] * b[1] + (u128)a[4] * b2_19 + (u128)a[3] * b3_19 + (u128)a[2] * b4_19;
  u128 c2 = (u128)a[2] * b[0] + (u128)a[1] * b[1] + (u128)a[0] * b[2] + (u128)a[4] * b3_19 + (u128)a[3] * b4_19;
  u128 c3 = (u128)a[3] * b[0] + (u128)a[2] * b[1] + (u128)a[1] * b[2] + (u128)a[0] * b[3] + (u128)a[4] * b4_19;
  u128 c4 = (u128)a[4] * b[0] + (u128)a[3] * b[1] + (u128)a[2] * b[2] + (u128)a[1] * b[3] + (u128)a[0] * b[4];
  c1 += (uint64_t)(c0 >> 51);
  uint64_t r0 = (uint64_t)c0 & MASK51;
  c2 += (uint64_t)(c1 >> 51);
  uint64_t r1 = (uint64_t)c1 & MASK51;
  c3 += (uint64_t)(c2 >> 51);
  uint64_t r2 = (uint64_t)c2 & MASK51;
  c4 += (uint64_t)(c3 >> 51);
  uint64_t r3 = (uint64_t)c3 & MASK51;
  uint64_t carry = (uint64_t)(c4 >> 51);
  uint64_t r4 = (uint64_t)c4 & MASK51;
  r0 += carry * 19;
  r1 += r0 >> 51;
  r0 &= MASK51;
  h->v[0] = r0; h->v[1] = r1; h->v[2] = r2; h->v[3] = r3; h->v[4] = r4;
}

static inline void fe_sq(fe51 *h, const fe51 *f) { fe_mul(h, f, f); }

static void fe_sqn(fe51 *h, const fe51 *f, int n) {
  *h = *f;
  for (int i = 0; i < n; ++i) fe_sq(h, h);
}

/* z^((p-5)/8) */
static void fe_pow22523(fe51 *out, const fe51 *z) {
  fe51 t0, t1, t2;
  fe_sq(&t0, z);
  fe_sqn(&t1, &t0, 2);
  fe_mul(&t1, z, &t1);
  fe_mul(&t0, &t0, &t1);
  fe_sq(&t0, &t0);
  fe_mul(&t0, &t1, &t0);
  fe_sqn(&t1, &t0, 5);
  fe_mul(&t0, &t1, &t0);
  fe_sqn(&t1, &t0, 10);
  fe_mul(&t1, &t1, &t0);
  fe_sqn(&t2, &t1, 20);
  fe_mul(&t1, &t2, &t1);
  fe_sqn(&t1, &t1, 10);
  fe_mul(&t0, &t1, &t0);
  fe_sqn(&t1, &t0, 50);
  fe_mul(&t1, &t1, &t0);
  fe_sqn(&t2, &t1, 100);
  fe_mul(&t1, &t2, &t1);
  fe_sqn(&t1, &t1, 50);
  fe_mul(&t0, &t1, &t0);
  fe_sqn(&t0, &t0, 2);
  fe_mul(out, &t0, z);
}

static int fe_eq(const fe51 *a, const fe51 *b) {
  uint8_t x[32], y[32];
  fe_tobytes(x, a);
  fe_tobytes(y, b);
  return memcmp(x, y, 32) == 0;
}

static int fe_isneg(const fe51 *a) {
  uint8_t x[32];
  fe_tobytes(x, a);
  return x[0] & 1;
}

static const fe51 FE_ONE = {{1, 0, 0, 0, 0}};
static fe51 FE_D, FE_D2, FE_SQRTM1;

/* --------------------------------------------------------------------- */
/* points: extended (X:Y:Z:T)                                              */
typedef struct { fe51 X, Y, Z, T; } ge;
typedef struct { fe51 YpX, YmX, Z2, T2d; } ge_cached;

static void ge_identity(ge *p) {
  memset(p, 0, sizeof *p);
  p->Y = FE_ONE;
  p->Z = FE_ONE;
}

static void ge_to_cached(ge_cached *c, const ge *p) {
  fe_add(&c->YpX, &p->Y, &p->X);
  fe_sub(&c->YmX, &p->Y, &p->X);
  fe_add(&c->Z2, &p->Z, &p->Z);
  fe_mul(&c->T2d, &p->T, &FE_D2);
}

static void ge_add(ge *r, const ge *p, const ge_cached *q) {
  fe51 a, b, c, d, e, f, g, h, t;
  fe_sub(&t, &p->Y, &p->X);
  fe_mul(&a, &t, &q->YmX);
  fe_add(&t, &p->Y, &p->X);
  fe_mul(&b, &t, &q->YpX);
  fe_mul(&c, &p->T, &q->T2d);
  fe_mul(&d, &p->Z, &q->Z2);
  fe_sub(&e, &b, &a);
  fe_sub(&f, &d, &c);
  fe_add(&g, &d, &c);
  fe_add(&h, &b, &a);
  fe_mul(&r->X, &e, &f);
  fe_mul(&r->Y, &g, &h);
  fe_mul(&r->Z, &f, &g);
  fe_mul(&r->T, &e, &h);
}

static void ge_sub(ge *r, const ge *p, const ge_cached *q) {
  ge_cached n;
  n.YpX = q->YmX;
  n.YmX = q->YpX;
  n.Z2 = q->Z2;
  fe_neg(&n.T2d, &q->T2d);
  ge_add(r, p, &n);
}

static void ge_dbl(ge *r, const ge *p) {
  fe51 a, b, c, h, e, g, f, t;
  fe_sq(&a, &p->X);
  fe_sq(&b, &p->Y);
  fe_sq(&c, &p->Z);
  fe_add(&c, &c, &c);
  fe_add(&h, &a, &b);
  fe_add(&t, &p->X, &p->Y);
  fe_sq(&t, &t);
  fe_sub(&e, &h, &t);
  fe_sub(&g, &a, &b);
  fe_add(&f, &c, &g);
  fe_mul(&r->X, &e, &f);
  fe_mul(&r->Y, &g, &h);
  fe_mul(&r->Z, &f, &g);
  fe_mul(&r->T, &e, &h);
}

static int ge_eq(const ge *p, const ge *q) {
  fe51 a, b;
  fe_mul(&a, &p->X, &q->Z);
  fe_mul(&b, &q->X, &p->Z);
  if (!fe_eq(&a, &b)) return 0;
  fe_mul(&a, &p->Y, &q->Z);
  fe_mul(&b, &q->Y, &p->Z);
  return fe_eq(&a, &b);
}

static int ge_is_identity(const ge *p) {
  ge o;
  ge_identity(&o);
  return ge_eq(p, &o);
}

static int ge_is_small_order(const ge *p) {
  ge t;
  ge_dbl(&t, p);
  ge_dbl(&t, &t);
  ge_dbl(&t, &t);
  return ge_is_identity(&t);
}

/* CompressedEdwardsY::decompress */
static int ge_decompress(ge *p, const uint8_t s[32]) {
  fe51 y, yy, u, v, v3, v7, r, chk, t, negu;
  fe_frombytes(&y, s);
  fe_sq(&yy, &y);
  fe_sub(&u, &yy, &FE_ONE);
  fe_mul(&v, &yy, &FE_D);
  fe_add(&v, &v, &FE_ONE);
  /* sqrt_ratio_i(u, v) */
  fe_sq(&v3, &v);
  fe_mul(&v3, &v3, &v);
  fe_sq(&v7, &v3);
  fe_mul(&v7, &v7, &v);
  fe_mul(&t, &u, &v7);
  fe_pow22523(&t, &t);
  fe_mul(&r, &u, &v3);
  fe_mul(&r, &r, &t);
  fe_sq(&chk, &r);
  fe_mul(&chk, &chk, &v);
  fe_neg(&negu, &u);
  int correct = fe_eq(&chk, &u);
  int flipped = fe_eq(&chk, &negu);
  fe_mul(&t, &negu, &FE_SQRTM1);
  int flipped_i = fe_eq(&chk, &t);
  if (flipped || flipped_i) fe_mul(&r, &r, &FE_SQRTM1);
  if (fe_isneg(&r)) fe_neg(&r, &r);
  if (!(correct || flipped)) return 0;
  if (s[31] >> 7) fe_neg(&r, &r);
  p->X = r;
  p->Y = y;
  p->Z = FE_ONE;
  fe_mul(&p->T, &r, &y);
  return 1;
}

/* --------------------------------------------------------------------- */
/* scalars mod l                                                           */
static const uint32_t L32[8] = {0x5cf5d3edu, 0x5812631au, 0xa2f79cd6u, 0x14def9deu,
                                0u,          0u,          0u,          0x10000000u};

static int sc_canonical(const uint8_t s[32]) {
  for (int i = 31; i >= 0; --i) {
    uint8_t lb = (uint8_t)(L32[i / 4] >> (8 * (i % 4)));
    if (s[i] < lb) return 1;
    if (s[i] > lb) return 0;
  }
  return 0; /* s == l */
}

/* x (64 bytes, little-endian) mod l -> 32 bytes: simple shift-subtract */
static void sc_reduce64(uint8_t out[32], const uint8_t x[64]) {
  /* r = x mod l via binary long division on 32-bit words (oracle: clarity over speed) */
  uint32_t r[9] = {0};
  for (int bit = 511; bit >= 0; --bit) {
    /* r = 2r + bit */
    uint32_t carry = (x[bit / 8] >> (bit % 8)) & 1;
    for (int i = 0; i < 9; ++i) {
      uint32_t nc = r[i] >> 31;
      r[i] = (r[i] << 1) | carry;
      carry = nc;
    }
    /* if r >= l: r -= l */
    int ge = 1;
    if (r[8]) ge = 1;
    else {
      for (int i = 7; i >= 0; --i) {
        if (r[i] > L32[i]) { ge = 1; break; }
        if (r[i] < L32[i]) { ge = 0; break; }
        if (i == 0) ge = 1;
      }
    }
    if (ge) {
      int64_t t = 0;
      for (int i = 0; i < 9; ++i) {
        t += (int64_t)r[i] - (int64_t)(i < 8 ? L32[i] : 0u);
        r[i] = (uint32_t)t;
        t >>= 32;
      }
    }
  }
  for (int i = 0; i < 32; ++i) out[i] = (uint8_t)(r[i / 4] >> (8 * (i % 4)));
}

/* width-w NAF of a 256-bit scalar (curve25519-dalek Scalar::non_adjacent_form) */
static void naf(int8_t out[256], const uint8_t s[32], int w) {
  uint64_t x[5] = {0};
  for (int i = 0; i < 4; ++i) x[i] = load64(s + 8 * i);
  memset(out, 0, 256);
  const uint64_t width = 1ull << w;
  const uint64_t window_mask = width - 1;
  int pos = 0;
  uint64_t carry = 0;
  while (pos < 256) {
    int u64_idx = pos / 64, bit_idx = pos % 64;
    uint64_t bit_buf;
    if (bit_idx < 64 - w) bit_buf = x[u64_idx] >> bit_idx;
    else bit_buf = (x[u64_idx] >> bit_idx) | (x[1 + u64_idx] << (64 - bit_idx));
    uint64_t window = carry + (bit_buf & window_mask);
    if ((window & 1) == 0) {
      pos += 1;
      continue;
    }
    if (window < width / 2) {
      carry = 0;
      out[pos] = (int8_t)window;
    } else {
      carry = 1;
      out[pos] = (int8_t)((int64_t)window - (int64_t)width);
    }
    pos += w;
  }
}

/* --------------------------------------------------------------------- */
/* SHA-512                                                                 */
static const uint64_t K512[80] = {
    0x428a2f98d728ae22ull, 0x7137449123ef65cdull, 0xb5c0fbcfec4d3b2full, 0xe9b5dba58189dbbcull,
    0x3956c25bf348b538ull, 0x59f111f1b605d019ull, 0x923f82a4af194f9bull, 0xab1c5ed5da6d8118ull,
    0xd807aa98a3030242ull, 0x12835b0145706fbeull, 0x243185be4ee4b28cull, 0x550c7dc3d5ffb4e2ull,
    0x72be5d74f27b896full, 0x80deb1fe3b1696b1ull, 0x9bdc06a725c71235ull, 0xc19bf174cf692694ull,
    0xe49b69c19ef14ad2ull, 0xefbe4786384f25e3ull, 0x0fc19dc68b8cd5b5ull, 0x240ca1cc77ac9c65ull,
    0x2de92c6f592b0275ull, 0x4a7484aa6ea6e483ull, 0x5cb0a9dcbd41fbd4ull, 0x76f988da831153b5ull,
    0x983e5152ee66dfabull, 0xa831c66d2db43210ull, 0xb00327c898fb213full, 0xbf597fc7beef0ee4ull,
    0xc6e00bf33da88fc2ull, 0xd5a79147930aa725ull, 0x06ca6351e003826full, 0x142929670a0e6e70ull,
    0x27b70a8546d22ffcull, 0x2e1b21385c26c926ull, 0x4d2c6dfc5ac42aedull, 0x53380d139d95b3dfull,
    0x650a73548baf63deull, 0x766a0abb3c77b2a8ull, 0x81c2c92e47edaee6ull, 0x92722c851482353bull,
    0xa2bfe8a14cf10364ull, 0xa81a664bbc423001ull, 0xc24b8b70d0f89791ull, 0xc76c51a30654be30ull,
    0xd192e819d6ef5218ull, 0xd69906245565a910ull, 0xf40e35855771202aull, 0x106aa07032bbd1b8ull,
    0x19a4c116b8d2d0c8ull, 0x1e376c085141ab53ull, 0x2748774cdf8eeb99ull, 0x34b0bcb5e19b48a8ull,
    0x391c0cb3c5c95a63ull, 0x4ed8aa4ae3418acbull, 0x5b9cca4f7763e373ull, 0x682e6ff3d6b2b8a3ull,
    0x748f82ee5defb2fcull, 0x78a5636f43172f60ull, 0x84c87814a1f0ab72ull, 0x8cc702081a6439ecull,
    0x90befffa23631e28ull, 0xa4506cebde82bde9ull, 0xbef9a3f7b2c67915ull, 0xc67178f2e372532bull,
    0xca273eceea26619cull, 0xd186b8c721c0c207ull, 0xeada7dd6cde0eb1eull, 0xf57d4f7fee6ed178ull,
    0x06f067aa72176fbaull, 0x0a637dc5a2c898a6ull, 0x113f9804bef90daeull, 0x1b710b35131c471bull,
    0x28db77f523047d84ull, 0x32caab7b40c72493ull, 0x3c9ebe0a15c9bebcull, 0x431d67c49c100d4cull,
    0x4cc5d4becb3e42b6ull, 0x597f299cfc657e2aull, 0x5fcb6fab3ad6faecull, 0x6c44198c4a475817ull};

#define ROTR(x, n) (((x) >> (n)) | ((x) << (64 - (n))))

static void sha512_block(uint64_t h[8], const uint8_t blk[128]) {
  uint64_t w[80];
  for (int i = 0; i < 16; ++i) {
    uint64_t x = 0;
    for (int j = 0; j < 8; ++j) x = (x << 8) | blk[8 * i + j];
    w[i] = x;
  }
  for (int i = 16; i < 80; ++i) {
    uint64_t s0 = ROTR(w[i - 15], 1) ^ ROTR(w[i - 15], 8) ^ (w[i - 15] >> 7);
    uint64_t s1 = ROTR(w[i - 2], 19) ^ ROTR(w[i - 2], 61) ^ (w[i - 2] >> 6);
    w[i] = w[i - 16] + s0 + w[i - 7] + s1;
  }
  uint64_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
  for (int i = 0; i < 80; ++i) {
    uint64_t S1 = ROTR(e, 14) ^ ROTR(e, 18) ^ ROTR(e, 41);
    uint64_t ch = (e & f) ^ (~e & g);
    uint64_t t1 = hh + S1 + ch + K512[i] + w[i];
    uint64_t S0 = ROTR(a, 28) ^ ROTR(a, 34) ^ ROTR(a, 39);
    uint64_t mj = (a & b) ^ (a & c) ^ (b & c);
    uint64_t t2 = S0 + mj;
    hh = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
  }
  h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += hh;
}

static void sha512(uint8_t out[64], const uint8_t *m, size_t len) {
  uint64_t h[8] = {0x6a09e667f3bcc908ull, 0xbb67ae8584caa73bull, 0x3c6ef372fe94f82bull,
                   0xa54ff53a5f1d36f1ull, 0x510e527fade682d1ull, 0x9b05688c2b3e6c1full,
                   0x1f83d9abfb41bd6bull, 0x5be0cd19137e2179ull};
  size_t nblk = (len + 17 + 127) / 128;
  for (size_t b = 0; b < nblk; ++b) {
    uint8_t blk[128];
    for (int i = 0; i < 128; ++i) {
      size_t pos = b * 128 + i;
      blk[i] = pos < len ? m[pos] : (pos == len ? 0x80 : 0);
    }
    if (b + 1 == nblk)
      for (int i = 0; i < 8; ++i) blk[127 - i] = (uint8_t)(((uint64_t)len * 8) >> (8 * i));
    sha512_block(h, blk);
  }
  for (int i = 0; i < 8; ++i)
    for (int j = 0; j < 8; ++j) out[8 * i + j] = (uint8_t)(h[i] >> (56 - 8 * j));
}

/* --------------------------------------------------------------------- */
/* constants and the basepoint NAF table                                   */
static ge_cached B_ODD[64]; /* [1,3,5,...,127]B */
static pthread_once_t g_once = PTHREAD_ONCE_INIT;

static void fe_from_hex_le(fe51 *f, const char *hex) {
  uint8_t b[32];
  for (int i = 0; i < 32; ++i) {
    unsigned v;
    char tmp[3] = {hex[2 * i], hex[2 * i + 1], 0};
    v = (unsigned)strtoul(tmp, NULL, 16);
    b[i] = (uint8_t)v;
  }
  fe_frombytes(f, b);
}

static void init_consts(void) {
  fe_from_hex_le(&FE_D, "a3785913ca4deb75abd841414d0a700098e879777940c78c73fe6f2bee6c0352");
  fe_from_hex_le(&FE_D2, "59f1b226949bd6eb56b183829a14e00030d1f3eef2808e19e7fcdf56dcd90624");
  fe_from_hex_le(&FE_SQRTM1, "b0a00e4a271beec478e42fad0618432fa7d7fb3d99004d2b0bdfc14f8024832b");
  uint8_t by[32];
  memset(by, 0x66, 32);
  by[0] = 0x58;
  ge B, B2, acc;
  ge_decompress(&B, by);
  ge_dbl(&B2, &B);
  ge_cached b2c;
  ge_to_cached(&b2c, &B2);
  acc = B;
  for (int i = 0; i < 64; ++i) {
    ge_to_cached(&B_ODD[i], &acc);
    ge_add(&acc, &acc, &b2c);
  }
}

/* --------------------------------------------------------------------- */
/* vartime_double_scalar_mul_basepoint: [a]A + [b]B                        */
static void double_scalar_mul(ge *r, const uint8_t a[32], const ge *A, const uint8_t b[32]) {
  int8_t an[256], bn[256];
  naf(an, a, 5);
  naf(bn, b, 8);
  ge_cached Atab[8]; /* [1,3,...,15]A */
  ge A2, acc;
  ge_cached a2c;
  ge_dbl(&A2, A);
  ge_to_cached(&a2c, &A2);
  acc = *A;
  for (int i = 0; i < 8; ++i) {
    ge_to_cached(&Atab[i], &acc);
    ge_add(&acc, &acc, &a2c);
  }
  int i = 255;
  while (i >= 0 && an[i] == 0 && bn[i] == 0) --i;
  ge q;
  ge_identity(&q);
  for (; i >= 0; --i) {
    ge_dbl(&q, &q);
    if (an[i] > 0) ge_add(&q, &q, &Atab[an[i] / 2]);
    else if (an[i] < 0) ge_sub(&q, &q, &Atab[-an[i] / 2]);
    if (bn[i] > 0) ge_add(&q, &q, &B_ODD[bn[i] / 2]);
    else if (bn[i] < 0) ge_sub(&q, &q, &B_ODD[-bn[i] / 2]);
  }
  *r = q;
}

void oracle_sc_reduce64_fast(uint8_t out[32], const uint8_t x[64]);

/* flag bits (include/hsv.h) */
enum { STRICT_OK = 1, EQ_OK = 2, PARSE_OK = 4, SMALL_A = 8, SMALL_R = 16, S_OK = 32, A_OK = 64, R_OK = 128 };

uint8_t oracle_verify_flags(const uint8_t pk[32], const uint8_t sig[64], const uint8_t *msg,
                            size_t msg_len) {
  pthread_once(&g_once, init_consts);
  uint8_t flags = 0;
  int s_ok = sc_canonical(sig + 32);
  ge A, R;
  int a_ok = ge_decompress(&A, pk);
  int r_ok = ge_decompress(&R, sig);
  if (s_ok) flags |= S_OK;
  if (a_ok) {
    flags |= A_OK;
    if (ge_is_small_order(&A)) flags |= SMALL_A;
  }
  if (r_ok) {
    flags |= R_OK;
    if (ge_is_small_order(&R)) flags |= SMALL_R;
  }
  if (!(s_ok && a_ok && r_ok)) return flags;
  flags |= PARSE_OK;
  uint8_t hbuf[64], k[32];
  uint8_t *buf = (uint8_t *)malloc(64 + msg_len);
  memcpy(buf, sig, 32);
  memcpy(buf + 32, pk, 32);
  memcpy(buf + 64, msg, msg_len);
  sha512(hbuf, buf, 64 + msg_len);
  free(buf);
  oracle_sc_reduce64_fast(k, hbuf); /* Barrett; equal to the bit-serial sc_reduce64 (tests/test_oracle.py) */
  ge negA = A;
  fe_neg(&negA.X, &A.X);
  fe_neg(&negA.T, &A.T);
  ge Rp;
  double_scalar_mul(&Rp, k, &negA, sig + 32);
  if (ge_eq(&Rp, &R)) {
    flags |= EQ_OK;
    if (!(flags & (SMALL_A | SMALL_R))) flags |= STRICT_OK;
  }
  return flags;
}

typedef struct {
  const uint8_t *pk, *sig, *msg;
  size_t msg_stride, lo, hi;
  uint8_t *flags;
} job_t;

static void *worker(void *arg) {
  job_t *j = (job_t *)arg;
  for (size_t i = j->lo; i < j->hi; ++i)
    j->flags[i] = oracle_verify_flags(j->pk + 32 * i, j->sig + 64 * i, j->msg + j->msg_stride * i, 32);
  return NULL;
}

/* n records (32-byte messages; msg_stride 0 = shared digest) on nthreads threads */
int oracle_verify_many(const uint8_t *pk, const uint8_t *sig, const uint8_t *msg, size_t msg_stride,
                       size_t n, uint8_t *flags, int nthreads) {
  pthread_once(&g_once, init_consts);
  if (nthreads < 1) nthreads = 1;
  if (nthreads > 256) nthreads = 256;
  pthread_t th[256];
  job_t jobs[256];
  for (int t = 0; t < nthreads; ++t) {
    jobs[t] = (job_t){pk, sig, msg, msg_stride, n * t / nthreads, n * (t + 1) / nthreads, flags};
    pthread_create(&th[t], NULL, worker, &jobs[t]);
  }
  for (int t = 0; t < nthreads; ++t) pthread_join(th[t], NULL);
  return 0;
}

/* crypto::Signature::verify_batch deterministic rule over one shared digest */
int oracle_verify_batch(const uint8_t digest[32], const uint8_t *pk, const uint8_t *sig, size_t n) {
  for (size_t i = 0; i < n; ++i) {
    uint8_t f = oracle_verify_flags(pk + 32 * i, sig + 64 * i, digest, 32);
    if ((f & (PARSE_OK | EQ_OK)) != (PARSE_OK | EQ_OK)) return 0;
  }
  return 1;
}

/* Mempool transaction check (reference mempool/src/batch_maker.rs:79-85):
 * tx = message || pk (32) || sig (64); flags of verify over
 * Digest(SHA-512(message)[..32]).  Transaction i = txs[offsets[i]..offsets[i+1]);
 * offsets NULL = fixed size tx_size.  A transaction shorter than 96 bytes gets
 * flags 0 (the reference's slice would panic). */
typedef struct {
  const uint8_t *txs;
  const uint64_t *offsets;
  size_t tx_size, lo, hi;
  uint8_t *flags;
} txjob_t;

static void *tx_worker(void *arg) {
  txjob_t *j = (txjob_t *)arg;
  for (size_t i = j->lo; i < j->hi; ++i) {
    const uint64_t a = j->offsets ? j->offsets[i] : (uint64_t)i * j->tx_size;
    const uint64_t b = j->offsets ? j->offsets[i + 1] : a + j->tx_size;
    if (b < a || b - a < 96) {
      j->flags[i] = 0;
      continue;
    }
    const uint8_t *tx = j->txs + a;
    const size_t mlen = (size_t)(b - a - 96);
    uint8_t h[64];
    sha512(h, tx, mlen);
    j->flags[i] = oracle_verify_flags(tx + mlen, tx + mlen + 32, h, 32);
  }
  return NULL;
}

int oracle_verify_tx_many(const uint8_t *txs, const uint64_t *offsets, size_t tx_size, size_t n, uint8_t *flags,
                          int nthreads) {
  pthread_once(&g_once, init_consts);
  if (nthreads < 1) nthreads = 1;
  if (nthreads > 256) nthreads = 256;
  pthread_t th[256];
  txjob_t jobs[256];
  for (int t = 0; t < nthreads; ++t) {
    jobs[t] = (txjob_t){txs, offsets, tx_size, n * t / nthreads, n * (t + 1) / nthreads, flags};
    pthread_create(&th[t], NULL, tx_worker, &jobs[t]);
  }
  for (int t = 0; t < nthreads; ++t) pthread_join(th[t], NULL);
  return 0;
}

/* ===================================================================== */
/* Fast mod-l arithmetic (Barrett, HAC 14.42 with b = 2^64, k = 4).       */
/* Cross-checked against the bit-serial sc_reduce64 in tests/test_oracle.  */
static const uint64_t L64[4] = {0x5812631a5cf5d3edull, 0x14def9dea2f79cd6ull, 0ull, 0x1000000000000000ull};
static const uint64_t MU64[5] = {0xed9ce5a30a2c131bull, 0x2106215d086329a7ull, 0xffffffffffffffebull,
                                 0xffffffffffffffffull, 0xfull};  /* floor(2^512 / l) */

static int geq_l(const uint64_t r[5]) {
  if (r[4]) return 1;
  for (int i = 3; i >= 0; --i) {
    if (r[i] > L64[i]) return 1;
    if (r[i] < L64[i]) return 0;
  }
  return 1;
}

/* x: 8 little-endian u64 limbs (< 2^512) -> x mod l in 4 limbs */
static void sc_barrett(uint64_t out[4], const uint64_t x[8]) {
  uint64_t q2[10] = {0};
  /* q2 = (x >> 192) * mu, only limbs >= 5 are needed but compute all */
  for (int i = 0; i < 5; ++i) {
    u128 c = 0;
    const uint64_t xi = x[3 + i];
    for (int j = 0; j < 5; ++j) {
      c += (u128)xi * MU64[j] + q2[i + j];
      q2[i + j] = (uint64_t)c;
      c >>= 64;
    }
    q2[i + 5] = (uint64_t)c;
  }
  const uint64_t *q3 = q2 + 5; /* q2 >> 320 */
  /* r2 = (q3 * l) mod 2^320 */
  uint64_t r2[5] = {0};
  for (int i = 0; i < 5; ++i) {
    u128 c = 0;
    for (int j = 0; i + j < 5 && j < 4; ++j) {
      c += (u128)q3[i] * L64[j] + r2[i + j];
      r2[i + j] = (uint64_t)c;
      c >>= 64;
    }
    if (i + 4 < 5) r2[i + 4] += (uint64_t)c;
  }
  /* r = (x mod 2^320) - r2 mod 2^320 */
  uint64_t r[5];
  u128 borrow = 0;
  for (int i = 0; i < 5; ++i) {
    const u128 t = (u128)x[i] - r2[i] - borrow;
    r[i] = (uint64_t)t;
    borrow = (t >> 64) ? 1 : 0;
  }
  while (geq_l(r)) {
    u128 b = 0;
    for (int i = 0; i < 5; ++i) {
      const u128 t = (u128)r[i] - (i < 4 ? L64[i] : 0) - b;
      r[i] = (uint64_t)t;
      b = (t >> 64) ? 1 : 0;
    }
  }
  memcpy(out, r, 32);
}

static void sc_from_bytes64(uint64_t out[8], const uint8_t x[64]) {
  for (int i = 0; i < 8; ++i) out[i] = load64(x + 8 * i);
}

static void sc_to_bytes(uint8_t out[32], const uint64_t s[4]) {
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 8; ++j) out[8 * i + j] = (uint8_t)(s[i] >> (8 * j));
}

static void sc_load(uint64_t s[4], const uint8_t b[32]) {
  for (int i = 0; i < 4; ++i) s[i] = load64(b + 8 * i);
}

/* (a * b) mod l for a, b < 2^256 */
static void sc_mul(uint64_t out[4], const uint64_t a[4], const uint64_t b[4]) {
  uint64_t p[8] = {0};
  for (int i = 0; i < 4; ++i) {
    u128 c = 0;
    for (int j = 0; j < 4; ++j) {
      c += (u128)a[i] * b[j] + p[i + j];
      p[i + j] = (uint64_t)c;
      c >>= 64;
    }
    p[i + 4] = (uint64_t)c;
  }
  sc_barrett(out, p);
}

/* (a + b) mod l for a, b < l */
static void sc_add(uint64_t out[4], const uint64_t a[4], const uint64_t b[4]) {
  uint64_t x[8] = {0};
  u128 c = 0;
  for (int i = 0; i < 4; ++i) {
    c += (u128)a[i] + b[i];
    x[i] = (uint64_t)c;
    c >>= 64;
  }
  x[4] = (uint64_t)c;
  sc_barrett(out, x);
}

/* exported for the cross-check test: both reductions of 64 bytes */
void oracle_sc_reduce64_fast(uint8_t out[32], const uint8_t x[64]) {
  uint64_t w[8], r[4];
  sc_from_bytes64(w, x);
  sc_barrett(r, w);
  sc_to_bytes(out, r);
}

void oracle_sc_reduce64_slow(uint8_t out[32], const uint8_t x[64]) { sc_reduce64(out, x); }

/* ===================================================================== */
/* ed25519-dalek 1.0.1 verify_batch (feature "batch"), the QC path of the  */
/* reference (crypto/src/lib.rs:210-223 -> dalek::verify_batch):           */
/*   parse every s (check_scalar) and A (PublicKey::from_bytes),           */
/*   k_i = SHA-512(R_i || A_i || M) mod l, random 128-bit z_i,             */
/*   [-sum z_i s_i]B + sum [z_i]R_i + sum [z_i k_i]A_i == O  (one MSM of   */
/*   2n+1 points; R_i decompressed inside the MSM's point list),           */
/*   curve25519-dalek 3.x VartimeMultiscalarMul: Straus with width-5 NAF   */
/*   tables below 190 points, Pippenger (w = 6/7/8 by size) above.         */
/* dalek draws z_i from a merlin transcript finalised with thread_rng; the */
/* port draws them from a seeded splitmix64 (same cost class, the verdict  */
/* differs only for pure-torsion failures).           */

static uint64_t splitmix64(uint64_t *s) {
  uint64_t z = (*s += 0x9e3779b97f4a7c15ull);
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}

/* Scalar::to_radix_2w (w in 5..8): signed digits in [-2^(w-1), 2^(w-1)) */
static int to_radix_2w(int16_t *digits, const uint64_t s[4], int w) {
  const uint64_t radix = 1ull << w, mask = radix - 1;
  const int count = (256 + w - 1) / w;
  uint64_t carry = 0;
  for (int i = 0; i < count; ++i) {
    const int bit_offset = i * w, u = bit_offset / 64, b = bit_offset % 64;
    uint64_t buf;
    if (b < 64 - w || u == 3) buf = s[u] >> b;
    else buf = (s[u] >> b) | (s[u + 1] << (64 - b));
    const uint64_t coef = carry + (buf & mask);
    carry = (coef + radix / 2) >> w;
    digits[i] = (int16_t)((int64_t)coef - (int64_t)(carry << w));
  }
  if (w == 8) {
    digits[count] = (int16_t)carry;
    return count + 1;
  }
  digits[count - 1] = (int16_t)(digits[count - 1] + (int16_t)(carry << w));
  return count;
}

static void ge_add_ext(ge *r, const ge *p, const ge *q) {
  ge_cached c;
  ge_to_cached(&c, q);
  ge_add(r, p, &c);
}

/* Straus: NAF width 5, tables [1,3,...,15]P per point */
static void msm_straus(ge *out, const uint64_t (*sc)[4], const ge *pts, size_t m) {
  int8_t(*nafs)[256] = malloc(m * sizeof *nafs);
  ge_cached(*tabs)[8] = malloc(m * sizeof *tabs);
  for (size_t i = 0; i < m; ++i) {
    uint8_t b[32];
    sc_to_bytes(b, sc[i]);
    naf(nafs[i], b, 5);
    ge p2, acc = pts[i];
    ge_cached c2;
    ge_dbl(&p2, &pts[i]);
    ge_to_cached(&c2, &p2);
    for (int k = 0; k < 8; ++k) {
      ge_to_cached(&tabs[i][k], &acc);
      ge_add(&acc, &acc, &c2);
    }
  }
  ge r;
  ge_identity(&r);
  for (int bit = 255; bit >= 0; --bit) {
    ge_dbl(&r, &r);
    for (size_t i = 0; i < m; ++i) {
      const int d = nafs[i][bit];
      if (d > 0) ge_add(&r, &r, &tabs[i][d / 2]);
      else if (d < 0) ge_sub(&r, &r, &tabs[i][-d / 2]);
    }
  }
  *out = r;
  free(nafs);
  free(tabs);
}

/* Pippenger: signed radix-2^w digits, 2^(w-1) buckets per column */
static void msm_pippenger(ge *out, const uint64_t (*sc)[4], const ge *pts, size_t m) {
  const int w = m < 500 ? 6 : (m < 800 ? 7 : 8);
  const int nb = 1 << (w - 1);
  int16_t(*digits)[64] = malloc(m * sizeof *digits);
  ge_cached *pc = malloc(m * sizeof *pc);
  int count = 0;
  for (size_t i = 0; i < m; ++i) {
    count = to_radix_2w(digits[i], sc[i], w);
    ge_to_cached(&pc[i], &pts[i]);
  }
  ge *buckets = malloc((size_t)nb * sizeof *buckets);
  ge total;
  ge_identity(&total);
  for (int col = count - 1; col >= 0; --col) {
    for (int b = 0; b < nb; ++b) ge_identity(&buckets[b]);
    for (size_t i = 0; i < m; ++i) {
      const int d = digits[i][col];
      if (d > 0) ge_add(&buckets[d - 1], &buckets[d - 1], &pc[i]);
      else if (d < 0) ge_sub(&buckets[-d - 1], &buckets[-d - 1], &pc[i]);
    }
    ge inter = buckets[nb - 1], sum = buckets[nb - 1];
    for (int b = nb - 2; b >= 0; --b) {
      ge_add_ext(&inter, &inter, &buckets[b]);
      ge_add_ext(&sum, &sum, &inter);
    }
    if (col == count - 1) {
      total = sum;
    } else {
      for (int k = 0; k < w; ++k) ge_dbl(&total, &total);
      ge_add_ext(&total, &total, &sum);
    }
  }
  *out = total;
  free(buckets);
  free(digits);
  free(pc);
}

/* 1 = Ok, 0 = Err, for dalek verify_batch over n (pk, sig, msg) triples with
 * 32-byte messages at msg + i * msg_stride (msg_stride 0: one shared digest,
 * crypto::Signature::verify_batch(digest, votes)) */
int oracle_verify_batch_dalek_msgs(const uint8_t *msg, size_t msg_stride, const uint8_t *pk, const uint8_t *sig,
                                   size_t n, uint64_t seed) {
  pthread_once(&g_once, init_consts);
  if (n == 0) return 1;
  const size_t m = 2 * n + 1;
  uint64_t(*sc)[4] = malloc(m * sizeof *sc);
  ge *pts = malloc(m * sizeof *pts);
  int ok = 1;
  uint64_t bcoef[4] = {0, 0, 0, 0};
  uint64_t rng = seed;
  for (size_t i = 0; i < n && ok; ++i) {
    const uint8_t *p = pk + 32 * i, *s = sig + 64 * i;
    if (!sc_canonical(s + 32)) { ok = 0; break; }          /* InternalSignature::try_from */
    if (!ge_decompress(&pts[1 + n + i], p)) { ok = 0; break; } /* PublicKey::from_bytes (glue) */
    if (!ge_decompress(&pts[1 + i], s)) { ok = 0; break; }     /* R inside the MSM point list */
    uint8_t buf[96], h[64];
    memcpy(buf, s, 32);
    memcpy(buf + 32, p, 32);
    memcpy(buf + 64, msg + msg_stride * i, 32);
    sha512(h, buf, 96);
    uint64_t hw[8], k[4], sv[4], z[4] = {0, 0, 0, 0}, t[4];
    sc_from_bytes64(hw, h);
    sc_barrett(k, hw);                                       /* Scalar::from_hash */
    sc_load(sv, s + 32);
    z[0] = splitmix64(&rng);
    z[1] = splitmix64(&rng);
    memcpy(sc[1 + i], z, 32);                                /* z_i R_i */
    sc_mul(sc[1 + n + i], z, k);                             /* z_i k_i A_i */
    sc_mul(t, z, sv);
    sc_add(bcoef, bcoef, t);                                 /* sum z_i s_i */
  }
  if (ok) {
    /* -B_coefficient */
    uint64_t zero[4] = {0, 0, 0, 0}, negb[4];
    if (memcmp(bcoef, zero, 32) == 0) {
      memset(negb, 0, 32);
    } else {
      u128 b = 0;
      for (int i = 0; i < 4; ++i) {
        const u128 t = (u128)L64[i] - bcoef[i] - b;
        negb[i] = (uint64_t)t;
        b = (t >> 64) ? 1 : 0;
      }
    }
    memcpy(sc[0], negb, 32);
    uint8_t by[32];
    memset(by, 0x66, 32);
    by[0] = 0x58;
    ge_decompress(&pts[0], by);
    ge r;
    if (m < 190) msm_straus(&r, (const uint64_t(*)[4])sc, pts, m);
    else msm_pippenger(&r, (const uint64_t(*)[4])sc, pts, m);
    ok = ge_is_identity(&r);
  }
  free(sc);
  free(pts);
  return ok;
}

int oracle_verify_batch_dalek(const uint8_t digest[32], const uint8_t *pk, const uint8_t *sig, size_t n,
                              uint64_t seed) {
  return oracle_verify_batch_dalek_msgs(digest, 0, pk, sig, n, seed);
}

/* Per-item accept vector the batch way (BASELINE.md CPU plan for C4/C5):
 * chunks of 64 through verify_batch; a chunk that fails is re-verified item
 * by item with verify_strict.  Fills flags with STRICT_OK bits only (1 / 0)
 * for the chunk-accepted items and the full flag byte for re-verified ones;
 * nthreads host threads over contiguous chunk ranges. */
typedef struct {
  const uint8_t *pk, *sig, *msg;
  size_t lo, hi;
  uint8_t *flags;
  uint64_t fallback_chunks;
} b64job_t;

static void *b64_worker(void *arg) {
  b64job_t *j = (b64job_t *)arg;
  for (size_t c = j->lo; c < j->hi; c += 64) {
    const size_t m = (j->hi - c) < 64 ? (j->hi - c) : 64;
    if (oracle_verify_batch_dalek_msgs(j->msg + 32 * c, 32, j->pk + 32 * c, j->sig + 64 * c, m, 0x5eed + c)) {
      memset(j->flags + c, STRICT_OK, m);
    } else {
      ++j->fallback_chunks;
      for (size_t i = c; i < c + m; ++i)
        j->flags[i] = oracle_verify_flags(j->pk + 32 * i, j->sig + 64 * i, j->msg + 32 * i, 32);
    }
  }
  return NULL;
}

uint64_t oracle_verify_many_batch64(const uint8_t *pk, const uint8_t *sig, const uint8_t *msg, size_t n,
                                    uint8_t *flags, int nthreads) {
  pthread_once(&g_once, init_consts);
  if (nthreads < 1) nthreads = 1;
  if (nthreads > 256) nthreads = 256;
  pthread_t th[256];
  b64job_t jobs[256];
  const size_t chunks = (n + 63) / 64;
  for (int t = 0; t < nthreads; ++t) {
    size_t lo = chunks * t / nthreads * 64, hi = chunks * (t + 1) / nthreads * 64;
    if (hi > n) hi = n;
    if (lo > n) lo = n;
    jobs[t] = (b64job_t){pk, sig, msg, lo, hi, flags, 0};
    pthread_create(&th[t], NULL, b64_worker, &jobs[t]);
  }
  uint64_t fb = 0;
  for (int t = 0; t < nthreads; ++t) {
    pthread_join(th[t], NULL);
    fb += jobs[t].fallback_chunks;
  }
  return fb;
}

/* consensus TC::verify's signature loop (consensus/src/messages.rs:307-313):
 * Signature::verify per vote over its own digest, in order, stopping at the
 * first failure.  1 = all Ok. */
int oracle_tc_verify(const uint8_t *pk, const uint8_t *sig, const uint8_t *digests, size_t n) {
  pthread_once(&g_once, init_consts);
  for (size_t i = 0; i < n; ++i)
    if (!(oracle_verify_flags(pk + 32 * i, sig + 64 * i, digests + 32 * i, 32) & STRICT_OK)) return 0;
  return 1;
}
