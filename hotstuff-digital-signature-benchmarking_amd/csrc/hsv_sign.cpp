// Host-side key generation and signing (RFC 8032 Ed25519), the CPU part of
// the reference's crypto API that the hot path does not cover:
//   crypto::generate_keypair  (reference crypto/src/lib.rs:167-175)
//   crypto::Signature::new    (reference crypto/src/lib.rs:185-191)
// Used by callers that sign, and by bench.py / tests to synthesise inputs.
// Fixed-base multiplication uses a per-position table
//   T[j][m] = [m * 256^j]B,  j < 32, m in 1..128   (cached form, built once)
// so [a]B costs 32 cached additions and one inversion for the encoding.
#include <cstring>
#include <mutex>
#include <thread>
#include <vector>

#include "hsv.h"
#include "hsv_point.hpp"
#include "hsv_scalar.hpp"
#include "hsv_sha512.hpp"

using namespace hsv;

namespace {

constexpr int kPos = 32, kEnt = 128;

std::vector<ge_cached> &fixed_base_table() {
  static std::vector<ge_cached> tab;
  static std::once_flag once;
  std::call_once(once, []() {
    tab.resize(kPos * kEnt);
    // B in extended coordinates
    const uint32_t by_words[8] = {0x66666658u, 0x66666666u, 0x66666666u, 0x66666666u,
                                  0x66666666u, 0x66666666u, 0x66666666u, 0x66666666u};
    fe bx, by;
    (void)ge_decompress(by_words, bx, by);
    ge_ext base;
    base.X = bx;
    base.Y = by;
    base.Z = fe_small(1);
    base.T = fe_mul(bx, by);
    for (int j = 0; j < kPos; ++j) {
      const ge_cached c1 = ge_to_cached(base);
      ge_ext acc = base;
      tab[j * kEnt + 0] = c1;
      for (int m = 2; m <= kEnt; ++m) {
        acc = ge_add_cached<true>(acc, c1);
        tab[j * kEnt + m - 1] = ge_to_cached(acc);
      }
      // next position: base * 256 = 2 * (128 * base)
      base = ge_dbl<true>(acc);
    }
  });
  return tab;
}

// [a]B for a < l (a as 8 little-endian limbs)
ge_ext fixed_base_mul(const sc &a) {
  const std::vector<ge_cached> &tab = fixed_base_table();
  // signed radix-256 digits via the recoding constant C8 = sum 128 * 256^j
  uint32_t r[9];
  uint64_t t = 0;
  for (int j = 0; j < 9; ++j) {
    uint32_t c = 0;
    for (int b = 0; b < 32; ++b) {
      const int bit = 32 * j + b;
      if (bit < 8 * kPos && bit % 8 == 7) c |= 1u << b;
    }
    t += (uint64_t)(j < 8 ? a.v[j] : 0u) + c;
    r[j] = (uint32_t)t;
    t >>= 32;
  }
  ge_ext q = ge_identity();
  for (int j = 0; j < kPos; ++j) {
    const int chunk = (int)((r[j / 4] >> (8 * (j % 4))) & 0xffu);
    const int d = chunk - 128;
    const uint32_t neg = d < 0;
    const int mag = neg ? -d : d;
    ge_cached c = mag ? tab[j * kEnt + mag - 1] : ge_cached_identity();
    q = ge_add_cached<true>(q, ge_cached_cneg(c, neg));
  }
  return q;
}

void words_to_bytes(const uint32_t *w, uint8_t *b, int nwords) {
  for (int i = 0; i < nwords; ++i)
    for (int k = 0; k < 4; ++k) b[4 * i + k] = (uint8_t)(w[i] >> (8 * k));
}

void bytes_to_words(const uint8_t *b, uint32_t *w, int nwords) {
  for (int i = 0; i < nwords; ++i)
    w[i] = (uint32_t)b[4 * i] | ((uint32_t)b[4 * i + 1] << 8) | ((uint32_t)b[4 * i + 2] << 16) |
           ((uint32_t)b[4 * i + 3] << 24);
}

sc reduce_bytes64(const uint8_t h[64]) {
  uint32_t w[16];
  bytes_to_words(h, w, 16);
  return sc_reduce512(w);
}

struct Expanded {
  sc a;             // clamped secret scalar reduced mod l
  uint8_t prefix[32];
  uint8_t pk[32];
};

void expand(const uint8_t seed[32], Expanded &e) {
  uint8_t h[64];
  sha512_bytes(seed, 32, h);
  h[0] &= 248;
  h[31] &= 127;
  h[31] |= 64;
  uint8_t wide[64] = {0};
  std::memcpy(wide, h, 32);
  e.a = reduce_bytes64(wide);
  std::memcpy(e.prefix, h + 32, 32);
  uint32_t enc[8];
  ge_compress(fixed_base_mul(e.a), enc);
  words_to_bytes(enc, e.pk, 8);
}

void sign_expanded(const Expanded &e, const uint8_t *msg, size_t len, uint8_t sig[64]) {
  std::vector<uint8_t> buf(64 + len);
  std::memcpy(buf.data(), e.prefix, 32);
  std::memcpy(buf.data() + 32, msg, len);
  uint8_t h[64];
  sha512_bytes(buf.data(), 32 + len, h);
  const sc r = reduce_bytes64(h);
  uint32_t renc[8];
  ge_compress(fixed_base_mul(r), renc);
  words_to_bytes(renc, sig, 8);
  std::memcpy(buf.data(), sig, 32);
  std::memcpy(buf.data() + 32, e.pk, 32);
  std::memcpy(buf.data() + 64, msg, len);
  sha512_bytes(buf.data(), 64 + len, h);
  const sc k = reduce_bytes64(h);
  const sc s = sc_muladd(k, e.a, r);
  words_to_bytes(s.v, sig + 32, 8);
}

// [t]T8 for a point T8 of order 8 (encoding c7176a70...ac037a, one of the
// eight torsion points), t in 1..7
ge_ext torsion_multiple(int t) {
  const uint8_t enc[32] = {0xc7, 0x17, 0x6a, 0x70, 0x3d, 0x4d, 0xd8, 0x4f, 0xba, 0x3c, 0x0b,
                           0x76, 0x0d, 0x10, 0x67, 0x0f, 0x2a, 0x20, 0x53, 0xfa, 0x2c, 0x39,
                           0xcc, 0xc6, 0x4e, 0xc7, 0xfd, 0x77, 0x92, 0xac, 0x03, 0x7a};
  uint32_t w[8];
  bytes_to_words(enc, w, 8);
  fe x, y;
  (void)ge_decompress(w, x, y);
  ge_ext p;
  p.X = x;
  p.Y = y;
  p.Z = fe_small(1);
  p.T = fe_mul(x, y);
  const ge_cached c = ge_to_cached(p);
  ge_ext q = p;
  for (int i = 1; i < t; ++i) q = ge_add_cached<true>(q, c);
  return q;
}

}  // namespace

extern "C" {

// Synthesis helper (not on the hot path): a
// mixed-order key A' = [a]B + [t]T8 (a from `seed` as in hsv_public_key, T8 of
// order 8, t odd: 2 * torsion + 1) and a signature over msg whose challenge
// k = SHA-512(R || A' || msg) mod l satisfies k = 0 (mod 8) when accept != 0
// -- then [s]B - [k]A' = R and verify_strict accepts (cofactorless) -- or
// k != 0 (mod 8) when accept == 0, where only a cofactored verifier would
// accept.  The nonce is RFC 8032's r = SHA-512(prefix || msg) for the first
// try and SHA-512(prefix || msg || try) after it (deterministic).
int hsv_sign_mixed_order(const uint8_t seed[32], const uint8_t *msg, size_t msg_len, int torsion, int accept,
                         uint8_t pk_out[32], uint8_t sig_out[64]) {
  if (!seed || (!msg && msg_len) || !pk_out || !sig_out || torsion < 0 || torsion > 3) return HSV_ERR_INVALID_ARG;
  (void)fixed_base_table();
  Expanded e;
  expand(seed, e);
  const ge_ext ap = ge_add_cached<true>(fixed_base_mul(e.a), ge_to_cached(torsion_multiple(2 * torsion + 1)));
  uint32_t enc[8];
  ge_compress(ap, enc);
  uint8_t pk[32];
  words_to_bytes(enc, pk, 8);
  std::vector<uint8_t> buf(96 + msg_len + 4);
  for (uint32_t attempt = 0; attempt < 4096; ++attempt) {
    std::memcpy(buf.data(), e.prefix, 32);
    if (msg_len) std::memcpy(buf.data() + 32, msg, msg_len);
    size_t len = 32 + msg_len;
    if (attempt) {
      for (int b = 0; b < 4; ++b) buf[len + b] = (uint8_t)(attempt >> (8 * b));
      len += 4;
    }
    uint8_t h[64];
    sha512_bytes(buf.data(), len, h);
    const sc r = reduce_bytes64(h);
    uint32_t renc[8];
    ge_compress(fixed_base_mul(r), renc);
    uint8_t sig[64];
    words_to_bytes(renc, sig, 8);
    std::memcpy(buf.data(), sig, 32);
    std::memcpy(buf.data() + 32, pk, 32);
    if (msg_len) std::memcpy(buf.data() + 64, msg, msg_len);
    sha512_bytes(buf.data(), 64 + msg_len, h);
    const sc k = reduce_bytes64(h);
    if (((k.v[0] & 7u) == 0) != (accept != 0)) continue;
    const sc s = sc_muladd(k, e.a, r);
    words_to_bytes(s.v, sig + 32, 8);
    std::memcpy(pk_out, pk, 32);
    std::memcpy(sig_out, sig, 64);
    return HSV_OK;
  }
  return HSV_ERR_INVALID_ARG;  // unreachable in practice (2^-550 for accept)
}

int hsv_public_key(const uint8_t seed[32], uint8_t pk_out[32]) {
  if (!seed || !pk_out) return HSV_ERR_INVALID_ARG;
  Expanded e;
  expand(seed, e);
  std::memcpy(pk_out, e.pk, 32);
  return HSV_OK;
}

int hsv_sign(const uint8_t seed[32], const uint8_t *msg, size_t msg_len, uint8_t sig_out[64]) {
  if (!seed || (!msg && msg_len) || !sig_out) return HSV_ERR_INVALID_ARG;
  Expanded e;
  expand(seed, e);
  sign_expanded(e, msg, msg_len, sig_out);
  return HSV_OK;
}

int hsv_sign_many(const uint8_t *seeds, const uint8_t *msgs, size_t msg_len, size_t n,
                  uint8_t *pk_out, uint8_t *sig_out, int nthreads) {
  if (n == 0) return HSV_OK;
  if (!seeds || (!msgs && msg_len) || !sig_out) return HSV_ERR_INVALID_ARG;
  (void)fixed_base_table();
  unsigned nt = nthreads > 0 ? (unsigned)nthreads : std::thread::hardware_concurrency();
  if (nthreads <= 0 && nt > 16) nt = 16;  // default: one GPU box's CPU share
  if (nt == 0) nt = 1;
  if ((size_t)nt > n) nt = (unsigned)n;
  std::vector<std::thread> th;
  for (unsigned t = 0; t < nt; ++t) {
    th.emplace_back([=]() {
      const size_t lo = n * t / nt, hi = n * (t + 1) / nt;
      for (size_t i = lo; i < hi; ++i) {
        Expanded e;
        expand(seeds + 32 * i, e);
        if (pk_out) std::memcpy(pk_out + 32 * i, e.pk, 32);
        sign_expanded(e, msgs + msg_len * i, msg_len, sig_out + 64 * i);
      }
    });
  }
  for (auto &x : th) x.join();
  return HSV_OK;
}

}  // extern "C"
