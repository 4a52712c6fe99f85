// SHA-512 (FIPS 180-4) specialised for the verification challenge
//   k = SHA-512(R || A || M) mod l
// On the hot path every message M is a 32-byte consensus Digest
// (reference crypto/src/lib.rs:22, signed as &digest.0 at lib.rs:185-191), so
// the input is exactly 96 bytes and the padded message is ONE 1024-bit block:
//   W[0..11] = R||A||M (big-endian 64-bit words), W[12] = 0x80 << 56,
//   W[13..14] = 0, W[15] = 768 (bit length).
// A generic multi-block variant (sha512_bytes) is kept for host-side signing.
#pragma once
#include "hsv_field.hpp"

// Host builds (g++: signing, the wire parser's certificate digests): the
// round and rotate helpers inlined, or each of the 80 rounds is a call that
// passes the state through memory (1.3 us per block on the container's host
// against ~0.4 us inlined).
#if defined(__HIPCC__)
#define HSV_SHA_INL HSV_INL
#else
#define HSV_SHA_INL static inline __attribute__((always_inline))
#endif

namespace hsv {

#if defined(__HIP_DEVICE_COMPILE__)
__constant__ static const uint64_t kSha512K[80] = {
#else
static const uint64_t kSha512K[80] = {
#endif
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

// 64-bit rotate; on gfx950 two v_alignbit_b32 on the halves (n is a constant
// at every call site, so the branch folds)
HSV_SHA_INL uint64_t sha_rotr(uint64_t x, int n) {
#if defined(__HIP_DEVICE_COMPILE__)
  const uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
  if (n < 32)
    return ((uint64_t)__builtin_amdgcn_alignbit(lo, hi, n) << 32) | __builtin_amdgcn_alignbit(hi, lo, n);
  return ((uint64_t)__builtin_amdgcn_alignbit(hi, lo, n - 32) << 32) | __builtin_amdgcn_alignbit(lo, hi, n - 32);
#else
  return (x >> n) | (x << (64 - n));
#endif
}

HSV_SHA_INL uint32_t bswap32(uint32_t x) {
  return (x >> 24) | ((x >> 8) & 0x0000ff00u) | ((x << 8) & 0x00ff0000u) | (x << 24);
}

HSV_SHA_INL void sha512_init(uint64_t h[8]) {
  h[0] = 0x6a09e667f3bcc908ull; h[1] = 0xbb67ae8584caa73bull;
  h[2] = 0x3c6ef372fe94f82bull; h[3] = 0xa54ff53a5f1d36f1ull;
  h[4] = 0x510e527fade682d1ull; h[5] = 0x9b05688c2b3e6c1full;
  h[6] = 0x1f83d9abfb41bd6bull; h[7] = 0x5be0cd19137e2179ull;
}

// Three-input bit functions of the 32-bit halves.  gfx950's v_bitop3_b32
// evaluates any 3-input function in one instruction (imm = its truth table
// over A = 0xf0, B = 0xcc, C = 0xaa): x ^ y ^ z is 0x96, maj 0xe8, ch 0xca.
// Without it the compiler forms v_bfi_b32 for ch but keeps the XOR pairs of
// the four sigma functions and the majority as two or three instructions.
// HSV_SHA_BITOP3=1 selects the v_bitop3 form: the mempool
// kernels define it (csrc/hsv_mempool.hip); the other translation units keep
// the XOR form.
#ifndef HSV_SHA_BITOP3
#define HSV_SHA_BITOP3 0
#endif
template <uint32_t IMM>
HSV_SHA_INL uint64_t sha_bitop3(uint64_t x, uint64_t y, uint64_t z) {
#if defined(__HIP_DEVICE_COMPILE__) && HSV_SHA_BITOP3
  const uint32_t lo = __builtin_amdgcn_bitop3_b32((uint32_t)x, (uint32_t)y, (uint32_t)z, IMM);
  const uint32_t hi = __builtin_amdgcn_bitop3_b32((uint32_t)(x >> 32), (uint32_t)(y >> 32), (uint32_t)(z >> 32), IMM);
  uint64_t r = ((uint64_t)hi << 32) | lo;
  // opaque pair: otherwise the compiler splits the 64-bit adds that consume
  // r into a low add, a separate high-half add and a v_mov (more instructions
  // than the XORs the bitop3 saves)
  asm("" : "+v"(r));
  return r;
#else
  if constexpr (IMM == 0x96) return x ^ y ^ z;
  if constexpr (IMM == 0xe8) return (x & y) ^ (x & z) ^ (y & z);
  if constexpr (IMM == 0xca) return (x & y) ^ (~x & z);
  return 0;
#endif
}
HSV_SHA_INL uint64_t sha_xor3(uint64_t x, uint64_t y, uint64_t z) { return sha_bitop3<0x96>(x, y, z); }

// One SHA-512 round with message word wj and round constant kj.
HSV_SHA_INL void sha512_round(uint64_t &a, uint64_t &b, uint64_t &c, uint64_t &d, uint64_t &e, uint64_t &f,
                          uint64_t &g, uint64_t &hh, uint64_t wj, uint64_t kj) {
  const uint64_t S1 = sha_xor3(sha_rotr(e, 14), sha_rotr(e, 18), sha_rotr(e, 41));
  const uint64_t ch = sha_bitop3<0xca>(e, f, g);  // (e & f) ^ (~e & g)
  const uint64_t t1 = hh + S1 + ch + kj + wj;
  const uint64_t S0 = sha_xor3(sha_rotr(a, 28), sha_rotr(a, 34), sha_rotr(a, 39));
  const uint64_t mj = sha_bitop3<0xe8>(a, b, c);  // (a & b) ^ (a & c) ^ (b & c)
  hh = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + S0 + mj;
}

// One compression of the 16-word block w (big-endian words already assembled).
// Rounds 0-15 use w directly; rounds 16-79 run as a loop of four 16-round
// groups that extend the schedule in place.  No branch inside a group: a
// per-round "first group?" test made the compiler copy the whole w array and
// state through phi moves every round.
HSV_SHA_INL void sha512_compress(uint64_t h[8], uint64_t w[16]) {
  uint64_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
  HSV_UNROLL
  for (int j = 0; j < 16; ++j) {
    sha512_round(a, b, c, d, e, f, g, hh, w[j], kSha512K[j]);
    // 16 rounds rotate the eight state names back to where they started
  }
  HSV_NOUNROLL
  for (int blk = 1; blk < 5; ++blk) {
    HSV_UNROLL
    for (int j = 0; j < 16; ++j) {
      const uint64_t w15 = w[(j + 1) & 15], w2 = w[(j + 14) & 15];
      const uint64_t s0 = sha_xor3(sha_rotr(w15, 1), sha_rotr(w15, 8), w15 >> 7);
      const uint64_t s1 = sha_xor3(sha_rotr(w2, 19), sha_rotr(w2, 61), w2 >> 6);
      const uint64_t wj = w[j] + s0 + w[(j + 9) & 15] + s1;
      w[j] = wj;
      sha512_round(a, b, c, d, e, f, g, hh, wj, kSha512K[blk * 16 + j]);
    }
  }
  h[0] += a; h[1] += b; h[2] += c; h[3] += d;
  h[4] += e; h[5] += f; h[6] += g; h[7] += hh;
}

// The same compression with one 16-round body: five passes of 16 rounds,
// each followed (but the last) by a separate extension of the schedule.  Same
// instruction count, about half the code: the latency kernels' lone waves
// execute it once, with every instruction fetched cold.
HSV_SHA_INL void sha512_compress_compact(uint64_t h[8], uint64_t w[16]) {
  uint64_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
  HSV_NOUNROLL
  for (int blk = 0; blk < 5; ++blk) {
    HSV_UNROLL
    for (int j = 0; j < 16; ++j) sha512_round(a, b, c, d, e, f, g, hh, w[j], kSha512K[blk * 16 + j]);
    if (blk == 4) break;
    HSV_UNROLL
    for (int j = 0; j < 16; ++j) {
      const uint64_t w15 = w[(j + 1) & 15], w2 = w[(j + 14) & 15];
      const uint64_t s0 = sha_xor3(sha_rotr(w15, 1), sha_rotr(w15, 8), w15 >> 7);
      const uint64_t s1 = sha_xor3(sha_rotr(w2, 19), sha_rotr(w2, 61), w2 >> 6);
      w[j] = w[j] + s0 + w[(j + 9) & 15] + s1;
    }
  }
  h[0] += a; h[1] += b; h[2] += c; h[3] += d;
  h[4] += e; h[5] += f; h[6] += g; h[7] += hh;
}

// Big-endian 64-bit word from two little-endian 32-bit loads of bytes b0..b7.
HSV_SHA_INL uint64_t be64_from_le32(uint32_t lo_bytes, uint32_t hi_bytes) {
  return ((uint64_t)bswap32(lo_bytes) << 32) | bswap32(hi_bytes);
}

// SHA-512 over R(32) || A(32) || M(32), each given as 8 little-endian words.
// Output: the 64-byte digest as 16 little-endian 32-bit limbs (the 512-bit
// little-endian integer that Scalar::from_hash reduces).
template <bool Compact = false>
HSV_SHA_INL void sha512_96(const uint32_t r[8], const uint32_t a[8], const uint32_t m[8],
                       uint32_t out[16]) {
  uint64_t w[16];
  HSV_UNROLL
  for (int i = 0; i < 4; ++i) {
    w[i] = be64_from_le32(r[2 * i], r[2 * i + 1]);
    w[4 + i] = be64_from_le32(a[2 * i], a[2 * i + 1]);
    w[8 + i] = be64_from_le32(m[2 * i], m[2 * i + 1]);
  }
  w[12] = 0x8000000000000000ull;
  w[13] = 0;
  w[14] = 0;
  w[15] = 768;
  uint64_t h[8];
  sha512_init(h);
#ifdef HSV_TIMING_STUB_SHA  // tools/phase_probe.py only: wrong results, timing share of SHA-512
  for (int i = 0; i < 8; ++i) h[i] ^= w[i] + w[i + 4];
#else
  if constexpr (Compact) sha512_compress_compact(h, w);
  else sha512_compress(h, w);
#endif
  HSV_UNROLL
  for (int i = 0; i < 8; ++i) {
    out[2 * i] = bswap32((uint32_t)(h[i] >> 32));
    out[2 * i + 1] = bswap32((uint32_t)h[i]);
  }
}

// Generic SHA-512 of a byte string (host-side signing / key expansion).
// Padded length = len + 1 (0x80) + zeros + 16 (length field), rounded to 128.
HSV_SHA_INL void sha512_bytes(const uint8_t *msg, uint64_t len, uint8_t out[64]) {
  uint64_t h[8];
  sha512_init(h);
  uint64_t w[16];
  const uint64_t nblocks = (len + 1 + 16 + 127) / 128;
  for (uint64_t b = 0; b < nblocks; ++b) {
    uint8_t block[128];
    for (int i = 0; i < 128; ++i) {
      const uint64_t pos = b * 128 + (uint64_t)i;
      uint8_t byte = 0;
      if (pos < len) byte = msg[pos];
      else if (pos == len) byte = 0x80;
      block[i] = byte;
    }
    if (b + 1 == nblocks) {
      const uint64_t bits = len * 8;
      for (int i = 0; i < 8; ++i) block[127 - i] = (uint8_t)(bits >> (8 * i));
    }
    for (int i = 0; i < 16; ++i) {
      uint64_t x = 0;
      for (int j = 0; j < 8; ++j) x = (x << 8) | block[8 * i + j];
      w[i] = x;
    }
    sha512_compress(h, w);
  }
  for (int i = 0; i < 8; ++i)
    for (int j = 0; j < 8; ++j) out[8 * i + j] = (uint8_t)(h[i] >> (56 - 8 * j));
}

}  // namespace hsv
