// Bincode parsers of QC / TC certificates (see hsv_wire_parse.h).
//
// Layouts (bincode 1.3 default options: little-endian, fixed-width integers,
// u64 length prefixes; the serde derives of the reference):
//   Digest            32 raw bytes            crypto/src/lib.rs:20-22
//   PublicKey         str: u64 len + base64   crypto/src/lib.rs:94-101
//   Signature         part1 (32) || part2 (32) crypto/src/lib.rs:176-182
//   QC  = hash: Digest | round: u64 | votes: Vec<(PublicKey, Signature)>
//   TC  = round: u64 | votes: Vec<(PublicKey, Signature, Round)>
// PublicKey::decode_base64 (crypto/src/lib.rs:73-79) runs base64 0.13's
// standard decoder and keeps the first 32 bytes; shorter decodings are an
// error.  This decoder follows the same rules: standard alphabet, optional
// '=' padding only at the end, no non-zero trailing bits.
#include "hsv_wire_parse.h"

#include <algorithm>
#include <array>
#include <cstring>
#include <unordered_map>

#if defined(__x86_64__) && !defined(HSVW_SCALAR_B64)
#include <immintrin.h>
#endif

#include "hsv_sha512.hpp"

namespace hsvw {
namespace {

struct Reader {
  const uint8_t *p;
  size_t left;
  bool u64(uint64_t &v) {
    if (left < 8) return false;
    v = 0;
    for (int i = 7; i >= 0; --i) v = (v << 8) | p[i];
    p += 8;
    left -= 8;
    return true;
  }
  bool bytes(const uint8_t *&out, size_t n) {
    if (left < n) return false;
    out = p;
    p += n;
    left -= n;
    return true;
  }
};

// base64 standard alphabet: value of each byte, 0xff for none
struct B64Table {
  uint8_t v[256];
  B64Table() {
    std::memset(v, 0xff, sizeof(v));
    const char *a = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/";
    for (int i = 0; i < 64; ++i) v[(uint8_t)a[i]] = (uint8_t)i;
  }
};
const B64Table kB64;

#if defined(__x86_64__) && !defined(HSVW_SCALAR_B64)
// 16 base64 characters -> 12 bytes with SSSE3 (nibble-table validation and
// translation, then two multiply-adds pack four 6-bit values into 3 bytes);
// false if any of the 16 is outside the standard alphabet ('=' included).
// A public key's 44-character string is two such blocks plus three quads, so
// a C3 QC's 667 keys decode in a fraction of the scalar loop's time.
__attribute__((target("ssse3"))) bool b64_block16(const uint8_t *s, uint8_t out[16]) {
  const __m128i in = _mm_loadu_si128(reinterpret_cast<const __m128i *>(s));
  const __m128i nib = _mm_set1_epi8(0x0f);
  const __m128i hi = _mm_and_si128(_mm_srli_epi32(in, 4), nib);
  const __m128i lo = _mm_and_si128(in, nib);
  // a character is valid iff lut_lo[lo] & lut_hi[hi] == 0
  const __m128i lut_lo = _mm_setr_epi8(0x15, 0x11, 0x11, 0x11, 0x11, 0x11, 0x11, 0x11, 0x11, 0x11, 0x13, 0x1a,
                                       0x1b, 0x1b, 0x1b, 0x1a);
  const __m128i lut_hi = _mm_setr_epi8(0x10, 0x10, 0x01, 0x02, 0x04, 0x08, 0x04, 0x08, 0x10, 0x10, 0x10, 0x10,
                                       0x10, 0x10, 0x10, 0x10);
  const __m128i bad = _mm_and_si128(_mm_shuffle_epi8(lut_lo, lo), _mm_shuffle_epi8(lut_hi, hi));
  if (_mm_movemask_epi8(_mm_cmpeq_epi8(bad, _mm_setzero_si128())) != 0xffff) return false;
  // value = c + roll[hi], with '/' (the one character of its nibble row
  // below '+') taking roll[hi - 1]
  const __m128i lut_roll = _mm_setr_epi8(0, 16, 19, 4, -65, -65, -71, -71, 0, 0, 0, 0, 0, 0, 0, 0);
  const __m128i slash = _mm_cmpeq_epi8(in, _mm_set1_epi8('/'));
  const __m128i v = _mm_add_epi8(in, _mm_shuffle_epi8(lut_roll, _mm_add_epi8(slash, hi)));
  // [a b c d] -> a<<18 | b<<12 | c<<6 | d per dword, then big-endian bytes
  const __m128i ab_cd = _mm_maddubs_epi16(v, _mm_set1_epi32(0x01400140));
  const __m128i abcd = _mm_madd_epi16(ab_cd, _mm_set1_epi32(0x00011000));
  const __m128i packed = _mm_shuffle_epi8(abcd, _mm_setr_epi8(2, 1, 0, 6, 5, 4, 10, 9, 8, 14, 13, 12, -1, -1, -1, -1));
  _mm_storeu_si128(reinterpret_cast<__m128i *>(out), packed);
  return true;
}

// (a static initializer: the cpu model must be initialised first)
const bool kHaveSsse3 = (__builtin_cpu_init(), __builtin_cpu_supports("ssse3"));
#endif

// Decodes s[0, n) under b64_decode's rules, keeping the first `keep` bytes in
// out; returns the decoded length, or -1 for an invalid string.
long b64_decode_prefix(const uint8_t *s, size_t n, uint8_t *out, size_t keep) {
  size_t end = n;
  while (end > 0 && s[end - 1] == '=') --end;
  if (n - end > 2) return -1;
  if (n != end && n % 4 != 0) return -1;  // padded input comes in whole quads
  const size_t rem = end % 4;
  if (rem == 1) return -1;
  size_t o = 0, i = 0;
  uint8_t bad = 0;
#if defined(__x86_64__) && !defined(HSVW_SCALAR_B64)
  if (kHaveSsse3) {  // whole 16-character blocks of the unpadded quads
    for (; i + 16 <= end - rem; i += 16) {
      uint8_t t[16];
      if (!b64_block16(s + i, t)) return -1;  // the quad loop below would reject it too
      if (o < keep) std::memcpy(out + o, t, std::min<size_t>(12, keep - o));
      o += 12;
    }
  }
#endif
  for (; i + 4 <= end; i += 4) {  // whole quads: 3 bytes each
    const uint8_t a = kB64.v[s[i]], b = kB64.v[s[i + 1]], c = kB64.v[s[i + 2]], d = kB64.v[s[i + 3]];
    bad |= a | b | c | d;
    const uint32_t q = ((uint32_t)a << 18) | ((uint32_t)b << 12) | ((uint32_t)c << 6) | d;
    if (o + 3 <= keep) {
      out[o] = (uint8_t)(q >> 16);
      out[o + 1] = (uint8_t)(q >> 8);
      out[o + 2] = (uint8_t)q;
    } else {
      for (int k = 0; k < 3; ++k)
        if (o + k < keep) out[o + k] = (uint8_t)(q >> (16 - 8 * k));
    }
    o += 3;
  }
  if (bad & 0xc0) return -1;  // a byte outside the alphabet (0xff) in a quad
  uint32_t acc = 0;
  int bits = 0;
  for (; i < end; ++i) {  // the last 2 or 3 characters
    const uint8_t v = kB64.v[s[i]];
    if (v > 63) return -1;
    acc = (acc << 6) | v;
    bits += 6;
    if (bits >= 8) {
      bits -= 8;
      if (o < keep) out[o] = (uint8_t)(acc >> bits);
      ++o;
      acc &= (1u << bits) - 1u;
    }
  }
  if (acc != 0) return -1;  // the leftover (trailing) bits must be zero
  return (long)o;
}

// PublicKey from its bincode str
bool read_public_key(Reader &r, uint8_t pk[32]) {
  uint64_t len = 0;
  const uint8_t *s = nullptr;
  if (!r.u64(len) || len > r.left || !r.bytes(s, (size_t)len)) return false;
  return b64_decode_prefix(s, (size_t)len, pk, 32) >= 32;
}

void put_le64(uint8_t *p, uint64_t v) {
  for (int b = 0; b < 8; ++b) p[b] = (uint8_t)(v >> (8 * b));
}

}  // namespace

bool b64_decode(const uint8_t *s, size_t n, std::vector<uint8_t> &out) {
  out.assign(n / 4 * 3 + 3, 0);
  const long m = b64_decode_prefix(s, n, out.data(), out.size());
  if (m < 0) {
    out.clear();
    return false;
  }
  out.resize((size_t)m);
  return true;
}

bool parse_qc(const uint8_t *buf, size_t len, QcParsed &out, std::string &err) {
  if (!buf && len) {
    err = "null buffer";
    return false;
  }
  Reader r{buf, len};
  const uint8_t *hash = nullptr;
  uint64_t nv = 0;
  if (!r.bytes(hash, 32) || !r.u64(out.round) || !r.u64(nv)) {
    err = "truncated QC header";
    return false;
  }
  if (nv > r.left / 72) {  // a vote is at least 8 + 0 + 64 bytes
    err = "vote count exceeds the buffer";
    return false;
  }
  out.n = (size_t)nv;
  out.votes.resize(out.n * 96);  // every byte is written below
  for (size_t i = 0; i < out.n; ++i) {
    uint8_t *v = out.votes.data() + i * 96;
    const uint8_t *sig = nullptr;
    if (!read_public_key(r, v)) {
      err = "vote " + std::to_string(i) + ": bad public key";
      return false;
    }
    if (!r.bytes(sig, 64)) {
      err = "vote " + std::to_string(i) + ": truncated signature";
      return false;
    }
    std::memcpy(v + 32, sig, 64);
  }
  if (r.left != 0) {
    err = "trailing bytes after the QC";
    return false;
  }
  uint8_t pre[40], h[64];
  std::memcpy(pre, hash, 32);
  put_le64(pre + 32, out.round);
  hsv::sha512_bytes(pre, sizeof(pre), h);
  std::memcpy(out.digest, h, 32);
  return true;
}

bool parse_tc(const uint8_t *buf, size_t len, TcParsed &out, std::string &err) {
  if (!buf && len) {
    err = "null buffer";
    return false;
  }
  Reader r{buf, len};
  uint64_t nv = 0;
  if (!r.u64(out.round) || !r.u64(nv)) {
    err = "truncated TC header";
    return false;
  }
  if (nv > r.left / 80) {  // 8 + 0 + 64 + 8 bytes at least
    err = "vote count exceeds the buffer";
    return false;
  }
  out.n = (size_t)nv;
  out.pks.resize(out.n * 32);  // every byte is written below
  out.sigs.resize(out.n * 64);
  out.digests.resize(out.n * 32);
  // the per-vote digest depends only on (round, high_qc_round), and a TC's
  // high_qc_rounds take few distinct values (the last rounds before a
  // timeout): hash each once.  A small array searched from the last hit, not
  // a hash map -- no allocation per call, and a C3 TC's 667 lookups cost a
  // few compares each (the map made the parse ~28 us of a 0.092 ms bincode
  // TC on the GPU box, profiles/r05e_bench_detail.json).
  constexpr size_t kMemo = 32;
  uint64_t memo_key[kMemo];
  uint8_t memo_dig[kMemo][32];
  size_t memo_n = 0, memo_last = 0;
  for (size_t i = 0; i < out.n; ++i) {
    const uint8_t *sig = nullptr;
    uint64_t hqc = 0;
    if (!read_public_key(r, out.pks.data() + i * 32)) {
      err = "vote " + std::to_string(i) + ": bad public key";
      return false;
    }
    if (!r.bytes(sig, 64) || !r.u64(hqc)) {
      err = "vote " + std::to_string(i) + ": truncated";
      return false;
    }
    std::memcpy(out.sigs.data() + i * 64, sig, 64);
    uint8_t *dig = out.digests.data() + i * 32;
    size_t k = memo_last;
    if (memo_n == 0 || memo_key[k] != hqc) {
      for (k = 0; k < memo_n && memo_key[k] != hqc; ++k) {
      }
    }
    if (k < memo_n) {
      memo_last = k;
      std::memcpy(dig, memo_dig[k], 32);
      continue;
    }
    uint8_t pre[16], h[64];
    put_le64(pre, out.round);
    put_le64(pre + 8, hqc);
    hsv::sha512_bytes(pre, sizeof(pre), h);
    std::memcpy(dig, h, 32);
    if (memo_n < kMemo) {  // beyond kMemo distinct values every new one is hashed
      memo_key[memo_n] = hqc;
      std::memcpy(memo_dig[memo_n], h, 32);
      memo_last = memo_n++;
    }
  }
  if (r.left != 0) {
    err = "trailing bytes after the TC";
    return false;
  }
  return true;
}

}  // namespace hsvw
