// Fuzz harness for the certificate parsers (csrc/hsv_wire_parse.cpp), built
// with -fsanitize=address,undefined by tests/test_wire_fuzz.py (host only, no
// GPU).  The parsers read untrusted network bytes: the reference receives
// QCs and TCs as TCP frames (network/src/receiver.rs:47-60) and bincode-
// deserialises them (consensus/src/consensus.rs:32-39).
//
// Inputs: valid QC / TC encodings (bincode 1.3 defaults, PublicKey as its
// base64 string) and, from each, every truncation, oversized vote counts and
// string lengths, bad base64 (symbols, padding, trailing bits), and random
// byte flips / insertions / deletions / splices.  Checks: no sanitizer report,
// valid inputs parse to exactly the encoded votes and digests, every strict
// prefix of a valid encoding is rejected.
//
// usage: wire_fuzz [iterations] [seed]
#include <array>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "hsv_sha512.hpp"
#include "hsv_wire_parse.h"

namespace {

using Bytes = std::vector<uint8_t>;

void put_u64(Bytes &b, uint64_t v) {
  for (int i = 0; i < 8; ++i) b.push_back((uint8_t)(v >> (8 * i)));
}

std::string b64_encode(const uint8_t *p, size_t n) {
  static const char *A = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/";
  std::string s;
  size_t i = 0;
  for (; i + 3 <= n; i += 3) {
    const uint32_t v = (p[i] << 16) | (p[i + 1] << 8) | p[i + 2];
    s += A[v >> 18];
    s += A[(v >> 12) & 63];
    s += A[(v >> 6) & 63];
    s += A[v & 63];
  }
  if (n - i == 1) {
    const uint32_t v = p[i] << 16;
    s += A[v >> 18];
    s += A[(v >> 12) & 63];
    s += "==";
  } else if (n - i == 2) {
    const uint32_t v = (p[i] << 16) | (p[i + 1] << 8);
    s += A[v >> 18];
    s += A[(v >> 12) & 63];
    s += A[(v >> 6) & 63];
    s += '=';
  }
  return s;
}

void put_key(Bytes &b, const uint8_t pk[32]) {
  const std::string s = b64_encode(pk, 32);
  put_u64(b, s.size());
  b.insert(b.end(), s.begin(), s.end());
}

struct Qc {
  uint8_t hash[32];
  uint64_t round;
  std::vector<std::array<uint8_t, 96>> votes;
  Bytes enc;
};

struct Tc {
  uint64_t round;
  std::vector<std::array<uint8_t, 96>> votes;
  std::vector<uint64_t> hqc;
  Bytes enc;
};

Qc make_qc(std::mt19937_64 &rng, size_t n) {
  Qc q;
  for (auto &b : q.hash) b = (uint8_t)rng();
  q.round = rng() % 1000000;
  q.votes.resize(n);
  for (auto &v : q.votes)
    for (auto &b : v) b = (uint8_t)rng();
  q.enc.assign(q.hash, q.hash + 32);
  put_u64(q.enc, q.round);
  put_u64(q.enc, n);
  for (auto &v : q.votes) {
    put_key(q.enc, v.data());
    q.enc.insert(q.enc.end(), v.begin() + 32, v.end());
  }
  return q;
}

Tc make_tc(std::mt19937_64 &rng, size_t n) {
  Tc t;
  t.round = 1000 + rng() % 1000;
  t.votes.resize(n);
  t.hqc.resize(n);
  put_u64(t.enc, t.round);
  put_u64(t.enc, n);
  for (size_t i = 0; i < n; ++i) {
    for (auto &b : t.votes[i]) b = (uint8_t)rng();
    t.hqc[i] = t.round - 1 - rng() % 10;
    put_key(t.enc, t.votes[i].data());
    t.enc.insert(t.enc.end(), t.votes[i].begin() + 32, t.votes[i].end());
    put_u64(t.enc, t.hqc[i]);
  }
  return t;
}

int failures = 0;
#define CHECK(c, ...)                                  \
  do {                                                 \
    if (!(c)) {                                        \
      std::fprintf(stderr, "CHECK failed: %s: ", #c);  \
      std::fprintf(stderr, __VA_ARGS__);               \
      std::fprintf(stderr, "\n");                      \
      ++failures;                                      \
    }                                                  \
  } while (0)

void check_valid_qc(const Qc &q) {
  hsvw::QcParsed p;
  std::string err;
  CHECK(hsvw::parse_qc(q.enc.data(), q.enc.size(), p, err), "valid QC rejected: %s", err.c_str());
  CHECK(p.n == q.votes.size() && p.round == q.round, "QC header");
  for (size_t i = 0; i < p.n && i < q.votes.size(); ++i)
    CHECK(std::memcmp(p.votes.data() + 96 * i, q.votes[i].data(), 96) == 0, "QC vote %zu", i);
  uint8_t pre[40], h[64];
  std::memcpy(pre, q.hash, 32);
  for (int b = 0; b < 8; ++b) pre[32 + b] = (uint8_t)(q.round >> (8 * b));
  hsv::sha512_bytes(pre, 40, h);
  CHECK(std::memcmp(p.digest, h, 32) == 0, "QC digest");
  // every strict prefix is truncated, every extension has trailing bytes
  for (size_t cut = 0; cut < q.enc.size(); ++cut) {
    hsvw::QcParsed x;
    CHECK(!hsvw::parse_qc(q.enc.data(), cut, x, err), "QC prefix %zu accepted", cut);
  }
  Bytes ext = q.enc;
  ext.push_back(0);
  hsvw::QcParsed x;
  CHECK(!hsvw::parse_qc(ext.data(), ext.size(), x, err), "QC with a trailing byte accepted");
}

void check_valid_tc(const Tc &t) {
  hsvw::TcParsed p;
  std::string err;
  CHECK(hsvw::parse_tc(t.enc.data(), t.enc.size(), p, err), "valid TC rejected: %s", err.c_str());
  CHECK(p.n == t.votes.size() && p.round == t.round, "TC header");
  for (size_t i = 0; i < p.n && i < t.votes.size(); ++i) {
    CHECK(std::memcmp(p.pks.data() + 32 * i, t.votes[i].data(), 32) == 0, "TC pk %zu", i);
    CHECK(std::memcmp(p.sigs.data() + 64 * i, t.votes[i].data() + 32, 64) == 0, "TC sig %zu", i);
    uint8_t pre[16], h[64];
    for (int b = 0; b < 8; ++b) {
      pre[b] = (uint8_t)(t.round >> (8 * b));
      pre[8 + b] = (uint8_t)(t.hqc[i] >> (8 * b));
    }
    hsv::sha512_bytes(pre, 16, h);
    CHECK(std::memcmp(p.digests.data() + 32 * i, h, 32) == 0, "TC digest %zu", i);
  }
  for (size_t cut = 0; cut < t.enc.size(); ++cut) {
    hsvw::TcParsed x;
    CHECK(!hsvw::parse_tc(t.enc.data(), cut, x, err), "TC prefix %zu accepted", cut);
  }
}

// parse anything; only the sanitizers judge (and a successful parse must be
// self-consistent)
void parse_any(const Bytes &b) {
  std::string err;
  hsvw::QcParsed q;
  if (hsvw::parse_qc(b.data(), b.size(), q, err)) CHECK(q.votes.size() == 96 * q.n, "QC sizes");
  hsvw::TcParsed t;
  if (hsvw::parse_tc(b.data(), b.size(), t, err))
    CHECK(t.pks.size() == 32 * t.n && t.sigs.size() == 64 * t.n && t.digests.size() == 32 * t.n, "TC sizes");
}

void set_u64(Bytes &b, size_t off, uint64_t v) {
  if (off + 8 > b.size()) return;
  for (int i = 0; i < 8; ++i) b[off + i] = (uint8_t)(v >> (8 * i));
}

Bytes mutate(const Bytes &in, std::mt19937_64 &rng, const std::vector<Bytes> &pool) {
  Bytes b = in;
  const int ops = 1 + (int)(rng() % 4);
  for (int k = 0; k < ops; ++k) {
    switch (rng() % 9) {
      case 0:  // bit flip
        if (!b.empty()) b[rng() % b.size()] ^= (uint8_t)(1u << (rng() % 8));
        break;
      case 1:  // random byte
        if (!b.empty()) b[rng() % b.size()] = (uint8_t)rng();
        break;
      case 2:  // truncate
        if (!b.empty()) b.resize(rng() % b.size());
        break;
      case 3:  // insert
        b.insert(b.begin() + (b.empty() ? 0 : rng() % (b.size() + 1)), (uint8_t)rng());
        break;
      case 4:  // delete
        if (!b.empty()) b.erase(b.begin() + rng() % b.size());
        break;
      case 5: {  // oversized / boundary u64 at a random 8-aligned-ish offset
        static const uint64_t vals[] = {~0ull, 1ull << 63, 1ull << 32, 0xffffffffull, 44, 43, 45, 0, 1,
                                        ~0ull / 96, ~0ull / 72 + 1};
        set_u64(b, b.empty() ? 0 : rng() % b.size(), vals[rng() % (sizeof(vals) / sizeof(vals[0]))]);
        break;
      }
      case 6:  // bad base64 symbol / padding inside the bytes
        if (!b.empty()) {
          static const uint8_t bad[] = {'=', '-', '_', ' ', '\n', 0, 0x80, '!', '/', '+'};
          b[rng() % b.size()] = bad[rng() % sizeof(bad)];
        }
        break;
      case 7: {  // splice with another input
        const Bytes &o = pool[rng() % pool.size()];
        if (!o.empty() && !b.empty()) {
          const size_t at = rng() % b.size(), from = rng() % o.size(), len = rng() % (o.size() - from + 1);
          b.resize(at);
          b.insert(b.end(), o.begin() + from, o.begin() + from + len);
        }
        break;
      }
      default:  // duplicate a chunk
        if (b.size() > 2) {
          const size_t a = rng() % b.size(), len = rng() % (b.size() - a);
          Bytes chunk(b.begin() + a, b.begin() + a + len);
          b.insert(b.begin() + a, chunk.begin(), chunk.end());
        }
    }
  }
  return b;
}

// An independent, character-at-a-time statement of the decoder's rules
// (base64 0.13 standard: alphabet A-Z a-z 0-9 + /, at most two '=' and only
// at the end of a whole-quad string, no length = 1 mod 4, zero trailing
// bits), against which the parser's block decoder (16 characters at a time
// with SSSE3 on x86-64) is checked verdict for verdict and byte for byte.
bool ref_b64_decode(const std::string &t, Bytes &out) {
  auto val = [](unsigned char c) -> int {
    if (c >= 'A' && c <= 'Z') return c - 'A';
    if (c >= 'a' && c <= 'z') return c - 'a' + 26;
    if (c >= '0' && c <= '9') return c - '0' + 52;
    if (c == '+') return 62;
    if (c == '/') return 63;
    return -1;
  };
  out.clear();
  size_t end = t.size();
  while (end > 0 && t[end - 1] == '=') --end;
  const size_t pad = t.size() - end;
  if (pad > 2 || (pad && t.size() % 4 != 0) || end % 4 == 1) return false;
  uint32_t acc = 0;
  int bits = 0;
  for (size_t i = 0; i < end; ++i) {
    const int v = val((unsigned char)t[i]);
    if (v < 0) return false;
    acc = (acc << 6) | (uint32_t)v;
    bits += 6;
    if (bits >= 8) {
      bits -= 8;
      out.push_back((uint8_t)(acc >> bits));
      acc &= (1u << bits) - 1u;
    }
  }
  return acc == 0;
}

void fuzz_base64_differential(std::mt19937_64 &rng, long iters) {
  static const char *alpha = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/";
  static const uint8_t odd[] = {'=', '-', '_', ' ', '\n', 0, 0x80, 0xff, '!', '@', '[', '`', '{', ':', '?', '*', '.'};
  Bytes got, want;
  for (long i = 0; i < iters; ++i) {
    std::string t;
    if (rng() % 2) {  // a canonical encoding (often a key's 44 characters), sometimes with one byte changed
      Bytes raw(rng() % 4 ? 32 : rng() % 80);
      for (auto &x : raw) x = (uint8_t)rng();
      t = b64_encode(raw.data(), raw.size());
      if (!t.empty() && rng() % 3 == 0) {
        const size_t at = rng() % t.size();
        t[at] = rng() % 2 ? (char)odd[rng() % sizeof(odd)] : alpha[rng() % 64];
      }
    } else {  // random alphabet strings up to 100 characters, some odd bytes, some padding
      t.resize(rng() % 101);
      for (auto &c : t) c = rng() % 40 ? alpha[rng() % 64] : (char)odd[rng() % sizeof(odd)];
      if (!t.empty() && rng() % 4 == 0) t.back() = '=';
      if (t.size() > 1 && rng() % 8 == 0) t[t.size() - 2] = '=';
    }
    const bool ok = hsvw::b64_decode(reinterpret_cast<const uint8_t *>(t.data()), t.size(), got);
    const bool ok_ref = ref_b64_decode(t, want);
    CHECK(ok == ok_ref, "base64 verdict %d against %d for a %zu-character string", ok, ok_ref, t.size());
    if (ok && ok_ref) CHECK(got == want, "base64 bytes differ for a %zu-character string", t.size());
  }
}

void fuzz_base64(std::mt19937_64 &rng, long iters) {
  static const char *sym = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/=-_ \n";
  std::vector<uint8_t> out;
  for (long i = 0; i < iters; ++i) {
    // round trip of random bytes
    std::vector<uint8_t> raw(rng() % 48);
    for (auto &x : raw) x = (uint8_t)rng();
    const std::string s = b64_encode(raw.data(), raw.size());
    CHECK(hsvw::b64_decode(reinterpret_cast<const uint8_t *>(s.data()), s.size(), out) && out == raw,
          "base64 round trip of %zu bytes", raw.size());
    // random strings: any verdict, no UB; an accepted string re-encodes to itself
    std::string t(rng() % 50, 'A');
    for (auto &c : t) c = sym[rng() % 68];
    if (hsvw::b64_decode(reinterpret_cast<const uint8_t *>(t.data()), t.size(), out)) {
      std::string back = b64_encode(out.data(), out.size());
      while (!back.empty() && back.back() == '=' && t.find('=') == std::string::npos) back.pop_back();
      CHECK(back == t, "base64 accepted a non-canonical string '%s'", t.c_str());
    }
  }
}

}  // namespace

int main(int argc, char **argv) {
  const long iters = argc > 1 ? std::atol(argv[1]) : 200000;
  std::mt19937_64 rng(argc > 2 ? std::strtoull(argv[2], nullptr, 10) : 20241016);
  std::vector<Bytes> pool;
  for (size_t n : {0, 1, 2, 3, 67}) {
    const Qc q = make_qc(rng, n);
    check_valid_qc(q);
    pool.push_back(q.enc);
    const Tc t = make_tc(rng, n);
    check_valid_tc(t);
    pool.push_back(t.enc);
  }
  pool.push_back(Bytes());
  for (long i = 0; i < iters; ++i) parse_any(mutate(pool[rng() % pool.size()], rng, pool));
  fuzz_base64(rng, iters / 10);
  fuzz_base64_differential(rng, iters);
  if (failures) {
    std::fprintf(stderr, "%d check(s) failed\n", failures);
    return 1;
  }
  std::printf("wire fuzz ok: %ld mutated inputs, %zu seeds\n", iters, pool.size());
  return 0;
}
