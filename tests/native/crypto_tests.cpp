// C++ port of the reference's crypto tests (crypto/src/tests/crypto_tests.rs)
// and consensus verify_valid_qc (consensus/src/tests/messages_tests.rs:8-10),
// written against include/hsv_crypto.hpp (the C++ mirror of the crate) and
// run on the GPU through libhsv.so.  Exit code 0 = all passed.
//
// --fallback installs the caller-side infrastructure-failure policy
// (crypto::set_infrastructure_fallback) with the C oracle
// (oracle/ed25519_oracle.c, test infrastructure standing in for the host
// ed25519-dalek a real shim would call) and prints how often it was used: on
// a machine without a GPU every verify goes to it and the tests still pass;
// on a GPU it must never be used.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "hsv_crypto.hpp"
#include "hsv_sha512.hpp"  // test-only: Hash for &[u8] = SHA-512(msg)[..32]

extern "C" {  // oracle/ed25519_oracle.c (linked only into this test binary)
uint8_t oracle_verify_flags(const uint8_t pk[32], const uint8_t sig[64], const uint8_t *msg, size_t msg_len);
}

using namespace crypto;

static int g_failed = 0;
#define CHECK(cond)                                                        \
  do {                                                                     \
    if (!(cond)) {                                                         \
      std::fprintf(stderr, "FAILED %s:%d: %s\n", __FILE__, __LINE__, #cond); \
      ++g_failed;                                                          \
    }                                                                      \
  } while (0)

// rand 0.7 StdRng::from_seed([0;32]) is ChaCha20 (djb variant, 64-bit counter);
// dalek SecretKey::generate fills 32 bytes from it.
static void chacha20_block(const uint8_t key[32], uint64_t counter, uint8_t out[64]) {
  auto rotl = [](uint32_t v, int c) { return (v << c) | (v >> (32 - c)); };
  uint32_t st[16] = {0x61707865u, 0x3320646eu, 0x79622d32u, 0x6b206574u};
  for (int i = 0; i < 8; ++i) std::memcpy(&st[4 + i], key + 4 * i, 4);
  st[12] = (uint32_t)counter;
  st[13] = (uint32_t)(counter >> 32);
  st[14] = st[15] = 0;
  uint32_t w[16];
  std::memcpy(w, st, sizeof w);
  auto qr = [&](int a, int b, int c, int d) {
    w[a] += w[b]; w[d] = rotl(w[d] ^ w[a], 16);
    w[c] += w[d]; w[b] = rotl(w[b] ^ w[c], 12);
    w[a] += w[b]; w[d] = rotl(w[d] ^ w[a], 8);
    w[c] += w[d]; w[b] = rotl(w[b] ^ w[c], 7);
  };
  for (int r = 0; r < 10; ++r) {
    qr(0, 4, 8, 12); qr(1, 5, 9, 13); qr(2, 6, 10, 14); qr(3, 7, 11, 15);
    qr(0, 5, 10, 15); qr(1, 6, 11, 12); qr(2, 7, 8, 13); qr(3, 4, 9, 14);
  }
  for (int i = 0; i < 16; ++i) {
    const uint32_t v = w[i] + st[i];
    std::memcpy(out + 4 * i, &v, 4);
  }
}

struct StdRng {
  uint8_t key[32];
  uint64_t counter = 0;
  std::vector<uint8_t> buf;
  size_t pos = 0;
  explicit StdRng(uint8_t seed_byte) { std::memset(key, seed_byte, 32); }
  void fill(uint8_t *out, size_t n) {
    for (size_t i = 0; i < n; ++i) {
      if (pos == buf.size()) {
        buf.assign(64, 0);
        chacha20_block(key, counter++, buf.data());
        pos = 0;
      }
      out[i] = buf[pos++];
    }
  }
};

static std::vector<std::pair<PublicKey, SecretKey>> keys() {
  StdRng rng(0);
  std::vector<std::pair<PublicKey, SecretKey>> out;
  for (int i = 0; i < 4; ++i)
    out.push_back(generate_keypair([&](uint8_t *p, size_t n) { rng.fill(p, n); }));
  return out;
}

static Digest digest_of(const std::string &msg) {
  uint8_t h[64];
  hsv::sha512_bytes(reinterpret_cast<const uint8_t *>(msg.data()), msg.size(), h);
  Digest d;
  std::memcpy(d.bytes.data(), h, 32);
  return d;
}

static void import_export_public_key() {
  auto ks = keys();
  const PublicKey public_key = ks.back().first;
  const std::string exported = public_key.encode_base64();
  CHECK(PublicKey::decode_base64(exported) == public_key);
}

static void import_export_secret_key() {
  auto ks = keys();
  const SecretKey &secret_key = ks.back().second;
  CHECK(SecretKey::decode_base64(secret_key.encode_base64()) == secret_key);
}

static void verify_valid_signature() {
  auto ks = keys();
  auto [public_key, secret_key] = ks.back();
  const Digest digest = digest_of("Hello, world!");
  const Signature signature = Signature::sign(digest, secret_key);
  CHECK(signature.verify(digest, public_key).is_ok());
}

static void verify_invalid_signature() {
  auto ks = keys();
  auto [public_key, secret_key] = ks.back();
  const Signature signature = Signature::sign(digest_of("Hello, world!"), secret_key);
  CHECK(signature.verify(digest_of("Bad message!"), public_key).is_err());
}

static void verify_valid_batch() {
  const Digest digest = digest_of("Hello, world!");
  auto ks = keys();
  std::vector<std::pair<PublicKey, Signature>> signatures;
  for (int i = 0; i < 3; ++i) {
    auto [pk, sk] = ks.back();
    ks.pop_back();
    signatures.emplace_back(pk, Signature::sign(digest, sk));
  }
  CHECK(Signature::verify_batch(digest, signatures).is_ok());
}

static void verify_invalid_batch() {
  const Digest digest = digest_of("Hello, world!");
  auto ks = keys();
  std::vector<std::pair<PublicKey, Signature>> signatures;
  for (int i = 0; i < 2; ++i) {
    auto [pk, sk] = ks.back();
    ks.pop_back();
    signatures.emplace_back(pk, Signature::sign(digest, sk));
  }
  signatures.emplace_back(ks.back().first, Signature());  // Signature::default()
  CHECK(Signature::verify_batch(digest, signatures).is_err());
}

static void signature_service() {
  auto ks = keys();
  auto [public_key, secret_key] = ks.back();
  SignatureService service(secret_key);
  const Digest digest = digest_of("Hello, world!");
  const Signature signature = service.request_signature(digest).get();
  CHECK(signature.verify(digest, public_key).is_ok());
}

// consensus qc(): hash = 0^32, round = 1, votes from keys[3], [2], [1]
static void verify_valid_qc() {
  uint8_t buf[40] = {0};
  buf[32] = 1;  // round 1, little-endian u64
  uint8_t h[64];
  hsv::sha512_bytes(buf, 40, h);
  Digest qc_digest;
  std::memcpy(qc_digest.bytes.data(), h, 32);
  CHECK(qc_digest.bytes[0] == 0xf2 && qc_digest.bytes[1] == 0xa4);  // f2a4a4b7...
  auto ks = keys();
  std::vector<std::pair<PublicKey, Signature>> votes;
  for (int i = 0; i < 3; ++i) {
    auto [pk, sk] = ks.back();
    ks.pop_back();
    votes.emplace_back(pk, Signature::sign(qc_digest, sk));
  }
  const size_t cached0 = hsv_auto_committee_size();
  CHECK(Signature::verify_batch(qc_digest, votes).is_ok());
  // QC::verify with one forged vote -> Err (InvalidSignature)
  votes[1].second.part2[5] ^= 0x10;
  const size_t cached1 = hsv_auto_committee_size();
  const bool forged_rejected = Signature::verify_batch(qc_digest, votes).is_err();
  if (!forged_rejected)
    std::fprintf(stderr, "forged QC accepted; automatic committee cache held %zu / %zu keys before the two QCs\n",
                 cached0, cached1);
  CHECK(forged_rejected);
  // empty vote list: dalek verify_batch over zero items is Ok
  CHECK(Signature::verify_batch(qc_digest, {}).is_ok());
}

static void install_oracle_fallback() {
  InfrastructureFallback f;
  f.verify_strict = [](const uint8_t *digest, const uint8_t *pk, const uint8_t *sig) {
    return (oracle_verify_flags(pk, sig, digest, 32) & HSV_STRICT_OK) != 0;
  };
  f.verify_batch = [](const uint8_t *digest, const uint8_t *votes, size_t n) {
    for (size_t i = 0; i < n; ++i) {
      const uint8_t fl = oracle_verify_flags(votes + 96 * i, votes + 96 * i + 32, digest, 32);
      if ((fl & (HSV_PARSE_OK | HSV_EQ_OK)) != (HSV_PARSE_OK | HSV_EQ_OK)) return false;
    }
    return true;
  };
  set_infrastructure_fallback(std::move(f));
}

// --route: QCs of at most 2 votes on the host verifier (the C oracle stands
// in for dalek), larger QCs on libhsv; single verifies on libhsv unless its
// resident latency service is off (crypto::single_verify_on_host_default)
static void install_host_route() {
  HostRoute r;
  r.single = single_verify_on_host_default();
  r.max_batch = 2;
  r.verify_strict = [](const uint8_t *digest, const uint8_t *pk, const uint8_t *sig) {
    return (oracle_verify_flags(pk, sig, digest, 32) & HSV_STRICT_OK) != 0;
  };
  r.verify_batch = [](const uint8_t *digest, const uint8_t *votes, size_t n) {
    for (size_t i = 0; i < n; ++i) {
      const uint8_t fl = oracle_verify_flags(votes + 96 * i, votes + 96 * i + 32, digest, 32);
      if ((fl & (HSV_PARSE_OK | HSV_EQ_OK)) != (HSV_PARSE_OK | HSV_EQ_OK)) return false;
    }
    return true;
  };
  set_host_route(std::move(r));
}

#ifdef HSV_TEST_HOOKS
// libhsv_test.so's fault injection hook (csrc/hsv_test_hooks.h; libhsv.so
// exports no hook, so the --inject build links libhsv_test.so)
#include "hsv_test_hooks.h"
#endif

int main(int argc, char **argv) {
  bool fallback = false;
  for (int i = 1; i < argc; ++i) {
    if (std::strcmp(argv[i], "--fallback") == 0) fallback = true;
    if (std::strcmp(argv[i], "--route") == 0) install_host_route();
#ifdef HSV_TEST_HOOKS
    // --inject MODE: every launch of this (the main) thread reads corrupted
    // tables (csrc/hsv_verify_core.hpp kInject*)
    if (std::strcmp(argv[i], "--inject") == 0 && i + 1 < argc) hsv_test_inject_fault(std::atoi(argv[++i]));
#endif
  }
  if (fallback) install_oracle_fallback();
  import_export_public_key();
  import_export_secret_key();
  verify_valid_signature();
  verify_invalid_signature();
  verify_valid_batch();
  verify_invalid_batch();
  signature_service();
  verify_valid_qc();
  if (g_failed) {
    std::fprintf(stderr, "%d check(s) failed\n", g_failed);
    return 1;
  }
  if (fallback) std::printf("infrastructure fallbacks: %llu\n", (unsigned long long)infrastructure_fallback_uses());
  std::printf("host-routed calls: %llu\n", (unsigned long long)host_route_uses());
  std::printf("crypto_tests: all passed\n");
  return 0;
}
