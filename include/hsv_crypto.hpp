// hsv_crypto.hpp -- C++ mirror of the reference's `crypto` crate over the C ABI.
//
// The reference (mwaurawakati/hotstuff-digital-signature-benchmarking) is Rust;
// no Rust toolchain exists in this image, so the host side above libhsv's C
// ABI is written in C++ with the crate's names, byte layouts, argument meaning
// and error behaviour (reference crypto/src/lib.rs):
//
//   Digest(pub [u8;32])                       lib.rs:22      -> crypto::Digest
//   PublicKey(pub [u8;32]) + base64 serde     lib.rs:66-118  -> crypto::PublicKey
//   SecretKey([u8;64]), zeroed on drop        lib.rs:121-161 -> crypto::SecretKey
//   generate_keypair(csprng)                  lib.rs:167-175 -> crypto::generate_keypair
//   Signature{part1, part2}                   lib.rs:179-182 -> crypto::Signature
//   Signature::new / from_bytes / flatten     lib.rs:185-202
//   Signature::verify        -> Result        lib.rs:204-208 (verify_strict semantics)
//   Signature::verify_batch  -> Result        lib.rs:210-223
//   SignatureService::request_signature       lib.rs:229-254 -> crypto::SignatureService
//
// `Result` carries Ok or Err(CryptoError) exactly like Result<(), CryptoError>.
// An infrastructure failure (no GPU, HIP error) is NOT an Err: by default it
// throws crypto::InfrastructureError, so a broken device can never look like a
// rejected signature.  A deployment that must keep running through a device
// fault installs an InfrastructureFallback (set_infrastructure_fallback): a
// host verifier with the same semantics (ed25519-dalek in the Rust shim,
// INTEGRATION.md section 2) that is consulted ONLY for calls libhsv could not
// run, never to second-guess a rejection; every use is counted.  libhsv itself
// has no CPU path.
#ifndef HSV_CRYPTO_HPP_
#define HSV_CRYPTO_HPP_

#include <array>
#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <functional>
#include <future>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <utility>
#include <vector>

#include "hsv.h"

namespace crypto {

class InfrastructureError : public std::runtime_error {
 public:
  explicit InfrastructureError(const std::string &what) : std::runtime_error(what) {}
};

inline int check_infra(int rc, const char *what) {
  if (rc < 0) throw InfrastructureError(std::string(what) + ": " + hsv_last_error());
  return rc;
}

// Infrastructure-failure policy of the caller (see the header comment).
// Install once at startup, before verify calls run on other threads.
struct InfrastructureFallback {
  // verify_strict over one 32-byte digest; true = Ok
  std::function<bool(const uint8_t *digest, const uint8_t *pk, const uint8_t *sig)> verify_strict;
  // the deterministic verify_batch rule over packed 96-byte pk || R || s votes
  std::function<bool(const uint8_t *digest, const uint8_t *votes, size_t n)> verify_batch;
};

inline InfrastructureFallback &infrastructure_fallback() {
  static InfrastructureFallback f;
  return f;
}
inline std::atomic<uint64_t> &infrastructure_fallback_uses() {
  static std::atomic<uint64_t> n{0};
  return n;
}
inline void set_infrastructure_fallback(InfrastructureFallback f) { infrastructure_fallback() = std::move(f); }

// Latency routing of the caller.
// One signature on the GPU costs a launch plus one dependent root chain
// (0.0395 ms for a cached committee key, 0.0357 ms through the resident
// service), one host core 0.037 ms (dalek port); a 3-vote QC is 0.04 ms on the
// GPU against 0.077 ms on the host.  A
// deployment installs a host verifier with the same semantics (dalek in the
// Rust shim) and a size limit: verify calls and verify_batch calls of at most
// max_batch votes go to it, everything larger to libhsv.  Unlike the
// infrastructure fallback this is a routing choice made before the call --
// libhsv's verdicts are never second-guessed.  Every routed call is counted.
struct HostRoute {
  size_t max_batch = 0;  // verify_batch calls of at most this many votes go to the host
  bool single = false;   // Signature::verify goes to the host
  std::function<bool(const uint8_t *digest, const uint8_t *pk, const uint8_t *sig)> verify_strict;
  std::function<bool(const uint8_t *digest, const uint8_t *votes, size_t n)> verify_batch;
};

inline HostRoute &host_route() {
  static HostRoute r;
  return r;
}
inline std::atomic<uint64_t> &host_route_uses() {
  static std::atomic<uint64_t> n{0};
  return n;
}
// Install once at startup, before verify calls run on other threads.
inline void set_host_route(HostRoute r) { host_route() = std::move(r); }

// The single-verify routing default (the Rust
// shim's hsv_single_on_host): a lone signature goes to libhsv, whose resident
// latency service is on by default (one cached-key verify_strict 0.034 ms
// against 0.036-0.037 ms for the dalek port on one host core,
// profiles/r05ah_bench.json).  It stays on the host only when the service is
// turned off (HSV_QC_RESIDENT=0: launched, 0.039 ms).  HSV_ROUTE_SINGLE =
// "gpu" / "host" overrides it.
inline bool single_verify_on_host_default() {
  if (const char *v = std::getenv("HSV_ROUTE_SINGLE")) return std::strcmp(v, "gpu") != 0;
  const char *r = std::getenv("HSV_QC_RESIDENT");
  return r && r[0] == '0';
}

// ed25519::Error: opaque.
struct CryptoError {
  std::string message = "signature error";
};

// Result<(), CryptoError>
class Result {
 public:
  static Result ok() { return Result(true); }
  static Result err() { return Result(false); }
  bool is_ok() const { return ok_; }
  bool is_err() const { return !ok_; }
  CryptoError unwrap_err() const { return CryptoError{}; }

 private:
  explicit Result(bool ok) : ok_(ok) {}
  bool ok_;
};

namespace detail {
inline std::string b64encode(const uint8_t *p, size_t n) {
  static const char *tbl = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/";
  std::string out;
  for (size_t i = 0; i < n; i += 3) {
    uint32_t v = (uint32_t)p[i] << 16;
    if (i + 1 < n) v |= (uint32_t)p[i + 1] << 8;
    if (i + 2 < n) v |= p[i + 2];
    out += tbl[(v >> 18) & 63];
    out += tbl[(v >> 12) & 63];
    out += i + 1 < n ? tbl[(v >> 6) & 63] : '=';
    out += i + 2 < n ? tbl[v & 63] : '=';
  }
  return out;
}

inline std::vector<uint8_t> b64decode(const std::string &s) {
  auto val = [](char c) -> int {
    if (c >= 'A' && c <= 'Z') return c - 'A';
    if (c >= 'a' && c <= 'z') return c - 'a' + 26;
    if (c >= '0' && c <= '9') return c - '0' + 52;
    if (c == '+') return 62;
    if (c == '/') return 63;
    return -1;
  };
  std::vector<uint8_t> out;
  uint32_t buf = 0;
  int bits = 0;
  for (char c : s) {
    if (c == '=') break;
    const int v = val(c);
    if (v < 0) throw std::invalid_argument("base64: invalid symbol");
    buf = (buf << 6) | (uint32_t)v;
    bits += 6;
    if (bits >= 8) {
      bits -= 8;
      out.push_back((uint8_t)(buf >> bits));
    }
  }
  return out;
}
}  // namespace detail

struct Digest {
  std::array<uint8_t, 32> bytes{};
  std::vector<uint8_t> to_vec() const { return {bytes.begin(), bytes.end()}; }
  size_t size() const { return bytes.size(); }
  bool operator==(const Digest &o) const { return bytes == o.bytes; }
};

struct PublicKey {
  std::array<uint8_t, 32> bytes{};
  std::string encode_base64() const { return detail::b64encode(bytes.data(), 32); }
  static PublicKey decode_base64(const std::string &s) {
    const std::vector<uint8_t> raw = detail::b64decode(s);
    if (raw.size() < 32) throw std::invalid_argument("InvalidLength");
    PublicKey k;
    std::memcpy(k.bytes.data(), raw.data(), 32);
    return k;
  }
  bool operator==(const PublicKey &o) const { return bytes == o.bytes; }
  bool operator<(const PublicKey &o) const { return bytes < o.bytes; }
};

// 64 bytes: secret seed (32) || public key (32); zeroed on destruction.
class SecretKey {
 public:
  SecretKey() = default;
  explicit SecretKey(const std::array<uint8_t, 64> &b) : bytes_(b) {}
  SecretKey(const SecretKey &) = default;
  SecretKey &operator=(const SecretKey &) = default;
  ~SecretKey() {
    volatile uint8_t *p = bytes_.data();
    for (size_t i = 0; i < bytes_.size(); ++i) p[i] = 0;
  }
  std::string encode_base64() const { return detail::b64encode(bytes_.data(), 64); }
  static SecretKey decode_base64(const std::string &s) {
    const std::vector<uint8_t> raw = detail::b64decode(s);
    if (raw.size() < 64) throw std::invalid_argument("InvalidLength");
    std::array<uint8_t, 64> b{};
    std::memcpy(b.data(), raw.data(), 64);
    return SecretKey(b);
  }
  const uint8_t *seed() const { return bytes_.data(); }
  bool operator==(const SecretKey &o) const { return bytes_ == o.bytes_; }

 private:
  std::array<uint8_t, 64> bytes_{};
};

// generate_keypair(csprng): `fill` writes 32 secret bytes (dalek SecretKey::generate).
inline std::pair<PublicKey, SecretKey> generate_keypair(const std::function<void(uint8_t *, size_t)> &fill) {
  std::array<uint8_t, 64> sk{};
  fill(sk.data(), 32);
  PublicKey pk;
  check_infra(hsv_public_key(sk.data(), pk.bytes.data()), "hsv_public_key");
  std::memcpy(sk.data() + 32, pk.bytes.data(), 32);
  return {pk, SecretKey(sk)};
}

class Signature {
 public:
  std::array<uint8_t, 32> part1{};  // R
  std::array<uint8_t, 32> part2{};  // s

  Signature() = default;  // Signature::default(): 64 zero bytes

  // Signature::new (lib.rs:185-191): RFC 8032 over digest.0
  static Signature sign(const Digest &digest, const SecretKey &secret) {
    uint8_t out[64];
    check_infra(hsv_sign(secret.seed(), digest.bytes.data(), 32, out), "hsv_sign");
    Signature s;
    std::memcpy(s.part1.data(), out, 32);
    std::memcpy(s.part2.data(), out + 32, 32);
    return s;
  }

  static Signature from_bytes(const std::array<uint8_t, 32> &p1, const std::array<uint8_t, 32> &p2) {
    Signature s;
    s.part1 = p1;
    s.part2 = p2;
    return s;
  }

  std::array<uint8_t, 64> flatten() const {
    std::array<uint8_t, 64> f{};
    std::memcpy(f.data(), part1.data(), 32);
    std::memcpy(f.data() + 32, part2.data(), 32);
    return f;
  }

  // Signature::verify (lib.rs:204-208): ed25519-dalek verify_strict semantics.
  Result verify(const Digest &digest, const PublicKey &public_key) const {
    const std::array<uint8_t, 64> f = flatten();
    const HostRoute &route = host_route();
    if (route.single && route.verify_strict) {
      ++host_route_uses();
      return route.verify_strict(digest.bytes.data(), public_key.bytes.data(), f.data()) ? Result::ok()
                                                                                         : Result::err();
    }
    int rc = hsv_verify_strict(digest.bytes.data(), public_key.bytes.data(), f.data());
    if (rc < 0 && infrastructure_fallback().verify_strict) {
      ++infrastructure_fallback_uses();
      rc = infrastructure_fallback().verify_strict(digest.bytes.data(), public_key.bytes.data(), f.data()) ? 1 : 0;
    }
    check_infra(rc, "hsv_verify_strict");
    return rc == 1 ? Result::ok() : Result::err();
  }

  // Signature::verify_batch (lib.rs:210-223): every vote signs the same digest.
  static Result verify_batch(const Digest &digest, const std::vector<std::pair<PublicKey, Signature>> &votes) {
    std::vector<uint8_t> packed(votes.size() * 96);
    for (size_t i = 0; i < votes.size(); ++i) {
      std::memcpy(packed.data() + 96 * i, votes[i].first.bytes.data(), 32);
      std::memcpy(packed.data() + 96 * i + 32, votes[i].second.part1.data(), 32);
      std::memcpy(packed.data() + 96 * i + 64, votes[i].second.part2.data(), 32);
    }
    const HostRoute &route = host_route();
    if (votes.size() <= route.max_batch && route.verify_batch) {
      ++host_route_uses();
      return route.verify_batch(digest.bytes.data(), packed.data(), votes.size()) ? Result::ok() : Result::err();
    }
    int rc = hsv_verify_batch_packed(digest.bytes.data(), packed.data(), votes.size());
    if (rc < 0 && infrastructure_fallback().verify_batch) {
      ++infrastructure_fallback_uses();
      rc = infrastructure_fallback().verify_batch(digest.bytes.data(), packed.data(), votes.size()) ? 1 : 0;
    }
    check_infra(rc, "hsv_verify_batch_packed");
    return rc == 1 ? Result::ok() : Result::err();
  }
};

// SignatureService (lib.rs:229-254): a worker owns the secret key and answers
// signature requests in order (tokio task + mpsc(100) in the reference).
class SignatureService {
 public:
  explicit SignatureService(SecretKey secret) : secret_(std::move(secret)), worker_([this] { run(); }) {}
  ~SignatureService() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    worker_.join();
  }
  std::future<Signature> request_signature(const Digest &digest) {
    std::promise<Signature> p;
    std::future<Signature> f = p.get_future();
    {
      std::lock_guard<std::mutex> lk(mu_);
      queue_.emplace_back(digest, std::move(p));
    }
    cv_.notify_one();
    return f;
  }

 private:
  void run() {
    for (;;) {
      std::pair<Digest, std::promise<Signature>> job;
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [this] { return stop_ || !queue_.empty(); });
        if (queue_.empty()) return;
        job = std::move(queue_.front());
        queue_.pop_front();
      }
      try {
        job.second.set_value(Signature::sign(job.first, secret_));
      } catch (...) {
        job.second.set_exception(std::current_exception());
      }
    }
  }
  SecretKey secret_;
  std::mutex mu_;
  std::condition_variable cv_;
  std::deque<std::pair<Digest, std::promise<Signature>>> queue_;
  bool stop_ = false;
  std::thread worker_;
};

}  // namespace crypto

#endif  // HSV_CRYPTO_HPP_
