// Wire formats: QC and TC certificates verified straight
// from their bincode bytes, so a node can check a certificate it received
// without first materialising the Rust structs.
//
// Layouts (bincode 1.3 default options: little-endian, fixed-width integers,
// u64 length prefixes; the serde derives of the reference):
//   Digest            32 raw bytes            crypto/src/lib.rs:20-22
//   PublicKey         str: u64 len + base64   crypto/src/lib.rs:94-101
//   Signature         part1 (32) || part2 (32) crypto/src/lib.rs:176-182
//   QC  = hash: Digest | round: u64 | votes: Vec<(PublicKey, Signature)>
//                                              consensus/src/messages.rs:162-167
//   TC  = round: u64 | votes: Vec<(PublicKey, Signature, Round)>
//                                              consensus/src/messages.rs:281-285
// The crypto part of QC::verify (messages.rs:196-197) is
//   Signature::verify_batch(&qc.digest(), &qc.votes),
//   qc.digest() = SHA-512(hash || round_le)[..32]            (messages.rs:201-207)
// and of TC::verify (messages.rs:306-313) one Signature::verify per vote over
//   SHA-512(round_le || high_qc_round_le)[..32].
// The TC's per-vote digests are exactly the mempool transaction digest of the
// 16-byte message round_le || high_qc_round_le, so a TC vote is verified as
// the 112-byte transaction  round_le || hqc_le || pk || sig  on the GPU
// (hsv_verify_transactions_fixed): no host hashing.
//
// PublicKey::decode_base64 (crypto/src/lib.rs:73-79) runs base64 0.13's
// standard decoder and keeps the first 32 bytes; shorter decodings are an
// error.  This decoder follows the same rules: standard alphabet, optional
// '=' padding only at the end, no non-zero trailing bits.  Malformed bytes
// return HSV_ERR_PARSE (the reference's bincode::deserialize error); the
// quorum / stake checks of QC::verify and TC::verify stay with the caller.
#include <cstring>
#include <string>
#include <vector>

#include "hsv.h"
#include "hsv_internal.h"
#include "hsv_sha512.hpp"

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

int b64_value(uint8_t c) {
  if (c >= 'A' && c <= 'Z') return c - 'A';
  if (c >= 'a' && c <= 'z') return c - 'a' + 26;
  if (c >= '0' && c <= '9') return c - '0' + 52;
  if (c == '+') return 62;
  if (c == '/') return 63;
  return -1;
}

// Standard-alphabet base64 -> bytes; false on an invalid symbol, misplaced
// padding, an impossible length or non-zero trailing bits.
bool b64_decode(const uint8_t *s, size_t n, std::vector<uint8_t> &out) {
  size_t end = n;
  while (end > 0 && s[end - 1] == '=') --end;
  if (n - end > 2) return false;
  if (n != end && n % 4 != 0) return false;  // padded input comes in whole quads
  const size_t rem = end % 4;
  if (rem == 1) return false;
  out.clear();
  out.reserve(end * 3 / 4);
  uint32_t acc = 0;
  int bits = 0;
  for (size_t i = 0; i < end; ++i) {
    const int v = b64_value(s[i]);
    if (v < 0) return false;
    acc = (acc << 6) | (uint32_t)v;
    bits += 6;
    if (bits >= 8) {
      bits -= 8;
      out.push_back((uint8_t)(acc >> bits));
      acc &= (1u << bits) - 1u;
    }
  }
  return acc == 0;  // the leftover (trailing) bits must be zero
}

// PublicKey from its bincode str
bool read_public_key(Reader &r, uint8_t pk[32]) {
  uint64_t len = 0;
  const uint8_t *s = nullptr;
  if (!r.u64(len) || len > r.left || !r.bytes(s, (size_t)len)) return false;
  std::vector<uint8_t> dec;
  if (!b64_decode(s, (size_t)len, dec) || dec.size() < 32) return false;
  std::memcpy(pk, dec.data(), 32);
  return true;
}

int parse_error(const std::string &what) { return hsv_set_error(HSV_ERR_PARSE, ("bincode: " + what).c_str()); }

}  // namespace

extern "C" {

int hsv_qc_verify_bincode(const uint8_t *buf, size_t len, size_t *n_votes_out, uint8_t *pks_out) {
  if (!buf && len) return hsv_set_error(HSV_ERR_INVALID_ARG, "null buffer");
  Reader r{buf, len};
  const uint8_t *hash = nullptr;
  uint64_t round = 0, nv = 0;
  if (!r.bytes(hash, 32) || !r.u64(round) || !r.u64(nv)) return parse_error("truncated QC header");
  if (nv > r.left / 72) return parse_error("vote count exceeds the buffer");
  std::vector<uint8_t> votes((size_t)nv * 96);
  for (uint64_t i = 0; i < nv; ++i) {
    uint8_t *v = votes.data() + i * 96;
    const uint8_t *sig = nullptr;
    if (!read_public_key(r, v)) return parse_error("vote " + std::to_string(i) + ": bad public key");
    if (!r.bytes(sig, 64)) return parse_error("vote " + std::to_string(i) + ": truncated signature");
    std::memcpy(v + 32, sig, 64);
  }
  if (r.left != 0) return parse_error("trailing bytes after the QC");
  if (n_votes_out) *n_votes_out = (size_t)nv;
  if (pks_out)
    for (uint64_t i = 0; i < nv; ++i) std::memcpy(pks_out + i * 32, votes.data() + i * 96, 32);
  // qc.digest() = SHA-512(hash || round_le)[..32]
  uint8_t pre[40], h[64];
  std::memcpy(pre, hash, 32);
  for (int i = 0; i < 8; ++i) pre[32 + i] = (uint8_t)(round >> (8 * i));
  hsv::sha512_bytes(pre, sizeof(pre), h);
  return hsv_verify_batch_packed(h, votes.data(), (size_t)nv);
}

int hsv_tc_verify_bincode(const uint8_t *buf, size_t len, size_t *n_votes_out, uint8_t *flags_out) {
  if (!buf && len) return hsv_set_error(HSV_ERR_INVALID_ARG, "null buffer");
  Reader r{buf, len};
  uint64_t round = 0, nv = 0;
  if (!r.u64(round) || !r.u64(nv)) return parse_error("truncated TC header");
  if (nv > r.left / 80) return parse_error("vote count exceeds the buffer");
  // each vote as the 112-byte transaction round_le || hqc_le || pk || sig
  std::vector<uint8_t> txs((size_t)nv * 112);
  for (uint64_t i = 0; i < nv; ++i) {
    uint8_t *t = txs.data() + i * 112;
    const uint8_t *sig = nullptr;
    uint64_t hqc = 0;
    if (!read_public_key(r, t + 16)) return parse_error("vote " + std::to_string(i) + ": bad public key");
    if (!r.bytes(sig, 64) || !r.u64(hqc)) return parse_error("vote " + std::to_string(i) + ": truncated");
    std::memcpy(t + 48, sig, 64);
    for (int b = 0; b < 8; ++b) {
      t[b] = (uint8_t)(round >> (8 * b));
      t[8 + b] = (uint8_t)(hqc >> (8 * b));
    }
  }
  if (r.left != 0) return parse_error("trailing bytes after the TC");
  if (n_votes_out) *n_votes_out = (size_t)nv;
  if (nv == 0) return 1;
  std::vector<uint8_t> flags((size_t)nv);
  uint8_t *f = flags_out ? flags_out : flags.data();
  const int rc = hsv_verify_transactions_fixed(txs.data(), 112, (size_t)nv, f);
  if (rc != HSV_OK) return rc;
  for (uint64_t i = 0; i < nv; ++i)
    if (!(f[i] & HSV_STRICT_OK)) return 0;
  return 1;
}

}  // extern "C"
