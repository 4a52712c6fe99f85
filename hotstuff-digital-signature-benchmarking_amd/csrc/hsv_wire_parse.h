// Parsers of the consensus certificates' bincode bytes (no GPU code): the
// part of hsv_qc_verify_bincode / hsv_tc_verify_bincode that reads untrusted
// network bytes (the reference receives them as TCP frames,
// network/src/receiver.rs:47-60, consensus/src/consensus.rs:32-39).  Kept in
// its own translation unit so tests/native/wire_fuzz.cpp can build it alone
// under AddressSanitizer / UndefinedBehaviorSanitizer.
#pragma once
#include <cstddef>
#include <cstdint>
#include <string>
#include <vector>

namespace hsvw {

// consensus::QC (consensus/src/messages.rs:162-167) -> packed pk||R||s votes
// and qc.digest() = SHA-512(hash || round_le)[..32] (messages.rs:201-207).
struct QcParsed {
  uint8_t digest[32];
  uint64_t round = 0;
  std::vector<uint8_t> votes;  // n * 96
  size_t n = 0;
};

// consensus::TC (messages.rs:281-285) -> per-vote pk, sig and digest
// SHA-512(round_le || high_qc_round_le)[..32] (messages.rs:306-313).
struct TcParsed {
  uint64_t round = 0;
  std::vector<uint8_t> pks, sigs, digests;  // n * 32, n * 64, n * 32
  size_t n = 0;
};

// true on success; on failure `err` says what was malformed
bool parse_qc(const uint8_t *buf, size_t len, QcParsed &out, std::string &err);
bool parse_tc(const uint8_t *buf, size_t len, TcParsed &out, std::string &err);

// base64 0.13 standard decoding (PublicKey::decode_base64, crypto/src/lib.rs:73-79)
bool b64_decode(const uint8_t *s, size_t n, std::vector<uint8_t> &out);

}  // namespace hsvw
