// Wire formats: QC and TC certificates verified straight
// from their bincode bytes, so a node can check a certificate it received
// without first materialising the Rust structs.  Parsing is in
// hsv_wire_parse.cpp (GPU-free, fuzzed under ASan/UBSan by
// tests/native/wire_fuzz.cpp); this file hands the parsed votes to the
// verification entry points.
//
// The crypto part of QC::verify (consensus/src/messages.rs:196-197) is
//   Signature::verify_batch(&qc.digest(), &qc.votes)
// and of TC::verify (messages.rs:306-313) one Signature::verify per vote over
// SHA-512(round_le || high_qc_round_le)[..32]; the TC goes through the
// batched strict API (hsv_verify), which uses the committee key cache when
// every key is cached.  Malformed bytes return HSV_ERR_PARSE (the reference's
// bincode::deserialize error); the quorum / stake checks of QC::verify and
// TC::verify stay with the caller.
#include <cstring>
#include <string>
#include <vector>

#include "hsv.h"
#include "hsv_host.h"
#include "hsv_internal.h"
#include "hsv_wire_parse.h"

namespace {

int parse_error(const std::string &what) { return hsvi_set_error(HSV_ERR_PARSE, ("bincode: " + what).c_str()); }

}  // namespace

extern "C" {

int hsv_qc_verify_bincode(const uint8_t *buf, size_t len, size_t *n_votes_out, uint8_t *pks_out) {
  hsvh::CallScope call;  // the host timeline includes the parse
  if (!buf && len) return hsvi_set_error(HSV_ERR_INVALID_ARG, "null buffer");
  thread_local hsvw::QcParsed qc;  // keeps its vote buffer from call to call
  std::string err;
  if (!hsvw::parse_qc(buf, len, qc, err)) return parse_error(err);
  if (n_votes_out) *n_votes_out = qc.n;
  if (pks_out)
    for (size_t i = 0; i < qc.n; ++i) std::memcpy(pks_out + i * 32, qc.votes.data() + i * 96, 32);
  return hsv_verify_batch_packed(qc.digest, qc.votes.data(), qc.n);
}

int hsv_tc_verify_bincode(const uint8_t *buf, size_t len, size_t *n_votes_out, uint8_t *flags_out) {
  hsvh::CallScope call;
  if (!buf && len) return hsvi_set_error(HSV_ERR_INVALID_ARG, "null buffer");
  thread_local hsvw::TcParsed tc;
  std::string err;
  if (!hsvw::parse_tc(buf, len, tc, err)) return parse_error(err);
  if (n_votes_out) *n_votes_out = tc.n;
  if (tc.n == 0) return 1;
  std::vector<uint8_t> flags(tc.n);
  uint8_t *f = flags_out ? flags_out : flags.data();
  const int rc = hsv_verify(tc.pks.data(), tc.sigs.data(), tc.digests.data(), 32, tc.n, f);
  if (rc != HSV_OK) return rc;
  for (size_t i = 0; i < tc.n; ++i)
    if (!(f[i] & HSV_STRICT_OK)) return 0;
  return 1;
}

}  // extern "C"
