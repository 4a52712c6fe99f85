// Mempool transaction digest.
//
// The reference's transaction check (mempool/src/batch_maker.rs:79-85 and
// consensus/src/core.rs:121-127, both guarded out in the shipped code) splits a
// client transaction as
//     tx = message || public_key (32 B) || signature (64 B, R || s)
// and verifies the signature over
//     Digest(SHA-512(message)[..32])
// with crypto::Signature::verify (crypto/src/lib.rs:204-208, verify_strict).
//
// One lane hashes one transaction.  The transaction starts at an arbitrary
// byte offset, so the lane reads the 16-byte-aligned chunks that contain its
// bytes (a chunk holding at least one byte of the transaction never crosses a
// page, so it is always mapped) and realigns them in registers: a word select
// for the offset's 4-byte part and a funnel shift for the byte part.  Message
// bytes past the end are replaced by the SHA-512 padding in the same pass.
//
// The routines take a chunk loader `ld(q, out[4])` so that the same code runs
// in the gfx950 kernel (hsv_mempool.hip) and in the host test build
// (tests/native/core_host.cpp, "txdigest").
#pragma once
#include "hsv_sha512.hpp"

namespace hsv {

// bytes [sh, sh+4) of the 8-byte little-endian pair lo||hi, sh in 0..3
HSV_INL uint32_t tx_funnel(uint32_t lo, uint32_t hi, uint32_t sh) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_alignbyte(hi, lo, sh);
#else
  return (uint32_t)((((uint64_t)hi << 32) | lo) >> (8 * sh));
#endif
}

// The NW little-endian words of bytes [sh16, sh16 + 4*NW) of raw (the words
// of NW/4 + 1 consecutive aligned chunks, plus one spare word).
template <int NW>
HSV_INL void tx_realign(const uint32_t raw[4 * (NW / 4 + 1) + 1], uint32_t sh16, uint32_t out[NW]) {
  const uint32_t s4 = sh16 >> 2, s1 = sh16 & 3u;
  // word-granular realignment by s4 (selects, no register indexing)
  uint32_t al[NW + 1];
  HSV_UNROLL
  for (int j = 0; j <= NW; ++j) {
    const uint32_t r0 = raw[j], r1 = raw[j + 1], r2 = raw[j + 2], r3 = raw[j + 3];
    al[j] = s4 == 0 ? r0 : s4 == 1 ? r1 : s4 == 2 ? r2 : r3;
  }
  HSV_UNROLL
  for (int j = 0; j < NW; ++j) out[j] = tx_funnel(al[j], al[j + 1], s1);
}

// The NW little-endian words of bytes [a, a + 4*NW) of the stream, where
// a = 16*q0 + sh16 (sh16 in 0..15) and ld(q, w) fills the aligned chunk q.
// Chunk indices are clamped to q_last (the last chunk holding a byte of the
// transaction), so every load is in bounds and unconditional; words built from
// a clamped chunk lie past the transaction's end and callers never use them
// (message padding replaces them, and the pk || sig words end at the end).
template <int NW, class LoadChunk>
HSV_INL void tx_load_words(LoadChunk &ld, uint64_t q0, uint32_t sh16, uint64_t q_last, uint32_t out[NW]) {
  constexpr int NQ = NW / 4 + 1;  // chunks covering 4*NW bytes at any offset
  uint32_t raw[4 * NQ + 1];
  HSV_UNROLL
  for (int k = 0; k < NQ; ++k) {
    uint32_t w[4];
    const uint64_t qk = q0 + (uint64_t)k;
    ld(qk < q_last ? qk : q_last, w);
    raw[4 * k + 0] = w[0];
    raw[4 * k + 1] = w[1];
    raw[4 * k + 2] = w[2];
    raw[4 * k + 3] = w[3];
  }
  raw[4 * NQ] = 0u;
  tx_realign<NW>(raw, sh16, out);
}

// Big-endian SHA-512 message word for bytes [p, p+8) of a message of mlen
// bytes, given the raw big-endian word x of the stream there: message bytes
// kept, then 0x80, then zeros (the length field is added by the caller).
// Branch-free (selects only): the compiler would otherwise emit exec-mask
// branches per word.
HSV_INL uint64_t tx_pad_word(uint64_t x, int64_t rem) {
  const uint32_t r = rem >= 8 ? 8u : rem < 0 ? 9u : (uint32_t)rem;  // 9: past the padding byte
  const uint32_t kb = r >= 8 ? (r == 8 ? 64u : 0u) : 8u * r;        // message bits kept, from the top
  const uint64_t keep = kb == 0 ? 0ull : ~0ull << (64u - kb);
  const uint64_t pad = r < 8 ? 0x80ull << (56u - 8u * r) : 0ull;
  return (x & keep) | pad;
}

// SHA-512 blocks of a message of mlen bytes: the padded message occupies
// (mlen + 17 + 127) / 128 blocks
HSV_INL uint64_t tx_num_blocks(uint64_t mlen) { return (mlen + 1 + 16 + 127) >> 7; }

// Compress block b of the padded message whose raw stream words (little-endian,
// bytes 128*b .. 128*b + 127 of the message) are `words`.
HSV_INL void tx_compress_block(uint64_t h[8], const uint32_t words[32], uint64_t mlen, uint64_t b,
                               uint64_t nblocks) {
  uint64_t w[16];
  HSV_UNROLL
  for (int j = 0; j < 16; ++j) {
    const int64_t rem = (int64_t)mlen - (int64_t)(b * 128 + 8 * (uint64_t)j);
    w[j] = tx_pad_word(be64_from_le32(words[2 * j], words[2 * j + 1]), rem);
  }
  if (b + 1 == nblocks) {
    w[14] = mlen >> 61;  // 128-bit big-endian bit length
    w[15] = mlen << 3;
  }
  sha512_compress(h, w);
}

// The same for a block wholly inside the message ((b + 1) * 128 <= mlen): no
// padding word, no length field.  The kernel takes it when every lane of the
// wave is in that case (wave-uniform branch), which is all but the last block
// of equal-sized transactions.
HSV_INL void tx_compress_full_block(uint64_t h[8], const uint32_t words[32]) {
  uint64_t w[16];
  HSV_UNROLL
  for (int j = 0; j < 16; ++j) w[j] = be64_from_le32(words[2 * j], words[2 * j + 1]);
  sha512_compress(h, w);
}

// First 32 digest bytes as 8 little-endian words.
HSV_INL void tx_digest_words(const uint64_t h[8], uint32_t out[8]) {
  HSV_UNROLL
  for (int i = 0; i < 4; ++i) {
    out[2 * i] = bswap32((uint32_t)(h[i] >> 32));
    out[2 * i + 1] = bswap32((uint32_t)h[i]);
  }
}

// digest = SHA-512(message)[..32] as 8 little-endian words (the byte order the
// verification kernels read a 32-byte Digest in), for a message of mlen bytes
// at stream byte address `start`; q_last = last chunk holding a byte of the
// transaction (bounds every load).
template <class LoadChunk>
HSV_INL void tx_message_digest(LoadChunk &ld, uint64_t start, uint64_t mlen, uint64_t q_last,
                               uint32_t out[8]) {
  uint64_t h[8];
  sha512_init(h);
  const uint64_t nblocks = tx_num_blocks(mlen);
  const uint32_t sh16 = (uint32_t)(start & 15u);
  HSV_NOUNROLL
  for (uint64_t b = 0; b < nblocks; ++b) {
    uint32_t words[32];
    tx_load_words<32>(ld, (start >> 4) + 8 * b, sh16, q_last, words);
    tx_compress_block(h, words, mlen, b, nblocks);
  }
  tx_digest_words(h, out);
}

// The 128-byte verification record of one transaction of tx_len >= 96 bytes at
// stream byte address `start`:  pk (32) || R || s (64) || digest (32), i.e.
// the packed-record layout hsv_verify_device reads with strides 128.
template <class LoadChunk>
HSV_INL void tx_record(LoadChunk &ld, uint64_t start, uint64_t tx_len, uint32_t rec[32]) {
  const uint64_t mlen = tx_len - 96;
  const uint64_t q_last = (start + tx_len - 1) >> 4;
  const uint64_t tail = start + mlen;  // pk || sig
  tx_load_words<24>(ld, tail >> 4, (uint32_t)(tail & 15u), q_last, rec);
  tx_message_digest(ld, start, mlen, q_last, rec + 24);
}

}  // namespace hsv
