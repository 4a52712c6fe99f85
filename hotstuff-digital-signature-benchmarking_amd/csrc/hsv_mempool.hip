// Mempool transaction verification kernels.
//
// Reference: the client-transaction check in mempool/src/batch_maker.rs:79-85
// (and the batch re-check in consensus/src/core.rs:121-127):
//     message = tx[..len-96], pk = tx[len-96..len-64], sig = tx[len-64..]
//     digest  = Digest(SHA-512(message)[..32])
//     Signature::from_bytes(sig[..32], sig[32..64]).verify(&digest, &PublicKey(pk))
//
// Stage 1 (hsv_tx_record_kernel, one lane per transaction, loads staged through
// LDS by the whole wave) hashes the message and writes the 128-byte record
// pk || R || s || digest; stage 2 is the
// generic verification launch over those records (strides 128, the same
// kernels and flags as hsv_verify_device).  The record pass is a small
// fraction of a verification: a 512-byte transaction is 4 SHA-512 blocks
// (about 4 x 80 rounds) against ~2,300 field operations for the signature.
#include <hip/hip_runtime.h>

// The message hash in this file runs gfx950's v_bitop3_b32 for the sigma XOR
// triples, the majority and the choice (hsv_sha512.hpp): with the bitop3
// results kept as opaque 64-bit pairs that is 754 instead of 991 instructions
// per 16 rounds, and the record kernel went from 0.99 to 0.82 ms per 2^20
// transactions together with the full-block fast path below
// (profiles/r06/r06k_*).  The latency kernels keep the XOR form (their lone
// waves measured no faster with it).
#define HSV_SHA_BITOP3 1
#include "hsv_internal.h"
#include "hsv_txhash.hpp"
#include "hsv_verify_hc.hpp"

namespace hsv {

constexpr int kTxBlock = 256;

// Transaction i spans [lo, hi) bytes of txs: offsets[i], offsets[i+1] when
// offsets is given, else i*tx_size, (i+1)*tx_size.  A transaction shorter
// than 96 bytes (the reference's slice would panic) gets an all-zero record
// here and flags 0 from hsv_tx_mask_kernel.
__device__ __forceinline__ bool tx_span(const uint64_t *offsets, uint64_t tx_size, uint32_t i, uint64_t &lo,
                                        uint64_t &hi) {
  if (offsets) {
    lo = offsets[i];
    hi = offsets[i + 1];
  } else {
    lo = (uint64_t)i * tx_size;
    hi = lo + tx_size;
  }
  return hi >= lo && hi - lo >= 96;
}

constexpr int kTxWaves = kTxBlock / 64;
constexpr int kTxQ = 9;                   // 16-B chunks under a 128-B window at any offset
constexpr uint64_t kNoChunk = ~0ull;      // lane without a transaction: loads nothing

__device__ __forceinline__ uint64_t shfl_u64(uint64_t v, int src) {
  const uint32_t lo = (uint32_t)__shfl((int)(uint32_t)v, src, 64);
  const uint32_t hi = (uint32_t)__shfl((int)(uint32_t)(v >> 32), src, 64);
  return ((uint64_t)hi << 32) | lo;
}

// The wave's NQ chunks starting at chunk first(t) (clamped to last(t)) for each
// of its 64 transactions t, staged through LDS with consecutive lanes reading
// consecutive chunks of one transaction (one load instruction covers about
// 64/NQ transactions' runs instead of 64 scattered lines); lane l gets the raw
// words of its own transaction.
template <int NQ>
__device__ __forceinline__ void tx_stage_chunks(const uint4 *__restrict__ q, uint4 *stage, uint32_t lane,
                                                uint64_t first, uint64_t last, uint32_t raw[4 * NQ + 1]) {
  HSV_UNROLL
  for (int it = 0; it < NQ; ++it) {
    const uint32_t e = (uint32_t)it * 64u + lane;  // = t * NQ + c
    const uint32_t t = e / NQ, c = e - t * NQ;
    const uint64_t f = shfl_u64(first, (int)t), l = shfl_u64(last, (int)t);
    uint4 v = make_uint4(0u, 0u, 0u, 0u);
    if (l != kNoChunk) {
      const uint64_t k = f + c;
      v = q[k < l ? k : l];
    }
    stage[e] = v;
  }
  __builtin_amdgcn_wave_barrier();
  HSV_UNROLL
  for (int k = 0; k < NQ; ++k) {
    const uint4 v = stage[lane * NQ + k];
    raw[4 * k] = v.x;
    raw[4 * k + 1] = v.y;
    raw[4 * k + 2] = v.z;
    raw[4 * k + 3] = v.w;
  }
  raw[4 * NQ] = 0u;
  __builtin_amdgcn_wave_barrier();  // every lane has read before the next staging round
}

// One lane per transaction; the wave's loads are cooperative (tx_stage_chunks).
// Waves are independent: each loops over its own longest message.
// PREP (large batches, hsv_launch_tx_prep): the same lane then runs the scalar
// prepass of the generic point pass on the record it holds in registers
// (SHA-512(R || A || digest), k mod l, lattice reduction, recoding;
// prep_scalars, hsv_verify_hc.hpp) and writes its SoA record, so a
// transaction's bytes are read once and no separate prepass reads the
// records back (round-2 VERDICT item 8).
template <bool PREP>
__global__ void __launch_bounds__(kTxBlock) hsv_tx_record_kernel(const uint8_t *__restrict__ txs,
                                                                  const uint64_t *__restrict__ offsets,
                                                                  uint64_t tx_size, uint32_t n,
                                                                  uint4 *__restrict__ rec,
                                                                  uint32_t *__restrict__ prep,
                                                                  uint32_t *__restrict__ fb_count,
                                                                  uint32_t *__restrict__ fb_list, int lat_bits) {
  __shared__ uint4 stage_all[kTxWaves][64 * kTxQ];
  if constexpr (PREP) __builtin_amdgcn_s_setprio(3);  // as hsv_prep_kernel: ahead of a running point pass
  const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
  if (blockIdx.x * kTxBlock + wv * 64u >= n) return;  // whole wave past the end
  uint4 *stage = stage_all[wv];
  const uint32_t i = blockIdx.x * kTxBlock + threadIdx.x;
  uint64_t lo = 0, hi = 0;
  const bool ok = i < n && tx_span(offsets, tx_size, i, lo, hi);
  const uintptr_t base = reinterpret_cast<uintptr_t>(txs);
  const uint4 *q = reinterpret_cast<const uint4 *>(base & ~uintptr_t(15));
  const uint64_t start = (uint64_t)(base & 15u) + lo;
  const uint64_t mlen = ok ? hi - lo - 96 : 0;
  const uint64_t q_last = ok ? (start + (hi - lo) - 1) >> 4 : kNoChunk;
  // SHA-512 of the message, block by block
  uint64_t h[8];
  sha512_init(h);
  const uint64_t nblocks = tx_num_blocks(mlen);
  uint32_t wave_blocks = (uint32_t)nblocks;
  HSV_UNROLL
  for (int m = 1; m < 64; m <<= 1) wave_blocks = max(wave_blocks, (uint32_t)__shfl_xor((int)wave_blocks, m, 64));
  const uint32_t sh16 = (uint32_t)(start & 15u);
  // wave-uniform fast paths: every transaction of the wave starts on a 16-byte
  // boundary (no realignment), and block b lies wholly inside every message
  // (no padding selects) -- the common case of equal-sized transactions
  const bool wave_aligned = __all(sh16 == 0u);
  HSV_NOUNROLL
  for (uint32_t b = 0; b < wave_blocks; ++b) {
    uint32_t raw[4 * kTxQ + 1];
    tx_stage_chunks<kTxQ>(q, stage, lane, (start >> 4) + 8ull * b, q_last, raw);
    const bool wave_full = __all((uint64_t)(b + 1u) * 128u <= mlen);
    if (b < nblocks) {
      uint32_t words[32];
      if (wave_aligned) {
        HSV_UNROLL
        for (int j = 0; j < 32; ++j) words[j] = raw[j];
      } else {
        tx_realign<32>(raw, sh16, words);
      }
      if (wave_full) tx_compress_full_block(h, words);
      else tx_compress_block(h, words, mlen, b, nblocks);
    }
  }
  // pk || R || s: the last 96 bytes (7 chunks at any offset), staged after
  // the hash so that its 24 words are not live across the message loop
  uint32_t r[32];
  {
    const uint64_t tail = start + mlen;
    uint32_t raw[4 * 7 + 1];
    tx_stage_chunks<7>(q, stage, lane, tail >> 4, q_last, raw);
    tx_realign<24>(raw, (uint32_t)(tail & 15u), r);
  }
  tx_digest_words(h, r + 24);
  if (i >= n) return;
  if (!ok) {
    HSV_UNROLL
    for (int j = 0; j < 32; ++j) r[j] = 0u;
  }
  uint4 *out = rec + (size_t)i * 8;
  HSV_UNROLL
  for (int j = 0; j < 8; ++j) out[j] = make_uint4(r[4 * j], r[4 * j + 1], r[4 * j + 2], r[4 * j + 3]);
  if constexpr (PREP) {
    // pk = r[0..8), R || s = r[8..24), digest = r[24..32)
    if (prep_scalars<4>(r, r + 8, r + 24, prep + i, n, lat_bits)) fb_list[atomicAdd(fb_count, 1u)] = i;
  }
}

// Zero the flags (and the STRICT_OK bit) of transactions shorter than 96 bytes.
__global__ void __launch_bounds__(kTxBlock) hsv_tx_mask_kernel(const uint64_t *__restrict__ offsets, uint32_t n,
                                                                uint8_t *flags, uint32_t *strict_bits) {
  const uint32_t i = blockIdx.x * kTxBlock + threadIdx.x;
  if (i >= n) return;
  uint64_t lo, hi;
  if (tx_span(offsets, 0, i, lo, hi)) return;
  if (flags) flags[i] = 0;
  if (strict_bits) atomicAnd(strict_bits + (i >> 5), ~(1u << (i & 31u)));
}

}  // namespace hsv

extern "C" hipError_t hsv_launch_tx_records(const uint8_t *txs, const uint64_t *offsets, uint64_t tx_size,
                                            uint32_t n, uint8_t *records, hipStream_t stream) {
  if (n == 0) return hipSuccess;
  const uint32_t grid = (n + hsv::kTxBlock - 1) / hsv::kTxBlock;
  hipLaunchKernelGGL((hsv::hsv_tx_record_kernel<false>), dim3(grid), dim3(hsv::kTxBlock), 0, stream, txs, offsets,
                     tx_size, n, reinterpret_cast<uint4 *>(records), nullptr, nullptr, nullptr, 0);
  return hipGetLastError();
}

extern "C" hipError_t hsv_launch_tx_prep(const uint8_t *txs, const uint64_t *offsets, uint64_t tx_size, uint32_t n,
                                         uint8_t *records, uint32_t *prep, uint32_t *fb_count, uint32_t *fb_list,
                                         int lat_bits, hipStream_t stream) {
  if (n == 0) return hipSuccess;
  const uint32_t grid = (n + hsv::kTxBlock - 1) / hsv::kTxBlock;
  hipLaunchKernelGGL((hsv::hsv_tx_record_kernel<true>), dim3(grid), dim3(hsv::kTxBlock), 0, stream, txs, offsets,
                     tx_size, n, reinterpret_cast<uint4 *>(records), prep, fb_count, fb_list, lat_bits);
  return hipGetLastError();
}

extern "C" hipError_t hsv_launch_tx_mask(const uint64_t *offsets, uint32_t n, uint8_t *flags,
                                         uint32_t *strict_bits, hipStream_t stream) {
  if (n == 0 || !offsets) return hipSuccess;
  const uint32_t grid = (n + hsv::kTxBlock - 1) / hsv::kTxBlock;
  hipLaunchKernelGGL(hsv::hsv_tx_mask_kernel, dim3(grid), dim3(hsv::kTxBlock), 0, stream, offsets, n, flags,
                     strict_bits);
  return hipGetLastError();
}
