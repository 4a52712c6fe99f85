// Mempool transaction verification kernels.
//
// Reference: the client-transaction check in mempool/src/batch_maker.rs:79-85
// (and the batch re-check in consensus/src/core.rs:121-127):
//     message = tx[..len-96], pk = tx[len-96..len-64], sig = tx[len-64..]
//     digest  = Digest(SHA-512(message)[..32])
//     Signature::from_bytes(sig[..32], sig[32..64]).verify(&digest, &PublicKey(pk))
//
// Stage 1 (hsv_tx_record_kernel, one lane per transaction) hashes the message
// and writes the 128-byte record pk || R || s || digest; stage 2 is the
// generic verification launch over those records (strides 128, the same
// kernels and flags as hsv_verify_device).  The record pass is a small
// fraction of a verification: a 512-byte transaction is 4 SHA-512 blocks
// (about 4 x 80 rounds) against ~2,300 field operations for the signature.
#include <hip/hip_runtime.h>

#include "hsv_internal.h"
#include "hsv_txhash.hpp"

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

__global__ void __launch_bounds__(kTxBlock) hsv_tx_record_kernel(const uint8_t *__restrict__ txs,
                                                                  const uint64_t *__restrict__ offsets,
                                                                  uint64_t tx_size, uint32_t n,
                                                                  uint4 *__restrict__ rec) {
  const uint32_t i = blockIdx.x * kTxBlock + threadIdx.x;
  if (i >= n) return;
  uint64_t lo, hi;
  uint32_t r[32];
  if (tx_span(offsets, tx_size, i, lo, hi)) {
    const uintptr_t base = reinterpret_cast<uintptr_t>(txs);
    const uint4 *q = reinterpret_cast<const uint4 *>(base & ~uintptr_t(15));
    auto ld = [q](uint64_t k, uint32_t w[4]) {
      const uint4 v = q[k];
      w[0] = v.x;
      w[1] = v.y;
      w[2] = v.z;
      w[3] = v.w;
    };
    tx_record(ld, (uint64_t)(base & 15u) + lo, hi - lo, r);
  } else {
    HSV_UNROLL
    for (int j = 0; j < 32; ++j) r[j] = 0u;
  }
  uint4 *out = rec + (size_t)i * 8;
  HSV_UNROLL
  for (int j = 0; j < 8; ++j) out[j] = make_uint4(r[4 * j], r[4 * j + 1], r[4 * j + 2], r[4 * j + 3]);
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
  hipLaunchKernelGGL(hsv::hsv_tx_record_kernel, dim3(grid), dim3(hsv::kTxBlock), 0, stream, txs, offsets, tx_size,
                     n, reinterpret_cast<uint4 *>(records));
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
