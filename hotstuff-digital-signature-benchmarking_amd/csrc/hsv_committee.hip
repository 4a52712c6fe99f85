// Committee key cache kernels, see hsv_comb.hpp.
//
//  hsv_comb_build_kernel   one lane per (key, position j): [2^(8j)](+/-P) by
//                          8j doublings (j is wave-uniform: keys are padded to
//                          a multiple of 64 per position), 127 additions, one
//                          batched inversion -> 128 affine Niels entries.
//  hsv_comb_verify_kernel  one verification per lane against a cached key:
//                          64 mixed additions from the key's table and the B
//                          table, then R decompression and the projective
//                          comparison.  Same flag byte as hsv_verify_kernel.
#include <hip/hip_runtime.h>

#include "hsv_comb.hpp"
#include "hsv_internal.h"

namespace hsv {

__global__ void __launch_bounds__(256)
hsv_comb_build_kernel(const uint8_t *__restrict__ encs, uint32_t nkeys, uint32_t npad, uint32_t negate,
                      uint32_t *__restrict__ tables, uint32_t *__restrict__ tmp,
                      uint8_t *__restrict__ key_flags) {
  const uint32_t id = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t j = id / npad, key = id % npad;
  if (j >= (uint32_t)kCombPos || key >= nkeys) return;
  uint32_t w[8];
  const uint4 *p = reinterpret_cast<const uint4 *>(encs + (uint64_t)key * 32);
  const uint4 p0 = p[0], p1 = p[1];
  w[0] = p0.x; w[1] = p0.y; w[2] = p0.z; w[3] = p0.w;
  w[4] = p1.x; w[5] = p1.y; w[6] = p1.z; w[7] = p1.w;
  fe x, y;
  const uint32_t ok = ge_decompress(w, x, y);
  if (j == 0 && key_flags) key_flags[key] = (uint8_t)((ok ? kKeyAOk : 0u) | (ok && y_is_small_order(y) ? kKeySmallA : 0u));
  const ge_ext base = comb_position_base(x, y, negate, (int)j);
  comb_build_position(base, tables + (uint64_t)key * kCombTableWords + (uint64_t)j * kCombEnt * kCombEntryWords,
                      tmp + (uint64_t)id * kCombEnt * 8);
}

__global__ void __launch_bounds__(256, 2)
hsv_comb_verify_kernel(const uint32_t *__restrict__ key_idx, const uint8_t *__restrict__ sig,
                       uint64_t sig_stride, const uint8_t *__restrict__ msg, uint64_t msg_stride,
                       uint32_t m, const uint8_t *__restrict__ pks, const uint8_t *__restrict__ key_flags,
                       uint32_t nkeys, const uint32_t *__restrict__ tables,
                       const uint32_t *__restrict__ btable, uint8_t *__restrict__ flags_out) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= m) return;
  const uint32_t kidx = key_idx[i];
  const bool kvalid = kidx < nkeys;
  const uint32_t kk = kvalid ? kidx : 0u;
  uint32_t pkw[8], sigw[16], msgw[8];
  {
    const uint4 *p = reinterpret_cast<const uint4 *>(pks + (uint64_t)kk * 32);
    const uint4 *s = reinterpret_cast<const uint4 *>(sig + (uint64_t)i * sig_stride);
    const uint4 *g = reinterpret_cast<const uint4 *>(msg + (uint64_t)i * msg_stride);
    const uint4 p0 = p[0], p1 = p[1];
    const uint4 s0 = s[0], s1 = s[1], s2 = s[2], s3 = s[3];
    const uint4 m0 = g[0], m1 = g[1];
    pkw[0] = p0.x; pkw[1] = p0.y; pkw[2] = p0.z; pkw[3] = p0.w;
    pkw[4] = p1.x; pkw[5] = p1.y; pkw[6] = p1.z; pkw[7] = p1.w;
    sigw[0] = s0.x; sigw[1] = s0.y; sigw[2] = s0.z; sigw[3] = s0.w;
    sigw[4] = s1.x; sigw[5] = s1.y; sigw[6] = s1.z; sigw[7] = s1.w;
    sigw[8] = s2.x; sigw[9] = s2.y; sigw[10] = s2.z; sigw[11] = s2.w;
    sigw[12] = s3.x; sigw[13] = s3.y; sigw[14] = s3.z; sigw[15] = s3.w;
    msgw[0] = m0.x; msgw[1] = m0.y; msgw[2] = m0.z; msgw[3] = m0.w;
    msgw[4] = m1.x; msgw[5] = m1.y; msgw[6] = m1.z; msgw[7] = m1.w;
  }
  const uint32_t f = verify_one_comb(pkw, key_flags[kk], sigw, msgw,
                                     tables + (uint64_t)kk * kCombTableWords, btable);
  flags_out[i] = kvalid ? (uint8_t)f : (uint8_t)0;
}

// one lane per (position j, chunk c) of the wide B table; j is wave-uniform
// (256 chunks per position)
__global__ void __launch_bounds__(256) hsv_comb16_build_kernel(uint32_t *__restrict__ table,
                                                             uint32_t *__restrict__ tmp) {
  const uint32_t id = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t j = id / (uint32_t)kComb16ChunksPerPos, c = id % (uint32_t)kComb16ChunksPerPos;
  if (j >= (uint32_t)kComb16Pos) return;
  const uint32_t bw[8] = {0x66666658u, 0x66666666u, 0x66666666u, 0x66666666u,
                          0x66666666u, 0x66666666u, 0x66666666u, 0x66666666u};
  fe x, y;
  (void)ge_decompress(bw, x, y);
  comb16_build_chunk(x, y, (int)j, c, table, tmp + (uint64_t)id * kComb16Chunk * 8);
}

}  // namespace hsv

extern "C" hipError_t hsv_launch_comb16_build(uint32_t *table, uint32_t *tmp, hipStream_t stream) {
  const uint32_t lanes = (uint32_t)(hsv::kComb16Pos * hsv::kComb16ChunksPerPos);
  hipLaunchKernelGGL(hsv::hsv_comb16_build_kernel, dim3(lanes / 256u), dim3(256), 0, stream, table, tmp);
  return hipGetLastError();
}

extern "C" uint64_t hsv_comb16_table_bytes(void) { return hsv::kComb16TableWords * 4ull; }
extern "C" uint64_t hsv_comb16_tmp_bytes(void) {
  return (uint64_t)hsv::kComb16Pos * hsv::kComb16ChunksPerPos * hsv::kComb16Chunk * 8ull * 4ull;
}

extern "C" hipError_t hsv_launch_comb_build(const uint8_t *encs, uint32_t nkeys, uint32_t negate,
                                            uint32_t *tables, uint32_t *tmp, uint8_t *key_flags,
                                            hipStream_t stream) {
  if (nkeys == 0) return hipSuccess;
  const uint32_t npad = (nkeys + 63u) / 64u * 64u;
  const uint32_t lanes = npad * (uint32_t)hsv::kCombPos;
  hipLaunchKernelGGL(hsv::hsv_comb_build_kernel, dim3((lanes + 255u) / 256u), dim3(256), 0, stream, encs,
                     nkeys, npad, negate, tables, tmp, key_flags);
  return hipGetLastError();
}

extern "C" hipError_t hsv_launch_comb_verify(const uint32_t *key_idx, const uint8_t *sig, uint64_t sig_stride,
                                             const uint8_t *msg, uint64_t msg_stride, uint32_t m,
                                             const uint8_t *pks, const uint8_t *key_flags, uint32_t nkeys,
                                             const uint32_t *tables, const uint32_t *btable,
                                             uint8_t *flags_out, hipStream_t stream) {
  if (m == 0) return hipSuccess;
  hipLaunchKernelGGL(hsv::hsv_comb_verify_kernel, dim3((m + 255u) / 256u), dim3(256), 0, stream, key_idx, sig,
                     sig_stride, msg, msg_stride, m, pks, key_flags, nkeys, tables, btable, flags_out);
  return hipGetLastError();
}

extern "C" uint64_t hsv_comb_table_bytes(void) { return hsv::kCombTableWords * 4ull; }
extern "C" uint64_t hsv_comb_tmp_bytes(uint32_t nkeys) {
  const uint64_t npad = (nkeys + 63u) / 64u * 64u;
  return npad * (uint64_t)hsv::kCombPos * hsv::kCombEnt * 8ull * 4ull;
}
