// Minimal reproducer of the strict-bits hang of the persistent point pass
// (round 1, commit 6e5c7e3).  Both kernels take 64-item
// batches from an atomic counter (lane 0 adds, the base is broadcast) and
// store the wave's 64-bit ballot into a bit array.  k_double stores both
// halves from lane 0 (two nested conditional stores); k_pair stores one word
// each from lanes 0 and 1.  hipcc for gfx950 compiles k_double's work loop as
// a DIVERGENT loop (exec-masked back edge, exit mask taken from the exec left
// by the lane-0 region) and k_pair's as a uniform loop (VCC-tested back edge).
// The hardware is never needed: tests/test_kernel_isa.py compiles this file
// with -S and checks both forms, and checks that the product kernels' work
// loops are uniform.  Not a product source; never launched.
#include <hip/hip_runtime.h>

#include <cstdint>

__global__ void k_double(uint32_t *next, uint32_t n, const uint32_t *in, uint32_t *bits) {
  const uint32_t lane = threadIdx.x & 63u;
  for (;;) {
    uint32_t base = 0;
    if (lane == 0) base = atomicAdd(next, 64u);
    base = __builtin_amdgcn_readfirstlane(__shfl(base, 0));
    if (base >= n) break;
    const uint32_t idx = base + lane;
    const bool valid = idx < n;
    uint32_t x = valid ? in[idx] : 0u;
    for (int i = 0; i < 64; ++i) x = x * 2654435761u + (x >> 7);
    const uint64_t mask = __ballot(valid && (x & 1u));
    const uint32_t nwords = (n + 31u) / 32u;
    if (lane == 0) {
      const uint32_t w0 = base / 32u;
      if (w0 < nwords) bits[w0] = (uint32_t)mask;
      if (w0 + 1 < nwords) bits[w0 + 1] = (uint32_t)(mask >> 32);
    }
  }
}
__global__ void k_pair(uint32_t *next, uint32_t n, const uint32_t *in, uint32_t *bits) {
  const uint32_t lane = threadIdx.x & 63u;
  for (;;) {
    uint32_t base = 0;
    if (lane == 0) base = atomicAdd(next, 64u);
    base = __builtin_amdgcn_readfirstlane(__shfl(base, 0));
    if (base >= n) break;
    const uint32_t idx = base + lane;
    const bool valid = idx < n;
    uint32_t x = valid ? in[idx] : 0u;
    for (int i = 0; i < 64; ++i) x = x * 2654435761u + (x >> 7);
    const uint64_t mask = __ballot(valid && (x & 1u));
    const uint32_t w = base / 32u + lane;
    if (lane < 2u && w < (n + 31u) / 32u) bits[w] = lane ? (uint32_t)(mask >> 32) : (uint32_t)mask;
  }
}
