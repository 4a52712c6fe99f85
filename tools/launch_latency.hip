// Latency pieces of the small-batch (QC) path on one MI355X, p50 over 2000
// calls each, host clock: an empty kernel launch + hipStreamSynchronize; the
// same with the output written to pinned host memory (zero-copy); and one
// wave decompressing one point (R's root chain, the cached QC path's critical
// piece, csrc/hsv_point.hpp ge_decompress) launched and synced the same way.
//
// Build: hipcc --offload-arch=gfx950 -O3 -fno-slp-vectorize -std=c++17
//        -I hotstuff-digital-signature-benchmarking_amd/csrc tools/launch_latency.hip -o tools/launch_latency
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <vector>

#include "hsv_point.hpp"

using namespace hsv;

__global__ void k_empty(uint8_t *out) {
  if (threadIdx.x == 0) out[0] = 1;
}

__global__ void k_decompress(const uint32_t *enc, uint8_t *out) {
  if (threadIdx.x != 0) return;
  uint32_t w[8];
  for (int i = 0; i < 8; ++i) w[i] = enc[i];
  fe x, y;
  const uint32_t ok = ge_decompress(w, x, y);
  out[0] = (uint8_t)(ok | (x.v[0] & 2u));
}

template <class F>
static double p50_us(F &&f, int reps = 2000) {
  std::vector<double> t(reps);
  for (int i = 0; i < 50; ++i) f();
  for (int i = 0; i < reps; ++i) {
    const auto a = std::chrono::steady_clock::now();
    f();
    t[i] = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - a).count();
  }
  std::sort(t.begin(), t.end());
  return t[reps / 2];
}

int main() {
  hipStream_t s;
  (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  uint8_t *d_out, *h_out;
  uint32_t *d_enc;
  (void)hipMalloc(&d_out, 64);
  (void)hipHostMalloc(&h_out, 64, hipHostMallocDefault);
  (void)hipMalloc(&d_enc, 32);
  const uint32_t bw[8] = {0x66666658u, 0x66666666u, 0x66666666u, 0x66666666u,
                          0x66666666u, 0x66666666u, 0x66666666u, 0x66666666u};  // B
  (void)hipMemcpy(d_enc, bw, 32, hipMemcpyHostToDevice);
  void *hd = nullptr;
  (void)hipHostGetDevicePointer(&hd, h_out, 0);
  const double e = p50_us([&] {
    hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, s, d_out);
    (void)hipStreamSynchronize(s);
  });
  const double z = p50_us([&] {
    hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, s, static_cast<uint8_t *>(hd));
    (void)hipStreamSynchronize(s);
  });
  const double g = p50_us([&] {
    void *p = nullptr;
    (void)hipHostGetDevicePointer(&p, h_out, 0);
  });
  const double d = p50_us([&] {
    hipLaunchKernelGGL(k_decompress, dim3(1), dim3(64), 0, s, d_enc, static_cast<uint8_t *>(hd));
    (void)hipStreamSynchronize(s);
  });
  std::printf("empty kernel launch + sync        p50 %.1f us\n", e);
  std::printf("  ... output to pinned host memory p50 %.1f us\n", z);
  std::printf("hipHostGetDevicePointer           p50 %.2f us\n", g);
  std::printf("one-lane ge_decompress + sync      p50 %.1f us (root chain ~ %.1f us)\n", d, d - z);
  return 0;
}
