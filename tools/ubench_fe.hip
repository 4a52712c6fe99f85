// Cost of the real field and point operations of the kernel (csrc/
// hsv_fe26x10.hpp, hsv_point.hpp) on gfx950, per wave-operation per SIMD, at
// 3 waves per SIMD (the point pass's occupancy): fe_mul, fe_sq, fe_carry,
// ge_dbl_rt (with / without T), ge_add_cached_rt (with / without T), and a
// bare 100-long v_mad_u64_u32 chain for scale.  Each lane runs one dependent
// chain of the operation, as the kernel does.  The VALU instruction count of
// each loop body is read from the ISA (tools/isa_mix.py) to turn the times
// into a mix-weighted ceiling.
//
// Build: hipcc --offload-arch=gfx950 -O3 -fno-slp-vectorize -std=c++17 [-DHSV_FE26_PARALLEL_CARRY | -DHSV_FE_RADIX=32]
//        -I hotstuff-digital-signature-benchmarking_amd/csrc tools/ubench_fe.hip -o tools/ubench_fe
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

#include "hsv_point.hpp"

using namespace hsv;

#define ITERS 256

__device__ __forceinline__ fe seed_fe(uint32_t t, uint32_t k) {
  fe r;
#if HSV_FE_RADIX == 32
  for (int i = 0; i < kFeLimbs; ++i) r.v[i] = (t * 2654435761u + k * 40503u + i * 977u) & (i == 7 ? 0x7fffffffu : ~0u);
#else
  for (int i = 0; i < kFeLimbs; ++i) r.v[i] = ((t * 2654435761u + k * 40503u + i * 977u) >> 7) & fe26_mask(i);
#endif
  return r;
}

__device__ __forceinline__ void sink_fe(uint32_t *sink, const fe &a) {
  uint32_t x = 0;
  for (int i = 0; i < kFeLimbs; ++i) x ^= a.v[i];
  if (x == 0x12345678u) sink[0] = x;
}

// shader-clock ticks of one wave's loop (s_memtime), summed over waves in cyc[0]
struct WaveClock {
  uint64_t t0;
  __device__ __forceinline__ WaveClock() { t0 = __builtin_amdgcn_s_memtime(); }
  __device__ __forceinline__ void done(unsigned long long *cyc) const {
    const uint64_t dt = __builtin_amdgcn_s_memtime() - t0;
    if ((threadIdx.x & 63u) == 0) atomicAdd(cyc, (unsigned long long)dt);
  }
};

__global__ void __launch_bounds__(256) k_mul(uint32_t *sink, uint32_t seed, unsigned long long *cyc) {
  const uint32_t t = threadIdx.x + blockIdx.x * 256u + seed;
  fe a = seed_fe(t, 1), b = seed_fe(t, 2);
WaveClock wc;
#pragma nounroll
  for (int it = 0; it < ITERS; ++it) a = fe_mul(a, b);
  wc.done(cyc);
  sink_fe(sink, a);
}

// both operands change every step (the prescaled 19 g of fe_mul is not hoisted)
__global__ void __launch_bounds__(256) k_mul_var(uint32_t *sink, uint32_t seed, unsigned long long *cyc) {
  const uint32_t t = threadIdx.x + blockIdx.x * 256u + seed;
  fe a = seed_fe(t, 1), b = seed_fe(t, 2);
WaveClock wc;
#pragma nounroll
  for (int it = 0; it < ITERS; ++it) {
    const fe c = fe_mul(a, b);
    b = a;
    a = c;
  }
  wc.done(cyc);
  sink_fe(sink, a);
}

// two independent chains per lane through the paired forms (per pair: 2 ops)
__global__ void __launch_bounds__(256) k_mul2(uint32_t *sink, uint32_t seed, unsigned long long *cyc) {
  const uint32_t t = threadIdx.x + blockIdx.x * 256u + seed;
  fe a = seed_fe(t, 1), b = seed_fe(t, 2), c = seed_fe(t, 3), d = seed_fe(t, 4);
  WaveClock wc;
#pragma nounroll
  for (int it = 0; it < ITERS; ++it) {
    fe x, y;
    fe_mul2(a, b, c, d, x, y);
    b = a;
    a = x;
    d = c;
    c = y;
  }
  wc.done(cyc);
  sink_fe(sink, a);
  sink_fe(sink, c);
}

__global__ void __launch_bounds__(256) k_sqp(uint32_t *sink, uint32_t seed, unsigned long long *cyc) {
  const uint32_t t = threadIdx.x + blockIdx.x * 256u + seed;
  fe a = seed_fe(t, 1), b = seed_fe(t, 2);
  WaveClock wc;
#pragma nounroll
  for (int it = 0; it < ITERS; ++it) {
    fe x, y;
    fe_sq2(a, b, x, y);
    a = x;
    b = y;
  }
  wc.done(cyc);
  sink_fe(sink, a);
  sink_fe(sink, b);
}

__global__ void __launch_bounds__(256) k_sq(uint32_t *sink, uint32_t seed, unsigned long long *cyc) {
  const uint32_t t = threadIdx.x + blockIdx.x * 256u + seed;
  fe a = seed_fe(t, 1);
WaveClock wc;
#pragma nounroll
  for (int it = 0; it < ITERS; ++it) a = fe_sq(a);
  wc.done(cyc);
  sink_fe(sink, a);
}

__global__ void __launch_bounds__(256) k_sq2(uint32_t *sink, uint32_t seed, unsigned long long *cyc) {
  const uint32_t t = threadIdx.x + blockIdx.x * 256u + seed;
  fe a = seed_fe(t, 1);
WaveClock wc;
#pragma nounroll
  for (int it = 0; it < ITERS / 2; ++it) a = fe_sq(fe_sq(a));
  wc.done(cyc);
  sink_fe(sink, a);
}

__global__ void __launch_bounds__(256) k_carry(uint32_t *sink, uint32_t seed, unsigned long long *cyc) {
  const uint32_t t = threadIdx.x + blockIdx.x * 256u + seed;
  fe a = seed_fe(t, 1);
WaveClock wc;
#pragma nounroll
  for (int it = 0; it < ITERS; ++it) a = fe_carry(fe_add(a, a));
  wc.done(cyc);
  sink_fe(sink, a);
}

template <bool WT>
__global__ void __launch_bounds__(256) k_dbl(uint32_t *sink, uint32_t seed, unsigned long long *cyc) {
  const uint32_t t = threadIdx.x + blockIdx.x * 256u + seed;
  ge_ext q;
  q.X = seed_fe(t, 1);
  q.Y = seed_fe(t, 2);
  q.Z = seed_fe(t, 3);
  q.T = seed_fe(t, 4);
WaveClock wc;
#pragma nounroll
  for (int it = 0; it < ITERS; ++it) q = ge_dbl_rt(q, WT ? true : (it & 0x40000000) != 0);
  wc.done(cyc);
  sink_fe(sink, q.X);
  sink_fe(sink, q.T);
}

template <bool WT>
__global__ void __launch_bounds__(256) k_add(uint32_t *sink, uint32_t seed, unsigned long long *cyc) {
  const uint32_t t = threadIdx.x + blockIdx.x * 256u + seed;
  ge_ext q;
  q.X = seed_fe(t, 1);
  q.Y = seed_fe(t, 2);
  q.Z = seed_fe(t, 3);
  q.T = seed_fe(t, 4);
  ge_cached c;
  c.YpX = seed_fe(t, 5);
  c.YmX = seed_fe(t, 6);
  c.Z2 = seed_fe(t, 7);
  c.T2d = seed_fe(t, 8);
WaveClock wc;
#pragma nounroll
  for (int it = 0; it < ITERS; ++it) q = ge_add_cached_rt(q, c, WT ? true : (it & 0x40000000) != 0);
  wc.done(cyc);
  sink_fe(sink, q.X);
  sink_fe(sink, q.T);
}

#define M1 "v_mad_u64_u32 %0, vcc, %1, %2, %0\n\t"
#define M10 M1 M1 M1 M1 M1 M1 M1 M1 M1 M1
__global__ void __launch_bounds__(256) k_mad100(uint32_t *sink, uint32_t seed, unsigned long long *cyc) {
  const uint32_t t = threadIdx.x + blockIdx.x * 256u + seed;
  uint64_t x = t;
  const uint32_t a = t | 1u, b = t * 7u + 3u;
WaveClock wc;
#pragma nounroll
  for (int it = 0; it < ITERS; ++it) asm volatile(M10 M10 M10 M10 M10 M10 M10 M10 M10 M10 : "+v"(x) : "v"(a), "v"(b) : "vcc");
  wc.done(cyc);
  if ((uint32_t)(x ^ (x >> 32)) == 0x12345678u) sink[0] = 1u;
}

typedef void (*kfn)(uint32_t *, uint32_t, unsigned long long *);

struct Cost {
  double ns, cyc;  // per wave-op per SIMD: wall time, and shader cycles of a wave's loop / waves per SIMD
};

static Cost cost_per_op(kfn k, int ops_per_iter, uint32_t *sink, unsigned long long *cyc, int ncu, int bpc) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const int grid = ncu * bpc;
  hipLaunchKernelGGL(k, dim3(grid), dim3(256), 0, 0, sink, 1u, cyc);
  hipLaunchKernelGGL(k, dim3(grid), dim3(256), 0, 0, sink, 2u, cyc);
  (void)hipDeviceSynchronize();
  (void)hipMemset(cyc, 0, 8);
  (void)hipEventRecord(e0);
  const int reps = 10;
  for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(k, dim3(grid), dim3(256), 0, 0, sink, (uint32_t)r, cyc);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, e0, e1);
  unsigned long long c = 0;
  (void)hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  const double waves_per_simd = (double)bpc;  // 256-thread block = 4 waves, one per SIMD
  const double ops = (double)reps * ITERS * ops_per_iter;
  const double waves = (double)reps * grid * 4;
  Cost r;
  r.ns = ms * 1e6 / (waves_per_simd * ops);
  r.cyc = (double)c / waves * reps / ops / waves_per_simd;
  return r;
}

int main(int argc, char **argv) {
  hipDeviceProp_t prop;
  (void)hipGetDeviceProperties(&prop, 0);
  uint32_t *sink;
  unsigned long long *cyc;
  (void)hipMalloc(&sink, 64);
  (void)hipMalloc(&cyc, 8);
  const int ncu = prop.multiProcessorCount;
  struct {
    const char *name;
    kfn k;
    int ops;
  } tab[] = {
      {"mad100 (100 v_mad_u64_u32)", k_mad100, 1}, {"fe_mul (g fixed)", k_mul, 1}, {"fe_mul (g varies)", k_mul_var, 1}, {"fe_mul2 (per product)", k_mul2, 2}, {"fe_sq", k_sq, 1}, {"fe_sq2 (per square)", k_sqp, 2},
      {"fe_sq x2 unrolled", k_sq2, 1}, {"fe_add+fe_carry", k_carry, 1}, {"ge_dbl_rt (no T)", k_dbl<false>, 1},
      {"ge_dbl_rt (with T)", k_dbl<true>, 1}, {"ge_add_cached_rt (no T)", k_add<false>, 1},
      {"ge_add_cached_rt (with T)", k_add<true>, 1},
  };
  // argv: waves per SIMD to measure (default 3 4 6 8; 1 = a lone wave, the
  // latency forms' situation)
  int list[8] = {3, 4, 6, 8}, nl = 4;
  if (argc > 1) {
    nl = 0;
    for (int i = 1; i < argc && nl < 8; ++i) list[nl++] = std::atoi(argv[i]);
  }
  for (int li = 0; li < nl; ++li) {
    const int bpc = list[li];
    std::printf("%s CUs=%d waves/SIMD=%d (per wave-op per SIMD: wall ns, shader cycles, implied GHz)\n",
                prop.gcnArchName, ncu, bpc);
    for (auto &e : tab) {
      const Cost c = cost_per_op(e.k, e.ops, sink, cyc, ncu, bpc);
      std::printf("  %-30s %9.2f ns %9.1f cyc  %.3f GHz\n", e.name, c.ns, c.cyc, c.cyc / c.ns);
    }
  }
  (void)hipFree(sink);
  (void)hipFree(cyc);
  return 0;
}
