// Issue rate of v_mad_u64_u32 chains on gfx950, measured without the s_nop
// the compiler puts after every inline-asm statement that writes an SGPR:
// each asm statement holds 16 mads (NCH interleaved dependency chains), so
// there is one s_nop per 16 mads.  Also: the same for the carry-step pair
// v_lshrrev_b64 + v_and_b32 interleaved with the chain (the sequential carry
// of hsv_fe26x10.hpp).
// Build: hipcc --offload-arch=gfx950 -O3 tools/ubench_chain.hip -o tools/ubench_chain
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

#define ITERS 4096

#define M1(c) "v_mad_u64_u32 %" #c ", s[40:41], %8, %9, %" #c "\n\t"

template <int NCH>
__global__ void __launch_bounds__(64) k_chain(uint32_t *sink, uint32_t seed) {
  const uint32_t t = threadIdx.x + seed;
  uint64_t x0 = t, x1 = t + 1, x2 = t + 2, x3 = t + 3, x4 = t + 4, x5 = t + 5, x6 = t + 6, x7 = t + 7;
  const uint32_t a = t | 1, b = t * 3 + 7;
  for (int it = 0; it < ITERS; ++it) {
    if constexpr (NCH == 1)
      asm volatile(M1(0) M1(0) M1(0) M1(0) M1(0) M1(0) M1(0) M1(0) M1(0) M1(0) M1(0) M1(0) M1(0) M1(0) M1(0) M1(0)
                   : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3), "+v"(x4), "+v"(x5), "+v"(x6), "+v"(x7)
                   : "v"(a), "v"(b) : "s40", "s41");
    else if constexpr (NCH == 2)
      asm volatile(M1(0) M1(1) M1(0) M1(1) M1(0) M1(1) M1(0) M1(1) M1(0) M1(1) M1(0) M1(1) M1(0) M1(1) M1(0) M1(1)
                   : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3), "+v"(x4), "+v"(x5), "+v"(x6), "+v"(x7)
                   : "v"(a), "v"(b) : "s40", "s41");
    else if constexpr (NCH == 4)
      asm volatile(M1(0) M1(1) M1(2) M1(3) M1(0) M1(1) M1(2) M1(3) M1(0) M1(1) M1(2) M1(3) M1(0) M1(1) M1(2) M1(3)
                   : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3), "+v"(x4), "+v"(x5), "+v"(x6), "+v"(x7)
                   : "v"(a), "v"(b) : "s40", "s41");
    else
      asm volatile(M1(0) M1(1) M1(2) M1(3) M1(4) M1(5) M1(6) M1(7) M1(0) M1(1) M1(2) M1(3) M1(4) M1(5) M1(6) M1(7)
                   : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3), "+v"(x4), "+v"(x5), "+v"(x6), "+v"(x7)
                   : "v"(a), "v"(b) : "s40", "s41");
  }
  const uint64_t r = x0 ^ x1 ^ x2 ^ x3 ^ x4 ^ x5 ^ x6 ^ x7;
  if ((uint32_t)(r ^ (r >> 32)) == 0x12345678u) sink[0] = 1;
}

// one chain of 10 mads followed by the carry step (shift + mask), like one
// column of the sequential-carry multiply; 16 instructions per asm block
__global__ void __launch_bounds__(64) k_column(uint32_t *sink, uint32_t seed) {
  const uint32_t t = threadIdx.x + seed;
  uint64_t x = t;
  uint32_t lo = 0, acc32 = 0;
  const uint32_t a = t | 1, b = t * 3 + 7;
  for (int it = 0; it < ITERS; ++it) {
    asm volatile("v_mad_u64_u32 %0, s[40:41], %3, %4, %0\n\t"
                 "v_mad_u64_u32 %0, s[40:41], %3, %4, %0\n\t"
                 "v_mad_u64_u32 %0, s[40:41], %3, %4, %0\n\t"
                 "v_mad_u64_u32 %0, s[40:41], %3, %4, %0\n\t"
                 "v_mad_u64_u32 %0, s[40:41], %3, %4, %0\n\t"
                 "v_mad_u64_u32 %0, s[40:41], %3, %4, %0\n\t"
                 "v_mad_u64_u32 %0, s[40:41], %3, %4, %0\n\t"
                 "v_mad_u64_u32 %0, s[40:41], %3, %4, %0\n\t"
                 "v_mad_u64_u32 %0, s[40:41], %3, %4, %0\n\t"
                 "v_mad_u64_u32 %0, s[40:41], %3, %4, %0\n\t"
                 "v_and_b32 %1, 0x3ffffff, %2\n\t"
                 "v_lshrrev_b64 %0, 26, %0\n\t"
                 "v_add_u32 %2, %2, %1\n\t"
                 "v_add_u32 %2, %2, %1\n\t"
                 "v_add_u32 %2, %2, %1\n\t"
                 "v_add_u32 %2, %2, %1\n\t"
                 : "+v"(x), "+v"(lo), "+v"(acc32)
                 : "v"(a), "v"(b) : "s40", "s41");
  }
  if ((uint32_t)(x ^ (x >> 32) ^ acc32) == 0x12345678u) sink[0] = 1;
}

typedef void (*kfn)(uint32_t *, uint32_t);

static void run(kfn k, const char *name, int waves_per_simd, uint32_t *sink, int ncu, double clk_ghz) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const int grid = ncu * 4 * waves_per_simd;
  hipLaunchKernelGGL(k, dim3(grid), dim3(64), 0, 0, sink, 1u);
  (void)hipDeviceSynchronize();
  (void)hipEventRecord(e0);
  const int reps = 3;
  for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(k, dim3(grid), dim3(64), 0, 0, sink, (uint32_t)r);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, e0, e1);
  const double instr_per_simd = (double)reps * waves_per_simd * ITERS * 16.0;
  printf("%-26s waves/SIMD=%d  %7.3f ms  %.2f cycles per instruction per SIMD\n", name, waves_per_simd, ms,
         ms * 1e-3 * clk_ghz * 1e9 / instr_per_simd);
}

int main() {
  hipDeviceProp_t prop;
  (void)hipGetDeviceProperties(&prop, 0);
  const double clk = prop.clockRate * 1e-6;
  printf("device %s CUs=%d clock=%.3f GHz\n", prop.gcnArchName, prop.multiProcessorCount, clk);
  uint32_t *sink;
  (void)hipMalloc(&sink, 64);
  const int ncu = prop.multiProcessorCount;
  for (int w : {1, 2, 3, 4}) {
    run(k_chain<1>, "mad chain x1 (dependent)", w, sink, ncu, clk);
    run(k_chain<2>, "mad chains x2", w, sink, ncu, clk);
    run(k_chain<4>, "mad chains x4", w, sink, ncu, clk);
    run(k_chain<8>, "mad chains x8", w, sink, ncu, clk);
    run(k_column, "column: 10 mad+and+shr+4add", w, sink, ncu, clk);
  }
  (void)hipFree(sink);
  return 0;
}
