// Dependent-issue latency of the field-multiply instructions on gfx950.
// One or two waves per SIMD run NCH interleaved dependency chains of the same
// instruction; cycles per instruction per SIMD = clock * time / (instrs per SIMD).
// Build: hipcc --offload-arch=gfx950 -O3 tools/ubench_lat.hip -o tools/ubench_lat
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

#define ITERS 8192

template <int NCH>
__global__ void __launch_bounds__(64) k_mad(uint32_t *sink, uint32_t seed) {
  uint32_t t = threadIdx.x + seed;
  uint64_t x[NCH];
  uint32_t a = t | 1, b = t * 3 + 7;
#pragma unroll
  for (int c = 0; c < NCH; ++c) x[c] = t + c;
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int r = 0; r < 16 / NCH; ++r)
#pragma unroll
      for (int c = 0; c < NCH; ++c)
        asm volatile("v_mad_u64_u32 %0, s[40:41], %1, %2, %0" : "+v"(x[c]) : "v"(a), "v"(b) : "s40", "s41");
  }
  uint32_t r = 0;
#pragma unroll
  for (int c = 0; c < NCH; ++c) r ^= (uint32_t)(x[c] ^ (x[c] >> 32));
  if (r == 0x12345678u) sink[0] = r;
}

template <int NCH>
__global__ void __launch_bounds__(64) k_add(uint32_t *sink, uint32_t seed) {
  uint32_t t = threadIdx.x + seed;
  uint32_t x[NCH];
  uint32_t a = t | 1;
#pragma unroll
  for (int c = 0; c < NCH; ++c) x[c] = t + c;
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int r = 0; r < 16 / NCH; ++r)
#pragma unroll
      for (int c = 0; c < NCH; ++c) asm volatile("v_add_u32 %0, %0, %1" : "+v"(x[c]) : "v"(a));
  }
  uint32_t r = 0;
#pragma unroll
  for (int c = 0; c < NCH; ++c) r ^= x[c];
  if (r == 0x12345678u) sink[0] = r;
}

template <int NCH>
__global__ void __launch_bounds__(64) k_lshl_add64(uint32_t *sink, uint32_t seed) {
  uint32_t t = threadIdx.x + seed;
  uint64_t x[NCH];
  uint64_t a = ((uint64_t)t << 32) | 5;
#pragma unroll
  for (int c = 0; c < NCH; ++c) x[c] = t + c;
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int r = 0; r < 16 / NCH; ++r)
#pragma unroll
      for (int c = 0; c < NCH; ++c) asm volatile("v_lshl_add_u64 %0, %0, 0, %1" : "+v"(x[c]) : "v"(a));
  }
  uint32_t r = 0;
#pragma unroll
  for (int c = 0; c < NCH; ++c) r ^= (uint32_t)(x[c] ^ (x[c] >> 32));
  if (r == 0x12345678u) sink[0] = r;
}


// carry-out SGPR pair rotated per chain (breaks a write-after-write chain on one pair)
template <int NCH>
__global__ void __launch_bounds__(64) k_mad_rot(uint32_t *sink, uint32_t seed) {
  uint32_t t = threadIdx.x + seed;
  uint64_t x[NCH];
  uint32_t a = t | 1, b = t * 3 + 7;
#pragma unroll
  for (int c = 0; c < NCH; ++c) x[c] = t + c;
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int r = 0; r < 16 / NCH; ++r) {
#pragma unroll
      for (int c = 0; c < NCH; ++c) {
        if (c % 4 == 0) asm volatile("v_mad_u64_u32 %0, s[40:41], %1, %2, %0" : "+v"(x[c]) : "v"(a), "v"(b) : "s40", "s41");
        if (c % 4 == 1) asm volatile("v_mad_u64_u32 %0, s[42:43], %1, %2, %0" : "+v"(x[c]) : "v"(a), "v"(b) : "s42", "s43");
        if (c % 4 == 2) asm volatile("v_mad_u64_u32 %0, s[44:45], %1, %2, %0" : "+v"(x[c]) : "v"(a), "v"(b) : "s44", "s45");
        if (c % 4 == 3) asm volatile("v_mad_u64_u32 %0, s[46:47], %1, %2, %0" : "+v"(x[c]) : "v"(a), "v"(b) : "s46", "s47");
      }
    }
  }
  uint32_t r = 0;
#pragma unroll
  for (int c = 0; c < NCH; ++c) r ^= (uint32_t)(x[c] ^ (x[c] >> 32));
  if (r == 0x12345678u) sink[0] = r;
}

template <int NCH>
__global__ void __launch_bounds__(64) k_mad_vcc(uint32_t *sink, uint32_t seed) {
  uint32_t t = threadIdx.x + seed;
  uint64_t x[NCH];
  uint32_t a = t | 1, b = t * 3 + 7;
#pragma unroll
  for (int c = 0; c < NCH; ++c) x[c] = t + c;
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int r = 0; r < 16 / NCH; ++r)
#pragma unroll
      for (int c = 0; c < NCH; ++c)
        asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(x[c]) : "v"(a), "v"(b) : "vcc");
  }
  uint32_t r = 0;
#pragma unroll
  for (int c = 0; c < NCH; ++c) r ^= (uint32_t)(x[c] ^ (x[c] >> 32));
  if (r == 0x12345678u) sink[0] = r;
}

// 24-bit multiplies (no carry-out): lo and hi halves into two 32-bit accumulators
template <int NCH>
__global__ void __launch_bounds__(64) k_mad24(uint32_t *sink, uint32_t seed) {
  uint32_t t = threadIdx.x + seed;
  uint32_t x[NCH];
  uint32_t a = t | 1, b = t * 3 + 7;
#pragma unroll
  for (int c = 0; c < NCH; ++c) x[c] = t + c;
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int r = 0; r < 16 / NCH; ++r)
#pragma unroll
      for (int c = 0; c < NCH; ++c) asm volatile("v_mad_u32_u24 %0, %1, %2, %0" : "+v"(x[c]) : "v"(a), "v"(b));
  }
  uint32_t r = 0;
#pragma unroll
  for (int c = 0; c < NCH; ++c) r ^= x[c];
  if (r == 0x12345678u) sink[0] = r;
}

typedef void (*kfn)(uint32_t *, uint32_t);

static void run(kfn k, const char *name, int nch, int waves_per_simd, uint32_t *sink, int ncu, double clk_ghz) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const int grid = ncu * 4 * waves_per_simd;  // 64-thread blocks: 4 SIMDs per CU
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
  const double cyc = ms * 1e-3 * clk_ghz * 1e9 / instr_per_simd;
  printf("%-16s chains=%d waves/SIMD=%d  %7.3f ms  %.2f cycles per wave-instruction per SIMD\n", name, nch,
         waves_per_simd, ms, cyc);
}

int main() {
  hipDeviceProp_t prop;
  (void)hipGetDeviceProperties(&prop, 0);
  const double clk = prop.clockRate * 1e-6;
  printf("device %s CUs=%d clock=%.3f GHz\n", prop.gcnArchName, prop.multiProcessorCount, clk);
  uint32_t *sink;
  (void)hipMalloc(&sink, 64);
  const int ncu = prop.multiProcessorCount;
  for (int w : {1, 2, 4}) {
    run(k_mad_rot<4>, "mad_u64 rot-sdst", 4, w, sink, ncu, clk);
    run(k_mad_rot<8>, "mad_u64 rot-sdst", 8, w, sink, ncu, clk);
    run(k_mad_vcc<8>, "mad_u64 vcc", 8, w, sink, ncu, clk);
    run(k_mad24<1>, "v_mad_u32_u24", 1, w, sink, ncu, clk);
    run(k_mad24<8>, "v_mad_u32_u24", 8, w, sink, ncu, clk);
  }
  for (int w : {1, 2, 3, 4}) {
    run(k_mad<1>, "v_mad_u64_u32", 1, w, sink, ncu, clk);
    run(k_mad<2>, "v_mad_u64_u32", 2, w, sink, ncu, clk);
    run(k_mad<4>, "v_mad_u64_u32", 4, w, sink, ncu, clk);
    run(k_mad<8>, "v_mad_u64_u32", 8, w, sink, ncu, clk);
    run(k_add<1>, "v_add_u32", 1, w, sink, ncu, clk);
    run(k_add<4>, "v_add_u32", 4, w, sink, ncu, clk);
    run(k_lshl_add64<1>, "v_lshl_add_u64", 1, w, sink, ncu, clk);
    run(k_lshl_add64<4>, "v_lshl_add_u64", 4, w, sink, ncu, clk);
  }
  (void)hipFree(sink);
  return 0;
}
