// VALU issue-rate microbenchmark for the instructions a 255-bit field multiply
// can be built from on gfx950.  Each lane runs NCHAIN independent dependency
// chains so the measurement is throughput, not latency.
// Build: hipcc --offload-arch=gfx950 -O3 tools/ubench_valu.hip -o tools/ubench_valu
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define NCHAIN 8
#define ITERS 4096

#define KERNEL(name, decl, body, out)                                              \
  __global__ void __launch_bounds__(256) name(uint32_t *sink, uint32_t seed) {     \
    uint32_t t = threadIdx.x + blockIdx.x * blockDim.x + seed;                     \
    decl;                                                                          \
    for (int it = 0; it < ITERS; ++it) {                                           \
      _Pragma("unroll") for (int c = 0; c < NCHAIN; ++c) { body; }                 \
    }                                                                              \
    uint32_t r = 0;                                                                \
    _Pragma("unroll") for (int c = 0; c < NCHAIN; ++c) { r ^= out; }               \
    if (r == 0x12345678u) sink[0] = r;                                             \
  }

KERNEL(k_mad_u64_u32, uint64_t x[NCHAIN]; uint32_t a = t | 1; uint32_t b = t * 3 + 7;
       for (int c = 0; c < NCHAIN; ++c) x[c] = t + c,
       asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(x[c]) : "v"(a), "v"(b) : "vcc"),
       (uint32_t)(x[c] ^ (x[c] >> 32)))

KERNEL(k_mul_lo_u32, uint32_t x[NCHAIN]; uint32_t a = t | 1;
       for (int c = 0; c < NCHAIN; ++c) x[c] = t + c,
       asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(x[c]) : "v"(a)), x[c])

KERNEL(k_mul_hi_u32, uint32_t x[NCHAIN]; uint32_t a = t | 1;
       for (int c = 0; c < NCHAIN; ++c) x[c] = t + c,
       asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(x[c]) : "v"(a)), x[c])

KERNEL(k_mad_u32_u24, uint32_t x[NCHAIN]; uint32_t a = t | 1; uint32_t b = t * 5;
       for (int c = 0; c < NCHAIN; ++c) x[c] = t + c,
       asm volatile("v_mad_u32_u24 %0, %1, %2, %0" : "+v"(x[c]) : "v"(a), "v"(b)), x[c])

KERNEL(k_mul_hi_u32_u24, uint32_t x[NCHAIN]; uint32_t a = t | 1;
       for (int c = 0; c < NCHAIN; ++c) x[c] = t + c,
       asm volatile("v_mul_hi_u32_u24 %0, %0, %1" : "+v"(x[c]) : "v"(a)), x[c])

KERNEL(k_add_co_u32, uint32_t x[NCHAIN]; uint32_t a = t | 1;
       for (int c = 0; c < NCHAIN; ++c) x[c] = t + c,
       asm volatile("v_add_co_u32 %0, vcc, %0, %1" : "+v"(x[c]) : "v"(a) : "vcc"), x[c])

KERNEL(k_addc_co_u32, uint32_t x[NCHAIN]; uint32_t a = t | 1;
       for (int c = 0; c < NCHAIN; ++c) x[c] = t + c,
       asm volatile("v_addc_co_u32 %0, vcc, %0, %1, vcc" : "+v"(x[c]) : "v"(a) : "vcc"), x[c])

KERNEL(k_lshl_add_u64, uint64_t x[NCHAIN]; uint64_t a = ((uint64_t)t << 32) | 5;
       for (int c = 0; c < NCHAIN; ++c) x[c] = t + c,
       asm volatile("v_lshl_add_u64 %0, %0, 1, %1" : "+v"(x[c]) : "v"(a)),
       (uint32_t)(x[c] ^ (x[c] >> 32)))

KERNEL(k_fma_f64, double x[NCHAIN]; double a = 1.0000001 + t * 1e-12; double b = 1e-9;
       for (int c = 0; c < NCHAIN; ++c) x[c] = t + c,
       asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(x[c]) : "v"(a), "v"(b)),
       (uint32_t)__double_as_longlong(x[c]))

KERNEL(k_fma_f32, float x[NCHAIN]; float a = 1.0000001f + t * 1e-12f; float b = 1e-9f;
       for (int c = 0; c < NCHAIN; ++c) x[c] = t + c,
       asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(x[c]) : "v"(a), "v"(b)),
       __float_as_uint(x[c]))

KERNEL(k_alignbit, uint32_t x[NCHAIN]; uint32_t a = t | 1;
       for (int c = 0; c < NCHAIN; ++c) x[c] = t + c,
       asm volatile("v_alignbit_b32 %0, %0, %1, 7" : "+v"(x[c]) : "v"(a)), x[c])

KERNEL(k_cndmask, uint32_t x[NCHAIN]; uint32_t a = t | 1;
       for (int c = 0; c < NCHAIN; ++c) x[c] = t + c,
       asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(x[c]) : "v"(a) : "vcc"), x[c])


KERNEL(k_cndmask_s, uint32_t x[NCHAIN]; uint32_t a = t | 1; uint64_t m;
       asm volatile("v_cmp_lt_u32 %0, %1, %2" : "=s"(m) : "v"(t & 63u), "v"(32u));
       for (int c = 0; c < NCHAIN; ++c) x[c] = t + c,
       asm volatile("v_cndmask_b32 %0, %0, %1, %2" : "+v"(x[c]) : "v"(a), "s"(m)), x[c])

KERNEL(k_add_u32, uint32_t x[NCHAIN]; uint32_t a = t | 1;
       for (int c = 0; c < NCHAIN; ++c) x[c] = t + c,
       asm volatile("v_add_u32 %0, %0, %1" : "+v"(x[c]) : "v"(a)), x[c])

KERNEL(k_and_b32, uint32_t x[NCHAIN]; uint32_t a = t | 1;
       for (int c = 0; c < NCHAIN; ++c) x[c] = t + c,
       asm volatile("v_and_b32 %0, %0, %1" : "+v"(x[c]) : "v"(a)), x[c])

KERNEL(k_mov_b32, uint32_t x[NCHAIN]; uint32_t a = t | 1;
       for (int c = 0; c < NCHAIN; ++c) x[c] = t + c,
       asm volatile("v_mov_b32 %0, %1" : "=v"(x[c]) : "v"(a + c)), x[c])

KERNEL(k_lshrrev_b64, uint64_t x[NCHAIN];
       for (int c = 0; c < NCHAIN; ++c) x[c] = ((uint64_t)t << 20) + c,
       asm volatile("v_lshrrev_b64 %0, 1, %0" : "+v"(x[c])), (uint32_t)(x[c] ^ (x[c] >> 32)))

KERNEL(k_add3_u32, uint32_t x[NCHAIN]; uint32_t a = t | 1; uint32_t b = t * 7;
       for (int c = 0; c < NCHAIN; ++c) x[c] = t + c,
       asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(x[c]) : "v"(a), "v"(b)), x[c])

KERNEL(k_bfe_u32, uint32_t x[NCHAIN];
       for (int c = 0; c < NCHAIN; ++c) x[c] = t + c,
       asm volatile("v_bfe_u32 %0, %0, 3, 26" : "+v"(x[c])), x[c])

KERNEL(k_mad_u64_u32_dep, uint64_t x[NCHAIN]; uint32_t a = t | 1; uint32_t b = t * 3 + 7;
       for (int c = 0; c < NCHAIN; ++c) x[c] = t + c,
       asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(x[0]) : "v"(a), "v"(b) : "vcc"),
       (uint32_t)(x[c] ^ (x[c] >> 32)))

KERNEL(k_pk_add_u16, uint32_t x[NCHAIN]; uint32_t a = t | 1;
       for (int c = 0; c < NCHAIN; ++c) x[c] = t + c,
       asm volatile("v_pk_add_u16 %0, %0, %1" : "+v"(x[c]) : "v"(a)), x[c])

KERNEL(k_fma_f64b, double x[NCHAIN]; double a = 1.0000001 + t * 1e-12; double b = 1e-9;
       for (int c = 0; c < NCHAIN; ++c) x[c] = t + c,
       asm volatile("v_fma_f64 %0, %1, %2, %0" : "+v"(x[c]) : "v"(a), "v"(b)),
       (uint32_t)(x[c]))

typedef void (*kfn)(uint32_t *, uint32_t);

static double run(kfn k, const char *name, int blocks_per_cu, uint32_t *sink, int ncu) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  int grid = ncu * blocks_per_cu;
  hipLaunchKernelGGL(k, dim3(grid), dim3(256), 0, 0, sink, 1u);  // warm
  hipDeviceSynchronize();
  hipEventRecord(e0);
  for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k, dim3(grid), dim3(256), 0, 0, sink, (uint32_t)r);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  double ops = 5.0 * grid * 256.0 * ITERS * NCHAIN;
  double rate = ops / (ms * 1e-3);
  printf("%-18s blocks/CU=%d  %8.3f ms  %8.3f T lane-ops/s\n", name, blocks_per_cu, ms, rate / 1e12);
  return rate;
}

int main() {
  hipDeviceProp_t prop;
  hipGetDeviceProperties(&prop, 0);
  printf("device %s  CUs=%d  clock=%d kHz\n", prop.gcnArchName, prop.multiProcessorCount, prop.clockRate);
  uint32_t *sink;
  hipMalloc(&sink, 64);
  int ncu = prop.multiProcessorCount;
  for (int bpc : {8, 16}) {
    run(k_fma_f32, "v_fma_f32", bpc, sink, ncu);
    run(k_add_co_u32, "v_add_co_u32", bpc, sink, ncu);
    run(k_addc_co_u32, "v_addc_co_u32", bpc, sink, ncu);
    run(k_cndmask, "v_cndmask_b32", bpc, sink, ncu);
    run(k_alignbit, "v_alignbit_b32", bpc, sink, ncu);
    run(k_mad_u64_u32, "v_mad_u64_u32", bpc, sink, ncu);
    run(k_mul_lo_u32, "v_mul_lo_u32", bpc, sink, ncu);
    run(k_mul_hi_u32, "v_mul_hi_u32", bpc, sink, ncu);
    run(k_mad_u32_u24, "v_mad_u32_u24", bpc, sink, ncu);
    run(k_mul_hi_u32_u24, "v_mul_hi_u32_u24", bpc, sink, ncu);
    run(k_lshl_add_u64, "v_lshl_add_u64", bpc, sink, ncu);
    run(k_fma_f64, "v_fma_f64", bpc, sink, ncu);
    run(k_cndmask_s, "v_cndmask_b32_sgpr", bpc, sink, ncu);
    run(k_add_u32, "v_add_u32", bpc, sink, ncu);
    run(k_and_b32, "v_and_b32", bpc, sink, ncu);
    run(k_mov_b32, "v_mov_b32", bpc, sink, ncu);
    run(k_lshrrev_b64, "v_lshrrev_b64", bpc, sink, ncu);
    run(k_add3_u32, "v_add3_u32", bpc, sink, ncu);
    run(k_bfe_u32, "v_bfe_u32", bpc, sink, ncu);
    run(k_mad_u64_u32_dep, "v_mad_u64_u32_dep1", bpc, sink, ncu);
    run(k_pk_add_u16, "v_pk_add_u16", bpc, sink, ncu);
    run(k_fma_f64b, "v_fma_f64_acc", bpc, sink, ncu);
  }
  hipFree(sink);
  return 0;
}
