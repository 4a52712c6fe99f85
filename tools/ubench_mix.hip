// Issue cost of instruction MIXES on gfx950: how a full-rate op (v_add_u32,
// v_and_b32, ...) interleaved with v_mad_u64_u32 costs, versus alone.  Each
// lane runs 4 independent chains of the pattern; 16 blocks x 256 per CU.
// Output: nanoseconds per wave-instruction per SIMD and cycles at the clock
// the probe measures with a pure v_mad_u64_u32 stream taken as 4 cycles.
//
// Build: hipcc --offload-arch=gfx950 -O3 tools/ubench_mix.hip -o tools/ubench_mix
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

#define ITERS 1024

// pattern P(x, y): one step on chain x (64-bit acc) with scratch y (32-bit)
#define KMIX(name, P)                                                                                  \
  __global__ void __launch_bounds__(256) name(uint32_t *sink, uint32_t seed) {                         \
    uint32_t t = threadIdx.x + blockIdx.x * blockDim.x + seed;                                         \
    uint64_t x0 = t, x1 = t + 1, x2 = t + 2, x3 = t + 3;                                               \
    uint32_t y0 = t * 3, y1 = t * 5, y2 = t * 7, y3 = t * 9;                                           \
    const uint32_t a = t | 1u, b = (t * 7u) | 3u;                                                      \
    for (int it = 0; it < ITERS; ++it)                                                                 \
      asm volatile(P("%0", "%4") P("%1", "%5") P("%2", "%6") P("%3", "%7")                             \
                   : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3), "+v"(y0), "+v"(y1), "+v"(y2), "+v"(y3)     \
                   : "v"(a), "v"(b)                                                                    \
                   : "vcc");                                                                           \
    const uint64_t r = x0 ^ x1 ^ x2 ^ x3 ^ y0 ^ y1 ^ y2 ^ y3;                                          \
    if ((uint32_t)(r ^ (r >> 32)) == 0x12345678u) sink[0] = 1u;                                        \
  }

#define MAD(x) "v_mad_u64_u32 " x ", vcc, %8, %9, " x "\n\t"
#define ADD(y) "v_add_u32_e32 " y ", %8, " y "\n\t"
#define AND(y) "v_and_b32_e32 " y ", %9, " y "\n\t"
#define LSHR(y) "v_lshrrev_b32_e32 " y ", 3, " y "\n\t"
#define LSHL(y) "v_lshlrev_b32_e32 " y ", 3, " y "\n\t"
#define MULLO(y) "v_mul_lo_u32 " y ", " y ", 19\n\t"
#define SHR64(x) "v_lshrrev_b64 " x ", 26, " x "\n\t"
#define CND(y) "v_cndmask_b32_e64 " y ", " y ", %8, vcc\n\t"

#define P_MAD(x, y) MAD(x) MAD(x)
#define P_ADD(x, y) ADD(y) ADD(y)
#define P_MAD_ADD(x, y) MAD(x) ADD(y)
#define P_MAD_AND(x, y) MAD(x) AND(y)
#define P_MAD_LSHR(x, y) MAD(x) LSHR(y)
#define P_MAD_LSHL(x, y) MAD(x) LSHL(y)
#define P_MAD_MULLO(x, y) MAD(x) MULLO(y)
#define P_MAD_SHR64(x, y) MAD(x) SHR64(x)
#define P_MAD2_ADD(x, y) MAD(x) MAD(x) ADD(y)
#define P_MAD4_ADD_AND(x, y) MAD(x) MAD(x) MAD(x) MAD(x) ADD(y) AND(y)
#define P_ADD_AND(x, y) ADD(y) AND(y)
#define P_MULLO(x, y) MULLO(y) MULLO(y)
#define P_MAD_CND(x, y) MAD(x) CND(y)
#define P_COLUMN(x, y) MAD(x) MAD(x) MAD(x) MAD(x) MAD(x) MAD(x) MAD(x) MAD(x) MAD(x) MAD(x) AND(y) SHR64(x)
#define P_COLUMN_NOP(x, y) P_COLUMN(x, y) "s_nop 0\n\t"
#define P_COL6(x, y) MAD(x) MAD(x) MAD(x) MAD(x) MAD(x) MAD(x) AND(y) SHR64(x)
#define P_ADDSUB(x, y) ADD(y) "v_sub_u32_e32 " y ", %9, " y "\n\t"

// one dependent chain per lane (as in the field multiply: the wave's only
// accumulator), the pattern repeated on it
#define KMIX1(name, P)                                                                                 \
  __global__ void __launch_bounds__(256) name(uint32_t *sink, uint32_t seed) {                         \
    uint32_t t = threadIdx.x + blockIdx.x * blockDim.x + seed;                                         \
    uint64_t x0 = t;                                                                                   \
    uint32_t y0 = t * 3;                                                                               \
    const uint32_t a = t | 1u, b = (t * 7u) | 3u;                                                      \
    for (int it = 0; it < ITERS; ++it)                                                                 \
      asm volatile(P("%0", "%1") P("%0", "%1") P("%0", "%1") P("%0", "%1")                             \
                   : "+v"(x0), "+v"(y0)                                                                \
                   : "v"(a), "v"(b)                                                                    \
                   : "vcc");                                                                           \
    const uint64_t r = x0 ^ y0;                                                                        \
    if ((uint32_t)(r ^ (r >> 32)) == 0x12345678u) sink[0] = 1u;                                        \
  }
#define MAD1(x) "v_mad_u64_u32 " x ", vcc, %2, %3, " x "\n\t"
#define AND1(y) "v_and_b32_e32 " y ", %3, " y "\n\t"
#define P1_COLUMN(x, y) MAD1(x) MAD1(x) MAD1(x) MAD1(x) MAD1(x) MAD1(x) MAD1(x) MAD1(x) MAD1(x) MAD1(x) AND1(y) SHR64(x)
#define P1_COLUMN_NOP(x, y) P1_COLUMN(x, y) "s_nop 0\n\t"
#define P1_MAD(x, y) MAD1(x) MAD1(x)

KMIX(k_mad, P_MAD)
KMIX(k_add, P_ADD)
KMIX(k_mad_add, P_MAD_ADD)
KMIX(k_mad_and, P_MAD_AND)
KMIX(k_mad_lshr, P_MAD_LSHR)
KMIX(k_mad_lshl, P_MAD_LSHL)
KMIX(k_mad_mullo, P_MAD_MULLO)
KMIX(k_mad_shr64, P_MAD_SHR64)
KMIX(k_mad2_add, P_MAD2_ADD)
KMIX(k_mad4_add_and, P_MAD4_ADD_AND)
KMIX(k_add_and, P_ADD_AND)
KMIX(k_mullo, P_MULLO)
KMIX(k_mad_cnd, P_MAD_CND)
KMIX(k_column, P_COLUMN)
KMIX(k_column_nop, P_COLUMN_NOP)
KMIX(k_col6, P_COL6)
KMIX(k_addsub, P_ADDSUB)
KMIX1(k1_mad, P1_MAD)
KMIX1(k1_column, P1_COLUMN)
KMIX1(k1_column_nop, P1_COLUMN_NOP)

typedef void (*kfn)(uint32_t *, uint32_t);

static double ns_per_inst(kfn k, int insts_per_pattern, uint32_t *sink, int ncu, int bpc) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const int grid = ncu * bpc;
  hipLaunchKernelGGL(k, dim3(grid), dim3(256), 0, 0, sink, 1u);
  (void)hipDeviceSynchronize();
  (void)hipEventRecord(e0);
  for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k, dim3(grid), dim3(256), 0, 0, sink, (uint32_t)r);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, e0, e1);
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  // wave-instructions per SIMD
  const double waves_per_simd = (double)grid * 4 / (ncu * 4);
  const double insts = 5.0 * waves_per_simd * ITERS * 4 * insts_per_pattern;
  return ms * 1e6 / insts;
}

int main() {
  hipDeviceProp_t prop;
  (void)hipGetDeviceProperties(&prop, 0);
  uint32_t *sink;
  (void)hipMalloc(&sink, 64);
  const int ncu = prop.multiProcessorCount;
  struct {
    const char *name;
    kfn k;
    int n;
  } tab[] = {
      {"mad,mad", k_mad, 2},           {"add,add", k_add, 2},           {"mad,add", k_mad_add, 2},
      {"mad,and", k_mad_and, 2},       {"mad,lshr32", k_mad_lshr, 2},   {"mad,lshl32", k_mad_lshl, 2},
      {"mad,mul_lo", k_mad_mullo, 2},  {"mad,shr64", k_mad_shr64, 2},   {"mad,mad,add", k_mad2_add, 3},
      {"4mad,add,and", k_mad4_add_and, 6}, {"add,and", k_add_and, 2},   {"mul_lo,mul_lo", k_mullo, 2},
      {"mad,cndmask_e64", k_mad_cnd, 2}, {"column 10mad,and,shr64", k_column, 12},
      {"column + s_nop 0", k_column_nop, 12}, {"column 6mad,and,shr64", k_col6, 8}, {"add,sub", k_addsub, 2},
      {"1 chain: mad,mad", k1_mad, 2}, {"1 chain: column", k1_column, 12}, {"1 chain: column + s_nop", k1_column_nop, 12},
  };
  for (int bpc : {2, 3, 4, 8}) {
    const double mad = ns_per_inst(k_mad, 2, sink, ncu, bpc);
    std::printf("%s CUs=%d blocks/CU=%d (waves/SIMD=%d); pure mad = 4 cycles -> %.3f GHz\n", prop.gcnArchName, ncu,
                bpc, bpc, 4.0 / mad);
    for (auto &e : tab) {
      const double ns = ns_per_inst(e.k, e.n, sink, ncu, bpc);
      std::printf("  %-26s %7.3f ns/inst  %5.2f cycles/inst  %6.2f cycles/pattern\n", e.name, ns, ns / mad * 4.0,
                  ns / mad * 4.0 * e.n);
    }
  }
  (void)hipFree(sink);
  return 0;
}
