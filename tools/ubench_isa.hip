// Issue cost of every VALU opcode in the hot loops of hsv_verify_hp_kernel on
// gfx950 (the opcode list comes from tools/isa_mix.py).  Each lane runs 8
// independent chains of one opcode, 16 blocks of 256 threads per CU (4 waves
// per SIMD), so the result is issue throughput, not latency.  Output: lane-ops
// per second and the cost relative to v_add_u32_e32 (the cheapest integer op);
// tools/isa_mix.py weighs the kernel's instruction mix with these costs.
//
// Build: hipcc --offload-arch=gfx950 -O3 tools/ubench_isa.hip -o tools/ubench_isa
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

#define ITERS 2048

// 32-bit chains x0..x7, sources a, b (VGPR)
#define K32(name, ins)                                                                            \
  __global__ void __launch_bounds__(256) name(uint32_t *sink, uint32_t seed) {                    \
    uint32_t t = threadIdx.x + blockIdx.x * blockDim.x + seed;                                    \
    uint32_t x0 = t, x1 = t + 1, x2 = t + 2, x3 = t + 3, x4 = t + 4, x5 = t + 5, x6 = t + 6,       \
             x7 = t + 7;                                                                          \
    const uint32_t a = t | 1u, b = (t * 7u) | 3u;                                                 \
    for (int it = 0; it < ITERS; ++it)                                                            \
      asm volatile(ins("%0") ins("%1") ins("%2") ins("%3") ins("%4") ins("%5") ins("%6") ins("%7") \
                   : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3), "+v"(x4), "+v"(x5), "+v"(x6), "+v"(x7) \
                   : "v"(a), "v"(b));                                                             \
    if ((x0 ^ x1 ^ x2 ^ x3 ^ x4 ^ x5 ^ x6 ^ x7) == 0x12345678u) sink[0] = 1u;                    \
  }

// 64-bit chains (register pairs), sources a (64-bit), b (32-bit)
#define K64(name, ins)                                                                            \
  __global__ void __launch_bounds__(256) name(uint32_t *sink, uint32_t seed) {                    \
    uint32_t t = threadIdx.x + blockIdx.x * blockDim.x + seed;                                    \
    uint64_t x0 = t, x1 = t + 1, x2 = t + 2, x3 = t + 3, x4 = t + 4, x5 = t + 5, x6 = t + 6,       \
             x7 = t + 7;                                                                          \
    const uint64_t a = ((uint64_t)t << 32) | 5u;                                                  \
    const uint32_t b = (t * 7u) | 3u;                                                             \
    for (int it = 0; it < ITERS; ++it)                                                            \
      asm volatile(ins("%0") ins("%1") ins("%2") ins("%3") ins("%4") ins("%5") ins("%6") ins("%7") \
                   : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3), "+v"(x4), "+v"(x5), "+v"(x6), "+v"(x7) \
                   : "v"(a), "v"(b)                                                               \
                   : "vcc", "s40", "s41");                                                        \
    const uint64_t r = x0 ^ x1 ^ x2 ^ x3 ^ x4 ^ x5 ^ x6 ^ x7;                                     \
    if ((uint32_t)(r ^ (r >> 32)) == 0x12345678u) sink[0] = 1u;                                   \
  }

#define I_ADD(x) "v_add_u32_e32 " x ", %8, " x "\n\t"
#define I_SUB(x) "v_sub_u32_e32 " x ", %8, " x "\n\t"
#define I_AND(x) "v_and_b32_e32 " x ", %8, " x "\n\t"
#define I_OR(x) "v_or_b32_e32 " x ", %8, " x "\n\t"
#define I_XOR(x) "v_xor_b32_e32 " x ", %8, " x "\n\t"
#define I_AND_K(x) "v_and_b32_e32 " x ", 0x3ffffff, " x "\n\t"
#define I_LSHR(x) "v_lshrrev_b32_e32 " x ", 25, " x "\n\t"
#define I_LSHL(x) "v_lshlrev_b32_e32 " x ", 1, " x "\n\t"
#define I_ASHR(x) "v_ashrrev_i32_e32 " x ", 3, " x "\n\t"
#define I_MOV(x) "v_mov_b32_e32 " x ", %8\n\t"
#define I_MULLO(x) "v_mul_lo_u32 " x ", " x ", 19\n\t"
#define I_MULU24(x) "v_mul_u32_u24_e32 " x ", 19, " x "\n\t"
#define I_MADU24(x) "v_mad_u32_u24 " x ", " x ", 19, %9\n\t"
#define I_LSHL_OR(x) "v_lshl_or_b32 " x ", " x ", 6, %8\n\t"
#define I_LSHL_ADD(x) "v_lshl_add_u32 " x ", " x ", 1, %8\n\t"
#define I_ADD_LSHL(x) "v_add_lshl_u32 " x ", " x ", %8, 1\n\t"
#define I_AND_OR(x) "v_and_or_b32 " x ", " x ", %8, %9\n\t"
#define I_OR3(x) "v_or3_b32 " x ", " x ", %8, %9\n\t"
#define I_ADD3(x) "v_add3_u32 " x ", " x ", %8, %9\n\t"
#define I_BFE(x) "v_bfe_u32 " x ", " x ", 3, 26\n\t"
#define I_BFI(x) "v_bfi_b32 " x ", %8, " x ", %9\n\t"
#define I_ALIGNBIT(x) "v_alignbit_b32 " x ", %8, " x ", 26\n\t"
#define I_PERM(x) "v_perm_b32 " x ", %8, " x ", %9\n\t"
#define I_CNDMASK(x) "v_cndmask_b32_e32 " x ", " x ", %8, vcc\n\t"
#define I_CNDMASK64(x) "v_cndmask_b32_e64 " x ", " x ", %8, s[40:41]\n\t"

#define I_MAD64(x) "v_mad_u64_u32 " x ", s[40:41], %9, %9, " x "\n\t"
#define I_LSHR64(x) "v_lshrrev_b64 " x ", 26, " x "\n\t"
#define I_LSHLADD64(x) "v_lshl_add_u64 " x ", " x ", 0, %8\n\t"
#define I_MOV64(x) "v_mov_b64_e32 " x ", %8\n\t"
// round 4: the f64 path's costs, and gfx950's three-input bit op
#define I_FMA64(x) "v_fma_f64 " x ", " x ", %8, %8\n\t"
#define I_ADDF64(x) "v_add_f64 " x ", " x ", %8\n\t"
#define I_MULF64(x) "v_mul_f64 " x ", " x ", %8\n\t"
#define I_BITOP3(x) "v_bitop3_b32 " x ", " x ", %8, %9 bitop3:0x96\n\t"
#define I_MULHI(x) "v_mul_hi_u32 " x ", " x ", %8\n\t"
#define I_ADDCO(x) "v_add_co_u32_e32 " x ", vcc, %8, " x "\n\t"
#define I_ADDC(x) "v_addc_co_u32_e32 " x ", vcc, %8, " x ", vcc\n\t"

K32(k_add, I_ADD)
K32(k_sub, I_SUB)
K32(k_and, I_AND)
K32(k_or, I_OR)
K32(k_xor, I_XOR)
K32(k_and_k, I_AND_K)
K32(k_lshr, I_LSHR)
K32(k_lshl, I_LSHL)
K32(k_ashr, I_ASHR)
K32(k_mov, I_MOV)
K32(k_mullo, I_MULLO)
K32(k_mulu24, I_MULU24)
K32(k_madu24, I_MADU24)
K32(k_lshl_or, I_LSHL_OR)
K32(k_lshl_add, I_LSHL_ADD)
K32(k_add_lshl, I_ADD_LSHL)
K32(k_and_or, I_AND_OR)
K32(k_or3, I_OR3)
K32(k_add3, I_ADD3)
K32(k_bfe, I_BFE)
K32(k_bfi, I_BFI)
K32(k_alignbit, I_ALIGNBIT)
K32(k_perm, I_PERM)
K64(k_mad64, I_MAD64)
K64(k_lshr64, I_LSHR64)
K64(k_lshladd64, I_LSHLADD64)
K64(k_mov64, I_MOV64)
K64(k_fma64, I_FMA64)
K64(k_addf64, I_ADDF64)
K64(k_mulf64, I_MULF64)
K32(k_bitop3, I_BITOP3)
K32(k_mulhi, I_MULHI)

// carry chains through VCC (v_add_co / v_addc_co: a 64-bit add is one of each)
__global__ void __launch_bounds__(256) k_addco(uint32_t *sink, uint32_t seed) {
  uint32_t t = threadIdx.x + blockIdx.x * blockDim.x + seed;
  uint32_t x0 = t, x1 = t + 1, x2 = t + 2, x3 = t + 3, x4 = t + 4, x5 = t + 5, x6 = t + 6, x7 = t + 7;
  const uint32_t a = t | 1u, b = t * 7u;
  for (int it = 0; it < ITERS; ++it)
    asm volatile(I_ADDCO("%0") I_ADDC("%1") I_ADDCO("%2") I_ADDC("%3") I_ADDCO("%4") I_ADDC("%5") I_ADDCO("%6")
                     I_ADDC("%7")
                 : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3), "+v"(x4), "+v"(x5), "+v"(x6), "+v"(x7)
                 : "v"(a), "v"(b)
                 : "vcc");
  if ((x0 ^ x1 ^ x2 ^ x3 ^ x4 ^ x5 ^ x6 ^ x7) == 0x12345678u) sink[0] = 1u;
}

// v_cndmask with VCC / an SGPR pair set once before the loop
__global__ void __launch_bounds__(256) k_cndmask(uint32_t *sink, uint32_t seed) {
  uint32_t t = threadIdx.x + blockIdx.x * blockDim.x + seed;
  uint32_t x0 = t, x1 = t + 1, x2 = t + 2, x3 = t + 3, x4 = t + 4, x5 = t + 5, x6 = t + 6, x7 = t + 7;
  const uint32_t a = t | 1u, b = t * 7u;
  asm volatile("v_cmp_lt_u32_e32 vcc, 31, %0\n\ts_nop 4" ::"v"(t & 63u) : "vcc");
  for (int it = 0; it < ITERS; ++it)
    asm volatile(I_CNDMASK("%0") I_CNDMASK("%1") I_CNDMASK("%2") I_CNDMASK("%3") I_CNDMASK("%4") I_CNDMASK("%5")
                     I_CNDMASK("%6") I_CNDMASK("%7")
                 : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3), "+v"(x4), "+v"(x5), "+v"(x6), "+v"(x7)
                 : "v"(a), "v"(b));
  if ((x0 ^ x1 ^ x2 ^ x3 ^ x4 ^ x5 ^ x6 ^ x7) == 0x12345678u) sink[0] = 1u;
}

__global__ void __launch_bounds__(256) k_cndmask64(uint32_t *sink, uint32_t seed) {
  uint32_t t = threadIdx.x + blockIdx.x * blockDim.x + seed;
  uint32_t x0 = t, x1 = t + 1, x2 = t + 2, x3 = t + 3, x4 = t + 4, x5 = t + 5, x6 = t + 6, x7 = t + 7;
  const uint32_t a = t | 1u, b = t * 7u;
  asm volatile("v_cmp_lt_u32_e64 s[40:41], 31, %0\n\ts_nop 4" ::"v"(t & 63u) : "s40", "s41");
  for (int it = 0; it < ITERS; ++it)
    asm volatile(I_CNDMASK64("%0") I_CNDMASK64("%1") I_CNDMASK64("%2") I_CNDMASK64("%3") I_CNDMASK64("%4")
                     I_CNDMASK64("%5") I_CNDMASK64("%6") I_CNDMASK64("%7")
                 : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3), "+v"(x4), "+v"(x5), "+v"(x6), "+v"(x7)
                 : "v"(a), "v"(b)
                 : "s40", "s41");
  if ((x0 ^ x1 ^ x2 ^ x3 ^ x4 ^ x5 ^ x6 ^ x7) == 0x12345678u) sink[0] = 1u;
}

typedef void (*kfn)(uint32_t *, uint32_t);

static double run(kfn k, int ops_per_iter, uint32_t *sink, int ncu) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int grid = ncu * 16;
  hipLaunchKernelGGL(k, dim3(grid), dim3(256), 0, 0, sink, 1u);  // warm
  hipDeviceSynchronize();
  hipEventRecord(e0);
  for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k, dim3(grid), dim3(256), 0, 0, sink, (uint32_t)r);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  hipEventDestroy(e0);
  hipEventDestroy(e1);
  return 5.0 * grid * 256.0 * ITERS * ops_per_iter / (ms * 1e-3);
}

int main() {
  hipDeviceProp_t prop;
  hipGetDeviceProperties(&prop, 0);
  uint32_t *sink;
  hipMalloc(&sink, 64);
  const int ncu = prop.multiProcessorCount;
  struct {
    const char *name;
    kfn k;
    int ops;
  } tab[] = {
      {"v_add_u32_e32", k_add, 8},         {"v_sub_u32_e32", k_sub, 8},         {"v_and_b32_e32", k_and, 8},
      {"v_or_b32_e32", k_or, 8},           {"v_xor_b32_e32", k_xor, 8},         {"v_and_b32_e32(lit)", k_and_k, 8},
      {"v_lshrrev_b32_e32", k_lshr, 8},    {"v_lshlrev_b32_e32", k_lshl, 8},    {"v_ashrrev_i32_e32", k_ashr, 8},
      {"v_mov_b32_e32", k_mov, 8},         {"v_mul_lo_u32", k_mullo, 8},        {"v_mul_u32_u24_e32", k_mulu24, 8},
      {"v_mad_u32_u24", k_madu24, 8},      {"v_lshl_or_b32", k_lshl_or, 8},     {"v_lshl_add_u32", k_lshl_add, 8},
      {"v_add_lshl_u32", k_add_lshl, 8},   {"v_and_or_b32", k_and_or, 8},       {"v_or3_b32", k_or3, 8},
      {"v_add3_u32", k_add3, 8},           {"v_bfe_u32", k_bfe, 8},             {"v_bfi_b32", k_bfi, 8},
      {"v_alignbit_b32", k_alignbit, 8},   {"v_perm_b32", k_perm, 8},           {"v_cndmask_b32_e32", k_cndmask, 8},
      {"v_cndmask_b32_e64", k_cndmask64, 8}, {"v_mad_u64_u32", k_mad64, 8},     {"v_lshrrev_b64", k_lshr64, 8},
      {"v_lshl_add_u64", k_lshladd64, 8},  {"v_mov_b64_e32", k_mov64, 8},
      {"v_fma_f64", k_fma64, 8},           {"v_add_f64", k_addf64, 8},          {"v_mul_f64", k_mulf64, 8},
      {"v_bitop3_b32", k_bitop3, 8},       {"v_mul_hi_u32", k_mulhi, 8},        {"v_add_co/v_addc_co (pairs)", k_addco, 8},
  };
  double base = 0;
  std::printf("device %s CUs=%d  (16 blocks x 256 per CU, 8 chains per lane)\n", prop.gcnArchName, ncu);
  for (auto &e : tab) {
    const double r = run(e.k, e.ops, sink, ncu);
    if (base == 0) base = r;
    std::printf("%-28s %8.3f T lane-ops/s   cost %.2f x v_add_u32\n", e.name, r / 1e12, base / r);
  }
  hipFree(sink);
  return 0;
}
