// Lane-split field arithmetic (csrc/hsv_fe16x16.hpp) against the one-lane
// radix-2^25.5 form on a lone wave: correctness of fl_mul / fl_pow22523 on
// random and edge inputs, and the clocks of one root chain (x^((p-5)/8), the
// critical piece of the committee QC path) in every form,
// including a four-row prototype (RowLane4, below) that the product lacks.
//
// Build: hipcc --offload-arch=gfx950 -O3 -fno-slp-vectorize -std=c++17
//        -I hotstuff-digital-signature-benchmarking_amd/csrc tools/ubench_lanesplit.hip -o tools/ubench_lanesplit
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "hsv_fe16x16.hpp"
#include "hsv_point.hpp"

using namespace hsv;

// ---- prototype: four rows per element (not in the product) -----------------
// Row r of the wave takes product steps 4r..4r+3: f turned so that
// row_newbcast:i yields f_(4r+i), g turned by 4r lanes with the wrapped limbs
// times 38 (a limb wraps at most once: 4r + 3 <= 15); the four rows' column
// sums meet through v_permlane16_swap (rows 0+1, 2+3) and v_permlane32_swap
// (01 + 23).  The summed halves have the two-row form's bounds (four rows of
// four steps against two rows of eight), so the same two carry passes apply.
namespace hsv {
struct RowLane4 : RowLane {
  uint32_t w4;  // 38 on lanes k < 4r of row r, else 1
  __device__ __forceinline__ RowLane4() : RowLane() {
    const uint32_t r = (__lane_id() >> 4) & 3u;
    w4 = k < 4u * r ? 38u : 1u;
  }
};
// row r: lane k <- lane (k + 4r) mod 16 (row_ror by 16 - 4r)
__device__ __forceinline__ uint32_t rows_turn_f(uint32_t x) {
  uint32_t t = (uint32_t)__builtin_amdgcn_update_dpp((int)x, (int)x, 0x12c, 0x2, 0xf, false);
  t = (uint32_t)__builtin_amdgcn_update_dpp((int)t, (int)x, 0x128, 0x4, 0xf, false);
  return (uint32_t)__builtin_amdgcn_update_dpp((int)t, (int)x, 0x124, 0x8, 0xf, false);
}
// row r: lane k <- lane (k - 4r) mod 16 (row_ror by 4r)
__device__ __forceinline__ uint32_t rows_turn_g(uint32_t x) {
  uint32_t t = (uint32_t)__builtin_amdgcn_update_dpp((int)x, (int)x, 0x124, 0x2, 0xf, false);
  t = (uint32_t)__builtin_amdgcn_update_dpp((int)t, (int)x, 0x128, 0x4, 0xf, false);
  return (uint32_t)__builtin_amdgcn_update_dpp((int)t, (int)x, 0x12c, 0x8, 0xf, false);
}
template <int I>
__device__ __forceinline__ void fl4_mul_step(uint64_t &acc, uint32_t &gr, uint32_t f, const RowLane &L) {
  if constexpr (I > 0) gr = __umul24(row_ror1(gr), L.win);
  acc += (uint64_t)row_bcast<I>(f) * gr;
  if constexpr (I < 3) fl4_mul_step<I + 1>(acc, gr, f, L);
}
__device__ __forceinline__ uint32_t fl4_mul(uint32_t f, uint32_t g, const RowLane4 &L) {
  HSV_SCHED_FENCE();
  uint64_t acc = 0;
  uint32_t gr = __umul24(rows_turn_g(g), L.w4);
  fl4_mul_step<0>(acc, gr, rows_turn_f(f), L);
  const uint32_t lo_h = (uint32_t)acc & 0xffffu;
  const uint32_t t_h = __builtin_amdgcn_alignbit((uint32_t)(acc >> 32), (uint32_t)acc, 16);
  const auto l1 = __builtin_amdgcn_permlane16_swap(lo_h, lo_h, false, false);
  const auto t1 = __builtin_amdgcn_permlane16_swap(t_h, t_h, false, false);
  const uint32_t lo2 = l1[0] + l1[1], t2 = t1[0] + t1[1];
  const auto l2 = __builtin_amdgcn_permlane32_swap(lo2, lo2, false, false);
  const auto t3 = __builtin_amdgcn_permlane32_swap(t2, t2, false, false);
  uint32_t x = (l2[0] + l2[1]) + row_ror1((t3[0] + t3[1]) * L.wout);
  const uint32_t lo16 = x & 0xffffu;
  const uint32_t t = x >> 16;
  x = lo16 + row_ror1(__umul24(t, L.wout));
  HSV_SCHED_FENCE();
  return x;
}
__device__ __forceinline__ uint32_t fl_mul(uint32_t f, uint32_t g, const RowLane4 &L) { return fl4_mul(f, g, L); }
__device__ __forceinline__ uint32_t fl_sq(uint32_t f, const RowLane4 &L) { return fl4_mul(f, f, L); }
}  // namespace hsv

__device__ __forceinline__ fe load_fe(const uint32_t *w) {
  uint32_t x[8];
  for (int i = 0; i < 8; ++i) x[i] = w[i];
  return fe_from_words_masked(x);
}

// row r of every wave: element pair (in[2r], in[2r+1]) -> product, square chain
// and root chain in both forms; out[r] = mismatch bits (1 mul, 2 pow, 4 sq chain)
__global__ void __launch_bounds__(64) k_check(const uint32_t *in, uint32_t *out, uint32_t rows) {
  const RowLane L;
  const uint32_t r = blockIdx.x * 4u + (threadIdx.x >> 4);
  const uint32_t rr = r < rows ? r : rows - 1u;
  const fe a = load_fe(in + 16u * rr), b = load_fe(in + 16u * rr + 8u);
  uint32_t bad = 0;
  {
    const fe ref = fe_mul(a, b);
    const fe got = fl_to_fe(fl_mul(fl_from_fe(a, L), fl_from_fe(b, L), L), L);
    bad |= fe_eq(ref, got) ? 0u : 1u;
  }
  {
    const fe ref = fe_pow22523(a);
    const fe got = fl_to_fe(fl_pow22523(fl_from_fe(a, L), L), L);
    bad |= fe_eq(ref, got) ? 0u : 2u;
  }
  {
    fe ref = b;
    uint32_t x = fl_from_fe(b, L);
    for (int i = 0; i < 40; ++i) {
      ref = fe_mul(fe_sq(ref), a);
      x = fl_mul(fl_sq(x, L), fl_from_fe(a, L), L);
    }
    bad |= fe_eq(ref, fl_to_fe(x, L)) ? 0u : 4u;
  }
  if (r < rows && (threadIdx.x & 15u) == 0u) out[r] = bad;
}

// rows 2j, 2j+1 hold element j (two rows per element, RowLane2): fl_mul / fl_pow22523
// against the one-lane form; out[j] bits as k_check
__global__ void __launch_bounds__(64) k_check2(const uint32_t *in, uint32_t *out, uint32_t pairs) {
  const RowLane2 L;
  const uint32_t r = blockIdx.x * 2u + (threadIdx.x >> 5);
  const uint32_t rr = r < pairs ? r : pairs - 1u;
  const fe a = load_fe(in + 16u * rr), b = load_fe(in + 16u * rr + 8u);
  uint32_t bad = 0;
  bad |= fe_eq(fe_mul(a, b), fl_to_fe(fl2_mul(fl_from_fe(a, L), fl_from_fe(b, L), L), L)) ? 0u : 1u;
  bad |= fe_eq(fe_pow22523(a), fl_to_fe(fl_pow22523(fl_from_fe(a, L), L), L)) ? 0u : 2u;
  if (r < pairs && (threadIdx.x & 31u) == 0u) out[r] = bad;
}

// one element per wave (four rows, RowLane4): out[j] bits 1 mul, 2 pow, 4 chain of 40
__global__ void __launch_bounds__(64) k_check4(const uint32_t *in, uint32_t *out, uint32_t n) {
  const RowLane4 L;
  const uint32_t r = blockIdx.x;
  const uint32_t rr = r < n ? r : n - 1u;
  const fe a = load_fe(in + 16u * rr), b = load_fe(in + 16u * rr + 8u);
  uint32_t bad = 0;
  bad |= fe_eq(fe_mul(a, b), fl_to_fe(fl4_mul(fl_from_fe(a, L), fl_from_fe(b, L), L), L)) ? 0u : 1u;
  bad |= fe_eq(fe_pow22523(a), fl_to_fe(fl_pow22523(fl_from_fe(a, L), L), L)) ? 0u : 2u;
  {
    fe ref = b;
    uint32_t x = fl_from_fe(b, L);
    for (int i = 0; i < 40; ++i) {
      ref = fe_mul(fe_sq(ref), a);
      x = fl_mul(fl_sq(x, L), fl_from_fe(a, L), L);
    }
    bad |= fe_eq(ref, fl_to_fe(x, L)) ? 0u : 4u;
  }
  if (r < n && threadIdx.x == 0u) out[r] = bad;
}

__global__ void __launch_bounds__(64) k_time_ls4(const uint32_t *in, uint32_t *sink, unsigned long long *clk, int reps) {
  const RowLane4 L;
  const fe a = load_fe(in);
  uint32_t x = fl_from_fe(a, L);
  const uint64_t t0 = __builtin_amdgcn_s_memtime(), w0 = wall_clock64();
  for (int i = 0; i < reps; ++i) x = fl_pow22523(x, L);
  const uint64_t t1 = __builtin_amdgcn_s_memtime(), w1 = wall_clock64();
  if (x == 0x12345678u) sink[0] = x;
  if (threadIdx.x == 0) {
    clk[0] = t1 - t0;
    clk[1] = w1 - w0;
  }
}

__global__ void __launch_bounds__(64) k_time_ls2(const uint32_t *in, uint32_t *sink, unsigned long long *clk, int reps) {
  const RowLane2 L;
  const fe a = load_fe(in + 16u * (threadIdx.x >> 5));
  uint32_t x = fl_from_fe(a, L);
  const uint64_t t0 = __builtin_amdgcn_s_memtime(), w0 = wall_clock64();
  for (int i = 0; i < reps; ++i) x = fl_pow22523(x, L);
  const uint64_t t1 = __builtin_amdgcn_s_memtime(), w1 = wall_clock64();
  if (x == 0x12345678u) sink[0] = x;
  if (threadIdx.x == 0) {
    clk[0] = t1 - t0;
    clk[1] = w1 - w0;
  }
}

// one wave: `reps` root chains in a row, each lane-split row its own input
__global__ void __launch_bounds__(64) k_time_ls(const uint32_t *in, uint32_t *sink, unsigned long long *clk, int reps) {
  const RowLane L;
  const fe a = load_fe(in + 16u * (threadIdx.x >> 4));
  uint32_t x = fl_from_fe(a, L);
  const uint64_t t0 = __builtin_amdgcn_s_memtime(), w0 = wall_clock64();
  for (int i = 0; i < reps; ++i) x = fl_pow22523(x, L);
  const uint64_t t1 = __builtin_amdgcn_s_memtime(), w1 = wall_clock64();
  if (x == 0x12345678u) sink[0] = x;
  if (threadIdx.x == 0) {
    clk[0] = t1 - t0;
    clk[1] = w1 - w0;
  }
}

// one wave: every lane its own one-lane root chain (radix 2^25.5)
__global__ void __launch_bounds__(64) k_time_one(const uint32_t *in, uint32_t *sink, unsigned long long *clk, int reps) {
  fe a = load_fe(in + 16u * (threadIdx.x & 3u));
  const uint64_t t0 = __builtin_amdgcn_s_memtime(), w0 = wall_clock64();
  for (int i = 0; i < reps; ++i) a = fe_pow22523(a);
  const uint64_t t1 = __builtin_amdgcn_s_memtime(), w1 = wall_clock64();
  uint32_t s = 0;
  for (int i = 0; i < kFeLimbs; ++i) s ^= a.v[i];
  if (s == 0x12345678u) sink[0] = s;
  if (threadIdx.x == 0) {
    clk[0] = t1 - t0;
    clk[1] = w1 - w0;
  }
}

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e_ = (x);                                                   \
    if (e_ != hipSuccess) {                                                \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));         \
      return 1;                                                            \
    }                                                                      \
  } while (0)

int main() {
  const uint32_t rows = 4096;
  std::vector<uint32_t> h(16u * rows);
  uint64_t s = 0x9e3779b97f4a7c15ull;
  for (auto &w : h) {
    s ^= s << 13;
    s ^= s >> 7;
    s ^= s << 17;
    w = (uint32_t)s;
  }
  // edge values: p - 1, p, 2^255 - 1 (masked input >= p), 0, 1, all limbs 0xffff
  const uint32_t edge[6][8] = {{0xffffffecu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0x7fffffffu},
                               {0xffffffedu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0x7fffffffu},
                               {0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu},
                               {0, 0, 0, 0, 0, 0, 0, 0},
                               {1, 0, 0, 0, 0, 0, 0, 0},
                               {0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0x7ffffffeu}};
  for (int e = 0; e < 6; ++e)
    for (int j = 0; j < 6; ++j)
      for (int i = 0; i < 8; ++i) {
        h[16u * (e * 6 + j) + i] = edge[e][i];
        h[16u * (e * 6 + j) + 8 + i] = edge[j][i];
      }
  uint32_t *d_in, *d_out, *d_sink;
  unsigned long long *d_clk;
  CK(hipMalloc(&d_in, h.size() * 4));
  CK(hipMalloc(&d_out, rows * 4));
  CK(hipMalloc(&d_sink, 4));
  CK(hipMalloc(&d_clk, 16));
  CK(hipMemcpy(d_in, h.data(), h.size() * 4, hipMemcpyHostToDevice));
  hipLaunchKernelGGL(k_check, dim3(rows / 4), dim3(64), 0, 0, d_in, d_out, rows);
  CK(hipGetLastError());
  CK(hipDeviceSynchronize());
  std::vector<uint32_t> out(rows);
  CK(hipMemcpy(out.data(), d_out, rows * 4, hipMemcpyDeviceToHost));
  int bad[3] = {0, 0, 0};
  for (uint32_t r = 0; r < rows; ++r)
    for (int b = 0; b < 3; ++b) bad[b] += (out[r] >> b) & 1u;
  std::printf("{\"check_rows\": %u, \"mul_mismatch\": %d, \"pow22523_mismatch\": %d, \"chain40_mismatch\": %d}\n", rows,
              bad[0], bad[1], bad[2]);
  hipLaunchKernelGGL(k_check2, dim3(rows / 2), dim3(64), 0, 0, d_in, d_out, rows);
  CK(hipGetLastError());
  CK(hipDeviceSynchronize());
  CK(hipMemcpy(out.data(), d_out, rows * 4, hipMemcpyDeviceToHost));
  int bad2[2] = {0, 0};
  for (uint32_t r = 0; r < rows; ++r)
    for (int b = 0; b < 2; ++b) bad2[b] += (out[r] >> b) & 1u;
  std::printf("{\"two_row_check\": %u, \"mul_mismatch\": %d, \"pow22523_mismatch\": %d}\n", rows, bad2[0], bad2[1]);
  bad[0] += bad2[0];
  bad[1] += bad2[1];
  hipLaunchKernelGGL(k_check4, dim3(rows), dim3(64), 0, 0, d_in, d_out, rows);
  CK(hipGetLastError());
  CK(hipDeviceSynchronize());
  CK(hipMemcpy(out.data(), d_out, rows * 4, hipMemcpyDeviceToHost));
  int bad4[3] = {0, 0, 0};
  for (uint32_t r = 0; r < rows; ++r)
    for (int b = 0; b < 3; ++b) bad4[b] += (out[r] >> b) & 1u;
  std::printf("{\"four_row_check\": %u, \"mul_mismatch\": %d, \"pow22523_mismatch\": %d, \"chain40_mismatch\": %d}\n",
              rows, bad4[0], bad4[1], bad4[2]);
  bad[0] += bad4[0];
  bad[1] += bad4[1];
  bad[2] += bad4[2];
  const int reps = 20;
  unsigned long long c[2];
  for (int form = 0; form < 4; ++form) {
    for (int warm = 0; warm < 2; ++warm) {
      if (form == 0) hipLaunchKernelGGL(k_time_ls, dim3(1), dim3(64), 0, 0, d_in, d_sink, d_clk, reps);
      else if (form == 1) hipLaunchKernelGGL(k_time_one, dim3(1), dim3(64), 0, 0, d_in, d_sink, d_clk, reps);
      else if (form == 2) hipLaunchKernelGGL(k_time_ls2, dim3(1), dim3(64), 0, 0, d_in, d_sink, d_clk, reps);
      else hipLaunchKernelGGL(k_time_ls4, dim3(1), dim3(64), 0, 0, d_in, d_sink, d_clk, reps);
      CK(hipGetLastError());
      CK(hipDeviceSynchronize());
    }
    CK(hipMemcpy(c, d_clk, 16, hipMemcpyDeviceToHost));
    std::printf("{\"form\": \"%s\", \"root_chain_clocks\": %.0f, \"root_chain_us\": %.2f}\n",
                form == 0 ? "lane_split_16x16" : form == 1 ? "one_lane_26x10" : form == 2 ? "two_rows_16x16" : "four_rows_16x16",
                (double)c[0] / reps,
                (double)c[1] / reps / 100.0);
  }
  return bad[0] + bad[1] + bad[2] ? 2 : 0;
}
