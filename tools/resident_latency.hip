// Round trip of the two ways a small verification could be started on one
// MI355X, p50 over 2000 requests each, host clock (the
// single-vote latency budget):
//   launch    hipLaunchKernelGGL of a one-wave kernel that writes a completion
//             marker into coherent pinned memory; the host spins on the marker
//             (the committee path's marker sync);
//   resident  one wave already running polls a request word in coherent pinned
//             memory (relaxed system-scope loads, s_sleep between polls) and
//             answers each new request with the same marker store.
// The resident wave leaves on a stop word, or by itself after 2 s without a
// request, so no grid outlives the process; every host wait has a timeout.
//
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/resident_latency.hip -o tools/resident_latency
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <vector>

constexpr uint32_t kStop = 0xffffffffu;

__global__ void __launch_bounds__(64) k_mark(uint32_t *done, uint32_t v) {
  if (threadIdx.x == 0) __hip_atomic_store(done, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ void __launch_bounds__(64) k_resident(uint32_t *cmd, uint32_t *done, uint64_t idle_ticks) {
  if (threadIdx.x != 0) return;
  uint32_t last = 0;
  uint64_t t_idle = wall_clock64();
  for (;;) {
    const uint32_t c = __hip_atomic_load(cmd, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if (c == kStop) break;
    if (c != last) {
      last = c;
      __hip_atomic_store(done, c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      t_idle = wall_clock64();
      continue;
    }
    if (wall_clock64() - t_idle > idle_ticks) break;  // idle exit
    __builtin_amdgcn_s_sleep(1);
  }
}

// The committee service's request shape without the verification: a block
// of four waves, thread 0 polls, the block meets at a barrier, every wave
// performs the agent-scope acquire, thread 0 releases and answers (the
// resident service's per-request overhead).
__global__ void __launch_bounds__(256) k_resident_block(uint32_t *cmd, uint32_t *done, uint64_t idle_ticks,
                                                        int acquire) {
  __shared__ uint32_t s_cmd, s_stop;
  uint32_t last = 0;
  for (;;) {
    if (threadIdx.x == 0) {
      const uint64_t t0 = wall_clock64();
      uint32_t c = last, stop = 0;
      for (;;) {
        c = __hip_atomic_load(cmd, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        if (c == kStop) { stop = 1; break; }
        if (c != last) break;
        if (wall_clock64() - t0 > idle_ticks) { stop = 1; break; }
        __builtin_amdgcn_s_sleep(1);
      }
      s_cmd = c;
      s_stop = stop;
      last = c;
    }
    __syncthreads();
    if (s_stop) break;
    if (acquire) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    const uint32_t c = s_cmd;
    __syncthreads();
    if (threadIdx.x == 0) {
      __atomic_thread_fence(__ATOMIC_RELEASE);
      __hip_atomic_store(done, c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
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

using clk = std::chrono::steady_clock;

// spin until *w == v; false after `limit`
static bool wait_for(volatile uint32_t *w, uint32_t v, std::chrono::microseconds limit) {
  const auto t0 = clk::now();
  while (*w != v)
    if (clk::now() - t0 > limit) return false;
  return true;
}

static double p50(std::vector<double> v) {
  std::sort(v.begin(), v.end());
  return v[v.size() / 2];
}

int main() {
  const int reps = 2000;
  uint32_t *h = nullptr;
  CK(hipHostMalloc(reinterpret_cast<void **>(&h), 4096, hipHostMallocCoherent));
  void *dv = nullptr;
  CK(hipHostGetDevicePointer(&dv, h, 0));
  uint32_t *d = static_cast<uint32_t *>(dv);
  volatile uint32_t *cmd = h, *done = h + 16, *mark = h + 32;
  *cmd = 0;
  *done = 0;
  *mark = 0;
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));

  // launch + marker
  std::vector<double> tl;
  for (int i = 1; i <= reps + 50; ++i) {
    const auto t0 = clk::now();
    hipLaunchKernelGGL(k_mark, dim3(1), dim3(64), 0, st, d + 32, (uint32_t)i);
    if (!wait_for(mark, (uint32_t)i, std::chrono::microseconds(100000))) {
      std::fprintf(stderr, "launch marker %d never came\n", i);
      return 2;
    }
    const auto t1 = clk::now();
    if (i > 50) tl.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count());
  }
  CK(hipStreamSynchronize(st));

  // resident wave
  hipLaunchKernelGGL(k_resident, dim3(1), dim3(64), 0, st, d, d + 16, (uint64_t)200000000ull);
  CK(hipGetLastError());
  *cmd = 1;
  if (!wait_for(done, 1u, std::chrono::microseconds(2000000))) {
    *cmd = kStop;
    std::fprintf(stderr, "resident wave never answered\n");
    (void)hipStreamSynchronize(st);
    return 3;
  }
  std::vector<double> tr;
  bool ok = true;
  for (int i = 2; i <= reps + 51 && ok; ++i) {
    const auto t0 = clk::now();
    *cmd = (uint32_t)i;
    ok = wait_for(done, (uint32_t)i, std::chrono::microseconds(100000));
    const auto t1 = clk::now();
    if (i > 51) tr.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count());
  }
  *cmd = kStop;
  CK(hipStreamSynchronize(st));
  if (!ok) {
    std::fprintf(stderr, "resident request timed out\n");
    return 4;
  }
  // the service's request shape: four waves, barrier, acquire (or not), release
  double tb[2] = {0, 0};
  for (int acq = 0; acq < 2; ++acq) {
    *cmd = 0;
    *done = 0;
    hipLaunchKernelGGL(k_resident_block, dim3(1), dim3(256), 0, st, d, d + 16, (uint64_t)200000000ull, acq);
    CK(hipGetLastError());
    *cmd = 1;
    if (!wait_for(done, 1u, std::chrono::microseconds(2000000))) {
      *cmd = kStop;
      (void)hipStreamSynchronize(st);
      std::fprintf(stderr, "resident block never answered\n");
      return 5;
    }
    std::vector<double> t;
    bool good = true;
    for (int i = 2; i <= reps + 51 && good; ++i) {
      const auto t0 = clk::now();
      *cmd = (uint32_t)i;
      good = wait_for(done, (uint32_t)i, std::chrono::microseconds(100000));
      const auto t1 = clk::now();
      if (i > 51) t.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count());
    }
    *cmd = kStop;
    CK(hipStreamSynchronize(st));
    if (!good) {
      std::fprintf(stderr, "resident block request timed out\n");
      return 6;
    }
    tb[acq] = p50(t);
  }
  std::printf("{\"launch_marker_p50_us\": %.2f, \"resident_round_trip_p50_us\": %.2f, "
              "\"resident_block_p50_us\": %.2f, \"resident_block_acquire_p50_us\": %.2f, \"reps\": %d}\n",
              p50(tl), p50(tr), tb[0], tb[1], reps);
  CK(hipStreamDestroy(st));
  CK(hipHostFree(h));
  return 0;
}
