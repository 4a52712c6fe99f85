// Round trip of a one-wave kernel that writes a completion marker into pinned
// host memory, the host spinning on the marker, p50 over 2000 calls each
// (the single-vote latency budget):
//   hip         hipLaunchKernelGGL on a HIP stream (the committee path today);
//   aql/...     an AQL dispatch packet written by this process into a user-mode
//               queue of its own (hsa_queue_create) and the doorbell rung
//               directly, the kernel loaded from a bare code object
//               (tools/aql_kernels.hsaco) -- with the packet's acquire /
//               release fences at system or agent scope, and the kernel
//               arguments in the system kernarg pool or in device memory;
//   aql-req     the same with a 100-byte vote carried in the kernel arguments.
// Every host wait has a timeout; a packet is written only into a free slot.
//
// Build: hipcc --offload-arch=gfx950 -O3 --offload-device-only --no-gpu-bundle-output -c tools/aql_kernels.hip -o tools/aql_kernels.hsaco
//        hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/aql_latency.hip -o tools/aql_latency -lhsa-runtime64
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>

#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <iterator>
#include <string>
#include <vector>

#include "aql_kernels.hip"

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e_ = (x);                                                   \
    if (e_ != hipSuccess) {                                                \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));         \
      return 1;                                                            \
    }                                                                      \
  } while (0)
#define HK(x)                                                              \
  do {                                                                     \
    hsa_status_t s_ = (x);                                                 \
    if (s_ != HSA_STATUS_SUCCESS) {                                        \
      const char *m_ = nullptr;                                            \
      hsa_status_string(s_, &m_);                                          \
      std::fprintf(stderr, "%s: %s\n", #x, m_ ? m_ : "?");                 \
      return 1;                                                            \
    }                                                                      \
  } while (0)

using clk = std::chrono::steady_clock;

static bool wait_for(volatile uint32_t *w, uint32_t v, std::chrono::microseconds limit) {
  const auto t0 = clk::now();
  while (*w != v)
    if (clk::now() - t0 > limit) return false;
  return true;
}

static double pct(std::vector<double> v, double q) {
  std::sort(v.begin(), v.end());
  return v[std::min(v.size() - 1, (size_t)(q * v.size()))];
}

struct Agents {
  std::vector<hsa_agent_t> gpus;
  hsa_agent_t cpu{};
};

static hsa_status_t agent_cb(hsa_agent_t a, void *p) {
  Agents *ag = static_cast<Agents *>(p);
  hsa_device_type_t t;
  if (hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t) != HSA_STATUS_SUCCESS) return HSA_STATUS_SUCCESS;
  if (t == HSA_DEVICE_TYPE_GPU) ag->gpus.push_back(a);
  if (t == HSA_DEVICE_TYPE_CPU && ag->cpu.handle == 0) ag->cpu = a;
  return HSA_STATUS_SUCCESS;
}

struct Pools {
  hsa_amd_memory_pool_t kernarg{}, vram{};
};

static hsa_status_t cpu_pool_cb(hsa_amd_memory_pool_t p, void *d) {
  hsa_amd_segment_t seg;
  hsa_amd_memory_pool_get_info(p, HSA_AMD_MEMORY_POOL_INFO_SEGMENT, &seg);
  if (seg != HSA_AMD_SEGMENT_GLOBAL) return HSA_STATUS_SUCCESS;
  uint32_t fl = 0;
  hsa_amd_memory_pool_get_info(p, HSA_AMD_MEMORY_POOL_INFO_GLOBAL_FLAGS, &fl);
  if ((fl & HSA_AMD_MEMORY_POOL_GLOBAL_FLAG_KERNARG_INIT) && static_cast<Pools *>(d)->kernarg.handle == 0)
    static_cast<Pools *>(d)->kernarg = p;
  return HSA_STATUS_SUCCESS;
}

static hsa_status_t gpu_pool_cb(hsa_amd_memory_pool_t p, void *d) {
  hsa_amd_segment_t seg;
  hsa_amd_memory_pool_get_info(p, HSA_AMD_MEMORY_POOL_INFO_SEGMENT, &seg);
  if (seg != HSA_AMD_SEGMENT_GLOBAL) return HSA_STATUS_SUCCESS;
  uint32_t fl = 0;
  hsa_amd_memory_pool_get_info(p, HSA_AMD_MEMORY_POOL_INFO_GLOBAL_FLAGS, &fl);
  if ((fl & HSA_AMD_MEMORY_POOL_GLOBAL_FLAG_COARSE_GRAINED) && static_cast<Pools *>(d)->vram.handle == 0)
    static_cast<Pools *>(d)->vram = p;
  return HSA_STATUS_SUCCESS;
}

struct Kern {
  uint64_t object = 0;
  uint32_t kernarg = 0, group = 0, priv = 0;
};

static int get_kernel(hsa_executable_t ex, hsa_agent_t gpu, const char *name, Kern *k) {
  hsa_executable_symbol_t sym;
  HK(hsa_executable_get_symbol_by_name(ex, name, &gpu, &sym));
  HK(hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_OBJECT, &k->object));
  HK(hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_KERNARG_SEGMENT_SIZE, &k->kernarg));
  HK(hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_GROUP_SEGMENT_SIZE, &k->group));
  HK(hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_PRIVATE_SEGMENT_SIZE, &k->priv));
  std::printf("# %s: kernarg %u B, group %u B, private %u B\n", name, k->kernarg, k->group, k->priv);
  return 0;
}

// one dispatch of `k` with kernel arguments `args` (copied into `ka`)
static bool dispatch(hsa_queue_t *q, const Kern &k, void *ka, const void *args, size_t nargs, uint16_t acq,
                     uint16_t rel) {
  const uint64_t idx = hsa_queue_add_write_index_screlease(q, 1);
  const auto t0 = clk::now();
  while (idx - hsa_queue_load_read_index_scacquire(q) >= q->size)
    if (clk::now() - t0 > std::chrono::milliseconds(100)) return false;
  std::memcpy(ka, args, nargs);
  auto *p = static_cast<hsa_kernel_dispatch_packet_t *>(q->base_address) + (idx & (q->size - 1));
  p->workgroup_size_x = 64;
  p->workgroup_size_y = 1;
  p->workgroup_size_z = 1;
  p->reserved0 = 0;
  p->grid_size_x = 64;
  p->grid_size_y = 1;
  p->grid_size_z = 1;
  p->private_segment_size = k.priv;
  p->group_segment_size = k.group;
  p->kernel_object = k.object;
  p->kernarg_address = ka;
  p->reserved2 = 0;
  p->completion_signal.handle = 0;
  const uint16_t header = (HSA_PACKET_TYPE_KERNEL_DISPATCH << HSA_PACKET_HEADER_TYPE) |
                          (1 << HSA_PACKET_HEADER_BARRIER) | (acq << HSA_PACKET_HEADER_SCACQUIRE_FENCE_SCOPE) |
                          (rel << HSA_PACKET_HEADER_SCRELEASE_FENCE_SCOPE);
  const uint16_t setup = 1 << HSA_KERNEL_DISPATCH_PACKET_SETUP_DIMENSIONS;
  __atomic_store_n(reinterpret_cast<uint32_t *>(p), (uint32_t)header | ((uint32_t)setup << 16), __ATOMIC_RELEASE);
  hsa_signal_store_screlease(q->doorbell_signal, (hsa_signal_value_t)idx);
  return true;
}

int main(int argc, char **argv) {
  const int reps = 2000;
  const std::string co_path = argc > 1 ? argv[1] : "tools/aql_kernels.hsaco";
  uint32_t *h = nullptr;
  CK(hipHostMalloc(reinterpret_cast<void **>(&h), 4096, hipHostMallocCoherent));
  void *dv = nullptr;
  CK(hipHostGetDevicePointer(&dv, h, 0));
  uint32_t *d = static_cast<uint32_t *>(dv);
  volatile uint32_t *mark = h;
  *mark = 0;
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));

  uint32_t seq = 0;
  std::vector<double> t(reps);
  // HIP launch + marker
  for (int i = -50; i < reps; ++i) {
    const uint32_t v = ++seq;
    const auto a = clk::now();
    hipLaunchKernelGGL(k_mark, dim3(1), dim3(64), 0, st, d, v);
    if (!wait_for(mark, v, std::chrono::milliseconds(100))) {
      std::fprintf(stderr, "hip: marker timeout\n");
      return 1;
    }
    if (i >= 0) t[i] = std::chrono::duration<double, std::micro>(clk::now() - a).count();
  }
  CK(hipStreamSynchronize(st));
  std::printf("{\"path\": \"hip\", \"p50_us\": %.2f, \"p99_us\": %.2f}\n", pct(t, 0.5), pct(t, 0.99));

  // HSA: our own queue and the same kernels from the bare code object
  HK(hsa_init());
  Agents ag;
  HK(hsa_iterate_agents(agent_cb, &ag));
  if (ag.gpus.empty()) {
    std::fprintf(stderr, "no GPU agent\n");
    return 1;
  }
  int hdev = 0;
  CK(hipGetDevice(&hdev));
  char bus[64] = {0};
  CK(hipDeviceGetPCIBusId(bus, sizeof(bus), hdev));
  hsa_agent_t gpu = ag.gpus[0];
  for (hsa_agent_t a : ag.gpus) {  // the agent of HIP's current device, by PCI location
    uint32_t bdf = 0;
    if (hsa_agent_get_info(a, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_BDFID, &bdf) != HSA_STATUS_SUCCESS) continue;
    unsigned dom = 0, b = 0, dv2 = 0, fn = 0;
    if (std::sscanf(bus, "%x:%x:%x.%x", &dom, &b, &dv2, &fn) == 4 && bdf == ((b << 8) | (dv2 << 3) | fn)) gpu = a;
  }
  Pools pools;
  HK(hsa_amd_agent_iterate_memory_pools(ag.cpu, cpu_pool_cb, &pools));
  HK(hsa_amd_agent_iterate_memory_pools(gpu, gpu_pool_cb, &pools));
  std::ifstream f(co_path, std::ios::binary);
  std::vector<char> co((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
  if (co.empty()) {
    std::fprintf(stderr, "cannot read %s\n", co_path.c_str());
    return 1;
  }
  hsa_code_object_reader_t rd;
  HK(hsa_code_object_reader_create_from_memory(co.data(), co.size(), &rd));
  hsa_executable_t ex;
  HK(hsa_executable_create_alt(HSA_PROFILE_FULL, HSA_DEFAULT_FLOAT_ROUNDING_MODE_DEFAULT, nullptr, &ex));
  HK(hsa_executable_load_agent_code_object(ex, gpu, rd, nullptr, nullptr));
  HK(hsa_executable_freeze(ex, nullptr));
  Kern km, kr;
  if (get_kernel(ex, gpu, "k_mark.kd", &km) || get_kernel(ex, gpu, "k_mark_req.kd", &kr)) return 1;
  hsa_queue_t *q = nullptr;
  HK(hsa_queue_create(gpu, 64, HSA_QUEUE_TYPE_MULTI, nullptr, nullptr, UINT32_MAX, UINT32_MAX, &q));
  void *ka_sys = nullptr, *ka_dev = nullptr;
  HK(hsa_amd_memory_pool_allocate(pools.kernarg, 64 * 1024, 0, &ka_sys));
  HK(hsa_amd_agents_allow_access(1, &gpu, nullptr, ka_sys));
  bool have_dev = false;
  if (pools.vram.handle) {
    if (hsa_amd_memory_pool_allocate(pools.vram, 64 * 1024, 0, &ka_dev) == HSA_STATUS_SUCCESS &&
        hsa_amd_agents_allow_access(1, &ag.cpu, nullptr, ka_dev) == HSA_STATUS_SUCCESS) {
      // a host store into device memory must be readable by the host back
      volatile uint32_t *pd = static_cast<volatile uint32_t *>(ka_dev);
      pd[0] = 0x12345678u;
      have_dev = pd[0] == 0x12345678u;
    }
  }
  std::printf("# device-memory kernargs: %s\n", have_dev ? "host-writable" : "unavailable");

  struct Case {
    const char *name;
    bool req, dev;
    uint16_t acq, rel;
  };
  const Case cases[] = {
      {"aql sys-kernarg acq=system rel=system", false, false, HSA_FENCE_SCOPE_SYSTEM, HSA_FENCE_SCOPE_SYSTEM},
      {"aql sys-kernarg acq=agent rel=agent", false, false, HSA_FENCE_SCOPE_AGENT, HSA_FENCE_SCOPE_AGENT},
      {"aql sys-kernarg acq=system rel=none", false, false, HSA_FENCE_SCOPE_SYSTEM, HSA_FENCE_SCOPE_NONE},
      {"aql dev-kernarg acq=system rel=system", false, true, HSA_FENCE_SCOPE_SYSTEM, HSA_FENCE_SCOPE_SYSTEM},
      {"aql dev-kernarg acq=system rel=none", false, true, HSA_FENCE_SCOPE_SYSTEM, HSA_FENCE_SCOPE_NONE},
      {"aql-req sys-kernarg acq=system rel=none", true, false, HSA_FENCE_SCOPE_SYSTEM, HSA_FENCE_SCOPE_NONE},
      {"aql-req dev-kernarg acq=system rel=none", true, true, HSA_FENCE_SCOPE_SYSTEM, HSA_FENCE_SCOPE_NONE},
  };
  for (const Case &c : cases) {
    if (c.dev && !have_dev) continue;
    uint8_t *ka_base = static_cast<uint8_t *>(c.dev ? ka_dev : ka_sys);
    const Kern &k = c.req ? kr : km;
    const size_t slot = 1024;
    for (int i = -50; i < reps; ++i) {
      const uint32_t v = ++seq;
      const auto a = clk::now();
      void *ka = ka_base + ((uint64_t)(i + 64) % 64) * slot;
      bool ok;
      if (c.req) {
        Req r{};
        r.done = d;
        r.v = v;
        r.kidx = (uint32_t)i;
        for (int j = 0; j < 16; ++j) r.sig[j] = v * 0x01000193u + j;
        for (int j = 0; j < 8; ++j) r.msg[j] = v ^ (uint32_t)j;
        ok = dispatch(q, k, ka, &r, sizeof(r), c.acq, c.rel);
      } else {
        struct {
          uint32_t *done;
          uint32_t v, pad;
        } args{d, v, 0};
        ok = dispatch(q, k, ka, &args, sizeof(args), c.acq, c.rel);
      }
      if (!ok || !wait_for(mark, v, std::chrono::milliseconds(100))) {
        std::fprintf(stderr, "%s: %s\n", c.name, ok ? "marker timeout" : "queue full");
        return 1;
      }
      if (i >= 0) t[i] = std::chrono::duration<double, std::micro>(clk::now() - a).count();
    }
    std::printf("{\"path\": \"%s\", \"p50_us\": %.2f, \"p99_us\": %.2f}\n", c.name, pct(t, 0.5), pct(t, 0.99));
  }
  // drain: every packet consumed before the queue goes
  const auto t0 = clk::now();
  while (hsa_queue_load_read_index_scacquire(q) != hsa_queue_load_write_index_scacquire(q))
    if (clk::now() - t0 > std::chrono::seconds(1)) break;
  hsa_queue_destroy(q);
  hsa_executable_destroy(ex);
  hsa_code_object_reader_destroy(rd);
  return 0;
}
