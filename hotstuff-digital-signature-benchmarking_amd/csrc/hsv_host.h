// Host-side state shared by the C-ABI translation units (hsv_capi.cpp,
// hsv_committee_api.cpp, hsv_tx.cpp).  Not part of the public ABI.
//
// Device model (include/hsv.h, hsv_init):
//   * one DevCtx per visible GPU, created lazily;
//   * each DevCtx owns a small pool of Slots (stream + pinned staging +
//     device buffer + mutex), so concurrent host-buffer calls -- several
//     tokio workers verifying QCs and votes at once -- run side by side
//     instead of queueing on one staging buffer;
//   * the fixed-base B tables (narrow comb for the committee kernels, wide
//     comb for the generic kernels) are per device and shared by its slots.
#pragma once
#include <hip/hip_runtime_api.h>

#include <atomic>
#include <cstddef>
#include <cstdint>
#include <cstring>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "hsv.h"
#include "hsv_internal.h"

#if defined(__SSE2__)
#include <emmintrin.h>
#endif

namespace hsvh {

// ---- errors ----------------------------------------------------------------
int fail(int code, const std::string &msg);
int hip_fail(const char *where, hipError_t e);
const std::string &last_error();

// ---- host timeline of a call (hsv_host_call_marks) ---------------------------
// Every public entry point that verifies opens a CallScope; the path below it
// stamps the HSV_MARK_* points it passes (ms from the entry), or, in a
// pipelined call, four marks per chunk.
class CallScope {
 public:
  CallScope();
  ~CallScope();
  CallScope(const CallScope &) = delete;
  CallScope &operator=(const CallScope &) = delete;
};
void call_mark(int which);
void call_chunk_mark();

// ---- sizes -------------------------------------------------------------------
constexpr size_t kAlign = 256;
constexpr size_t kChunk = size_t(1) << 22;        // items per verification launch
constexpr size_t kShardMin = size_t(1) << 16;     // shard host batches across devices at or above this
constexpr size_t kZeroCopyMax = size_t(1) << 12;  // small batches read straight from pinned memory
inline size_t round_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

// Inputs a kernel reads straight from pinned memory (the zero-copy latency
// form) are written with streaming stores, so they sit in DRAM and not in the
// writing core's cache: the GPU's reads then need no snoop of a remote core's
// cache, whose cost grows with the distance from that core to the PCIe root
// (after a host load had moved the calling thread, the C3 QC read 0.0634
// against 0.0543 ms, profiles/r05q_idle.txt).  dst 16-byte aligned; the tail
// of n that is not a multiple of 16 is a plain copy.  stage_fence() orders the
// streaming stores before the launch that reads them.
inline void stage_copy(uint8_t *dst, const void *src, size_t n) {
  const uint8_t *s = static_cast<const uint8_t *>(src);
#if defined(__SSE2__)
  size_t i = 0;
  for (; i + 16 <= n; i += 16)
    _mm_stream_si128(reinterpret_cast<__m128i *>(dst + i), _mm_loadu_si128(reinterpret_cast<const __m128i *>(s + i)));
  if (i < n) std::memcpy(dst + i, s + i, n - i);
#else
  std::memcpy(dst, s, n);
#endif
}
inline void stage_fence() {
#if defined(__SSE2__)
  _mm_sfence();
#endif
}

// ---- device contexts ---------------------------------------------------------
struct Slot {
  std::mutex mu;
  hipStream_t stream = nullptr;
  hipStream_t stream2 = nullptr;  // second compute stream of large host batches
  hipStream_t copy = nullptr;     // host-to-device stream of large host batches
  hipEvent_t ev[5] = {nullptr, nullptr, nullptr, nullptr, nullptr};  // staged[2], unused, joined[2] (run_pipelined)
  uint8_t *d_ws[3] = {nullptr, nullptr, nullptr};  // launch workspaces of the compute streams (run_pipelined)
  size_t ws_cap = 0;
  uint8_t *d_buf = nullptr;
  size_t d_cap = 0;
  uint8_t *h_buf = nullptr;
  uint8_t *h_buf_dev = nullptr;  // h_buf's device address (zero-copy launches), looked up once
  size_t h_cap = 0;
  // flag bytes, self-check words and completion markers of the committee
  // latency form (committee_run), in COHERENT pinned memory: the host reads
  // them while the kernel may still be running (marker sync), so they must not
  // sit in the GPU's L2 -- correctness does not rest on the release fence's
  // write-back of non-coherent lines (round-4 advice)
  uint8_t *h_sync = nullptr;
  uint8_t *h_sync_dev = nullptr;
  size_t h_sync_cap = 0;
  size_t pipe_warm_n = 0;  // items of the last completed pipelined call (HSV_PIPE_NOCOPY)
};

struct DevCtx {
  int device = 0;
  int cus = 0;
  std::mutex table_mu;             // guards the two B tables and d_fault below
  uint32_t *d_btable = nullptr;    // narrow comb of B (committee kernels)
  uint32_t *d_btable16 = nullptr;  // wide comb of B (generic kernels)
  uint32_t *d_fault = nullptr;     // self-check words of the device-resident calls (hsv_device_faults);
                                   // words kFaultOutWord.. receive the read-and-clear exchange
  std::mutex fault_mu;             // one read-and-clear of d_fault at a time
  std::vector<std::unique_ptr<Slot>> slots;
  std::atomic<unsigned> rr{0};
  std::mutex side_mu;                    // guards the side-stream pool
  std::vector<hipStream_t> side_free;    // idle second streams of multi-chunk device-API batches
  std::vector<hipStream_t> side_all;     // every side stream created (hsv_shutdown)
};

// Makes `device` current for the calling thread and restores the previous
// current device on destruction (the library never leaves the caller's
// thread on another device).
class DeviceGuard {
 public:
  explicit DeviceGuard(int device);
  ~DeviceGuard();
  hipError_t status() const { return status_; }

 private:
  int prev_ = -1;
  hipError_t status_ = hipSuccess;
};

int ensure_init();  // HSV_OK or HSV_ERR_NO_DEVICE
int device_count_inited();
DevCtx &ctx(int device);
int variant();

// Device a host-buffer call of n items that is not sharded runs on: the
// bound device (hsv_init(d) / HSV_DEVICE), else the calling thread's
// current HIP device.
int home_device();
// Number of shards a host batch of n items is split into (1 = no sharding)
// and the device shard s runs on.
int shard_count(size_t n);
int shard_device(int shard, int nshards);

// Lock a free slot of `c` (try every slot, then wait on one).
class SlotLease {
 public:
  explicit SlotLease(DevCtx &c);
  Slot &slot() { return *s_; }

 private:
  Slot *s_;
  std::unique_lock<std::mutex> lk_;
};

// Stream and buffers of a slot (current device must be c.device).
int slot_prepare(Slot &s, size_t dev_bytes, size_t host_bytes);
int slot_stream2(Slot &s);
int slot_pipeline(Slot &s);  // stream2, the copy stream, the events of run_pipelined
// the slot's coherent sync region (Slot::h_sync) of at least `bytes`
int slot_sync_region(Slot &s, size_t bytes);

// Device self-check words (hsv_kernels.hip report_faults): two words per
// launch, zeroed before it; non-zero after it -> HSV_ERR_DEVICE_FAULT.
constexpr size_t kFaultBytes = 8;
int check_faults(const uint8_t *words, const char *where);
// The per-device words of the stream-ordered device API (current device
// must be c.device); allocated and zeroed on first use.
int device_fault_words(DevCtx &c, uint32_t **out);
constexpr size_t kFaultOutWord = 4;  // d_fault[4..5]: output of hsv_launch_fault_exchange
// The words a device-API call reports into: the caller's d_fault (zeroed on
// `stream` here), or the per-device words when d_fault is NULL.
int call_fault_words(DevCtx &c, uint32_t *d_fault, hipStream_t stream, uint32_t **out);

// A side stream of device c for one call (current device must be c.device),
// returned to the pool when the lease ends: concurrent device-API calls never
// share one, so a call's join event only waits for its own chunks.
class SideStreamLease {
 public:
  explicit SideStreamLease(DevCtx &c);
  ~SideStreamLease();
  hipStream_t stream() const { return s_; }

 private:
  DevCtx &c_;
  hipStream_t s_ = nullptr;
};

// B tables of device c (current device must be c.device).
int ensure_btable(DevCtx &c);
int ensure_btable16(DevCtx &c);
int comb_table_for(DevCtx &c, int variant, const uint32_t **out);

// memcpy into pinned staging; large copies split over the pack pool of the
// current device (its helpers run on the GPU's NUMA node)
void stage_copy(uint8_t *dst, const uint8_t *src, size_t bytes);

// ---- host placement (hsv_numa.cpp) -------------------------------------------
struct HostPlace {
  int node = -1;          // NUMA node of the GPU's PCIe function (-1: unknown / single node)
  std::vector<int> cpus;  // that node's CPUs the process may use (empty: threads stay unpinned)
  int pack_threads = 0;   // helpers of the device's pack pool
};
bool parse_cpulist(const std::string &text, std::vector<int> &out);
std::vector<int> current_affinity();
bool pin_current_thread(const std::vector<int> &cpus);
int default_pack_threads();
// For PCI functions `bdfs` under the sysfs tree `root`: each one's node, the
// node's CPUs within `allowed` (sorted), and the pack-pool size (the node's
// CPUs split among its GPUs, at most pack_default)
std::vector<HostPlace> plan_host_places(const std::string &root, const std::vector<std::string> &bdfs,
                                        const std::vector<int> &allowed, int pack_default);
// The placement of a visible device (sysfs under /sys, the process affinity
// at first use); a device without NUMA information gets an unpinned place.
const HostPlace &device_place(int device);

// Run fn(shard, device) for shards [0, k) of a host batch, each on the
// persistent shard worker of its index, pinned to the NUMA node of its
// device; returns HSV_OK or the first shard's error.  The caller's fault
// injection mode (tests) reaches the workers.
int run_sharded(int k, const std::function<int(int shard, int device)> &fn);

// Device owning a device pointer (hipPointerGetAttributes); -1 if unknown.
int pointer_device(const void *p);
// Resolve the device a device-API call runs on: the device of its input
// pointers, checked against the stream's device.  Returns HSV_OK and sets
// *dev, or an error.
int device_for_call(const void *d_ptr, void *stream, int *dev);

// ---- hooks shared with hsv_test_hooks.cpp (exported by libhsv_test.so only) ----
int auto_committee_corrupt_tables();  // zero the cached tables of the automatic committee

// ---- the automatic committee cache (hsv_committee_api.cpp) --------------------
// Strict verification of small batches whose keys are all cached: HSV_OK
// when done, 1 when the caller should take the generic path, < 0 on error.
int auto_committee_try(const uint8_t *pk, const uint8_t *sig, const uint8_t *msg, size_t msg_stride, size_t n,
                       uint8_t *flags_out);
void auto_committee_shutdown();
// resident latency service (on by default, hsv_committee_api.cpp)
// A scope in which its kernel does not run: stopped at construction, and no
// request or relaunch until destruction (small calls launch meanwhile).  Held
// around every hipFree / hipHostFree of the library -- they wait for every
// grid on the device -- and around device-wide waits.
class ResidentPause {
 public:
  ResidentPause();
  ~ResidentPause();
  ResidentPause(const ResidentPause &) = delete;
  ResidentPause &operator=(const ResidentPause &) = delete;
};
void resident_quiesce();  // stop its kernel now (the next request relaunches it)
void resident_counts(uint64_t *posted, uint64_t *answered);
int resident_post_bad(uint32_t m);  // test hook: a request the kernel must refuse
int resident_set_mode(int on);      // hsv_set_resident_service

// The generic host-buffer path (hsv_capi.cpp): records at the given strides.
int run_host(const uint8_t *pk, size_t pk_stride, const uint8_t *sig, size_t sig_stride, const uint8_t *msg,
             size_t msg_stride, size_t n, uint8_t *flags_out);
int batch_verdict(const uint8_t *flags, size_t n);

}  // namespace hsvh
