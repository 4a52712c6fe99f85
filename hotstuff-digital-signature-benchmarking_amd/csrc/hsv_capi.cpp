// C ABI of libhsv.so (declared in include/hsv.h): device contexts and their
// slot pools, device binding, sharding across GPUs, and the generic
// reference-shaped entry points.
//
// Host-buffer calls stage inputs into the pinned buffer of a free slot,
// copy them to HBM on the slot's stream, launch the verification kernels and
// copy the flag bytes back.  Batches of at least kShardMin items are split
// into contiguous ranges, one per device (or per virtual shard, a test hook),
// each driven by its own host thread; the per-item flags are written straight
// into the caller's output (the "host gather").  There is no CPU
// verification path: without a GPU every call returns HSV_ERR_NO_DEVICE.
#include <hip/hip_runtime_api.h>
#if defined(__SSE2__)
#include <emmintrin.h>
#endif

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "hsv.h"
#include "hsv_host.h"
#include "hsv_internal.h"

namespace hsvh {

namespace {

thread_local std::string t_last_error;

constexpr int kUnbound = -2;

// Host timeline of the calling thread's current / last public call
// (hsv_host_call_marks).  CallScope opens it at every public entry point; a
// nested entry (hsv_verify_strict -> hsv_verify) joins the outer call.
struct CallClock {
  int depth = 0;
  std::chrono::steady_clock::time_point t0;
  std::vector<double> marks;
};
thread_local CallClock t_clock;

struct Global {
  std::mutex mu;
  bool inited = false;
  int ndev = 0;
  std::vector<DevCtx *> ctx;
  // fastest measured: scalar prepass + half-size point pass, wide B comb, WA=4,
  // 3 waves/SIMD; two lanes per item for batches of at most 2^13 (QC latency)
  std::atomic<int> variant{21};
  std::atomic<int> bound{kUnbound};  // >= 0: one device; -1: every device
  std::atomic<int> virtual_shards{0};  // test hook: k > 0 shards on the bound/home devices
  int nslots = 4;
};

Global &G() {
  static Global g;
  return g;
}

int env_int(const char *name, int dflt) {
  const char *v = std::getenv(name);
  if (!v || !*v) return dflt;
  return std::atoi(v);
}

}  // namespace

int fail(int code, const std::string &msg) {
  t_last_error = msg;
  return code;
}

int hip_fail(const char *where, hipError_t e) {
  // out of device memory (after hsv_ws_malloc's trim and retry) is the
  // allocation error of include/hsv.h, every other HIP failure HSV_ERR_HIP
  return fail(e == hipErrorOutOfMemory ? HSV_ERR_ALLOC : HSV_ERR_HIP, std::string(where) + ": " + hipGetErrorString(e));
}

const std::string &last_error() { return t_last_error; }

CallScope::CallScope() {
  CallClock &c = t_clock;
  if (c.depth++ == 0) {
    c.t0 = std::chrono::steady_clock::now();
    c.marks.assign(HSV_MARKS, -1.0);
  }
}

CallScope::~CallScope() { --t_clock.depth; }

static double clock_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_clock.t0).count();
}

void call_mark(int which) {
  CallClock &c = t_clock;
  if (c.depth > 0 && which >= 0 && (size_t)which < c.marks.size()) c.marks[which] = clock_ms();
}

void call_chunk_mark() {
  if (t_clock.depth > 0) t_clock.marks.push_back(clock_ms());
}

int ensure_init() {
  Global &g = G();
  std::lock_guard<std::mutex> lk(g.mu);
  if (g.inited) return g.ndev > 0 ? HSV_OK : fail(HSV_ERR_NO_DEVICE, "no HIP device visible");
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
  (void)hipGetLastError();
  g.ndev = n;
  g.nslots = std::min(16, std::max(1, env_int("HSV_SLOTS", 4)));
  for (int i = 0; i < n; ++i) {
    DevCtx *c = new DevCtx();
    c->device = i;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, i) == hipSuccess) c->cus = prop.multiProcessorCount;
    for (int s = 0; s < g.nslots; ++s) c->slots.emplace_back(new Slot());
    g.ctx.push_back(c);
  }
  const int d = env_int("HSV_DEVICE", kUnbound);
  if (g.bound.load() == kUnbound && d >= -1 && d < n) g.bound = d;
  g.inited = true;
  return n > 0 ? HSV_OK : fail(HSV_ERR_NO_DEVICE, "no HIP device visible");
}

int device_count_inited() { return G().ndev; }
DevCtx &ctx(int device) { return *G().ctx[device]; }
int variant() { return G().variant.load(); }

int home_device() {
  Global &g = G();
  const int b = g.bound.load();
  if (b >= 0 && b < g.ndev) return b;
  int d = 0;
  if (hipGetDevice(&d) != hipSuccess || d < 0 || d >= g.ndev) d = 0;
  return d;
}

int shard_count(size_t n) {
  Global &g = G();
  if (n < kShardMin) return 1;
  const int vs = g.virtual_shards.load();
  if (vs > 0) return vs;
  return g.bound.load() >= 0 ? 1 : g.ndev;
}

int shard_device(int shard, int nshards) {
  Global &g = G();
  const int b = g.bound.load();
  if (b >= 0 && b < g.ndev) return b;
  if (g.virtual_shards.load() > 0 || nshards > g.ndev) return shard % g.ndev;
  return shard;
}

DeviceGuard::DeviceGuard(int device) {
  if (hipGetDevice(&prev_) != hipSuccess) prev_ = -1;
  if (prev_ != device) status_ = hipSetDevice(device);
}

DeviceGuard::~DeviceGuard() {
  int cur = -1;
  if (prev_ >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev_) (void)hipSetDevice(prev_);
}

SlotLease::SlotLease(DevCtx &c) {
  // lowest free slot first: a lone caller keeps reusing slot 0 and its warm
  // staging buffers; concurrent callers spill over to the next slots
  const size_t k = c.slots.size();
  for (size_t i = 0; i < k; ++i) {
    Slot &s = *c.slots[i];
    std::unique_lock<std::mutex> l(s.mu, std::try_to_lock);
    if (l.owns_lock()) {
      s_ = &s;
      lk_ = std::move(l);
      return;
    }
  }
  s_ = c.slots[c.rr.fetch_add(1) % k].get();  // all busy: queue on one, round-robin
  lk_ = std::unique_lock<std::mutex>(s_->mu);
}

// A slot's streams are created at the greatest stream priority.  HIP spreads
// streams over a few hardware queues per priority (GPU_MAX_HW_QUEUES, 4 on
// the box); at normal priority a slot whose streams were created after the
// application's own shared their queues, and the pipelined 2^20 host call
// took 10.9-11.0 ms against 10.1-10.3 ms at the greatest priority, with the
// application's three-stream C4 line unchanged (8.89-8.92 ms per step;
// tools/eager_streams_ab.sh, profiles/r03zm_eager_streams_ab.txt).
hipError_t pipe_stream_create(hipStream_t *s) {
  int least = 0, greatest = 0;
  if (hipDeviceGetStreamPriorityRange(&least, &greatest) == hipSuccess)
    return hipStreamCreateWithPriority(s, hipStreamNonBlocking, greatest);
  return hipStreamCreateWithFlags(s, hipStreamNonBlocking);
}

int slot_prepare(Slot &s, size_t dev_bytes, size_t host_bytes) {
  hipError_t e;
  if (!s.stream) {
    e = pipe_stream_create(&s.stream);
    if (e != hipSuccess) return hip_fail("hipStreamCreate", e);
  }
  std::unique_ptr<ResidentPause> pause;  // hipFree / hipHostFree wait for every grid on the device
  if ((dev_bytes > s.d_cap && s.d_buf) || (host_bytes > s.h_cap && s.h_buf)) pause.reset(new ResidentPause());
  if (dev_bytes > s.d_cap) {
    if (s.d_buf) (void)hipFree(s.d_buf);
    s.d_buf = nullptr;
    s.d_cap = 0;
    const size_t cap = round_up(dev_bytes, size_t(1) << 20);
    e = hipMalloc(&s.d_buf, cap);
    if (e != hipSuccess) return hip_fail("hipMalloc", e);
    s.d_cap = cap;
  }
  if (host_bytes > s.h_cap) {
    if (s.h_buf) (void)hipHostFree(s.h_buf);
    s.h_buf = s.h_buf_dev = nullptr;
    s.h_cap = 0;
    const size_t cap = round_up(host_bytes, size_t(1) << 20);
    e = hipHostMalloc(&s.h_buf, cap, hipHostMallocDefault);
    if (e != hipSuccess) return hip_fail("hipHostMalloc", e);
    s.h_cap = cap;
    // the zero-copy latency path needs the device address at every call
    void *hd = nullptr;
    if (hipHostGetDevicePointer(&hd, s.h_buf, 0) == hipSuccess) s.h_buf_dev = static_cast<uint8_t *>(hd);
  }
  return HSV_OK;
}

int slot_sync_region(Slot &s, size_t bytes) {
  if (bytes <= s.h_sync_cap) return HSV_OK;
  if (s.h_sync) {
    ResidentPause pause;  // hipHostFree waits for every grid on the device
    (void)hipHostFree(s.h_sync);
  }
  s.h_sync = s.h_sync_dev = nullptr;
  s.h_sync_cap = 0;
  const size_t cap = round_up(bytes, size_t(64) << 10);
  hipError_t e = hipHostMalloc(&s.h_sync, cap, hipHostMallocCoherent | hipHostMallocMapped);
  if (e != hipSuccess) return hip_fail("hipHostMalloc (coherent sync region)", e);
  void *hd = nullptr;
  e = hipHostGetDevicePointer(&hd, s.h_sync, 0);
  if (e != hipSuccess || !hd) {
    ResidentPause pause;
    (void)hipHostFree(s.h_sync);
    s.h_sync = nullptr;
    return hip_fail("hipHostGetDevicePointer (coherent sync region)", e);
  }
  s.h_sync_dev = static_cast<uint8_t *>(hd);
  s.h_sync_cap = cap;
  return HSV_OK;
}

int slot_stream2(Slot &s) {
  if (s.stream2) return HSV_OK;
  const hipError_t e = pipe_stream_create(&s.stream2);
  return e == hipSuccess ? HSV_OK : hip_fail("hipStreamCreate", e);
}

int slot_pipeline(Slot &s) {
  int rc = slot_stream2(s);
  if (rc != HSV_OK) return rc;
  hipError_t e = hipSuccess;
  if (!s.copy) e = pipe_stream_create(&s.copy);
  for (int i = 0; i < 5 && e == hipSuccess; ++i)
    if (!s.ev[i]) e = hipEventCreateWithFlags(&s.ev[i], hipEventDisableTiming);
  return e == hipSuccess ? HSV_OK : hip_fail("creating the pipeline streams and events", e);
}

namespace {

const uint8_t kBasepointEncoding[32] = {0x58, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66,
                                        0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66,
                                        0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66};

// one-off table builds run on a stream of their own
int build_on_private_stream(const std::function<hipError_t(hipStream_t)> &enqueue) {
  hipStream_t st = nullptr;
  hipError_t e = hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
  if (e != hipSuccess) return hip_fail("hipStreamCreate", e);
  e = enqueue(st);
  if (e == hipSuccess) e = hipStreamSynchronize(st);
  (void)hipStreamDestroy(st);
  return e == hipSuccess ? HSV_OK : hip_fail("building a B comb table", e);
}

}  // namespace

int ensure_btable(DevCtx &c) {
  std::lock_guard<std::mutex> lk(c.table_mu);
  if (c.d_btable) return HSV_OK;
  uint8_t *d_enc = nullptr;
  uint32_t *d_tab = nullptr, *d_tmp = nullptr;
  hipError_t e = hipMalloc(&d_enc, 32);
  if (e == hipSuccess) e = hipMalloc(&d_tab, hsv_comb_table_bytes());
  if (e == hipSuccess) e = hipMalloc(&d_tmp, hsv_comb_tmp_bytes(1));
  if (e == hipSuccess) e = hipMemcpy(d_enc, kBasepointEncoding, 32, hipMemcpyHostToDevice);
  int rc = e == hipSuccess ? HSV_OK : hip_fail("allocating the B comb table", e);
  if (rc == HSV_OK)
    rc = build_on_private_stream([&](hipStream_t st) { return hsv_launch_comb_build(d_enc, 1, 0, d_tab, d_tmp, nullptr, st); });
  ResidentPause pause;  // hipFree waits for every grid on the device
  if (d_enc) (void)hipFree(d_enc);
  if (d_tmp) (void)hipFree(d_tmp);
  if (rc != HSV_OK) {
    if (d_tab) (void)hipFree(d_tab);
    return rc;
  }
  c.d_btable = d_tab;
  return HSV_OK;
}

int ensure_btable16(DevCtx &c) {
  std::lock_guard<std::mutex> lk(c.table_mu);
  if (c.d_btable16) return HSV_OK;
  uint32_t *d_tab = nullptr, *d_tmp = nullptr;
  hipError_t e = hipMalloc(&d_tab, hsv_comb16_table_bytes());
  if (e == hipSuccess) e = hipMalloc(&d_tmp, hsv_comb16_tmp_bytes());
  int rc = e == hipSuccess ? HSV_OK : hip_fail("allocating the wide B comb table", e);
  if (rc == HSV_OK) rc = build_on_private_stream([&](hipStream_t st) { return hsv_launch_comb16_build(d_tab, d_tmp, st); });
  ResidentPause pause;  // hipFree waits for every grid on the device
  if (d_tmp) (void)hipFree(d_tmp);
  if (rc != HSV_OK) {
    if (d_tab) (void)hipFree(d_tab);
    return rc;
  }
  c.d_btable16 = d_tab;
  return HSV_OK;
}

int comb_table_for(DevCtx &c, int v, const uint32_t **out) {
  *out = nullptr;
  const int bits = hsv_variant_needs_comb(v);
  if (bits == 0) return HSV_OK;
  const int rc = bits == 16 ? ensure_btable16(c) : ensure_btable(c);
  if (rc != HSV_OK) return rc;
  *out = bits == 16 ? c.d_btable16 : c.d_btable;
  return HSV_OK;
}

// ---- persistent host threads for the staging copies ----------------------------
// A host-buffer batch must be packed into pinned memory before the DMA engine
// can read it (128 MiB for 2^20 triples).  One thread copies ~10 GB/s, which
// made the pack -- not PCIe -- the bound of the drop-in path in round 2.  Each
// device has a pool of helper threads, pinned to the CPUs of that GPU's NUMA
// node (hsv_numa.cpp), which split every pack with the caller; a caller that
// finds its device's pool busy (another thread's pack) copies its parts
// itself.  With one pool per device, the shards of a multi-GPU batch pack
// side by side, each on its GPU's socket (round 5 had one process-wide pool,
// so at eight shards one shard had the helpers and seven packed alone).
namespace {

class PackPool {
 public:
  PackPool(int nthreads, std::vector<int> cpus) {
    for (int i = 0; i < nthreads; ++i)
      workers_.emplace_back([this, cpus] {
        pin_current_thread(cpus);  // no-op for an empty set
        loop();
      });
  }
  ~PackPool() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto &t : workers_) t.join();
  }
  int threads() const { return (int)workers_.size(); }
  // fn(part) for part in [0, nparts), spread over the pool and the caller
  void run(int nparts, const std::function<void(int)> &fn) {
    std::unique_lock<std::mutex> busy(job_mu_, std::try_to_lock);
    if (!busy.owns_lock() || workers_.empty() || nparts < 2) {
      for (int p = 0; p < nparts; ++p) fn(p);
      return;
    }
    auto job = std::make_shared<Job>();
    job->fn = &fn;
    job->nparts = nparts;
    {
      std::lock_guard<std::mutex> lk(mu_);
      job_ = job;
    }
    cv_.notify_all();
    work(*job);
    std::unique_lock<std::mutex> lk(mu_);
    done_cv_.wait(lk, [&] { return job->done == job->nparts; });
    job_.reset();
  }

 private:
  // A job outlives late workers: one that wakes after the job finished finds
  // its part counter exhausted and never calls fn.
  struct Job {
    const std::function<void(int)> *fn = nullptr;
    int nparts = 0;
    int done = 0;  // guarded by mu_
    std::atomic<int> next{0};
  };

  void work(Job &j) {
    int mine = 0;
    for (int p; (p = j.next.fetch_add(1)) < j.nparts;) {
      (*j.fn)(p);
      ++mine;
    }
    std::lock_guard<std::mutex> lk(mu_);
    j.done += mine;
    if (j.done == j.nparts) done_cv_.notify_all();
  }
  void loop() {
    std::shared_ptr<Job> last;
    std::unique_lock<std::mutex> lk(mu_);
    for (;;) {
      cv_.wait(lk, [&] { return stop_ || (job_ && job_ != last); });
      if (stop_) return;
      last = job_;
      lk.unlock();
      work(*last);
      lk.lock();
    }
  }

  std::mutex job_mu_;  // one pack at a time
  std::mutex mu_;
  std::condition_variable cv_, done_cv_;
  std::shared_ptr<Job> job_;
  bool stop_ = false;
  std::vector<std::thread> workers_;
};

// The pack pool of `device` (created on first use with that device's
// placement; -1: an unpinned pool for a caller without a device).  Pools live
// for the process.
PackPool &pack_pool(int device) {
  static std::mutex mu;
  static std::map<int, std::unique_ptr<PackPool>> pools;
  std::lock_guard<std::mutex> lk(mu);
  auto it = pools.find(device);
  if (it == pools.end()) {
    const HostPlace &p = device_place(device);
    it = pools.emplace(device, std::unique_ptr<PackPool>(new PackPool(p.pack_threads, p.cpus))).first;
  }
  return *it->second;
}

PackPool &pack_pool_current() {
  int d = -1;
  if (hipGetDevice(&d) != hipSuccess) d = -1;
  return pack_pool(d);
}

// ---- shard workers ----------------------------------------------------------------
// One persistent thread per shard index of a multi-GPU host batch: shard i
// runs on GPU i (run_host, run_tx_host), so its worker is pinned to that GPU's
// NUMA node, and the slot buffers it allocates there (pinned staging, first
// touched by this thread) sit on that node too.  Round 5 started one
// unpinned std::thread per shard per call.
class ShardWorker {
 public:
  ShardWorker() : th_([this] { loop(); }) {}
  ~ShardWorker() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    th_.join();
  }
  void post(int device, std::function<void()> fn) {
    {
      std::lock_guard<std::mutex> lk(mu_);
      q_.push_back({device, std::move(fn)});
    }
    cv_.notify_all();
  }

 private:
  void loop() {
    int placed = -2;  // the device this thread is pinned for
    std::unique_lock<std::mutex> lk(mu_);
    for (;;) {
      cv_.wait(lk, [&] { return stop_ || !q_.empty(); });
      if (q_.empty()) return;  // stop_ with nothing left
      auto job = std::move(q_.front());
      q_.erase(q_.begin());
      lk.unlock();
      if (job.first != placed) {
        const HostPlace &p = device_place(job.first);
        if (!pin_current_thread(p.cpus)) pin_current_thread(current_affinity_at_start_);
        placed = job.first;
      }
      job.second();
      lk.lock();
    }
  }
  std::vector<int> current_affinity_at_start_ = current_affinity();
  std::mutex mu_;
  std::condition_variable cv_;
  std::vector<std::pair<int, std::function<void()>>> q_;
  bool stop_ = false;
  std::thread th_;  // last: starts once the members above exist
};

ShardWorker &shard_worker(int shard) {
  static std::mutex mu;
  static std::vector<std::unique_ptr<ShardWorker>> workers;
  std::lock_guard<std::mutex> lk(mu);
  while ((int)workers.size() <= shard) workers.emplace_back(new ShardWorker());
  return *workers[shard];
}

}  // namespace

int run_sharded(int k, const std::function<int(int, int)> &fn) {
  struct Join {
    std::mutex mu;
    std::condition_variable cv;
    int left = 0;
  } join;
  join.left = k;
  std::vector<int> rcs(k, HSV_OK);
  std::vector<std::string> errs(k);
  const int inject = hsvi_inject_mode();  // the caller's (test) injection reaches its shards
  for (int d = 0; d < k; ++d) {
    const int dev = shard_device(d, k);
    shard_worker(d).post(dev, [&, d, dev, inject] {
      const int prev = hsvi_set_inject(inject);
      try {
        rcs[d] = fn(d, dev);
        if (rcs[d] != HSV_OK) errs[d] = t_last_error;
      } catch (const std::exception &e) {  // a host allocation failed: the shard's error, not the worker's end
        rcs[d] = HSV_ERR_ALLOC;
        errs[d] = e.what();
      }
      (void)hsvi_set_inject(prev < 0 ? 0 : prev);
      std::lock_guard<std::mutex> lk(join.mu);
      if (--join.left == 0) join.cv.notify_all();
    });
  }
  std::unique_lock<std::mutex> lk(join.mu);
  join.cv.wait(lk, [&] { return join.left == 0; });
  for (int d = 0; d < k; ++d)
    if (rcs[d] != HSV_OK) return fail(rcs[d], "shard " + std::to_string(d) + ": " + errs[d]);
  return HSV_OK;
}

namespace {

constexpr size_t kPackPart = size_t(1) << 20;  // bytes per part of a split copy

// 32 bytes with streaming (non-temporal) stores; dst 16-byte aligned.  The
// staging is written once and read next by the DMA engine, so a cached store
// only pays a read-for-ownership of a line nobody reads back: one thread packs
// records at 37 GB/s this way against 16 GB/s with memcpy
// (profiles/r03v_pack_probe.txt).  SSE2, baseline x86-64.
// Other hosts: plain copies (the kernels do not depend on this).
#if defined(__SSE2__)
inline void nt_copy32(uint8_t *dst, const uint8_t *src) {
  const __m128i a = _mm_loadu_si128(reinterpret_cast<const __m128i *>(src));
  const __m128i b = _mm_loadu_si128(reinterpret_cast<const __m128i *>(src + 16));
  _mm_stream_si128(reinterpret_cast<__m128i *>(dst), a);
  _mm_stream_si128(reinterpret_cast<__m128i *>(dst + 16), b);
}
inline void nt_fence() { _mm_sfence(); }
#else
inline void nt_copy32(uint8_t *dst, const uint8_t *src) { std::memcpy(dst, src, 32); }
inline void nt_fence() {}
#endif

// items [lo, hi) as records pk | R || s (| digest) at dst + rec * i; dst and
// rec multiples of 16 (pinned staging is page-aligned, rec is 96 or 128)
void pack_records(uint8_t *dst, size_t rec, const uint8_t *pk, size_t pk_stride, const uint8_t *sig,
                  size_t sig_stride, const uint8_t *msg, size_t msg_stride, size_t lo, size_t hi) {
  for (size_t i = lo; i < hi; ++i) {
    uint8_t *r = dst + rec * i;
    nt_copy32(r, pk + i * pk_stride);
    nt_copy32(r + 32, sig + i * sig_stride);
    nt_copy32(r + 64, sig + i * sig_stride + 32);
    if (msg_stride) nt_copy32(r + 96, msg + i * msg_stride);
  }
  nt_fence();  // streaming stores are weakly ordered: visible before the copy is enqueued
}

// bytes from src to dst, with streaming stores for large copies to a
// 16-byte-aligned dst (small ones, e.g. a QC's votes, stay cached)
void nt_copy(uint8_t *dst, const uint8_t *src, size_t bytes) {
  if (bytes < (size_t(64) << 10) || (reinterpret_cast<uintptr_t>(dst) & 15) != 0) {
    std::memcpy(dst, src, bytes);
    return;
  }
  size_t o = 0;
  for (; o + 32 <= bytes; o += 32) nt_copy32(dst + o, src + o);
  nt_fence();
  if (o < bytes) std::memcpy(dst + o, src + o, bytes - o);
}

}  // namespace

void stage_copy(uint8_t *dst, const uint8_t *src, size_t bytes) {
  const int nparts = (int)std::min<size_t>(64, (bytes + kPackPart - 1) / kPackPart);
  if (nparts < 2) {
    nt_copy(dst, src, bytes);
    return;
  }
  pack_pool_current().run(nparts, [&](int p) {
    const size_t lo = bytes * p / nparts & ~size_t(63), hi = p + 1 == nparts ? bytes : bytes * (p + 1) / nparts & ~size_t(63);
    nt_copy(dst + lo, src + lo, hi - lo);
  });
}

// ---- device self-check words ------------------------------------------------------
int check_faults(const uint8_t *words, const char *where) {
  uint32_t w[2];
  std::memcpy(w, words, sizeof(w));
  if (!(w[0] | w[1])) return HSV_OK;
  std::string why;
  if (w[0]) why = "a final point failed the curve self-check";
  if (w[1]) why += std::string(why.empty() ? "" : "; ") + "a workspace canary changed";
  return fail(HSV_ERR_DEVICE_FAULT, std::string(where) + ": device self-check failed (" + why +
                                        "): the flags of this launch are not a verdict");
}

int device_fault_words(DevCtx &c, uint32_t **out) {
  std::lock_guard<std::mutex> lk(c.table_mu);
  if (!c.d_fault) {
    uint32_t *p = nullptr;
    hipError_t e = hipMalloc(&p, 256);
    if (e == hipSuccess) e = hipMemset(p, 0, 256);
    if (e != hipSuccess) {
      if (p) {
        ResidentPause pause;
        (void)hipFree(p);
      }
      return hip_fail("allocating the device self-check words", e);
    }
    c.d_fault = p;
  }
  *out = c.d_fault;
  return HSV_OK;
}

int call_fault_words(DevCtx &c, uint32_t *d_fault, hipStream_t stream, uint32_t **out) {
  if (!d_fault) return device_fault_words(c, out);
  if (reinterpret_cast<uintptr_t>(d_fault) & 3u) return fail(HSV_ERR_ALIGN, "d_fault must be 4-byte aligned");
  const hipError_t e = hipMemsetAsync(d_fault, 0, kFaultBytes, stream);
  if (e != hipSuccess) return hip_fail("zeroing the call's self-check words", e);
  *out = d_fault;
  return HSV_OK;
}

SideStreamLease::SideStreamLease(DevCtx &c) : c_(c) {
  std::lock_guard<std::mutex> lk(c.side_mu);
  if (!c.side_free.empty()) {
    s_ = c.side_free.back();
    c.side_free.pop_back();
    return;
  }
  if (pipe_stream_create(&s_) != hipSuccess) {  // own queue pool, as the slots' streams
    s_ = nullptr;
    return;
  }
  c.side_all.push_back(s_);
}

SideStreamLease::~SideStreamLease() {
  if (!s_) return;
  std::lock_guard<std::mutex> lk(c_.side_mu);
  c_.side_free.push_back(s_);
}

int pointer_device(const void *p) {
  hipPointerAttribute_t attr;
  if (hipPointerGetAttributes(&attr, p) != hipSuccess) {
    (void)hipGetLastError();  // plain host memory: clear the sticky error
    return -1;
  }
  if (attr.type == hipMemoryTypeDevice || attr.type == hipMemoryTypeManaged) return attr.device;
  return -1;
}

int device_for_call(const void *d_ptr, void *stream, int *dev) {
  int d = pointer_device(d_ptr);
  if (d < 0) {
    if (hipGetDevice(&d) != hipSuccess) return fail(HSV_ERR_HIP, "hipGetDevice failed");
  }
  if (d < 0 || d >= device_count_inited()) return fail(HSV_ERR_INVALID_ARG, "device of the input pointers out of range");
  if (stream) {
    int sd = -1;
    if (hipStreamGetDevice(reinterpret_cast<hipStream_t>(stream), &sd) == hipSuccess && sd >= 0 && sd != d)
      return fail(HSV_ERR_INVALID_ARG, "inputs live on device " + std::to_string(d) + " but the stream belongs to device " +
                                           std::to_string(sd));
    (void)hipGetLastError();
  }
  *dev = d;
  return HSV_OK;
}

namespace {

// Records at pk + i*pk_stride etc. (msg_stride 0 = shared), [0, n) on one
// device, chunk by chunk.  Batches of at least 2 * kPipeChunk items run as a
// two-stage pipeline: two staging buffers and two streams, so the host packs
// chunk i+1 and the DMA engine copies it while the kernels verify chunk i.
std::atomic<bool> g_pipe_nocopy{false};  // set only through hsv_test_pipe_nocopy

// 16 MiB of inputs per pipelined chunk (2^17 items): 10.10 ms per 2^20
// against 10.25 for 2^16 and 10.31 for 2^18 (profiles/r03y_host_pipeline_schedules.txt)
constexpr size_t kPipeChunk = size_t(1) << 17;

// The slot's launch workspaces (one per compute stream): the first `count`
// exist and hold at least `need` bytes each; kept across calls, so no launch
// allocates.
int slot_workspaces(Slot &s, size_t need, int count) {
  int have = 0;
  while (have < 3 && s.d_ws[have]) ++have;
  if (need <= s.ws_cap && count <= have) return HSV_OK;
  const size_t cap = std::max(need, s.ws_cap);
  const int n = std::max(count, have);
  std::unique_ptr<ResidentPause> pause;  // hipFree waits for every grid on the device
  if (have) pause.reset(new ResidentPause());
  for (uint8_t *&w : s.d_ws) {
    if (w) (void)hipFree(w);
    w = nullptr;
  }
  s.ws_cap = 0;
  for (int i = 0; i < n; ++i) {
    const hipError_t ea = hipMalloc(&s.d_ws[i], cap);
    if (ea != hipSuccess) return hip_fail("allocating the launch workspaces", ea);
  }
  s.ws_cap = cap;
  return HSV_OK;
}

// Launch chunks of a pipelined call over n items (n >= 2 kPipeChunk).  The
// inputs cross PCIe in pieces of at most kPipeChunk items (57 GB/s: 0.29 ms
// per piece), four times as fast as the kernels verify them (1.1 ms per
// piece), so a launch need not wait for one piece each: every chunk is three
// times all the chunks before it -- 2^16, 3 x 2^16, 12 x 2^16 items for 2^20
// -- and the next chunk's pieces have landed before the previous chunk's
// launch ends.  Three launches instead of one per piece: each launch boundary
// costs a grid end and a prepass the point pass waits for (round 5's
// schedule of nine 2^17-item chunks took 9.85 ms per 2^20 against 8.91 ms for
// one launch alone, BENCH r06a).  Only the first piece (2^16 items, 8 MiB:
// 0.08 ms pack + 0.15 ms copy) is exposed.  hsv_test_pipe_schedule (test
// library) substitutes a schedule for measurement.
constexpr size_t kPipeFirst = size_t(1) << 16;
std::mutex g_pipe_sched_mu;
std::vector<size_t> g_pipe_sched;  // hsv_test_pipe_schedule; empty: the default

std::vector<size_t> pipe_schedule(size_t n) {
  std::vector<size_t> want;
  {
    std::lock_guard<std::mutex> lk(g_pipe_sched_mu);
    want = g_pipe_sched;
  }
  std::vector<size_t> sizes;
  for (size_t done = 0, k = 0; done < n; ++k) {
    size_t w;
    if (!want.empty()) w = want[std::min(k, want.size() - 1)];  // the last size repeats
    else w = done == 0 ? kPipeFirst : 3 * done;
    sizes.push_back(std::min(std::max<size_t>(w, 1), n - done));
    done += sizes.back();
  }
  return sizes;
}

// Stats of the calling thread's last host-buffer call (hsv_host_call_stats,
// a measurement hook): host time spent packing into pinned staging, bytes
// copied host-to-device, and the call's wall time.
thread_local double t_pack_ms = 0, t_call_ms = 0;
thread_local uint64_t t_h2d_bytes = 0;
double ms_since(std::chrono::steady_clock::time_point t0) {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

// Large host batches (n >= 2 kPipeChunk, n <= kChunk): the inputs stream
// to HBM chunk by chunk while earlier chunks verify.
//   * HBM holds the whole batch as records pk | R || s | digest (96 B with a
//     shared digest, staged once), then all flags and the self-check words.
//     A device region is never reused within the call, so a chunk's launch
//     depends only on its own copy -- one copy per chunk, the first chunk
//     half-size;
//   * two pinned staging buffers alternate on the host: chunk k is packed
//     while chunk k-1 copies, and a staging buffer is reused as soon as its
//     copy is done (event), not when its chunk's kernels are;
//   * copies run on the slot's copy stream; launches alternate over two
//     compute streams (a chunk's launch starts in the previous one's grid
//     end), each waiting for its chunk's copy by event, each with a launch
//     workspace the slot keeps (no allocation in the loop);
//   * one copy back of all flags and the self-check words at the end.
// The host's part (pack + enqueue) runs ahead of the GPU; the call costs the
// GPU's time for the chunks plus the first chunk's pack and copy and the copy
// back ("host buffers").
int run_pipelined(Slot &s, int v, const uint32_t *comb_b, const uint8_t *pk, size_t pk_stride, const uint8_t *sig,
                  size_t sig_stride, const uint8_t *msg, size_t msg_stride, size_t n, uint8_t *flags_out) {
  const std::vector<size_t> sizes = pipe_schedule(n);
  const size_t maxm = *std::max_element(sizes.begin(), sizes.end());
  const size_t rec = msg_stride ? 128 : 96;  // record bytes per item (a shared digest is staged once)
  // HBM: records n*rec | shared digest | flags n | self-check words
  const size_t d_dig = round_up(n * rec, kAlign);
  const size_t d_flag = d_dig + kAlign;
  const size_t d_fault = d_flag + round_up(n, kAlign);
  const size_t d_total = d_fault + kAlign;
  // host: two staging buffers of one piece | flags n | self-check words
  const size_t h_stage = round_up(kPipeChunk * rec, kAlign);
  const size_t h_flag = 2 * h_stage;
  const size_t h_fault = h_flag + round_up(n, kAlign);
  const size_t h_total = h_fault + kAlign;
  int rc = slot_prepare(s, d_total, h_total);
  if (rc != HSV_OK) return rc;
  // Launches alternate over two compute streams, so a chunk's memset and
  // prepass can run in the previous chunk's grid end (a third stream measured
  // slower with round 4's schedule: 10.27 against 10.04 ms per 2^20,
  // profiles/r04m_host_streams_ab.txt).
  constexpr int nstreams = 2;
  rc = slot_pipeline(s);
  if (rc != HSV_OK) return rc;
  // one launch workspace per compute stream, kept by the slot: a pool
  // allocation per launch made the enqueue of each chunk wait ~1 ms for an
  // earlier chunk (tools/host_api_probe.py marks)
  rc = slot_workspaces(s, hsv_launch_ws_bytes(v, (uint32_t)maxm), nstreams);
  if (rc != HSV_OK) return rc;
  hipStream_t comp[nstreams] = {s.stream, s.stream2};
  hipEvent_t staged[2] = {s.ev[0], s.ev[1]};
  auto drain = [&](int code) -> int {
    (void)hipStreamSynchronize(s.copy);
    (void)hipStreamSynchronize(s.stream);
    (void)hipStreamSynchronize(s.stream2);
    return code;
  };
  uint8_t *d = s.d_buf;
  // flags and self-check words start at zero (unwritten flags read as
  // rejections); ordered before every launch through the staged events
  hipError_t e = hipMemsetAsync(d + d_flag, 0, d_total - d_flag, s.copy);
  if (e == hipSuccess && msg_stride == 0) e = hipMemcpyAsync(d + d_dig, msg, 32, hipMemcpyHostToDevice, s.copy);
  if (e != hipSuccess) return drain(hip_fail("hipMemsetAsync", e));
  bool used[2] = {false, false};
  // hsv_test_pipe_nocopy (libhsv_test.so only, tools/host_api_ab.py): a call
  // of the same size as the slot's last one skips the pack and the copies and
  // verifies what the last call left in HBM -- the chunk schedule's GPU time
  // alone, for the same inputs called again
  const bool nocopy = g_pipe_nocopy.load(std::memory_order_relaxed) && s.pipe_warm_n == n;
  s.pipe_warm_n = 0;
  t_clock.marks.clear();  // four marks per piece instead of the HSV_MARK_* points
  size_t piece = 0;
  for (size_t base = 0, k = 0, m = 0; k < sizes.size(); base += m, ++k) {
    m = sizes[k];
    int last = 0;  // staging buffer of the chunk's last piece
    // Items as records pk | R || s (| digest), so any item range is one
    // contiguous copy.  The pieces of a chunk go out one by one, each as
    // soon as it is packed; the chunk's launch waits for its last piece
    // (copies run in order on the copy stream).
    for (size_t pb = 0; pb < m; pb += kPipeChunk, ++piece) {
      const size_t pm = std::min(kPipeChunk, m - pb);
      const int b = (int)(piece & 1);
      last = b;
      uint8_t *h = s.h_buf + (size_t)b * h_stage;
      if (used[b]) {  // the copy that last read this staging buffer has finished
        e = hipEventSynchronize(staged[b]);
        if (e != hipSuccess) return drain(hip_fail("hipEventSynchronize", e));
      }
      call_chunk_mark();
      const size_t ib = base + pb;  // first item of the piece
      if (!nocopy) {
        const auto t_pack = std::chrono::steady_clock::now();
        const int nparts = (int)std::min<size_t>(64, (pm * rec + kPackPart - 1) / kPackPart);
        auto part = [&](int p) {
          const size_t lo = pm * p / nparts, hi = pm * (p + 1) / nparts;
          pack_records(h, rec, pk + ib * pk_stride, pk_stride, sig + ib * sig_stride, sig_stride,
                       msg + ib * msg_stride, msg_stride, lo, hi);
        };
        if (nparts < 2) part(0);
        else pack_pool_current().run(nparts, part);
        t_pack_ms += ms_since(t_pack);
        call_chunk_mark();
        e = hipMemcpyAsync(d + ib * rec, h, pm * rec, hipMemcpyHostToDevice, s.copy);
        if (e != hipSuccess) return drain(hip_fail("hipMemcpyAsync H2D", e));
        t_h2d_bytes += pm * rec;
      } else {
        call_chunk_mark();
      }
      e = hipEventRecord(staged[b], s.copy);
      if (e != hipSuccess) return drain(hip_fail("staging a piece", e));
      used[b] = true;
      call_chunk_mark();
      if (pb + pm < m) call_chunk_mark();  // not the chunk's last piece: no launch behind it
    }
    const int cs = (int)(k % (size_t)nstreams);  // this chunk's compute stream and workspace
    uint8_t *dc = d + base * rec;                // chunk k's records in HBM
    e = hipStreamWaitEvent(comp[cs], staged[last], 0);
    if (e != hipSuccess) return drain(hip_fail("staging a chunk", e));
    e = hsv_launch_verify_ws(v, dc, rec, dc + 32, rec, msg_stride ? dc + 96 : d + d_dig, msg_stride ? rec : 0,
                             (uint32_t)m, d + d_flag + base, nullptr, comb_b,
                             reinterpret_cast<uint32_t *>(d + d_fault), s.d_ws[cs], s.ws_cap, comp[cs]);
    if (e != hipSuccess) return drain(hip_fail("verify kernel launch", e));
    call_chunk_mark();
  }
  // join: the flags come back once every compute stream is done
  for (int j = 1; j < nstreams && e == hipSuccess; ++j) {
    e = hipEventRecord(s.ev[2 + j], comp[j]);
    if (e == hipSuccess) e = hipStreamWaitEvent(s.stream, s.ev[2 + j], 0);
  }
  if (e == hipSuccess)
    e = hipMemcpyAsync(s.h_buf + h_flag, d + d_flag, d_total - d_flag, hipMemcpyDeviceToHost, s.stream);
  if (e != hipSuccess) return drain(hip_fail("hipMemcpyAsync D2H", e));
  e = hipStreamSynchronize(s.stream);
  if (e != hipSuccess) return drain(hip_fail("hipStreamSynchronize", e));
  const int frc = check_faults(s.h_buf + h_fault, "verify");
  if (frc != HSV_OK) return drain(frc);
  std::memcpy(flags_out, s.h_buf + h_flag, n);
  s.pipe_warm_n = n;
  return HSV_OK;
}

int run_on_device(DevCtx &c, const uint8_t *pk, size_t pk_stride, const uint8_t *sig, size_t sig_stride,
                  const uint8_t *msg, size_t msg_stride, size_t n, uint8_t *flags_out) {
  const auto t_call = std::chrono::steady_clock::now();
  t_pack_ms = 0;
  t_h2d_bytes = 0;
  DeviceGuard guard(c.device);
  if (guard.status() != hipSuccess) return hip_fail("hipSetDevice", guard.status());
  const int v = variant();
  const uint32_t *comb_b = nullptr;
  int rc = comb_table_for(c, v, &comb_b);
  if (rc != HSV_OK) return rc;
  SlotLease lease(c);
  Slot &s = lease.slot();
  call_mark(HSV_MARK_SLOT);
  if (n >= 2 * kPipeChunk) {  // the copy pipeline (HBM holds the whole batch)
    for (size_t base = 0; base < n; base += kChunk) {
      const size_t m = std::min(kChunk, n - base);
      rc = run_pipelined(s, v, comb_b, pk + base * pk_stride, pk_stride, sig + base * sig_stride, sig_stride,
                         msg + base * msg_stride, msg_stride, m, flags_out + base);
      if (rc != HSV_OK) return rc;
    }
    t_call_ms = ms_since(t_call);
    return HSV_OK;
  }
  // below the pipeline's size: one staging buffer,
  // chunk by chunk -- pk 32 | sig 64 | msg 32 (or one shared digest) | flags 1
  // | self-check words (kFaultBytes); the same layout in HBM
  const size_t chunk = std::min(n, kChunk);
  const size_t pk_off = 0;
  const size_t sig_off = round_up(chunk * 32, kAlign);
  const size_t msg_off = sig_off + round_up(chunk * 64, kAlign);
  const size_t msg_bytes = msg_stride ? chunk * 32 : 32;
  const size_t flag_off = msg_off + round_up(msg_bytes, kAlign);
  const size_t fault_off = flag_off + round_up(chunk, kAlign);
  const size_t total = fault_off + kAlign;
  rc = slot_prepare(s, total, total);
  if (rc != HSV_OK) return rc;
  uint8_t *h = s.h_buf, *d = s.d_buf;
  hipStream_t st = s.stream;
  for (size_t base = 0; base < n; base += chunk) {
    const size_t m = std::min(chunk, n - base);
    const auto t_pack = std::chrono::steady_clock::now();
    const int nparts = (int)std::min<size_t>(64, (m * 128 + kPackPart - 1) / kPackPart);
    auto part = [&](int p) {
      const size_t lo = m * p / nparts, hi = m * (p + 1) / nparts;
      // streaming stores (stage_copy, hsv_host.h): the kernels or the DMA
      // engine read these lines next, from DRAM rather than from this core's
      // cache; each part fences its own stores
      if (pk_stride == 32) stage_copy(h + pk_off + 32 * lo, pk + (base + lo) * 32, (hi - lo) * 32);
      else for (size_t i = lo; i < hi; ++i) stage_copy(h + pk_off + 32 * i, pk + (base + i) * pk_stride, 32);
      if (sig_stride == 64) stage_copy(h + sig_off + 64 * lo, sig + (base + lo) * 64, (hi - lo) * 64);
      else for (size_t i = lo; i < hi; ++i) stage_copy(h + sig_off + 64 * i, sig + (base + i) * sig_stride, 64);
      if (msg_stride == 32) stage_copy(h + msg_off + 32 * lo, msg + (base + lo) * 32, (hi - lo) * 32);
      else if (msg_stride != 0)
        for (size_t i = lo; i < hi; ++i) stage_copy(h + msg_off + 32 * i, msg + (base + i) * msg_stride, 32);
      stage_fence();
    };
    if (nparts < 2) part(0);
    else pack_pool(c.device).run(nparts, part);
    if (msg_stride == 0) std::memcpy(h + msg_off, msg, 32);
    // a flag the kernels failed to write reads as a rejection, never as an
    // earlier call's verdict; the self-check words start at zero
    std::memset(h + flag_off, 0, m);
    std::memset(h + fault_off, 0, kFaultBytes);
    t_pack_ms += ms_since(t_pack);
    call_mark(HSV_MARK_STAGED);
    hipError_t e;
    void *hd = nullptr;
    if (n <= kZeroCopyMax && (hd = s.h_buf_dev) != nullptr) {
      // small batches (a QC of non-cached keys, a single vote): the kernels read
      // the pinned staging buffer and write the flags through its device
      // mapping, so no copy launches sit on the latency path
      uint8_t *dh = static_cast<uint8_t *>(hd);
      // the launch workspace the slot keeps: no pool allocation on the latency path
      rc = slot_workspaces(s, hsv_launch_ws_bytes(v, (uint32_t)m), 1);
      if (rc != HSV_OK) return rc;
      e = hsv_launch_verify_ws(v, dh + pk_off, 32, dh + sig_off, 64, dh + msg_off, msg_stride ? 32 : 0, (uint32_t)m,
                               dh + flag_off, nullptr, comb_b, reinterpret_cast<uint32_t *>(dh + fault_off), s.d_ws[0],
                               s.ws_cap, st);
    } else {
      // inputs, the zeroed flags and the zeroed self-check words in one copy
      const size_t in_bytes = fault_off + kFaultBytes;
      e = hipMemcpyAsync(d, h, in_bytes, hipMemcpyHostToDevice, st);
      t_h2d_bytes += in_bytes;
      if (e == hipSuccess)
        e = hsv_launch_verify(v, d + pk_off, 32, d + sig_off, 64, d + msg_off, msg_stride ? 32 : 0, (uint32_t)m,
                              d + flag_off, nullptr, comb_b, reinterpret_cast<uint32_t *>(d + fault_off), st);
      if (e == hipSuccess)
        e = hipMemcpyAsync(h + flag_off, d + flag_off, fault_off + kFaultBytes - flag_off, hipMemcpyDeviceToHost,
                           st);
    }
    call_mark(HSV_MARK_LAUNCH);
    const hipError_t es = hipStreamSynchronize(st);  // nothing of this call stays in flight
    call_mark(HSV_MARK_SYNC);
    if (e != hipSuccess) return hip_fail("verify launch", e);
    if (es != hipSuccess) return hip_fail("hipStreamSynchronize", es);
    rc = check_faults(h + fault_off, "verify");
    if (rc != HSV_OK) return rc;
    std::memcpy(flags_out + base, h + flag_off, m);
    call_mark(HSV_MARK_DONE);
  }
  t_call_ms = ms_since(t_call);
  return HSV_OK;
}

}  // namespace

int run_host(const uint8_t *pk, size_t pk_stride, const uint8_t *sig, size_t sig_stride, const uint8_t *msg,
             size_t msg_stride, size_t n, uint8_t *flags_out) {
  if (n == 0) return HSV_OK;
  if (!pk || !sig || !msg || !flags_out) return fail(HSV_ERR_INVALID_ARG, "null pointer");
  int rc = ensure_init();
  if (rc != HSV_OK) return rc;
  const int k = shard_count(n);
  if (k <= 1) return run_on_device(ctx(home_device()), pk, pk_stride, sig, sig_stride, msg, msg_stride, n, flags_out);
  // contiguous shards, each on the shard worker of its GPU's node
  return run_sharded(k, [&](int d, int dev) {
    const size_t lo = n * d / k, hi = n * (d + 1) / k;
    if (hi <= lo) return HSV_OK;
    return run_on_device(ctx(dev), pk + lo * pk_stride, pk_stride, sig + lo * sig_stride, sig_stride,
                         msg + lo * msg_stride, msg_stride, hi - lo, flags_out + lo);
  });
}

int batch_verdict(const uint8_t *flags, size_t n) {
  for (size_t i = 0; i < n; ++i)
    if ((flags[i] & (HSV_PARSE_OK | HSV_EQ_OK)) != (HSV_PARSE_OK | HSV_EQ_OK)) return 0;
  return 1;
}

}  // namespace hsvh

using namespace hsvh;

extern "C" {

int hsv_init(int device) {
  int rc = ensure_init();
  if (rc != HSV_OK) return rc;
  Global &g = G();
  if (device >= g.ndev || device < -1) return fail(HSV_ERR_INVALID_ARG, "device index out of range");
  g.bound = device;
  return device < 0 ? g.ndev : 1;
}

int hsv_bound_device(void) {
  if (ensure_init() != HSV_OK) return HSV_ERR_NO_DEVICE;
  const int b = G().bound.load();
  return b == kUnbound ? -1 : b;
}

// Test hook (exported by libhsv_test.so only): split host batches of >= 2^16
// items into k contiguous shards, each on its own host thread and slot, mapped
// onto the bound device (or round-robin over the visible devices); k = 0
// restores the default.  Lets the multi-device gather path run on a one-GPU box.
int hsvi_set_virtual_shards(int k) {
  if (k < 0 || k > 64) return fail(HSV_ERR_INVALID_ARG, "virtual shards must be in [0, 64]");
  (void)ensure_init();
  G().virtual_shards = k;
  return HSV_OK;
}

int hsvi_set_pipe_nocopy(int on) { return hsvh::g_pipe_nocopy.exchange(on != 0) ? 1 : 0; }

int hsvi_set_pipe_schedule(const uint64_t *sizes, int count) {
  if (count < 0 || count > 64 || (count > 0 && !sizes)) return fail(HSV_ERR_INVALID_ARG, "schedule of 0..64 sizes");
  std::lock_guard<std::mutex> lk(hsvh::g_pipe_sched_mu);
  hsvh::g_pipe_sched.assign(sizes, sizes + count);
  return HSV_OK;
}

// Lifecycle call: must not run concurrently with verify calls (hsv.h).  It
// still quiesces first -- every slot locked and drained, every side stream
// drained, the device idle -- before it frees the tables those calls read.
void hsv_shutdown(void) {
  auto_committee_shutdown();
  ResidentPause pause;  // no relaunch while the buffers go
  Global &g = G();
  std::lock_guard<std::mutex> lk(g.mu);
  for (DevCtx *c : g.ctx) {
    DeviceGuard guard(c->device);
    std::vector<std::unique_lock<std::mutex>> held;
    for (auto &sp : c->slots) held.emplace_back(sp->mu);
    std::lock_guard<std::mutex> ls(c->side_mu);
    for (auto &sp : c->slots) {
      if (sp->stream) (void)hipStreamSynchronize(sp->stream);
      if (sp->stream2) (void)hipStreamSynchronize(sp->stream2);
      if (sp->copy) (void)hipStreamSynchronize(sp->copy);
    }
    for (hipStream_t st : c->side_all) (void)hipStreamSynchronize(st);
    (void)hipDeviceSynchronize();
    {
      std::lock_guard<std::mutex> lt(c->table_mu);
      if (c->d_btable) (void)hipFree(c->d_btable);
      if (c->d_btable16) (void)hipFree(c->d_btable16);
      if (c->d_fault) (void)hipFree(c->d_fault);
      c->d_btable = nullptr;
      c->d_btable16 = nullptr;
      c->d_fault = nullptr;
    }
    for (auto &sp : c->slots) {
      Slot &s = *sp;
      if (s.stream) (void)hipStreamDestroy(s.stream);
      if (s.stream2) (void)hipStreamDestroy(s.stream2);
      if (s.copy) (void)hipStreamDestroy(s.copy);
      for (hipEvent_t &ev : s.ev) {
        if (ev) (void)hipEventDestroy(ev);
        ev = nullptr;
      }
      s.copy = nullptr;
      for (uint8_t *&w : s.d_ws) {
        if (w) (void)hipFree(w);
        w = nullptr;
      }
      s.ws_cap = 0;
      if (s.d_buf) (void)hipFree(s.d_buf);
      if (s.h_buf) (void)hipHostFree(s.h_buf);
      if (s.h_sync) (void)hipHostFree(s.h_sync);
      s.h_sync = s.h_sync_dev = nullptr;
      s.h_sync_cap = 0;
      s.stream = s.stream2 = nullptr;
      s.d_buf = s.h_buf = s.h_buf_dev = nullptr;
      s.d_cap = s.h_cap = 0;
    }
    for (hipStream_t st : c->side_all) (void)hipStreamDestroy(st);
    c->side_all.clear();
    c->side_free.clear();
  }
  hsv_ws_trim();
}

int hsv_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) {
    (void)hipGetLastError();
    return 0;
  }
  return n;
}

const char *hsv_last_error(void) { return t_last_error.c_str(); }

const char *hsv_version(void) { return "hsv 0.3.0 (gfx950)"; }

int hsv_abi_version(void) { return HSV_ABI_VERSION; }

// Measurement/test hook (exported by libhsv_test.so only): pick the kernel variant.
int hsvi_set_variant(int v) {
  if (!hsvi_variant_available(v)) return fail(HSV_ERR_INVALID_ARG, "variant not built into this library");
  G().variant = v;
  return HSV_OK;
}

int hsv_get_variant(void) { return G().variant.load(); }

int hsv_verify(const uint8_t *pk, const uint8_t *sig, const uint8_t *msg, size_t msg_stride, size_t n,
               uint8_t *flags_out) {
  CallScope call;
  if (msg_stride != 0 && msg_stride != 32) return fail(HSV_ERR_INVALID_ARG, "msg_stride must be 0 or 32");
  if (n && pk && sig && msg && flags_out) {
    const int rc = auto_committee_try(pk, sig, msg, msg_stride, n, flags_out);
    if (rc != 1) return rc;  // handled (HSV_OK) or an error
  }
  return run_host(pk, 32, sig, 64, msg, msg_stride, n, flags_out);
}

int hsv_verify_strict(const uint8_t digest[32], const uint8_t pk[32], const uint8_t sig[64]) {
  uint8_t f = 0;
  int rc = hsv_verify(pk, sig, digest, 0, 1, &f);
  if (rc != HSV_OK) return rc;
  return (f & HSV_STRICT_OK) ? 1 : 0;
}

int hsv_verify_batch(const uint8_t digest[32], const uint8_t *pk, const uint8_t *sig, size_t n) {
  CallScope call;
  if (n == 0) return 1;  // dalek verify_batch over zero items is Ok
  if (!digest || !pk || !sig) return fail(HSV_ERR_INVALID_ARG, "null argument");
  std::vector<uint8_t> packed(n * 96);
  for (size_t i = 0; i < n; ++i) {
    std::memcpy(packed.data() + 96 * i, pk + 32 * i, 32);
    std::memcpy(packed.data() + 96 * i + 32, sig + 64 * i, 64);
  }
  return hsv_verify_batch_packed(digest, packed.data(), n);
}

int hsv_verify_device_bits(const uint8_t *d_pk, size_t pk_stride, const uint8_t *d_sig, size_t sig_stride,
                           const uint8_t *d_msg, size_t msg_stride, size_t n, uint8_t *d_flags,
                           uint32_t *d_strict_bits, uint32_t *d_fault, void *stream) {
  if (n == 0) return HSV_OK;
  if (!d_pk || !d_sig || !d_msg) return fail(HSV_ERR_INVALID_ARG, "null input pointer");
  if (!d_flags && !d_strict_bits) return fail(HSV_ERR_INVALID_ARG, "no output");
  const uintptr_t mis = (reinterpret_cast<uintptr_t>(d_pk) | reinterpret_cast<uintptr_t>(d_sig) |
                         reinterpret_cast<uintptr_t>(d_msg) | pk_stride | sig_stride | msg_stride) & 15u;
  if (mis) return fail(HSV_ERR_ALIGN, "device pointers and strides must be multiples of 16");
  if (pk_stride < 32 || sig_stride < 64 || (msg_stride != 0 && msg_stride < 32))
    return fail(HSV_ERR_INVALID_ARG, "record strides overlap");
  int rc = ensure_init();
  if (rc != HSV_OK) return rc;
  int dev = 0;
  rc = device_for_call(d_pk, stream, &dev);
  if (rc != HSV_OK) return rc;
  DeviceGuard guard(dev);
  if (guard.status() != hipSuccess) return hip_fail("hipSetDevice", guard.status());
  const int v = variant();
  const uint32_t *comb_b = nullptr;
  DevCtx &c = ctx(dev);
  rc = comb_table_for(c, v, &comb_b);
  if (rc != HSV_OK) return rc;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  uint32_t *fault = nullptr;
  rc = call_fault_words(c, d_fault, s, &fault);
  if (rc != HSV_OK) return rc;
  // Batches of several kChunk launches alternate them over the caller's stream
  // and a second library stream leased for this call (fork/join through
  // events on the caller's stream): a chunk's launch starts on the SIMDs the
  // previous chunk's point pass leaves idle at its grid end.  Chunks write
  // disjoint outputs (kChunk is a multiple of 32, so no strict-bits word is
  // shared).
  hipStream_t s2 = s;
  hipEvent_t fork = nullptr, join = nullptr;
  std::unique_ptr<SideStreamLease> side;
  if (n > kChunk) {
    side.reset(new SideStreamLease(c));
    if (side->stream() && hipEventCreateWithFlags(&fork, hipEventDisableTiming) == hipSuccess &&
        hipEventCreateWithFlags(&join, hipEventDisableTiming) == hipSuccess &&
        hipEventRecord(fork, s) == hipSuccess && hipStreamWaitEvent(side->stream(), fork, 0) == hipSuccess)
      s2 = side->stream();
  }
  hipError_t e = hipSuccess;
  size_t k = 0;
  for (size_t base = 0; base < n && e == hipSuccess; base += kChunk, ++k) {
    const size_t m = std::min(kChunk, n - base);
    e = hsv_launch_verify(v, d_pk + base * pk_stride, pk_stride, d_sig + base * sig_stride, sig_stride,
                          d_msg + base * msg_stride, msg_stride, (uint32_t)m, d_flags ? d_flags + base : nullptr,
                          d_strict_bits ? d_strict_bits + base / 32 : nullptr, comb_b, fault, (k & 1) ? s2 : s);
  }
  if (s2 != s) {  // join: the caller's stream waits for the side stream's chunks
    hipError_t ej = hipEventRecord(join, s2);
    if (ej == hipSuccess) ej = hipStreamWaitEvent(s, join, 0);
    if (e == hipSuccess) e = ej;
  }
  if (fork) (void)hipEventDestroy(fork);
  if (join) (void)hipEventDestroy(join);
  return e == hipSuccess ? HSV_OK : hip_fail("verify kernel launch", e);
}

int hsv_verify_device(const uint8_t *d_pk, size_t pk_stride, const uint8_t *d_sig, size_t sig_stride,
                      const uint8_t *d_msg, size_t msg_stride, size_t n, uint8_t *d_flags, void *stream) {
  if (!d_flags && n) return fail(HSV_ERR_INVALID_ARG, "null d_flags");
  return hsv_verify_device_bits(d_pk, pk_stride, d_sig, sig_stride, d_msg, msg_stride, n, d_flags, nullptr, nullptr,
                                stream);
}

int hsv_device_faults(int device, int clear) {
  int rc = ensure_init();
  if (rc != HSV_OK) return rc;
  const int nd = device_count_inited();
  if (device < -1 || device >= nd) return fail(HSV_ERR_INVALID_ARG, "device index out of range");
  int bits = 0;
  for (int d = device < 0 ? 0 : device; d < (device < 0 ? nd : device + 1); ++d) {
    DevCtx &c = ctx(d);
    uint32_t *words = nullptr;
    {
      std::lock_guard<std::mutex> lk(c.table_mu);
      words = c.d_fault;
    }
    if (!words) continue;  // no device-resident call has run there
    DeviceGuard guard(d);
    if (guard.status() != hipSuccess) return hip_fail("hipSetDevice", guard.status());
    uint32_t w[2] = {0, 0};
    hipError_t e;
    if (clear) {
      // one atomic exchange per word on the device: a fault that a launch on
      // another stream records concurrently is either in `w` or stays in the
      // word for the next read -- never cleared unseen (a copy followed by a
      // memset could lose it).  Readers of one device take turns on the
      // exchange's output words.
      std::lock_guard<std::mutex> lk(c.fault_mu);
      SideStreamLease side(c);
      if (!side.stream()) return fail(HSV_ERR_HIP, "no stream for the fault-word exchange");
      e = hsv_launch_fault_exchange(words, words + kFaultOutWord, side.stream());
      if (e == hipSuccess) e = hipMemcpyAsync(w, words + kFaultOutWord, sizeof(w), hipMemcpyDeviceToHost, side.stream());
      if (e == hipSuccess) e = hipStreamSynchronize(side.stream());
    } else {
      e = hipMemcpy(w, words, sizeof(w), hipMemcpyDeviceToHost);
    }
    if (e != hipSuccess) return hip_fail("reading the device self-check words", e);
    bits |= (w[0] ? 1 : 0) | (w[1] ? 2 : 0);
  }
  return bits;
}

// The calling thread's last host-buffer verification (hsv.h): host
// milliseconds spent packing into pinned staging, bytes copied host-to-device,
// and the call's wall milliseconds.
void hsv_host_call_stats(double *pack_ms, double *h2d_bytes, double *call_ms) {
  if (pack_ms) *pack_ms = t_pack_ms;
  if (h2d_bytes) *h2d_bytes = (double)t_h2d_bytes;
  if (call_ms) *call_ms = t_call_ms;
}

int hsv_pack_threads(void) {
  const int d = ensure_init() == HSV_OK ? home_device() : -1;
  return pack_pool(d).threads();
}

// The host timeline of the calling thread's last call (hsv.h HSV_MARK_*, or
// four marks per chunk of a pipelined call); returns the count.
int hsv_host_call_marks(double *out, int cap) {
  const std::vector<double> &m = t_clock.marks;
  const int n = (int)m.size();
  for (int i = 0; out && i < n && i < cap; ++i) out[i] = m[i];
  return n;
}

double hsv_measure_mad_peak(void) {
  if (ensure_init() != HSV_OK) return -1.0;
  const int dev = home_device();
  DeviceGuard guard(dev);
  if (guard.status() != hipSuccess) return -1.0;
  return hsv_launch_mad_peak(ctx(dev).cus);
}

int hsvi_set_error(int code, const char *msg) { return fail(code, msg ? msg : ""); }

}  // extern "C"
