// Committee key cache behind the C ABI:
//   * hsv_committee_*: an explicit committee (tables for a given key list);
//   * the automatic cache behind hsv_verify_batch[_packed] / small strict
//     batches, which learns the recurring consensus keys by itself.
//
// Both hand the committee kernels (hsv_committee.hip) a device array of
// per-key table pointers, so the automatic cache grows by appending 64-key
// table blocks: existing tables never move, a build for new keys never copies
// the old ones, and peak table memory is one copy of the cache.
#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <array>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <random>
#include <string>
#include <thread>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "hsv.h"
#include "hsv_host.h"
#include "hsv_internal.h"

namespace hsvh {
namespace {

// ---- key index -----------------------------------------------------------------
using Key32 = std::array<uint8_t, 32>;

Key32 key_of(const uint8_t *p) {
  Key32 k;
  std::memcpy(k.data(), p, 32);
  return k;
}

// Keys are attacker-chosen bytes (they arrive in certificates from the
// network), so the hash is keyed with a per-process random seed.
struct KeyHash {
  static uint64_t seed() {
    static const uint64_t s = [] {
      std::random_device rd;
      return ((uint64_t)rd() << 32) ^ rd() ^ 0x9e3779b97f4a7c15ull;
    }();
    return s;
  }
  size_t operator()(const Key32 &k) const {
    uint64_t h = seed();
    for (int i = 0; i < 4; ++i) {
      uint64_t w;
      std::memcpy(&w, k.data() + 8 * i, 8);
      h = (h ^ w) * 0xbf58476d1ce4e5b9ull;
      h ^= h >> 31;
    }
    return (size_t)h;
  }
};

// Member index by key, on the QC hot path (a C3 QC looks up 667 keys): an
// open-addressing table, load <= 1/2, linear probing, the keys kept
// contiguously.  A probe compares the key's first 8 bytes from the slot's tag
// before the full 32; no node chasing as in std::unordered_map (3.2 us per
// C3 lookup on the GPU box's host with it).  Copyable, so a new cache view
// starts from its base's index.
class KeyIndex {
 public:
  // the member index of pk, or -1
  int64_t find(const uint8_t *pk) const {
    if (count_ == 0) return -1;
    uint64_t w0;
    std::memcpy(&w0, pk, 8);
    for (size_t h = slot_of(pk);; h = (h + 1) & mask_) {
      const uint32_t e = slot_[h];
      if (e == 0) return -1;
      if (tag_[h] == w0 && std::memcmp(keys_.data() + (size_t)(e - 1) * 32, pk, 32) == 0) return val_[e - 1];
    }
  }
  // first insertion of a key wins (as unordered_map::emplace)
  void emplace(const Key32 &k, uint32_t v) {
    if (find(k.data()) >= 0) return;
    if (2 * (count_ + 1) > slot_.size()) grow();
    keys_.insert(keys_.end(), k.begin(), k.end());
    val_.push_back(v);
    ++count_;
    place(count_ - 1);
  }
  size_t size() const { return count_; }

 private:
  size_t slot_of(const uint8_t *pk) const {
    Key32 k;
    std::memcpy(k.data(), pk, 32);
    return KeyHash()(k) & mask_;
  }
  void place(size_t e) {
    const uint8_t *pk = keys_.data() + e * 32;
    size_t h = slot_of(pk);
    while (slot_[h] != 0) h = (h + 1) & mask_;
    slot_[h] = (uint32_t)e + 1;
    std::memcpy(&tag_[h], pk, 8);
  }
  void grow() {
    const size_t cap = std::max<size_t>(64, slot_.size() * 2);
    slot_.assign(cap, 0u);
    tag_.assign(cap, 0u);
    mask_ = cap - 1;
    for (size_t e = 0; e < count_; ++e) place(e);
  }
  std::vector<uint8_t> keys_;   // count_ * 32, in insertion order
  std::vector<uint32_t> val_;   // member index of each key
  std::vector<uint32_t> slot_;  // 1 + position in keys_, 0 = empty
  std::vector<uint64_t> tag_;   // first 8 bytes of the slot's key
  size_t mask_ = 0, count_ = 0;
};

// ---- committee tables on one device ----------------------------------------------
struct CommitteeDev {
  int device = 0;
  uint32_t n = 0;
  const uint8_t *h_pks = nullptr;  // host copy of the n key encodings, by member index
  const uint8_t *d_pks = nullptr;
  const uint8_t *d_kflags = nullptr;
  const uint32_t *const *d_tabptr = nullptr;
};

// ---- resident latency service (on by default; HSV_QC_RESIDENT=0 turns it off) ------
// One block of hsv_comb_resident_kernel stays on a CU of the home device and
// answers requests of at most hsv_comb_resident_votes() votes posted in
// coherent pinned memory (QcResidentReq): 2.2 us round trip for a block of its
// shape against 5.8 us for a launch with marker sync
// (profiles/r05a_aql_latency.txt), so one verify_strict of a cached key costs
// 0.034 ms instead of 0.039 ms launched (0.037 ms for the dalek port on one
// host core).  It holds that one CU while it runs.  The kernel leaves on the
// stop word -- hsv_shutdown, hsv_set_resident_service(0), an atexit handler,
// and every ResidentPause: the library pauses the service around each of its
// own hipFree / hipHostFree (on ROCm they wait for every grid on the device)
// and before each launch of the persistent point pass, whose grid is sized to
// fill every CU -- or after the idle time (HSV_QC_RESIDENT_IDLE_MS, default
// 50 ms) without a request; the next request relaunches it.  A request
// unanswered within kResidentWait, or a relaunch that does not start, takes
// the call to the launch path and keeps the service off for a backoff, so the
// service can cost latency but never a verdict.  An application that
// synchronises the whole device (hipDeviceSynchronize, torch.cuda.synchronize)
// waits at most the idle time after the last request.
constexpr auto kResidentWait = std::chrono::milliseconds(50);
constexpr int kResidentUnavailable = 1;
constexpr int kResidentMaxFailures = 4;  // then the service stays off for the process

struct ResidentQc {
  std::mutex mu;
  int device = -1;
  QcResidentReq *h = nullptr;  // coherent pinned
  QcResidentReq *d = nullptr;  // its device address
  hipStream_t stream = nullptr;
  uint32_t seq = 0;
  int failures = 0;                                   // relaunch / answer failures so far
  std::chrono::steady_clock::time_point retry_after;  // backoff after a failure
  int paused = 0;   // live ResidentPause scopes: no request, no relaunch
  // 1 on, 0 off (hsv_set_resident_service); -1: HSV_QC_RESIDENT on first use.
  // Read without the lock: a call that finds it on and the lock busy launches.
  std::atomic<int> mode{-1};
  bool atexit_registered = false;
  std::atomic<bool> started{false};   // its block has run in this process (hsvi_resident_started)
  uint64_t posted = 0, answered = 0;  // requests posted / answered (hsvi_resident_counts)
};

ResidentQc &RQ() {
  static ResidentQc r;
  return r;
}

bool resident_on(ResidentQc &r) {
  int m = r.mode.load(std::memory_order_relaxed);
  if (m < 0) {
    const char *v = std::getenv("HSV_QC_RESIDENT");
    int want = (v && v[0] == '0') ? 0 : 1;
    r.mode.compare_exchange_strong(m, want);  // a concurrent hsv_set_resident_service wins
    m = r.mode.load(std::memory_order_relaxed);
  }
  return m == 1;
}

uint64_t resident_idle_ticks() {
  static const uint64_t t = [] {
    long ms = 50;
    if (const char *v = std::getenv("HSV_QC_RESIDENT_IDLE_MS")) ms = std::atol(v);
    ms = std::max(1L, std::min(ms, 10000L));
    return (uint64_t)ms * 100000ull;  // the kernel's 100 MHz clock
  }();
  return t;
}

// stop the kernel and wait for its grid (mu held)
void resident_stop_locked(ResidentQc &r) {
  if (!r.h || !r.stream) return;
  __atomic_store_n(&r.h->stop, 1u, __ATOMIC_RELEASE);
  DeviceGuard guard(r.device);
  (void)hipStreamSynchronize(r.stream);
  __atomic_store_n(&r.h->stop, 0u, __ATOMIC_RELEASE);
}

// a failed relaunch or an unanswered request (mu held): off for a growing
// backoff, for good after kResidentMaxFailures
void resident_failed_locked(ResidentQc &r) {
  ++r.failures;
  r.retry_after = std::chrono::steady_clock::now() + std::chrono::milliseconds(250 << std::min(r.failures, 6));
}

void resident_atexit() {
  ResidentQc &r = RQ();
  std::lock_guard<std::mutex> lk(r.mu);
  resident_stop_locked(r);
}

// the kernel running on `device` (mu held): HSV_OK or kResidentUnavailable
int resident_ensure_locked(ResidentQc &r, int device) {
  if (r.paused || !resident_on(r) || r.failures >= kResidentMaxFailures) return kResidentUnavailable;
  if (r.failures && std::chrono::steady_clock::now() < r.retry_after) return kResidentUnavailable;
  if (r.h && r.device != device) return kResidentUnavailable;  // one device per process
  if (!r.h) {
    void *h = nullptr, *d = nullptr;
    // coherent pinned memory: the running kernel reads what the host writes
    // after it started (a non-coherent area let it read a stale request
    // header and fault, profiles/r04res_pytest_sub2.txt)
    if (hipHostMalloc(&h, sizeof(QcResidentReq), hipHostMallocCoherent) != hipSuccess) {
      r.failures = kResidentMaxFailures;
      return kResidentUnavailable;
    }
    if (hipHostGetDevicePointer(&d, h, 0) != hipSuccess || !d ||
        hipStreamCreateWithFlags(&r.stream, hipStreamNonBlocking) != hipSuccess) {
      (void)hipHostFree(h);  // the kernel never ran: nothing to wait for
      r.failures = kResidentMaxFailures;
      return kResidentUnavailable;
    }
    std::memset(h, 0, sizeof(QcResidentReq));
    r.h = static_cast<QcResidentReq *>(h);
    r.d = static_cast<QcResidentReq *>(d);
    r.device = device;
    r.seq = 0;
  }
  if (__atomic_load_n(&r.h->alive, __ATOMIC_ACQUIRE) == 1u) return HSV_OK;
  // not running (first use, or it left after its idle time): relaunch
  (void)hipStreamSynchronize(r.stream);  // the previous grid has fully ended
  __atomic_store_n(&r.h->stop, 0u, __ATOMIC_RELEASE);
  if (hsv_launch_comb_resident(r.d, resident_idle_ticks(), r.stream) != hipSuccess) {
    resident_failed_locked(r);
    return kResidentUnavailable;
  }
  r.started.store(true);
  if (!r.atexit_registered) {  // after HIP's own: runs before the runtime tears down
    std::atexit(resident_atexit);
    r.atexit_registered = true;
  }
  // The block announces itself once it holds a CU.  A device busy with other
  // grids may not give it one soon: then this call launches instead, the
  // stop word makes the block leave as soon as it starts, and the service
  // backs off.
  const auto t0 = std::chrono::steady_clock::now();
  while (__atomic_load_n(&r.h->alive, __ATOMIC_ACQUIRE) != 1u)
    if (std::chrono::steady_clock::now() - t0 > kResidentWait) {
      resident_stop_locked(r);
      resident_failed_locked(r);
      return kResidentUnavailable;
    }
  return HSV_OK;
}

// One request of at most hsv_comb_resident_votes() votes: HSV_OK, an error
// (HSV_ERR_DEVICE_FAULT from the self-checks or the kernel's request check),
// or kResidentUnavailable (the caller launches instead).
int resident_run(const CommitteeDev &cd, const uint32_t *key_idx, const uint8_t *sig, size_t sig_stride,
                 const uint8_t *msg, size_t msg_stride, size_t m, uint8_t *flags_out, const uint32_t *btable) {
  ResidentQc &r = RQ();
  // one request at a time: a concurrent caller launches instead of queueing
  // behind this one (the launch path takes 0.039 ms, a queue could take more)
  std::unique_lock<std::mutex> lk(r.mu, std::try_to_lock);
  if (!lk.owns_lock()) return kResidentUnavailable;
  if (resident_ensure_locked(r, cd.device) != HSV_OK) return kResidentUnavailable;
  QcResidentReq &q = *r.h;
  QcResidentBody b{};  // the payload, chunked into the request area at each post
  b.m = (uint32_t)m;
  b.nkeys = cd.n;
  b.inject = (uint32_t)hsvi_inject_mode();
  b.msg_per_vote = msg_stride ? 1u : 0u;
  b.pks = cd.d_pks;
  b.key_flags = cd.d_kflags;
  b.key_tables = cd.d_tabptr;
  b.btable = btable;
  const size_t mm = std::min<size_t>(m, kResidentVotes);  // m > kResidentVotes is the kernel's to refuse
  for (size_t i = 0; i < mm; ++i) {
    b.key_idx[i] = key_idx[i];
    if (key_idx[i] < cd.n) std::memcpy(b.pk[i], cd.h_pks + (size_t)key_idx[i] * 32, 32);  // else flag 0
    std::memcpy(b.sig[i], sig + i * sig_stride, 64);
    if (msg_stride) std::memcpy(b.msg[i], msg + i * msg_stride, 32);
  }
  if (!msg_stride) std::memcpy(b.msg[0], msg, 32);
  uint32_t words[kResidentChunks * 3];
  std::memcpy(words, &b, sizeof(b));
  call_mark(HSV_MARK_STAGED);
  // Each chunk {seq, three payload words} in ONE aligned 16-byte store, the
  // width of the kernel's read of it: a read can then never pair a new seq
  // with an older payload word (16-byte aligned SSE stores are single
  // accesses on x86-64 processors with AVX).  The compiler fence keeps the
  // chunks' stores in program order; x86 makes them visible in that order.
  auto post = [&](uint32_t sq) {
    std::atomic_signal_fence(std::memory_order_release);
    for (int c = 0; c < kResidentChunks; ++c) {
      QcResidentChunk *ch = &q.chunk[c];
#if defined(__SSE2__)
      _mm_store_si128(reinterpret_cast<__m128i *>(ch),
                      _mm_set_epi32((int)words[3 * c + 2], (int)words[3 * c + 1], (int)words[3 * c], (int)sq));
#else
      ch->w[0] = words[3 * c];
      ch->w[1] = words[3 * c + 1];
      ch->w[2] = words[3 * c + 2];
      __atomic_store_n(&ch->seq, sq, __ATOMIC_RELEASE);
#endif
    }
    std::atomic_signal_fence(std::memory_order_release);
  };
  // One retry: the kernel may leave on its idle timer just as a request is
  // posted (it read the doorbell before the store); then it is relaunched
  // and the same request posted again under a new number.
  uint64_t a0 = 0, a1 = 0;
  for (int attempt = 0;; ++attempt) {
    const uint32_t sq = ++r.seq == 0 ? ++r.seq : r.seq;  // never 0
    post(sq);
    ++r.posted;
    call_mark(HSV_MARK_LAUNCH);
    const auto t0 = std::chrono::steady_clock::now();
    bool answered = false;
    for (;;) {  // both 8-byte answer words carry this request's seq
      a0 = __atomic_load_n(&q.answer[0], __ATOMIC_ACQUIRE);
      a1 = __atomic_load_n(&q.answer[1], __ATOMIC_ACQUIRE);
      if ((uint32_t)a0 == sq && (uint32_t)a1 == sq) {
        answered = true;
        break;
      }
      if (std::chrono::steady_clock::now() - t0 > kResidentWait) break;
    }
    if (answered) break;
    if (attempt == 0 && __atomic_load_n(&q.alive, __ATOMIC_ACQUIRE) == 0u &&
        resident_ensure_locked(r, cd.device) == HSV_OK)
      continue;
    // no answer from a running kernel: stop it and back off, the launch
    // path answers
    resident_stop_locked(r);
    resident_failed_locked(r);
    return kResidentUnavailable;
  }
  ++r.answered;
  call_mark(HSV_MARK_SYNC);
  const uint32_t fb = (uint32_t)(a1 >> 32), fl = (uint32_t)(a0 >> 32);
  if (fb & kResidentBadRequest)
    return fail(HSV_ERR_DEVICE_FAULT, "committee verify (resident): the kernel refused the request header");
  const uint32_t fw[2] = {fb & kResidentFaultCurve, fb & kResidentFaultCanary};
  const int rc = check_faults(reinterpret_cast<const uint8_t *>(fw), "committee verify (resident)");
  if (rc != HSV_OK) return rc;
  for (size_t i = 0; i < m; ++i) flags_out[i] = (uint8_t)(fl >> (8 * i));
  call_mark(HSV_MARK_DONE);
  return HSV_OK;
}

bool resident_enabled() { return resident_on(RQ()); }

}  // namespace

// A scope in which the resident kernel does not run: the constructor stops it
// (when it runs) and, until the destructor, no request is posted and no
// relaunch happens -- a concurrent small call takes the launch path.  Around
// every hipFree / hipHostFree of the library (they wait for every grid on the
// device, and would otherwise wait for the service's idle exit, or forever
// under steady requests) and before each launch of the persistent point pass.
ResidentPause::ResidentPause() {
  ResidentQc &r = RQ();
  std::lock_guard<std::mutex> lk(r.mu);
  ++r.paused;
  if (r.h && __atomic_load_n(&r.h->alive, __ATOMIC_ACQUIRE) == 1u) resident_stop_locked(r);
}

ResidentPause::~ResidentPause() {
  ResidentQc &r = RQ();
  std::lock_guard<std::mutex> lk(r.mu);
  --r.paused;
}

// Stop the resident kernel now, without keeping it paused (the next request
// relaunches it).  A no-op when it does not run.
void resident_quiesce() { ResidentPause p; }

void resident_counts(uint64_t *posted, uint64_t *answered) {
  ResidentQc &r = RQ();
  std::lock_guard<std::mutex> lk(r.mu);
  if (posted) *posted = r.posted;
  if (answered) *answered = r.answered;
}

// hsv_set_resident_service: 1 on, 0 off (the kernel stops now); the previous mode
int resident_set_mode(int on) {
  ResidentQc &r = RQ();
  std::lock_guard<std::mutex> lk(r.mu);
  const int prev = resident_on(r) ? 1 : 0;
  r.mode.store(on ? 1 : 0);
  if (!on) resident_stop_locked(r);
  if (on) r.failures = 0;  // an explicit re-enable clears the backoff
  return prev;
}

}  // namespace hsvh

extern "C" void hsvi_resident_pause(int on) {
  using namespace hsvh;
  ResidentQc &r = RQ();
  std::lock_guard<std::mutex> lk(r.mu);
  if (on) {
    ++r.paused;
    if (r.h && __atomic_load_n(&r.h->alive, __ATOMIC_ACQUIRE) == 1u) resident_stop_locked(r);
  } else if (r.paused > 0) {
    --r.paused;
  }
}

extern "C" int hsvi_resident_started(void) {
  hsvh::ResidentQc &r = hsvh::RQ();
  return r.started.load() && hsvh::resident_on(r) ? 1 : 0;
}

namespace hsvh {

// Test hook: one resident request whose header claims m votes (0 or above
// the limit: the kernel must refuse it with HSV_ERR_DEVICE_FAULT, never read
// through it); needs the automatic cache's committee (nkeys, tables).
int resident_post_bad(uint32_t m) {
  if (!resident_enabled()) return fail(HSV_ERR_INVALID_ARG, "the resident service is off");
  int rc = ensure_init();
  if (rc != HSV_OK) return rc;
  DevCtx &c = ctx(home_device());
  DeviceGuard guard(c.device);
  rc = ensure_btable(c);
  if (rc != HSV_OK) return rc;
  // resident_run copies min(m, kResidentVotes) votes: arrays of that size
  const uint32_t idx[kResidentVotes] = {};
  uint8_t sig[kResidentVotes * 64] = {}, msg[32] = {}, flags[16];
  CommitteeDev cd;
  cd.device = c.device;
  cd.n = 1;
  static const uint8_t zero_key[32] = {0};
  cd.h_pks = zero_key;
  cd.d_pks = reinterpret_cast<const uint8_t *>(c.d_btable);  // valid device memory, never read: m is refused
  cd.d_kflags = cd.d_pks;
  cd.d_tabptr = reinterpret_cast<const uint32_t *const *>(c.d_btable);
  rc = resident_run(cd, idx, sig, 64, msg, 0, m, flags, c.d_btable);
  return rc == kResidentUnavailable ? fail(HSV_ERR_HIP, "resident service unavailable") : rc;
}

namespace {

// Votes by member index on the committee's device, through a slot of that
// device: the kernels read the pinned staging buffer directly for batches of
// at most kZeroCopyMax votes (the latency path), otherwise via copies.
int committee_run(const CommitteeDev &cd, const uint32_t *key_idx, const uint8_t *sig, size_t sig_stride,
                  const uint8_t *msg, size_t msg_stride, size_t m, uint8_t *flags_out) {
  int rc = ensure_init();
  if (rc != HSV_OK) return rc;
  DevCtx &c = ctx(cd.device);
  DeviceGuard guard(c.device);
  if (guard.status() != hipSuccess) return hip_fail("hipSetDevice", guard.status());
  rc = ensure_btable(c);  // also after an hsv_shutdown
  if (rc != HSV_OK) return rc;
  if (resident_enabled() && m <= hsv_comb_resident_votes()) {
    rc = resident_run(cd, key_idx, sig, sig_stride, msg, msg_stride, m, flags_out, c.d_btable);
    if (rc != kResidentUnavailable) return rc;
  }
  SlotLease lease(c);
  Slot &s = lease.slot();
  call_mark(HSV_MARK_SLOT);
  for (size_t base = 0; base < m; base += kChunk) {
    const size_t k = std::min(kChunk, m - base);
    const size_t idx_off = 0;
    const size_t sig_off = round_up(k * 4, kAlign);
    const size_t msg_off = sig_off + round_up(k * 64, kAlign);
    const size_t msg_bytes = msg_stride ? k * 32 : 32;
    const size_t flag_off = msg_off + round_up(msg_bytes, kAlign);
    const size_t fault_off = flag_off + round_up(k, kAlign);
    const size_t total = fault_off + kAlign;
    rc = slot_prepare(s, total, total);
    if (rc != HSV_OK) return rc;
    uint8_t *h = s.h_buf;
    stage_copy(h + idx_off, key_idx + base, k * 4);
    if (sig_stride == 64) {
      stage_copy(h + sig_off, sig + base * 64, k * 64);
    } else {  // signatures inside packed votes: gathered straight into the staging
      for (size_t i = 0; i < k; ++i) stage_copy(h + sig_off + i * 64, sig + (base + i) * sig_stride, 64);
    }
    stage_copy(h + msg_off, msg + base * msg_stride, msg_bytes);
    stage_fence();
    // The zero-copy latency form (<= kZeroCopyMax votes) reads the inputs from
    // the pinned staging through its device mapping (copying them to HBM first
    // made C1 0.0444 -> 0.0498 ms and C3 0.0592 -> 0.0689 ms,
    // profiles/r03zz7_qc_ab_zc.txt) and writes its flags, self-check words and
    // one completion marker per block into the slot's coherent sync region;
    // the host spins on the markers instead of hipStreamSynchronize: the flags
    // are final once every block has released them, several microseconds
    // before the kernel's completion signal (same box, alternating processes,
    // profiles/r04b_qc_ab_marker.txt: C1 0.0444 -> 0.0394 ms, C3 0.0587 ->
    // 0.0559 ms, one verify_strict 0.0443 -> 0.0395 ms).
    const bool zero_copy = k <= kZeroCopyMax && s.h_buf_dev != nullptr;
    uint8_t *flags_h, *flags_d, *fault_h, *fault_d;
    uint32_t nmark = 0;
    volatile uint32_t *marks = nullptr;
    uint32_t *marks_d = nullptr;
    if (zero_copy) {
      nmark = hsv_comb_marker_blocks((uint32_t)k);
      const size_t sf = round_up(k, kAlign), sm = sf + kAlign, need = sm + round_up((size_t)nmark * 4 + 4, kAlign);
      rc = slot_sync_region(s, need);
      if (rc != HSV_OK) return rc;
      flags_h = s.h_sync;
      flags_d = s.h_sync_dev;
      fault_h = s.h_sync + sf;
      fault_d = s.h_sync_dev + sf;
      marks = reinterpret_cast<volatile uint32_t *>(s.h_sync + sm);
      marks_d = reinterpret_cast<uint32_t *>(s.h_sync_dev + sm);
      for (uint32_t b = 0; b < nmark; ++b) marks[b] = 0u;
    } else {
      flags_h = h + flag_off;
      flags_d = s.d_buf + flag_off;
      fault_h = h + fault_off;
      fault_d = s.d_buf + fault_off;
    }
    // unwritten flags read as rejections; self-check words start at zero
    std::memset(flags_h, 0, k);
    std::memset(fault_h, 0, kFaultBytes);
    call_mark(HSV_MARK_STAGED);
    const uint8_t *dbuf = zero_copy ? s.h_buf_dev : s.d_buf;
    hipError_t e = hipSuccess;
    if (!zero_copy) e = hipMemcpyAsync(s.d_buf, h, fault_off + kFaultBytes, hipMemcpyHostToDevice, s.stream);
    if (e == hipSuccess)
      e = hsv_launch_comb_verify(reinterpret_cast<const uint32_t *>(dbuf + idx_off), dbuf + sig_off, 64,
                                 dbuf + msg_off, msg_stride ? 32 : 0, (uint32_t)k, cd.d_pks, cd.d_kflags, cd.n,
                                 cd.d_tabptr, c.d_btable, flags_d, reinterpret_cast<uint32_t *>(fault_d), marks_d,
                                 s.stream);
    if (e == hipSuccess && !zero_copy)
      e = hipMemcpyAsync(h + flag_off, s.d_buf + flag_off, fault_off + kFaultBytes - flag_off, hipMemcpyDeviceToHost,
                         s.stream);
    call_mark(HSV_MARK_LAUNCH);
    hipError_t es = hipSuccess;
    bool marked = false;
    if (nmark && e == hipSuccess) {
      // every block past its reads and its stores released: the flags are
      // final, and nothing of this call reads the staging any more (the next
      // call on this slot is ordered behind the kernel on the stream); a
      // kernel that never marks (a device fault) falls back to the stream sync
      const auto t0 = std::chrono::steady_clock::now();
      for (uint32_t b = 0;;) {
        while (b < nmark && marks[b] == 1u) ++b;
        if (b == nmark) {
          marked = true;
          break;
        }
        if (std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(50)) break;
      }
      std::atomic_thread_fence(std::memory_order_acquire);
    }
    if (!marked) es = hipStreamSynchronize(s.stream);  // nothing of this call stays in flight
    call_mark(HSV_MARK_SYNC);
    if (e != hipSuccess) return hip_fail("committee verify launch", e);
    if (es != hipSuccess) return hip_fail("hipStreamSynchronize", es);
    rc = check_faults(fault_h, "committee verify");
    if (rc != HSV_OK) return rc;
    std::memcpy(flags_out + base, flags_h, k);
    call_mark(HSV_MARK_DONE);
  }
  return HSV_OK;
}

// Builds comb tables for `nkeys` encodings already in HBM at d_encs into
// tables[i] (device pointers, host array), flags into d_kflags, on stream st.
// Keys are built in runs of contiguous table memory.
hipError_t build_tables(const uint8_t *d_encs, uint32_t nkeys, uint32_t *const *tables, uint8_t *d_kflags,
                        uint32_t *d_tmp, uint32_t tmp_keys, hipStream_t st) {
  const uint64_t words = hsv_comb_table_bytes() / 4;
  uint32_t i = 0;
  while (i < nkeys) {
    uint32_t j = i + 1;
    while (j < nkeys && j - i < tmp_keys && tables[j] == tables[j - 1] + words) ++j;
    const hipError_t e = hsv_launch_comb_build(d_encs + (size_t)i * 32, j - i, 1, tables[i], d_tmp, d_kflags + i, st);
    if (e != hipSuccess) return e;
    i = j;
  }
  return hipSuccess;
}

}  // namespace
}  // namespace hsvh

using namespace hsvh;

// ---- explicit committee ------------------------------------------------------------
struct hsv_committee {
  CommitteeDev dev;
  std::vector<uint8_t> h_pks;
  uint8_t *d_pks = nullptr;
  uint8_t *d_kflags = nullptr;
  uint32_t *d_tables = nullptr;
  uint32_t **d_tabptr = nullptr;
  KeyIndex index;
};

extern "C" {

int hsv_committee_create(const uint8_t *pks, size_t n, hsv_committee **out) {
  if (!out || (!pks && n)) return fail(HSV_ERR_INVALID_ARG, "null argument");
  if (n > (1u << 20)) return fail(HSV_ERR_INVALID_ARG, "committee too large");
  int rc = ensure_init();
  if (rc != HSV_OK) return rc;
  const int dev = home_device();
  DeviceGuard guard(dev);
  if (guard.status() != hipSuccess) return hip_fail("hipSetDevice", guard.status());
  rc = ensure_btable(ctx(dev));
  if (rc != HSV_OK) return rc;
  std::unique_ptr<hsv_committee> cm(new hsv_committee());
  cm->dev.device = dev;
  cm->dev.n = (uint32_t)n;
  cm->h_pks.assign(pks, pks + 32 * n);
  cm->dev.h_pks = cm->h_pks.data();
  for (size_t i = 0; i < n; ++i) cm->index.emplace(key_of(pks + 32 * i), (uint32_t)i);
  if (n) {
    const uint64_t words = hsv_comb_table_bytes() / 4;
    uint32_t *d_tmp = nullptr;
    hipStream_t st = nullptr;
    std::vector<uint32_t *> ptrs(n);
    hipError_t e = hipMalloc(&cm->d_pks, n * 32);
    if (e == hipSuccess) e = hipMalloc(&cm->d_kflags, n);
    if (e == hipSuccess) e = hipMalloc(&cm->d_tables, n * hsv_comb_table_bytes());
    if (e == hipSuccess) e = hipMalloc(&cm->d_tabptr, n * sizeof(uint32_t *));
    if (e == hipSuccess) e = hipMalloc(&d_tmp, hsv_comb_tmp_bytes(std::min<uint32_t>((uint32_t)n, 1024)));
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
    for (size_t i = 0; e == hipSuccess && i < n; ++i) ptrs[i] = cm->d_tables + i * words;
    if (e == hipSuccess) e = hipMemcpyAsync(cm->d_pks, pks, n * 32, hipMemcpyHostToDevice, st);
    if (e == hipSuccess)
      e = hipMemcpyAsync(cm->d_tabptr, ptrs.data(), n * sizeof(uint32_t *), hipMemcpyHostToDevice, st);
    if (e == hipSuccess)
      e = build_tables(cm->d_pks, (uint32_t)n, ptrs.data(), cm->d_kflags, d_tmp, std::min<uint32_t>((uint32_t)n, 1024), st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    if (st) (void)hipStreamDestroy(st);
    if (d_tmp) {
      ResidentPause pause;  // hipFree waits for every grid on the device
      (void)hipFree(d_tmp);
    }
    if (e != hipSuccess) {
      hsv_committee_destroy(cm.release());
      return hip_fail("building committee tables", e);
    }
    cm->dev.d_pks = cm->d_pks;
    cm->dev.d_kflags = cm->d_kflags;
    cm->dev.d_tabptr = cm->d_tabptr;
  }
  *out = cm.release();
  return HSV_OK;
}

void hsv_committee_destroy(hsv_committee *cm) {
  if (!cm) return;
  ResidentPause pause;  // hipFree waits for every grid on the device
  DeviceGuard guard(cm->dev.device);
  if (cm->d_pks) (void)hipFree(cm->d_pks);
  if (cm->d_kflags) (void)hipFree(cm->d_kflags);
  if (cm->d_tables) (void)hipFree(cm->d_tables);
  if (cm->d_tabptr) (void)hipFree(cm->d_tabptr);
  delete cm;
}

size_t hsv_committee_size(const hsv_committee *cm) { return cm ? cm->dev.n : 0; }

int64_t hsv_committee_index(const hsv_committee *cm, const uint8_t pk[32]) {
  if (!cm || !pk) return -1;
  return cm->index.find(pk);
}

int hsv_committee_verify_device(const hsv_committee *cm, const uint32_t *d_key_idx, const uint8_t *d_sig,
                                size_t sig_stride, const uint8_t *d_msg, size_t msg_stride, size_t m, uint8_t *d_flags,
                                uint32_t *d_fault, void *stream) {
  if (m == 0) return HSV_OK;
  if (!cm || !d_key_idx || !d_sig || !d_msg || !d_flags) return fail(HSV_ERR_INVALID_ARG, "null argument");
  if (((reinterpret_cast<uintptr_t>(d_sig) | reinterpret_cast<uintptr_t>(d_msg) | sig_stride | msg_stride) & 15u) != 0)
    return fail(HSV_ERR_ALIGN, "device pointers and strides must be multiples of 16");
  if (sig_stride < 64 || (msg_stride != 0 && msg_stride < 32)) return fail(HSV_ERR_INVALID_ARG, "record strides overlap");
  if (m > 0xffffffffu) return fail(HSV_ERR_INVALID_ARG, "batch too large");
  int rc = ensure_init();
  if (rc != HSV_OK) return rc;
  const int pd = pointer_device(d_sig);
  if (pd >= 0 && pd != cm->dev.device)
    return fail(HSV_ERR_INVALID_ARG, "inputs live on device " + std::to_string(pd) + ", the committee on device " +
                                         std::to_string(cm->dev.device));
  DevCtx &c = ctx(cm->dev.device);
  DeviceGuard guard(c.device);
  if (guard.status() != hipSuccess) return hip_fail("hipSetDevice", guard.status());
  rc = ensure_btable(c);  // the B table is rebuilt if hsv_shutdown released it
  if (rc != HSV_OK) return rc;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  uint32_t *fault = nullptr;
  rc = call_fault_words(c, d_fault, s, &fault);
  if (rc != HSV_OK) return rc;
  const hipError_t e = hsv_launch_comb_verify(d_key_idx, d_sig, sig_stride, d_msg, msg_stride, (uint32_t)m, cm->dev.d_pks,
                                              cm->dev.d_kflags, cm->dev.n, cm->dev.d_tabptr, c.d_btable, d_flags, fault,
                                              nullptr, s);
  return e == hipSuccess ? HSV_OK : hip_fail("committee verify launch", e);
}

int hsv_committee_verify(hsv_committee *cm, const uint32_t *key_idx, const uint8_t *sig, const uint8_t *msg,
                         size_t msg_stride, size_t m, uint8_t *flags_out) {
  CallScope call;
  if (m == 0) return HSV_OK;
  if (!cm || !key_idx || !sig || !msg || !flags_out) return fail(HSV_ERR_INVALID_ARG, "null argument");
  if (msg_stride != 0 && msg_stride != 32) return fail(HSV_ERR_INVALID_ARG, "msg_stride must be 0 or 32");
  return committee_run(cm->dev, key_idx, sig, 64, msg, msg_stride, m, flags_out);
}

int hsv_committee_verify_batch_packed(hsv_committee *cm, const uint8_t digest[32], const uint8_t *votes, size_t m) {
  CallScope call;
  if (m == 0) return 1;
  if (!cm || !digest || !votes) return fail(HSV_ERR_INVALID_ARG, "null argument");
  thread_local std::vector<uint32_t> idx;  // per-call scratch kept by the thread
  thread_local std::vector<uint8_t> flags;
  idx.resize(m);
  flags.resize(m);
  for (size_t i = 0; i < m; ++i) {
    const int64_t k = cm->index.find(votes + 96 * i);
    if (k < 0) {  // a non-member key: the generic kernels
      const int rc = run_host(votes, 96, votes + 32, 96, digest, 0, m, flags.data());
      return rc != HSV_OK ? rc : batch_verdict(flags.data(), m);
    }
    idx[i] = (uint32_t)k;
  }
  const int rc = committee_run(cm->dev, idx.data(), votes + 32, 96, digest, 0, m, flags.data());
  return rc != HSV_OK ? rc : batch_verdict(flags.data(), m);
}

}  // extern "C"

// ---- automatic committee cache behind the drop-in verify_batch ---------------------
// Consensus keys are fixed per epoch (consensus/src/config.rs:39-43), so the
// keys of every QC repeat round after round.  A key missing from the cache
// is counted once per batch it appears in; from its second batch on it is
// queued, and a background thread builds the queued keys' tables on a stream
// of its own, appends them to the cache and publishes a new immutable view.
// A verify call never waits for a build: it takes the committee kernels when
// every key of its batch is in the published view and the generic kernels
// otherwise, with identical flags either way (tests/test_committee.py).
// Capacity kAutoMaxKeys keys; batches larger than that are never counted.
// When the cache is full and batches keep missing it (a new epoch), it is
// dropped and relearnt.  A failed build is a cache miss, never an error.
// HSV_AUTO_COMMITTEE=0 or hsv_set_auto_committee(0) turns it off.
namespace hsvh {
namespace {

constexpr uint32_t kAutoMaxKeys = 8192;      // 3 GiB of tables at most
constexpr uint32_t kBlockKeys = 64;          // tables allocated 64 keys (24 MiB) at a time
constexpr size_t kCommitteeTryMax = 4096;    // hsv_verify / verify_strict batches that try the cache
constexpr size_t kLearnStrictMax = 16;       // ... and that teach it their keys (votes, single verifies)
constexpr uint32_t kResetAfterMisses = 256;  // missing batches against a full cache before a relearn
constexpr int kMaxBuildFailures = 3;         // then the cache stays off until hsv_set_auto_committee(1)

struct AutoStore {  // append-only device storage, freed with the last view using it
  int device = 0;
  uint8_t *d_pks = nullptr;
  uint8_t *d_kflags = nullptr;
  uint32_t **d_tabptr = nullptr;
  uint32_t *d_tmp = nullptr;
  hipStream_t stream = nullptr;  // builds only
  std::vector<uint32_t *> blocks;
  // host copy of the encodings (kAutoMaxKeys * 32 B, allocated once: a view's
  // pointer into it stays valid as later builds append)
  std::unique_ptr<uint8_t[]> h_pks{new uint8_t[(size_t)kAutoMaxKeys * 32]};
  ~AutoStore() {
    ResidentPause pause;  // hipFree waits for every grid on the device
    DeviceGuard guard(device);
    if (stream) (void)hipStreamDestroy(stream);
    for (uint32_t *b : blocks) (void)hipFree(b);
    if (d_pks) (void)hipFree(d_pks);
    if (d_kflags) (void)hipFree(d_kflags);
    if (d_tabptr) (void)hipFree(d_tabptr);
    if (d_tmp) (void)hipFree(d_tmp);
  }
};

struct AutoView {  // immutable snapshot: keys [0, n) of `store` are built
  std::shared_ptr<AutoStore> store;
  CommitteeDev dev;
  KeyIndex index;
};

struct AutoCommittee {
  std::mutex mu;  // everything below; `view` is also read lock-free (atomic_load)
  std::shared_ptr<const AutoView> view;
  std::unordered_map<Key32, uint32_t, KeyHash> seen;  // uncached key -> batches it appeared in
  std::vector<Key32> pending;
  std::unordered_set<Key32, KeyHash> pending_set;
  bool building = false;
  uint64_t generation = 0;  // bumped by a reset; a build of an older generation is discarded
  // batches that missed a full cache in a row; written under mu on a miss,
  // reset without the lock on a hit (the QC hot path takes no lock)
  std::atomic<uint32_t> miss_streak{0};
  int failures = 0;
  std::thread worker;
  std::condition_variable idle;
  std::atomic<int> enabled{-1};  // -1: read HSV_AUTO_COMMITTEE on first use
  std::atomic<uint64_t> builds{0};
  std::atomic<uint64_t> faults{0};  // cached-path launches whose self-check failed
  ~AutoCommittee() {
    std::unique_lock<std::mutex> lk(mu);
    idle.wait(lk, [&] { return !building; });
    lk.unlock();
    if (worker.joinable()) worker.join();
  }
};

AutoCommittee &AC() {
  static AutoCommittee a;
  return a;
}

bool auto_enabled() {
  AutoCommittee &a = AC();
  int e = a.enabled.load();
  if (e < 0) {
    const char *v = std::getenv("HSV_AUTO_COMMITTEE");
    e = (v && v[0] == '0') ? 0 : 1;
    a.enabled.store(e);
  }
  return e == 1;
}

std::shared_ptr<const AutoView> current_view() { return std::atomic_load(&AC().view); }

// Build tables for `keys` on top of `base` (nullptr: a fresh store on
// `device`).  Runs without the cache lock.
int build_view(const std::shared_ptr<const AutoView> &base, int device, const std::vector<Key32> &keys,
               std::shared_ptr<const AutoView> &out) {
  DeviceGuard guard(device);
  if (guard.status() != hipSuccess) return hip_fail("hipSetDevice", guard.status());
  std::shared_ptr<AutoStore> store = base ? base->store : std::make_shared<AutoStore>();
  const uint32_t n0 = base ? base->dev.n : 0;
  const uint32_t m = std::min<uint32_t>((uint32_t)keys.size(), kAutoMaxKeys - n0);
  hipError_t e = hipSuccess;
  if (!base) {
    store->device = device;
    e = hipMalloc(&store->d_pks, (size_t)kAutoMaxKeys * 32);
    if (e == hipSuccess) e = hipMalloc(&store->d_kflags, kAutoMaxKeys);
    if (e == hipSuccess) e = hipMalloc(&store->d_tabptr, (size_t)kAutoMaxKeys * sizeof(uint32_t *));
    if (e == hipSuccess) e = hipMalloc(&store->d_tmp, hsv_comb_tmp_bytes(kBlockKeys));
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&store->stream, hipStreamNonBlocking);
    if (e != hipSuccess) return hip_fail("allocating the committee cache", e);
  }
  const uint64_t words = hsv_comb_table_bytes() / 4;
  while ((uint64_t)store->blocks.size() * kBlockKeys < (uint64_t)n0 + m) {
    uint32_t *blk = nullptr;
    e = hipMalloc(&blk, (size_t)kBlockKeys * hsv_comb_table_bytes());
    if (e != hipSuccess) return hip_fail("allocating committee tables", e);
    store->blocks.push_back(blk);
  }
  std::vector<uint8_t> encs((size_t)m * 32);
  std::vector<uint32_t *> ptrs(m);
  for (uint32_t i = 0; i < m; ++i) {
    std::memcpy(encs.data() + (size_t)i * 32, keys[i].data(), 32);
    const uint32_t slot = n0 + i;
    ptrs[i] = store->blocks[slot / kBlockKeys] + (uint64_t)(slot % kBlockKeys) * words;
  }
  std::memcpy(store->h_pks.get() + (size_t)n0 * 32, encs.data(), encs.size());  // slots no published view reads yet
  e = hipMemcpyAsync(store->d_pks + (size_t)n0 * 32, encs.data(), encs.size(), hipMemcpyHostToDevice, store->stream);
  if (e == hipSuccess)
    e = hipMemcpyAsync(store->d_tabptr + n0, ptrs.data(), m * sizeof(uint32_t *), hipMemcpyHostToDevice, store->stream);
  if (e == hipSuccess)
    e = build_tables(store->d_pks + (size_t)n0 * 32, m, ptrs.data(), store->d_kflags + n0, store->d_tmp, kBlockKeys,
                     store->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(store->stream);
  if (e != hipSuccess) return hip_fail("building committee tables", e);
  auto v = std::make_shared<AutoView>();
  v->store = store;
  v->dev.device = store->device;
  v->dev.n = n0 + m;
  v->dev.h_pks = store->h_pks.get();
  v->dev.d_pks = store->d_pks;
  v->dev.d_kflags = store->d_kflags;
  v->dev.d_tabptr = store->d_tabptr;
  if (base) v->index = base->index;
  for (uint32_t i = 0; i < m; ++i) v->index.emplace(keys[i], n0 + i);
  out = v;
  return HSV_OK;
}

void worker_main() {
  AutoCommittee &a = AC();
  std::unique_lock<std::mutex> lk(a.mu);
  for (;;) {
    if (a.pending.empty() || a.enabled.load() != 1) {
      a.pending.clear();
      a.pending_set.clear();
      a.building = false;
      a.idle.notify_all();
      return;
    }
    std::vector<Key32> keys;
    keys.swap(a.pending);
    const uint64_t gen = a.generation;
    std::shared_ptr<const AutoView> base = a.view;
    const int device = base ? base->dev.device : home_device();
    lk.unlock();
    std::shared_ptr<const AutoView> built;
    const int rc = build_view(base, device, keys, built);
    lk.lock();
    for (const Key32 &k : keys) {
      a.pending_set.erase(k);
      a.seen.erase(k);
    }
    if (rc == HSV_OK && gen == a.generation) {
      std::atomic_store(&a.view, built);
      a.builds.fetch_add(1);
    } else if (rc != HSV_OK && ++a.failures >= kMaxBuildFailures) {
      a.enabled.store(0);  // verification goes on through the generic kernels
    }
  }
}

// The view to verify this batch with (every key in it; idx receives the
// member indices), or nullptr: the generic path.  Records misses.
std::shared_ptr<const AutoView> auto_lookup(const uint8_t *pk, size_t pk_stride, size_t n, uint32_t *idx,
                                            bool count_misses) {
  std::shared_ptr<const AutoView> v = current_view();
  std::vector<Key32> missing;
  for (size_t i = 0; i < n; ++i) {
    if (v) {
      const int64_t m = v->index.find(pk + i * pk_stride);
      if (m >= 0) {
        idx[i] = (uint32_t)m;
        continue;
      }
    }
    if (!count_misses) return nullptr;
    missing.push_back(key_of(pk + i * pk_stride));
  }
  AutoCommittee &a = AC();
  if (missing.empty()) {
    if (v && v->dev.device != home_device()) return nullptr;  // cache lives on another device
    if (a.miss_streak.load(std::memory_order_relaxed)) a.miss_streak.store(0, std::memory_order_relaxed);
    return v;
  }
  if (n > kAutoMaxKeys) return nullptr;  // not a committee-sized batch
  std::sort(missing.begin(), missing.end());
  missing.erase(std::unique(missing.begin(), missing.end()), missing.end());  // once per batch
  std::unique_lock<std::mutex> lk(a.mu);
  const uint32_t cached = v ? v->dev.n : 0;
  if (cached + a.pending_set.size() >= kAutoMaxKeys && a.miss_streak.fetch_add(1) + 1 >= kResetAfterMisses) {
    // a full cache that keeps missing: a new epoch, relearn from scratch
    std::atomic_store(&a.view, std::shared_ptr<const AutoView>());
    a.seen.clear();
    a.pending.clear();
    a.pending_set.clear();
    a.miss_streak = 0;
    ++a.generation;
    return nullptr;
  }
  for (const Key32 &k : missing) {
    if (a.pending_set.count(k)) continue;
    if (++a.seen[k] >= 2 && cached + a.pending_set.size() < kAutoMaxKeys) {
      a.pending.push_back(k);
      a.pending_set.insert(k);
    }
  }
  if (a.seen.size() > 4 * (size_t)kAutoMaxKeys) a.seen.clear();
  if (!a.pending.empty() && !a.building && a.enabled.load() == 1) {
    a.building = true;
    if (a.worker.joinable()) a.worker.join();  // the previous build thread has finished
    a.worker = std::thread(worker_main);
  }
  return nullptr;
}

// The cached path's self-check failed: its tables (or the memory under them)
// are no longer trusted.  Drop the view the failing call used -- unless a
// newer one was published meanwhile -- and relearn from scratch; the call
// itself is answered by the generic kernels.  Counted (hsv_auto_committee_faults).
void auto_invalidate(const std::shared_ptr<const AutoView> &bad) {
  AutoCommittee &a = AC();
  a.faults.fetch_add(1);
  std::lock_guard<std::mutex> lk(a.mu);
  if (std::atomic_load(&a.view) != bad) return;
  std::atomic_store(&a.view, std::shared_ptr<const AutoView>());
  a.seen.clear();
  a.pending.clear();
  a.pending_set.clear();
  a.miss_streak = 0;
  ++a.generation;
}

// Run a batch on the cached tables.  HSV_OK, 1 (take the generic path:
// the self-check failed, the view is dropped), or another error.
int auto_run(const std::shared_ptr<const AutoView> &v, const uint32_t *idx, const uint8_t *sig, size_t sig_stride,
             const uint8_t *msg, size_t msg_stride, size_t n, uint8_t *flags_out) {
  const int rc = committee_run(v->dev, idx, sig, sig_stride, msg, msg_stride, n, flags_out);
  if (rc == HSV_ERR_DEVICE_FAULT) {
    auto_invalidate(v);
    return 1;
  }
  return rc;
}

void auto_reset(bool enable) {
  AutoCommittee &a = AC();
  std::unique_lock<std::mutex> lk(a.mu);
  a.enabled.store(enable ? 1 : 0);
  if (!enable) {
    a.pending.clear();
    a.idle.wait(lk, [&] { return !a.building; });
    std::atomic_store(&a.view, std::shared_ptr<const AutoView>());
    a.seen.clear();
    a.pending_set.clear();
    a.miss_streak = 0;
    a.failures = 0;
    ++a.generation;
  } else {
    a.failures = 0;
  }
}

}  // namespace

int auto_committee_try(const uint8_t *pk, const uint8_t *sig, const uint8_t *msg, size_t msg_stride, size_t n,
                       uint8_t *flags_out) {
  // only the latency range (a vote, a TC); large batches of fresh keys would
  // pay a hash lookup per item for nothing.  Calls of a few signatures --
  // Vote::verify on every incoming vote (consensus/src/core.rs:240), the
  // proposer's Block::verify -- count their keys as sightings too, so a
  // committee whose votes arrive before its first QCs is learnt from them;
  // larger strict batches only read the cache (their keys need not recur).
  if (n > kCommitteeTryMax || !auto_enabled()) return 1;
  thread_local std::vector<uint32_t> idx;  // per-call scratch kept by the thread
  idx.resize(n);
  std::shared_ptr<const AutoView> v = auto_lookup(pk, 32, n, idx.data(), n <= kLearnStrictMax);
  call_mark(HSV_MARK_LOOKUP);
  if (!v || v->dev.device != home_device()) return 1;
  return auto_run(v, idx.data(), sig, 64, msg, msg_stride, n, flags_out);
}

int auto_committee_corrupt_tables() {
  std::shared_ptr<const AutoView> v = current_view();
  if (!v || v->store->blocks.empty()) return 0;
  DeviceGuard guard(v->dev.device);
  for (uint32_t *b : v->store->blocks) {
    const hipError_t e = hipMemset(b, 0, (size_t)kBlockKeys * hsv_comb_table_bytes());
    if (e != hipSuccess) return hip_fail("hipMemset", e);
  }
  return (int)v->dev.n;
}

void auto_committee_shutdown() {
  {
    ResidentQc &r = RQ();
    std::lock_guard<std::mutex> lk(r.mu);
    resident_stop_locked(r);
  }
  auto_reset(false);
  AutoCommittee &a = AC();
  std::lock_guard<std::mutex> lk(a.mu);
  a.enabled.store(-1);  // re-read the environment on next use
}

}  // namespace hsvh

extern "C" {

int hsv_verify_batch_packed(const uint8_t digest[32], const uint8_t *votes, size_t n) {
  CallScope call;
  if (n == 0) return 1;
  if (!digest || !votes) return fail(HSV_ERR_INVALID_ARG, "null argument");
  int rc = ensure_init();
  if (rc != HSV_OK) return rc;
  thread_local std::vector<uint8_t> flags;  // per-call scratch kept by the thread
  thread_local std::vector<uint32_t> idx;
  flags.resize(n);
  if (n >= 2 && auto_enabled()) {
    idx.resize(n);
    std::shared_ptr<const AutoView> v = auto_lookup(votes, 96, n, idx.data(), true);
    call_mark(HSV_MARK_LOOKUP);
    if (v) {
      rc = auto_run(v, idx.data(), votes + 32, 96, digest, 0, n, flags.data());
      if (rc == HSV_OK) return batch_verdict(flags.data(), n);
      // the self-check failed (the cache is dropped) or another infrastructure
      // error on the cached path: the generic path answers
    }
  }
  rc = run_host(votes, 96, votes + 32, 96, digest, 0, n, flags.data());
  return rc != HSV_OK ? rc : batch_verdict(flags.data(), n);
}

int hsv_set_resident_service(int mode) { return resident_set_mode(mode != 0); }

int hsv_set_auto_committee(int enable) {
  auto_reset(enable != 0);
  return HSV_OK;
}

size_t hsv_auto_committee_size(void) {
  std::shared_ptr<const AutoView> v = current_view();
  return v ? v->dev.n : 0;
}

uint64_t hsv_auto_committee_faults(void) { return AC().faults.load(); }

int hsv_auto_committee_wait(int timeout_ms) {
  AutoCommittee &a = AC();
  std::unique_lock<std::mutex> lk(a.mu);
  const bool done = a.idle.wait_for(lk, std::chrono::milliseconds(timeout_ms < 0 ? 0 : timeout_ms),
                                    [&] { return !a.building; });
  return done ? 1 : 0;
}

}  // extern "C"
