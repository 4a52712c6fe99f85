// C ABI of libhsv.so (declared in include/hsv.h): device contexts, staging
// buffers, sharding across GPUs, and the reference-shaped entry points.
//
// Host-buffer calls stage inputs into pinned memory, copy them to HBM on a
// per-device stream, launch the verification kernel and copy the flag bytes
// back.  Batches above kShardMin items are split into contiguous ranges, one
// per visible GPU, each driven by its own host thread; the per-item flags are
// written straight into the caller's output (the "host gather").
// There is no CPU verification path: without a GPU every call returns
// HSV_ERR_NO_DEVICE.
#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "hsv.h"
#include "hsv_internal.h"

namespace {

thread_local std::string t_last_error = "";

int fail(int code, const std::string &msg) {
  t_last_error = msg;
  return code;
}

int hip_fail(const char *where, hipError_t e) {
  return fail(HSV_ERR_HIP, std::string(where) + ": " + hipGetErrorString(e));
}

constexpr size_t kAlign = 256;
constexpr size_t kChunk = size_t(1) << 22;     // items per launch (512 MiB of inputs max)
constexpr size_t kShardMin = size_t(1) << 16;  // shard host batches across GPUs above this
constexpr size_t kZeroCopyMax = size_t(1) << 12;  // committee batches read straight from pinned memory

size_t round_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

struct DevCtx {
  int device = 0;
  int cus = 0;
  uint32_t *d_btable = nullptr;  // comb table of B (committee path), built lazily
  uint32_t *d_btable16 = nullptr;  // wide comb table of B (generic kernels 15, 16), built lazily
  hipStream_t stream = nullptr;
  hipStream_t stream2 = nullptr;  // second pipeline stage of large host batches
  uint8_t *d_buf = nullptr;
  size_t d_cap = 0;
  uint8_t *h_buf = nullptr;
  size_t h_cap = 0;
  std::mutex mu;
};

struct Global {
  std::mutex mu;
  bool inited = false;
  int ndev = 0;
  std::vector<DevCtx *> ctx;
  // fastest measured: scalar prepass + half-size point pass, wide B comb, WA=4,
  // 3 waves/SIMD; two lanes per item for batches of at most 2^13 (QC latency)
  std::atomic<int> variant{21};
};

Global &G() {
  static Global g;
  return g;
}

int ensure_init() {
  Global &g = G();
  std::lock_guard<std::mutex> lk(g.mu);
  if (g.inited) return g.ndev > 0 ? HSV_OK : fail(HSV_ERR_NO_DEVICE, "no HIP device visible");
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
  g.ndev = n;
  for (int i = 0; i < n; ++i) {
    DevCtx *c = new DevCtx();
    c->device = i;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, i) == hipSuccess) c->cus = prop.multiProcessorCount;
    g.ctx.push_back(c);
  }
  if (const char *v = std::getenv("HSV_VARIANT")) {
    const int vi = std::atoi(v);
    if (vi >= 0 && vi < hsv_num_variants()) g.variant = vi;
  }
  g.inited = true;
  return n > 0 ? HSV_OK : fail(HSV_ERR_NO_DEVICE, "no HIP device visible");
}

int ctx_prepare(DevCtx &c, size_t dev_bytes, size_t host_bytes) {
  hipError_t e = hipSetDevice(c.device);
  if (e != hipSuccess) return hip_fail("hipSetDevice", e);
  if (!c.stream) {
    e = hipStreamCreateWithFlags(&c.stream, hipStreamNonBlocking);
    if (e != hipSuccess) return hip_fail("hipStreamCreate", e);
  }
  if (dev_bytes > c.d_cap) {
    if (c.d_buf) (void)hipFree(c.d_buf);
    c.d_buf = nullptr;
    c.d_cap = 0;
    const size_t cap = round_up(dev_bytes, size_t(1) << 20);
    e = hipMalloc(&c.d_buf, cap);
    if (e != hipSuccess) return hip_fail("hipMalloc", e);
    c.d_cap = cap;
  }
  if (host_bytes > c.h_cap) {
    if (c.h_buf) (void)hipHostFree(c.h_buf);
    c.h_buf = nullptr;
    c.h_cap = 0;
    const size_t cap = round_up(host_bytes, size_t(1) << 20);
    e = hipHostMalloc(&c.h_buf, cap, hipHostMallocDefault);
    if (e != hipSuccess) return hip_fail("hipHostMalloc", e);
    c.h_cap = cap;
  }
  return HSV_OK;
}

const uint8_t kBasepointEncoding[32] = {0x58, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66,
                                        0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66,
                                        0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66};

// comb table of B on this device (caller holds c.mu and has set the device)
int ensure_btable(DevCtx &c) {
  if (c.d_btable) return HSV_OK;
  uint8_t *d_enc = nullptr;
  uint32_t *d_tab = nullptr, *d_tmp = nullptr;
  hipError_t e = hipMalloc(&d_enc, 32);
  if (e == hipSuccess) e = hipMalloc(&d_tab, hsv_comb_table_bytes());
  if (e == hipSuccess) e = hipMalloc(&d_tmp, hsv_comb_tmp_bytes(1));
  if (e == hipSuccess) e = hipMemcpy(d_enc, kBasepointEncoding, 32, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hsv_launch_comb_build(d_enc, 1, 0, d_tab, d_tmp, nullptr, c.stream);
  if (e == hipSuccess) e = hipStreamSynchronize(c.stream);
  if (d_enc) (void)hipFree(d_enc);
  if (d_tmp) (void)hipFree(d_tmp);
  if (e != hipSuccess) {
    if (d_tab) (void)hipFree(d_tab);
    return hip_fail("building the B comb table", e);
  }
  c.d_btable = d_tab;
  return HSV_OK;
}

// wide (16-bit digit) comb table of B on this device (caller holds c.mu and
// has set the device): 48 MiB, built once
int ensure_btable16(DevCtx &c) {
  if (c.d_btable16) return HSV_OK;
  uint32_t *d_tab = nullptr, *d_tmp = nullptr;
  hipError_t e = hipMalloc(&d_tab, hsv_comb16_table_bytes());
  if (e == hipSuccess) e = hipMalloc(&d_tmp, hsv_comb16_tmp_bytes());
  if (e == hipSuccess) e = hsv_launch_comb16_build(d_tab, d_tmp, c.stream);
  if (e == hipSuccess) e = hipStreamSynchronize(c.stream);
  if (d_tmp) (void)hipFree(d_tmp);
  if (e != hipSuccess) {
    if (d_tab) (void)hipFree(d_tab);
    return hip_fail("building the wide B comb table", e);
  }
  c.d_btable16 = d_tab;
  return HSV_OK;
}

// the B comb table `variant` reads (nullptr when none); caller holds c.mu
int comb_table_for(DevCtx &c, int variant, const uint32_t **out) {
  *out = nullptr;
  const int bits = hsv_variant_needs_comb(variant);
  if (bits == 0) return HSV_OK;
  const int rc = bits == 16 ? ensure_btable16(c) : ensure_btable(c);
  if (rc != HSV_OK) return rc;
  *out = bits == 16 ? c.d_btable16 : c.d_btable;
  return HSV_OK;
}


// Host records: item i at pk + i*pk_stride, sig + i*sig_stride, msg + i*msg_stride
// (msg_stride 0 = shared).  Runs [0, n) on one device, chunk by chunk.
// Batches of at least 2 * kPipeChunk items run as a two-stage pipeline: two
// staging buffers and two streams, so the host packs chunk i+1 and the DMA
// engine copies it while the kernels verify chunk i.
constexpr size_t kPipeChunk = size_t(1) << 18;  // 32 MiB of inputs per pipelined chunk

// memcpy into pinned staging; large copies are split over a few host threads
// (one thread copies ~10 GB/s, slower than the GPU consumes a chunk)
void stage_copy(uint8_t *dst, const uint8_t *src, size_t bytes) {
  constexpr size_t kSplit = size_t(8) << 20;
  const size_t nt = std::min<size_t>(4, bytes / kSplit);
  if (nt < 2) {
    std::memcpy(dst, src, bytes);
    return;
  }
  std::vector<std::thread> th;
  const size_t part = (bytes / nt + 63) & ~size_t(63);
  for (size_t t = 1; t < nt; ++t) {
    const size_t lo = std::min(bytes, t * part), hi = std::min(bytes, (t + 1) * part);
    if (hi > lo) th.emplace_back([=] { std::memcpy(dst + lo, src + lo, hi - lo); });
  }
  std::memcpy(dst, src, std::min(bytes, part));
  for (auto &x : th) x.join();
}

int run_on_device(DevCtx &c, const uint8_t *pk, size_t pk_stride, const uint8_t *sig,
                  size_t sig_stride, const uint8_t *msg, size_t msg_stride, size_t n,
                  uint8_t *flags_out) {
  std::lock_guard<std::mutex> lk(c.mu);
  static const bool no_pipe = std::getenv("HSV_NO_PIPELINE") != nullptr;  // measurement switch
  static const bool no_zero_copy = std::getenv("HSV_NO_ZERO_COPY") != nullptr;  // measurement switch
  const bool pipe = !no_pipe && n >= 2 * kPipeChunk;
  const size_t chunk = pipe ? kPipeChunk : std::min(n, kChunk);
  const int nbuf = pipe ? 2 : 1;
  const size_t pk_off = 0;
  const size_t sig_off = round_up(chunk * 32, kAlign);
  const size_t msg_off = sig_off + round_up(chunk * 64, kAlign);
  const size_t msg_bytes = msg_stride ? chunk * 32 : 32;
  const size_t flag_off = msg_off + round_up(msg_bytes, kAlign);
  const size_t total = flag_off + round_up(chunk, kAlign);
  int rc = ctx_prepare(c, total * nbuf, total * nbuf);
  if (rc != HSV_OK) return rc;
  if (pipe && !c.stream2) {
    const hipError_t e = hipStreamCreateWithFlags(&c.stream2, hipStreamNonBlocking);
    if (e != hipSuccess) return hip_fail("hipStreamCreate", e);
  }
  const int variant = G().variant.load();
  const uint32_t *comb_b = nullptr;
  rc = comb_table_for(c, variant, &comb_b);
  if (rc != HSV_OK) return rc;
  size_t pend_base[2] = {0, 0}, pend_m[2] = {0, 0};
  // wait for buffer b's chunk and hand its flags to the caller
  auto retire = [&](int b) -> int {
    if (pend_m[b] == 0) return HSV_OK;
    const hipError_t e = hipStreamSynchronize(b ? c.stream2 : c.stream);
    if (e != hipSuccess) return hip_fail("hipStreamSynchronize", e);
    std::memcpy(flags_out + pend_base[b], c.h_buf + (size_t)b * total + flag_off, pend_m[b]);
    pend_m[b] = 0;
    return HSV_OK;
  };
  int b = 0;
  for (size_t base = 0; base < n; base += chunk, b = (b + 1) % nbuf) {
    const size_t m = std::min(chunk, n - base);
    rc = retire(b);
    if (rc != HSV_OK) return rc;
    hipStream_t s = b ? c.stream2 : c.stream;
    uint8_t *h = c.h_buf + (size_t)b * total;
    uint8_t *d = c.d_buf + (size_t)b * total;
    // pack into the dense layout the kernel reads (pk 32 | sig 64 | msg 32)
    if (pk_stride == 32) stage_copy(h + pk_off, pk + base * 32, m * 32);
    else for (size_t i = 0; i < m; ++i) std::memcpy(h + pk_off + 32 * i, pk + (base + i) * pk_stride, 32);
    if (sig_stride == 64) stage_copy(h + sig_off, sig + base * 64, m * 64);
    else for (size_t i = 0; i < m; ++i) std::memcpy(h + sig_off + 64 * i, sig + (base + i) * sig_stride, 64);
    if (msg_stride == 0) std::memcpy(h + msg_off, msg, 32);
    else if (msg_stride == 32) stage_copy(h + msg_off, msg + base * 32, m * 32);
    else for (size_t i = 0; i < m; ++i) std::memcpy(h + msg_off + 32 * i, msg + (base + i) * msg_stride, 32);
    const size_t in_bytes = msg_off + (msg_stride ? m * 32 : 32);
    // small batches (a QC of non-cached keys, a single vote): as on the
    // committee path, the kernels read the pinned staging buffer and write the
    // flags through its device mapping, so no copy launches sit on the
    // latency path
    void *hd = nullptr;
    if (!no_zero_copy && n <= kZeroCopyMax && hipHostGetDevicePointer(&hd, h, 0) == hipSuccess && hd) {
      uint8_t *dh = static_cast<uint8_t *>(hd);
      hipError_t e = hsv_launch_verify(variant, dh + pk_off, 32, dh + sig_off, 64, dh + msg_off,
                                       msg_stride ? 32 : 0, (uint32_t)m, dh + flag_off, nullptr, comb_b, s);
      if (e != hipSuccess) return hip_fail("verify kernel launch", e);
      pend_base[b] = base;
      pend_m[b] = m;
      continue;
    }
    hipError_t e = hipMemcpyAsync(d, h, in_bytes, hipMemcpyHostToDevice, s);
    if (e != hipSuccess) return hip_fail("hipMemcpyAsync H2D", e);
    e = hsv_launch_verify(variant, d + pk_off, 32, d + sig_off, 64, d + msg_off, msg_stride ? 32 : 0,
                          (uint32_t)m, d + flag_off, nullptr, comb_b, s);
    if (e != hipSuccess) return hip_fail("verify kernel launch", e);
    e = hipMemcpyAsync(h + flag_off, d + flag_off, m, hipMemcpyDeviceToHost, s);
    if (e != hipSuccess) return hip_fail("hipMemcpyAsync D2H", e);
    pend_base[b] = base;
    pend_m[b] = m;
  }
  for (int k = 0; k < nbuf; ++k) {
    rc = retire(k);
    if (rc != HSV_OK) return rc;
  }
  return HSV_OK;
}

int run_host(const uint8_t *pk, size_t pk_stride, const uint8_t *sig, size_t sig_stride,
             const uint8_t *msg, size_t msg_stride, size_t n, uint8_t *flags_out) {
  if (n == 0) return HSV_OK;
  if (!pk || !sig || !msg || !flags_out) return fail(HSV_ERR_INVALID_ARG, "null pointer");
  int rc = ensure_init();
  if (rc != HSV_OK) return rc;
  Global &g = G();
  const int ndev = g.ndev;
  if (ndev == 1 || n < kShardMin) return run_on_device(*g.ctx[0], pk, pk_stride, sig, sig_stride, msg, msg_stride, n, flags_out);
  // contiguous shards, one host thread per GPU
  std::vector<int> rcs(ndev, HSV_OK);
  std::vector<std::string> errs(ndev);
  std::vector<std::thread> th;
  for (int d = 0; d < ndev; ++d) {
    const size_t lo = n * d / ndev, hi = n * (d + 1) / ndev;
    th.emplace_back([&, d, lo, hi]() {
      if (hi > lo)
        rcs[d] = run_on_device(*g.ctx[d], pk + lo * pk_stride, pk_stride, sig + lo * sig_stride,
                               sig_stride, msg + lo * msg_stride, msg_stride, hi - lo,
                               flags_out + lo);
      if (rcs[d] != HSV_OK) errs[d] = t_last_error;
    });
  }
  for (auto &t : th) t.join();
  for (int d = 0; d < ndev; ++d)
    if (rcs[d] != HSV_OK) return fail(rcs[d], "device " + std::to_string(d) + ": " + errs[d]);
  return HSV_OK;
}

}  // namespace

void release_auto_committee();  // hsv_verify_batch_packed's cache, defined below
// Strict verification of small batches whose keys are all in that cache, via
// the committee kernels: HSV_OK when done, 1 when the caller should take the
// generic path, < 0 on an error.
int auto_committee_try(const uint8_t *pk, const uint8_t *sig, const uint8_t *msg, size_t msg_stride, size_t n,
                       uint8_t *flags_out);

extern "C" {

int hsv_init(int device) {
  int rc = ensure_init();
  if (rc != HSV_OK) return rc;
  Global &g = G();
  if (device >= g.ndev) return fail(HSV_ERR_INVALID_ARG, "device index out of range");
  return device < 0 ? g.ndev : 1;
}

void hsv_shutdown(void) {
  release_auto_committee();
  Global &g = G();
  std::lock_guard<std::mutex> lk(g.mu);
  for (DevCtx *c : g.ctx) {
    std::lock_guard<std::mutex> lk2(c->mu);
    if (hipSetDevice(c->device) == hipSuccess) {
      if (c->stream) (void)hipStreamDestroy(c->stream);
      if (c->stream2) (void)hipStreamDestroy(c->stream2);
      if (c->d_buf) (void)hipFree(c->d_buf);
      if (c->h_buf) (void)hipHostFree(c->h_buf);
      if (c->d_btable) (void)hipFree(c->d_btable);
      if (c->d_btable16) (void)hipFree(c->d_btable16);
    }
    c->d_btable = nullptr;
    c->d_btable16 = nullptr;
    c->stream = c->stream2 = nullptr;
    c->d_buf = c->h_buf = nullptr;
    c->d_cap = c->h_cap = 0;
  }
}

int hsv_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

const char *hsv_last_error(void) { return t_last_error.c_str(); }

const char *hsv_version(void) { return "hsv 0.1.0 (gfx950)"; }

// Measurement/test hook (not in hsv.h): pick the kernel variant.
int hsv_set_variant(int v) {
  if (v < 0 || v >= hsv_num_variants()) return fail(HSV_ERR_INVALID_ARG, "bad variant");
  G().variant = v;
  return HSV_OK;
}

int hsv_get_variant(void) { return G().variant.load(); }

int hsv_verify(const uint8_t *pk, const uint8_t *sig, const uint8_t *msg, size_t msg_stride,
               size_t n, uint8_t *flags_out) {
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

static int batch_verdict(const std::vector<uint8_t> &flags) {
  for (uint8_t f : flags)
    if ((f & (HSV_PARSE_OK | HSV_EQ_OK)) != (HSV_PARSE_OK | HSV_EQ_OK)) return 0;
  return 1;
}

// crypto::Signature::verify_batch through the generic kernels
static int verify_batch_generic(const uint8_t digest[32], const uint8_t *pk, size_t pk_stride, const uint8_t *sig,
                                size_t sig_stride, size_t n) {
  std::vector<uint8_t> flags(n);
  int rc = run_host(pk, pk_stride, sig, sig_stride, digest, 0, n, flags.data());
  if (rc != HSV_OK) return rc;
  return batch_verdict(flags);
}

int hsv_verify_batch(const uint8_t digest[32], const uint8_t *pk, const uint8_t *sig, size_t n) {
  if (n == 0) return 1;  // dalek verify_batch over zero items is Ok
  if (!digest || !pk || !sig) return fail(HSV_ERR_INVALID_ARG, "null argument");
  std::vector<uint8_t> packed(n * 96);
  for (size_t i = 0; i < n; ++i) {
    std::memcpy(packed.data() + 96 * i, pk + 32 * i, 32);
    std::memcpy(packed.data() + 96 * i + 32, sig + 64 * i, 64);
  }
  return hsv_verify_batch_packed(digest, packed.data(), n);
}

int hsv_verify_device_bits(const uint8_t *d_pk, size_t pk_stride, const uint8_t *d_sig,
                           size_t sig_stride, const uint8_t *d_msg, size_t msg_stride, size_t n,
                           uint8_t *d_flags, uint32_t *d_strict_bits, void *stream) {
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
  const int variant = G().variant.load();
  const uint32_t *comb_b = nullptr;
  if (hsv_variant_needs_comb(variant)) {
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return hip_fail("hipGetDevice", e);
    if (dev < 0 || dev >= G().ndev) return fail(HSV_ERR_INVALID_ARG, "current device out of range");
    DevCtx &c = *G().ctx[dev];
    std::lock_guard<std::mutex> lk(c.mu);
    rc = ctx_prepare(c, 0, 0);
    if (rc == HSV_OK) rc = comb_table_for(c, variant, &comb_b);
    if (rc != HSV_OK) return rc;
  }
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  for (size_t base = 0; base < n; base += kChunk) {
    const size_t m = std::min(kChunk, n - base);
    hipError_t e = hsv_launch_verify(
        variant, d_pk + base * pk_stride, pk_stride, d_sig + base * sig_stride, sig_stride,
        d_msg + base * msg_stride, msg_stride, (uint32_t)m, d_flags ? d_flags + base : nullptr,
        d_strict_bits ? d_strict_bits + base / 32 : nullptr, comb_b, s);
    if (e != hipSuccess) return hip_fail("verify kernel launch", e);
  }
  return HSV_OK;
}

int hsv_verify_device(const uint8_t *d_pk, size_t pk_stride, const uint8_t *d_sig,
                      size_t sig_stride, const uint8_t *d_msg, size_t msg_stride, size_t n,
                      uint8_t *d_flags, void *stream) {
  if (!d_flags && n) return fail(HSV_ERR_INVALID_ARG, "null d_flags");
  return hsv_verify_device_bits(d_pk, pk_stride, d_sig, sig_stride, d_msg, msg_stride, n, d_flags,
                                nullptr, stream);
}

double hsv_measure_mad_peak(void) {
  if (ensure_init() != HSV_OK) return -1.0;
  int dev = 0;
  (void)hipGetDevice(&dev);
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, dev) != hipSuccess) return -1.0;
  return hsv_launch_mad_peak(prop.multiProcessorCount);
}

}  // extern "C"

// ---- committee key cache -------------------------------------------------
namespace {

}  // namespace

struct hsv_committee {
  int device = 0;
  uint32_t n = 0;
  uint8_t *d_pks = nullptr;
  uint8_t *d_kflags = nullptr;
  uint32_t *d_tables = nullptr;
  std::unordered_map<std::string, uint32_t> index;
};

extern "C" {

int hsv_committee_create(const uint8_t *pks, size_t n, hsv_committee **out) {
  if (!out || (!pks && n)) return fail(HSV_ERR_INVALID_ARG, "null argument");
  if (n > (1u << 20)) return fail(HSV_ERR_INVALID_ARG, "committee too large");
  int rc = ensure_init();
  if (rc != HSV_OK) return rc;
  int dev = 0;
  (void)hipGetDevice(&dev);
  if (dev < 0 || dev >= G().ndev) dev = 0;
  DevCtx &c = *G().ctx[dev];
  std::lock_guard<std::mutex> lk(c.mu);
  rc = ctx_prepare(c, 0, 0);
  if (rc != HSV_OK) return rc;
  rc = ensure_btable(c);
  if (rc != HSV_OK) return rc;
  hsv_committee *cm = new hsv_committee();
  cm->device = dev;
  cm->n = (uint32_t)n;
  for (size_t i = 0; i < n; ++i) cm->index.emplace(std::string(reinterpret_cast<const char *>(pks + 32 * i), 32), (uint32_t)i);
  uint32_t *d_tmp = nullptr;
  hipError_t e = hipSuccess;
  if (n) {
    e = hipMalloc(&cm->d_pks, n * 32);
    if (e == hipSuccess) e = hipMalloc(&cm->d_kflags, n);
    if (e == hipSuccess) e = hipMalloc(&cm->d_tables, n * hsv_comb_table_bytes());
    if (e == hipSuccess) e = hipMalloc(&d_tmp, hsv_comb_tmp_bytes((uint32_t)n));
    if (e == hipSuccess) e = hipMemcpy(cm->d_pks, pks, n * 32, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hsv_launch_comb_build(cm->d_pks, (uint32_t)n, 1, cm->d_tables, d_tmp, cm->d_kflags, c.stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c.stream);
    if (d_tmp) (void)hipFree(d_tmp);
  }
  if (e != hipSuccess) {
    hsv_committee_destroy(cm);
    return hip_fail("building committee tables", e);
  }
  *out = cm;
  return HSV_OK;
}

void hsv_committee_destroy(hsv_committee *cm) {
  if (!cm) return;
  if (hipSetDevice(cm->device) == hipSuccess) {
    if (cm->d_pks) (void)hipFree(cm->d_pks);
    if (cm->d_kflags) (void)hipFree(cm->d_kflags);
    if (cm->d_tables) (void)hipFree(cm->d_tables);
  }
  delete cm;
}

size_t hsv_committee_size(const hsv_committee *cm) { return cm ? cm->n : 0; }

int64_t hsv_committee_index(const hsv_committee *cm, const uint8_t pk[32]) {
  if (!cm || !pk) return -1;
  auto it = cm->index.find(std::string(reinterpret_cast<const char *>(pk), 32));
  return it == cm->index.end() ? -1 : (int64_t)it->second;
}

int hsv_committee_verify_device(const hsv_committee *cm, const uint32_t *d_key_idx, const uint8_t *d_sig,
                                size_t sig_stride, const uint8_t *d_msg, size_t msg_stride, size_t m,
                                uint8_t *d_flags, void *stream) {
  if (m == 0) return HSV_OK;
  if (!cm || !d_key_idx || !d_sig || !d_msg || !d_flags) return fail(HSV_ERR_INVALID_ARG, "null argument");
  if (((reinterpret_cast<uintptr_t>(d_sig) | reinterpret_cast<uintptr_t>(d_msg) | sig_stride | msg_stride) & 15u) != 0)
    return fail(HSV_ERR_ALIGN, "device pointers and strides must be multiples of 16");
  if (sig_stride < 64 || (msg_stride != 0 && msg_stride < 32)) return fail(HSV_ERR_INVALID_ARG, "record strides overlap");
  if (m > 0xffffffffu) return fail(HSV_ERR_INVALID_ARG, "batch too large");
  DevCtx &c = *G().ctx[cm->device];
  hipError_t e = hsv_launch_comb_verify(d_key_idx, d_sig, sig_stride, d_msg, msg_stride, (uint32_t)m, cm->d_pks,
                                        cm->d_kflags, cm->n, cm->d_tables, c.d_btable, d_flags,
                                        reinterpret_cast<hipStream_t>(stream));
  return e == hipSuccess ? HSV_OK : hip_fail("committee verify launch", e);
}

int hsv_committee_verify(hsv_committee *cm, const uint32_t *key_idx, const uint8_t *sig, const uint8_t *msg,
                         size_t msg_stride, size_t m, uint8_t *flags_out) {
  if (m == 0) return HSV_OK;
  if (!cm || !key_idx || !sig || !msg || !flags_out) return fail(HSV_ERR_INVALID_ARG, "null argument");
  if (msg_stride != 0 && msg_stride != 32) return fail(HSV_ERR_INVALID_ARG, "msg_stride must be 0 or 32");
  DevCtx &c = *G().ctx[cm->device];
  std::lock_guard<std::mutex> lk(c.mu);
  for (size_t base = 0; base < m; base += kChunk) {
    const size_t k = std::min(kChunk, m - base);
    const size_t idx_off = 0;
    const size_t sig_off = round_up(k * 4, kAlign);
    const size_t msg_off = sig_off + round_up(k * 64, kAlign);
    const size_t msg_bytes = msg_stride ? k * 32 : 32;
    const size_t flag_off = msg_off + round_up(msg_bytes, kAlign);
    const size_t total = flag_off + round_up(k, kAlign);
    int rc = ctx_prepare(c, total, total);
    if (rc != HSV_OK) return rc;
    uint8_t *h = c.h_buf;
    std::memcpy(h + idx_off, key_idx + base, k * 4);
    std::memcpy(h + sig_off, sig + base * 64, k * 64);
    std::memcpy(h + msg_off, msg + base * msg_stride, msg_bytes);
    // small batches (a QC, a vote): the kernel reads the pinned staging buffer
    // and writes the flags back through its device mapping (zero-copy), which
    // saves the two copy launches on the latency path
    void *hd = nullptr;
    if (k <= kZeroCopyMax && hipHostGetDevicePointer(&hd, h, 0) == hipSuccess && hd) {
      uint8_t *dh = static_cast<uint8_t *>(hd);
      hipError_t e = hsv_launch_comb_verify(reinterpret_cast<const uint32_t *>(dh + idx_off), dh + sig_off, 64,
                                            dh + msg_off, msg_stride ? 32 : 0, (uint32_t)k, cm->d_pks, cm->d_kflags,
                                            cm->n, cm->d_tables, c.d_btable, dh + flag_off, c.stream);
      if (e != hipSuccess) return hip_fail("committee verify launch", e);
      e = hipStreamSynchronize(c.stream);
      if (e != hipSuccess) return hip_fail("hipStreamSynchronize", e);
      std::memcpy(flags_out + base, h + flag_off, k);
      continue;
    }
    hipError_t e = hipMemcpyAsync(c.d_buf, h, msg_off + msg_bytes, hipMemcpyHostToDevice, c.stream);
    if (e != hipSuccess) return hip_fail("hipMemcpyAsync H2D", e);
    e = hsv_launch_comb_verify(reinterpret_cast<const uint32_t *>(c.d_buf + idx_off), c.d_buf + sig_off, 64,
                               c.d_buf + msg_off, msg_stride ? 32 : 0, (uint32_t)k, cm->d_pks, cm->d_kflags,
                               cm->n, cm->d_tables, c.d_btable, c.d_buf + flag_off, c.stream);
    if (e != hipSuccess) return hip_fail("committee verify launch", e);
    e = hipMemcpyAsync(h + flag_off, c.d_buf + flag_off, k, hipMemcpyDeviceToHost, c.stream);
    if (e != hipSuccess) return hip_fail("hipMemcpyAsync D2H", e);
    e = hipStreamSynchronize(c.stream);
    if (e != hipSuccess) return hip_fail("hipStreamSynchronize", e);
    std::memcpy(flags_out + base, h + flag_off, k);
  }
  return HSV_OK;
}

int hsv_committee_verify_batch_packed(hsv_committee *cm, const uint8_t digest[32], const uint8_t *votes, size_t m) {
  if (m == 0) return 1;
  if (!cm || !digest || !votes) return fail(HSV_ERR_INVALID_ARG, "null argument");
  std::vector<uint32_t> idx(m);
  std::vector<uint8_t> sigs(m * 64);
  for (size_t i = 0; i < m; ++i) {
    const int64_t k = hsv_committee_index(cm, votes + 96 * i);
    if (k < 0) return verify_batch_generic(digest, votes, 96, votes + 32, 96, m);  // a non-member key: generic kernel
    idx[i] = (uint32_t)k;
    std::memcpy(sigs.data() + 64 * i, votes + 96 * i + 32, 64);
  }
  std::vector<uint8_t> flags(m);
  int rc = hsv_committee_verify(cm, idx.data(), sigs.data(), digest, 0, m, flags.data());
  if (rc != HSV_OK) return rc;
  return batch_verdict(flags);
}

}  // extern "C"

// ---- automatic committee cache behind the drop-in verify_batch ------------
// Consensus keys are fixed per epoch (consensus/src/config.rs:39-43), so the
// keys of every QC repeat round after round.  verify_batch therefore keeps one
// committee key cache of its own: once a batch carries keys that were already
// seen in an earlier batch, it builds comb tables for the union of the cached
// keys and the batch's keys (one-time cost, ~4 ms per 1000 keys), and from
// then on batches whose keys are all cached take the committee kernels
// (four lanes per vote below 2^12 votes).  Flags are identical to the generic
// path's (tests/test_committee.py), so the verdict is unchanged.
// HSV_AUTO_COMMITTEE=0 or hsv_set_auto_committee(0) turns it off.
namespace {

constexpr size_t kAutoMaxKeys = 8192;      // 3 GiB of tables at most
constexpr size_t kCommitteeTryMax = 4096;  // hsv_verify / verify_strict batches that try the cache

struct AutoCommittee {
  std::mutex mu;
  std::shared_ptr<hsv_committee> cm;
  std::unordered_map<std::string, uint32_t> seen;  // uncached key -> batches it appeared in
  std::atomic<int> enabled{-1};                   // -1: read HSV_AUTO_COMMITTEE on first use
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

void add_batch_keys(const uint8_t *votes, size_t n, std::vector<std::string> &keys,
                    std::unordered_map<std::string, bool> &have) {
  for (size_t i = 0; i < n; ++i) {
    std::string k(reinterpret_cast<const char *>(votes + 96 * i), 32);
    if (!have.count(k)) {
      have[k] = true;
      keys.push_back(k);
    }
  }
}

// The cache to verify this batch with, or nullptr (generic path).  May build
// or rebuild the cache; rc receives an infrastructure error.
std::shared_ptr<hsv_committee> auto_committee_for(const uint8_t *votes, size_t n, int &rc) {
  rc = HSV_OK;
  AutoCommittee &a = AC();
  std::lock_guard<std::mutex> lk(a.mu);
  std::vector<std::string> missing;
  for (size_t i = 0; i < n; ++i) {
    const uint8_t *pk = votes + 96 * i;
    if (!a.cm || hsv_committee_index(a.cm.get(), pk) < 0)
      missing.emplace_back(reinterpret_cast<const char *>(pk), 32);
  }
  if (missing.empty()) return a.cm;
  bool recurring = false;
  for (const std::string &k : missing) recurring |= ++a.seen[k] >= 2;
  if (a.seen.size() > 4 * kAutoMaxKeys) a.seen.clear();
  if (!recurring) return nullptr;
  // rebuild over the cached keys and this batch's keys
  std::vector<std::string> keys;
  std::unordered_map<std::string, bool> have;
  if (a.cm) {
    for (const auto &kv : a.cm->index) {
      keys.push_back(kv.first);
      have[kv.first] = true;
    }
  }
  add_batch_keys(votes, n, keys, have);
  if (keys.size() > kAutoMaxKeys) {  // a new epoch: keep only this batch's keys
    keys.clear();
    have.clear();
    add_batch_keys(votes, n, keys, have);
  }
  std::vector<uint8_t> flat(keys.size() * 32);
  for (size_t i = 0; i < keys.size(); ++i) std::memcpy(flat.data() + 32 * i, keys[i].data(), 32);
  hsv_committee *c = nullptr;
  rc = hsv_committee_create(flat.data(), keys.size(), &c);
  if (rc != HSV_OK) return nullptr;
  a.cm = std::shared_ptr<hsv_committee>(c, [](hsv_committee *p) { hsv_committee_destroy(p); });
  a.seen.clear();
  return a.cm;
}

}  // namespace

extern "C" {

int hsv_verify_batch_packed(const uint8_t digest[32], const uint8_t *votes, size_t n) {
  if (n == 0) return 1;
  if (!digest || !votes) return fail(HSV_ERR_INVALID_ARG, "null argument");
  if (n >= 2 && auto_enabled()) {
    int rc = ensure_init();
    if (rc != HSV_OK) return rc;
    std::shared_ptr<hsv_committee> cm = auto_committee_for(votes, n, rc);
    if (rc != HSV_OK) return rc;
    if (cm) return hsv_committee_verify_batch_packed(cm.get(), digest, votes, n);
  }
  return verify_batch_generic(digest, votes, 96, votes + 32, 96, n);
}

}  // extern "C"

int auto_committee_try(const uint8_t *pk, const uint8_t *sig, const uint8_t *msg, size_t msg_stride, size_t n,
                       uint8_t *flags_out) {
  // only the latency range (a vote, a TC); large batches of fresh keys would
  // pay a hash lookup per item for nothing
  if (n > kCommitteeTryMax || !auto_enabled()) return 1;
  std::shared_ptr<hsv_committee> cm;
  {
    AutoCommittee &a = AC();
    std::lock_guard<std::mutex> lk(a.mu);
    cm = a.cm;
  }
  if (!cm) return 1;
  std::vector<uint32_t> idx(n);
  for (size_t i = 0; i < n; ++i) {
    const int64_t k = hsv_committee_index(cm.get(), pk + 32 * i);
    if (k < 0) return 1;
    idx[i] = (uint32_t)k;
  }
  return hsv_committee_verify(cm.get(), idx.data(), sig, msg, msg_stride, n, flags_out);
}

void release_auto_committee() {
  AutoCommittee &a = AC();
  std::lock_guard<std::mutex> lk(a.mu);
  a.cm.reset();
  a.seen.clear();
}

extern "C" {

int hsv_set_auto_committee(int enable) {
  AutoCommittee &a = AC();
  std::lock_guard<std::mutex> lk(a.mu);
  a.enabled.store(enable ? 1 : 0);
  if (!enable) {
    a.cm.reset();
    a.seen.clear();
  }
  return HSV_OK;
}

size_t hsv_auto_committee_size(void) {
  AutoCommittee &a = AC();
  std::lock_guard<std::mutex> lk(a.mu);
  return a.cm ? a.cm->n : 0;
}

}  // extern "C"

// ---- mempool transactions ------------------------------
// tx = message || pk (32) || sig (64); the signature is checked over
// Digest(SHA-512(message)[..32]) with Signature::verify, as in
// mempool/src/batch_maker.rs:79-85 and consensus/src/core.rs:121-127.
namespace {

constexpr size_t kTxChunkBytes = size_t(1) << 29;  // transaction bytes staged per launch

// records, verification and the short-transaction mask for m <= kChunk
// transactions already in HBM (d_offsets relative to d_txs, or NULL = fixed size)
int tx_enqueue(int variant, const uint32_t *comb_b, const uint8_t *d_txs, const uint64_t *d_offsets,
               size_t tx_size, size_t m, uint8_t *d_rec, uint8_t *d_flags, uint32_t *d_bits, hipStream_t s) {
  hipError_t e = hsv_launch_tx_records(d_txs, d_offsets, tx_size, (uint32_t)m, d_rec, s);
  if (e != hipSuccess) return hip_fail("transaction record kernel launch", e);
  e = hsv_launch_verify(variant, d_rec, 128, d_rec + 32, 128, d_rec + 96, 128, (uint32_t)m, d_flags, d_bits,
                        comb_b, s);
  if (e != hipSuccess) return hip_fail("verify kernel launch", e);
  e = hsv_launch_tx_mask(d_offsets, (uint32_t)m, d_flags, d_bits, s);
  if (e != hipSuccess) return hip_fail("transaction mask kernel launch", e);
  return HSV_OK;
}

size_t tx_bytes(const uint64_t *offsets, size_t tx_size, size_t a, size_t b) {
  return offsets ? (size_t)(offsets[b] - offsets[a]) : (b - a) * tx_size;
}

// transactions [lo, hi) of the caller's arrays on device c, chunk by chunk
int run_tx_on_device(DevCtx &c, const uint8_t *txs, const uint64_t *offsets, size_t tx_size, size_t lo,
                     size_t hi, uint8_t *flags_out) {
  std::vector<std::pair<size_t, size_t>> chunks;
  size_t max_items = 0, max_bytes = 0;
  if (!offsets) {
    const size_t per = std::max<size_t>(1, std::min(kChunk, kTxChunkBytes / tx_size));
    for (size_t a = lo; a < hi; a += per) chunks.emplace_back(a, std::min(hi, a + per));
  } else {
    for (size_t a = lo; a < hi;) {
      size_t b = a + 1;
      while (b < hi && b - a < kChunk && tx_bytes(offsets, 0, a, b + 1) <= kTxChunkBytes) ++b;
      chunks.emplace_back(a, b);
      a = b;
    }
  }
  for (auto &ch : chunks) {
    max_items = std::max(max_items, ch.second - ch.first);
    max_bytes = std::max(max_bytes, tx_bytes(offsets, tx_size, ch.first, ch.second));
  }
  // device: tx bytes | offsets | records | flags;  host: tx bytes | offsets | flags
  const size_t off_off = round_up(max_bytes, kAlign);
  const size_t rec_off = off_off + round_up((max_items + 1) * 8, kAlign);
  const size_t flag_off = rec_off + round_up(max_items * 128, kAlign);
  const size_t d_total = flag_off + round_up(max_items, kAlign);
  const size_t h_flag_off = rec_off;
  const size_t h_total = h_flag_off + round_up(max_items, kAlign);
  std::lock_guard<std::mutex> lk(c.mu);
  int rc = ctx_prepare(c, d_total, h_total);
  if (rc != HSV_OK) return rc;
  const int variant = G().variant.load();
  const uint32_t *comb_b = nullptr;
  rc = comb_table_for(c, variant, &comb_b);
  if (rc != HSV_OK) return rc;
  for (auto &ch : chunks) {
    const size_t a = ch.first, m = ch.second - ch.first;
    const size_t bytes = tx_bytes(offsets, tx_size, a, ch.second);
    const size_t first = offsets ? (size_t)offsets[a] : a * tx_size;
    uint8_t *h = c.h_buf;
    stage_copy(h, txs + first, bytes);
    size_t in_bytes = bytes;
    if (offsets) {
      uint64_t *ho = reinterpret_cast<uint64_t *>(h + off_off);
      for (size_t k = 0; k <= m; ++k) ho[k] = offsets[a + k] - offsets[a];
      in_bytes = off_off + (m + 1) * 8;
    }
    hipError_t e = hipMemcpyAsync(c.d_buf, h, in_bytes, hipMemcpyHostToDevice, c.stream);
    if (e != hipSuccess) return hip_fail("hipMemcpyAsync H2D", e);
    rc = tx_enqueue(variant, comb_b, c.d_buf, offsets ? reinterpret_cast<const uint64_t *>(c.d_buf + off_off) : nullptr,
                    tx_size, m, c.d_buf + rec_off, c.d_buf + flag_off, nullptr, c.stream);
    if (rc != HSV_OK) return rc;
    e = hipMemcpyAsync(h + h_flag_off, c.d_buf + flag_off, m, hipMemcpyDeviceToHost, c.stream);
    if (e != hipSuccess) return hip_fail("hipMemcpyAsync D2H", e);
    e = hipStreamSynchronize(c.stream);
    if (e != hipSuccess) return hip_fail("hipStreamSynchronize", e);
    std::memcpy(flags_out + (a - lo), h + h_flag_off, m);
  }
  return HSV_OK;
}

int run_tx_host(const uint8_t *txs, const uint64_t *offsets, size_t tx_size, size_t n, uint8_t *flags_out) {
  if (n == 0) return HSV_OK;
  if (!txs || !flags_out) return fail(HSV_ERR_INVALID_ARG, "null pointer");
  if (offsets) {
    for (size_t i = 0; i < n; ++i)
      if (offsets[i + 1] < offsets[i] || offsets[i + 1] - offsets[i] < 96)
        return fail(HSV_ERR_INVALID_ARG, "transaction " + std::to_string(i) + " is shorter than 96 bytes");
  } else if (tx_size < 96) {
    return fail(HSV_ERR_INVALID_ARG, "transactions are shorter than 96 bytes");
  }
  int rc = ensure_init();
  if (rc != HSV_OK) return rc;
  Global &g = G();
  const int ndev = g.ndev;
  if (ndev == 1 || n < kShardMin) return run_tx_on_device(*g.ctx[0], txs, offsets, tx_size, 0, n, flags_out);
  std::vector<int> rcs(ndev, HSV_OK);
  std::vector<std::string> errs(ndev);
  std::vector<std::thread> th;
  for (int d = 0; d < ndev; ++d) {
    const size_t lo = n * d / ndev, hi = n * (d + 1) / ndev;
    th.emplace_back([&, d, lo, hi]() {
      if (hi > lo) rcs[d] = run_tx_on_device(*g.ctx[d], txs, offsets, tx_size, lo, hi, flags_out + lo);
      if (rcs[d] != HSV_OK) errs[d] = t_last_error;
    });
  }
  for (auto &t : th) t.join();
  for (int d = 0; d < ndev; ++d)
    if (rcs[d] != HSV_OK) return fail(rcs[d], "device " + std::to_string(d) + ": " + errs[d]);
  return HSV_OK;
}

}  // namespace

extern "C" {

int hsv_set_error(int code, const char *msg) { return fail(code, msg ? msg : ""); }

int hsv_verify_transactions(const uint8_t *txs, const uint64_t *offsets, size_t n, uint8_t *flags_out) {
  if (n && !offsets) return fail(HSV_ERR_INVALID_ARG, "null offsets");
  return run_tx_host(txs, offsets, 0, n, flags_out);
}

int hsv_verify_transactions_fixed(const uint8_t *txs, size_t tx_size, size_t n, uint8_t *flags_out) {
  return run_tx_host(txs, nullptr, tx_size, n, flags_out);
}

int hsv_verify_transactions_device(const uint8_t *d_txs, const uint64_t *d_offsets, size_t tx_size, size_t n,
                                   uint8_t *d_flags, uint32_t *d_strict_bits, void *stream) {
  if (n == 0) return HSV_OK;
  if (!d_txs) return fail(HSV_ERR_INVALID_ARG, "null d_txs");
  if (!d_flags && !d_strict_bits) return fail(HSV_ERR_INVALID_ARG, "no output");
  if (!d_offsets && tx_size < 96) return fail(HSV_ERR_INVALID_ARG, "transactions are shorter than 96 bytes");
  int rc = ensure_init();
  if (rc != HSV_OK) return rc;
  const int variant = G().variant.load();
  const uint32_t *comb_b = nullptr;
  if (hsv_variant_needs_comb(variant)) {
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return hip_fail("hipGetDevice", e);
    if (dev < 0 || dev >= G().ndev) return fail(HSV_ERR_INVALID_ARG, "current device out of range");
    DevCtx &c = *G().ctx[dev];
    std::lock_guard<std::mutex> lk(c.mu);
    rc = ctx_prepare(c, 0, 0);
    if (rc == HSV_OK) rc = comb_table_for(c, variant, &comb_b);
    if (rc != HSV_OK) return rc;
  }
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const size_t per = std::min(n, kChunk);
  void *rec = nullptr;
  hipError_t e = hipMallocAsync(&rec, per * 128, s);
  if (e != hipSuccess) return hip_fail("hipMallocAsync (transaction records)", e);
  for (size_t base = 0; base < n && rc == HSV_OK; base += per) {
    const size_t m = std::min(per, n - base);
    rc = tx_enqueue(variant, comb_b, d_offsets ? d_txs : d_txs + base * tx_size,
                    d_offsets ? d_offsets + base : nullptr, tx_size, m, static_cast<uint8_t *>(rec),
                    d_flags ? d_flags + base : nullptr, d_strict_bits ? d_strict_bits + base / 32 : nullptr, s);
  }
  e = hipFreeAsync(rec, s);
  if (rc != HSV_OK) return rc;
  return e == hipSuccess ? HSV_OK : hip_fail("hipFreeAsync", e);
}

}  // extern "C"
