// Mempool transactions behind the C ABI.
// tx = message || pk (32) || sig (64); the signature is checked over
// Digest(SHA-512(message)[..32]) with Signature::verify, as in
// mempool/src/batch_maker.rs:79-85 and consensus/src/core.rs:121-127.
#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <cstring>
#include <string>
#include <thread>
#include <utility>
#include <vector>

#include "hsv.h"
#include "hsv_host.h"
#include "hsv_internal.h"

namespace hsvh {
namespace {

constexpr size_t kTxChunkBytes = size_t(1) << 29;  // transaction bytes staged per launch

// records, verification and the short-transaction mask for m <= kChunk
// transactions already in HBM (d_offsets relative to d_txs, or NULL = fixed size)
int tx_enqueue(int v, const uint32_t *comb_b, const uint8_t *d_txs, const uint64_t *d_offsets, size_t tx_size,
               size_t m, uint8_t *d_rec, uint8_t *d_flags, uint32_t *d_bits, uint32_t *d_fault, hipStream_t s) {
  hipError_t e = hsv_launch_verify_tx(v, d_txs, d_offsets, tx_size, (uint32_t)m, d_rec, d_flags, d_bits, comb_b,
                                      d_fault, s);
  if (e != hipSuccess) return hip_fail("transaction verify launch", e);
  e = hsv_launch_tx_mask(d_offsets, (uint32_t)m, d_flags, d_bits, s);
  if (e != hipSuccess) return hip_fail("transaction mask kernel launch", e);
  return HSV_OK;
}

size_t tx_bytes(const uint64_t *offsets, size_t tx_size, size_t a, size_t b) {
  return offsets ? (size_t)(offsets[b] - offsets[a]) : (b - a) * tx_size;
}

// transactions [lo, hi) of the caller's arrays on device c, chunk by chunk
int run_tx_on_device(DevCtx &c, const uint8_t *txs, const uint64_t *offsets, size_t tx_size, size_t lo, size_t hi,
                     uint8_t *flags_out) {
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
  // device: tx bytes | offsets | records | flags | self-check words;
  // host: tx bytes | offsets | flags | self-check words
  const size_t off_off = round_up(max_bytes, kAlign);
  const size_t rec_off = off_off + round_up((max_items + 1) * 8, kAlign);
  const size_t flag_off = rec_off + round_up(max_items * 128, kAlign);
  const size_t fault_off = flag_off + round_up(max_items, kAlign);
  const size_t d_total = fault_off + kAlign;
  const size_t h_flag_off = rec_off;
  const size_t h_fault_off = h_flag_off + round_up(max_items, kAlign);
  const size_t h_total = h_fault_off + kAlign;
  DeviceGuard guard(c.device);
  if (guard.status() != hipSuccess) return hip_fail("hipSetDevice", guard.status());
  const int v = variant();
  const uint32_t *comb_b = nullptr;
  int rc = comb_table_for(c, v, &comb_b);
  if (rc != HSV_OK) return rc;
  SlotLease lease(c);
  Slot &s = lease.slot();
  rc = slot_prepare(s, d_total, h_total);
  if (rc != HSV_OK) return rc;
  for (auto &ch : chunks) {
    const size_t a = ch.first, m = ch.second - ch.first;
    const size_t bytes = tx_bytes(offsets, tx_size, a, ch.second);
    const size_t first = offsets ? (size_t)offsets[a] : a * tx_size;
    uint8_t *h = s.h_buf;
    stage_copy(h, txs + first, bytes);
    size_t in_bytes = bytes;
    if (offsets) {
      uint64_t *ho = reinterpret_cast<uint64_t *>(h + off_off);
      for (size_t k = 0; k <= m; ++k) ho[k] = offsets[a + k] - offsets[a];
      in_bytes = off_off + (m + 1) * 8;
    }
    hipError_t e = hipMemcpyAsync(s.d_buf, h, in_bytes, hipMemcpyHostToDevice, s.stream);
    // unwritten flags read as rejections; self-check words start at zero
    if (e == hipSuccess) e = hipMemsetAsync(s.d_buf + flag_off, 0, fault_off + kFaultBytes - flag_off, s.stream);
    if (e != hipSuccess) {
      (void)hipStreamSynchronize(s.stream);
      return hip_fail("hipMemcpyAsync H2D", e);
    }
    rc = tx_enqueue(v, comb_b, s.d_buf, offsets ? reinterpret_cast<const uint64_t *>(s.d_buf + off_off) : nullptr,
                    tx_size, m, s.d_buf + rec_off, s.d_buf + flag_off, nullptr,
                    reinterpret_cast<uint32_t *>(s.d_buf + fault_off), s.stream);
    if (rc == HSV_OK) {
      e = hipMemcpyAsync(h + h_flag_off, s.d_buf + flag_off, fault_off + kFaultBytes - flag_off,
                         hipMemcpyDeviceToHost, s.stream);
      if (e != hipSuccess) rc = hip_fail("hipMemcpyAsync D2H", e);
    }
    e = hipStreamSynchronize(s.stream);  // nothing of this call stays in flight
    if (rc != HSV_OK) return rc;
    if (e != hipSuccess) return hip_fail("hipStreamSynchronize", e);
    rc = check_faults(h + h_fault_off, "transaction verify");
    if (rc != HSV_OK) return rc;
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
  const int k = shard_count(n);
  if (k <= 1) return run_tx_on_device(ctx(home_device()), txs, offsets, tx_size, 0, n, flags_out);
  // contiguous shards, each on the shard worker of its GPU's node
  return run_sharded(k, [&](int d, int dev) {
    const size_t lo = n * d / k, hi = n * (d + 1) / k;
    return hi > lo ? run_tx_on_device(ctx(dev), txs, offsets, tx_size, lo, hi, flags_out + lo) : HSV_OK;
  });
}

}  // namespace
}  // namespace hsvh

using namespace hsvh;

extern "C" {

int hsv_verify_transactions(const uint8_t *txs, const uint64_t *offsets, size_t n, uint8_t *flags_out) {
  CallScope call;
  if (n && !offsets) return fail(HSV_ERR_INVALID_ARG, "null offsets");
  return run_tx_host(txs, offsets, 0, n, flags_out);
}

int hsv_verify_transactions_fixed(const uint8_t *txs, size_t tx_size, size_t n, uint8_t *flags_out) {
  CallScope call;
  return run_tx_host(txs, nullptr, tx_size, n, flags_out);
}

int hsv_verify_transactions_device(const uint8_t *d_txs, const uint64_t *d_offsets, size_t tx_size, size_t n,
                                   uint8_t *d_flags, uint32_t *d_strict_bits, uint32_t *d_fault, void *stream) {
  if (n == 0) return HSV_OK;
  if (!d_txs) return fail(HSV_ERR_INVALID_ARG, "null d_txs");
  if (!d_flags && !d_strict_bits) return fail(HSV_ERR_INVALID_ARG, "no output");
  if (!d_offsets && tx_size < 96) return fail(HSV_ERR_INVALID_ARG, "transactions are shorter than 96 bytes");
  int rc = ensure_init();
  if (rc != HSV_OK) return rc;
  int dev = 0;
  rc = device_for_call(d_txs, stream, &dev);
  if (rc != HSV_OK) return rc;
  DeviceGuard guard(dev);
  if (guard.status() != hipSuccess) return hip_fail("hipSetDevice", guard.status());
  const int v = variant();
  const uint32_t *comb_b = nullptr;
  rc = comb_table_for(ctx(dev), v, &comb_b);
  if (rc != HSV_OK) return rc;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  uint32_t *fault = nullptr;
  rc = call_fault_words(ctx(dev), d_fault, s, &fault);
  if (rc != HSV_OK) return rc;
  const size_t per = std::min(n, kChunk);
  void *rec = nullptr;
  hipError_t e = hsv_ws_malloc(reinterpret_cast<void **>(&rec), per * 128, s);
  if (e != hipSuccess) return hip_fail("workspace allocation (transaction records)", e);
  for (size_t base = 0; base < n && rc == HSV_OK; base += per) {
    const size_t m = std::min(per, n - base);
    rc = tx_enqueue(v, comb_b, d_offsets ? d_txs : d_txs + base * tx_size, d_offsets ? d_offsets + base : nullptr,
                    tx_size, m, static_cast<uint8_t *>(rec), d_flags ? d_flags + base : nullptr,
                    d_strict_bits ? d_strict_bits + base / 32 : nullptr, fault, s);
  }
  e = hipFreeAsync(rec, s);
  if (rc != HSV_OK) return rc;
  return e == hipSuccess ? HSV_OK : hip_fail("hipFreeAsync", e);
}

}  // extern "C"
