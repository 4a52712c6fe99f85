// Internal interfaces between the C-ABI layer (hsv_capi.cpp) and the kernels.
#pragma once
#include <hip/hip_runtime_api.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

// Stream-ordered workspace for a launch on `stream` (current device), freed
// with hipFreeAsync on the same stream.  It comes from a memory pool the
// library owns per device, which keeps its freed blocks (release threshold
// max).  With hipMallocAsync on the default pool (release threshold 0), the
// QC latency kernel of one thread, run while another thread made the
// process's first committee-cache allocations, accepted a forged vote in 8 of
// 16 runs of tests/native/crypto_tests.cpp; with this pool, 0 of 16
// (tools/forgery_debug.sh).  The
// default-pool switch of the measurement build (HSV_WS_POOL=default) left
// the source with that build in round 5; the library always uses its own pool.
hipError_t hsv_ws_malloc(void **p, size_t bytes, hipStream_t stream);
void hsv_ws_trim(void);  // hsv_shutdown: release the pools' free blocks

// The resident latency service (hsv_committee_api.cpp) from the kernel
// launchers: pause (on = 1) / resume (on = 0) it around a device-wide wait,
// as hsvh::ResidentPause; hsvi_resident_started() is 1 once its block has run
// in this process with the service on -- the persistent point pass then
// leaves one CU's worth of blocks out of its grid, so every block of that
// grid finds a place while the resident block holds its CU.
void hsvi_resident_pause(int on);
int hsvi_resident_started(void);

// Everything declared here is internal: the library is built with
// -fvisibility=hidden, so none of it is exported from libhsv.so (only the
// HSV_API functions of include/hsv.h are).  The test and measurement hooks of
// csrc/hsv_test_hooks.h are exported by libhsv_test.so only; they call the
// hsvi_* functions below.

// Enqueue one verification launch on `stream` (no synchronisation).
int hsvi_num_variants(void);            // id space
int hsvi_variant_list(int *out, int cap);  // ids built into this library; returns their count
int hsvi_variant_available(int variant);
// fault: two device-visible words the caller zeroed before the launch; the
// kernels set fault[0] (an item's final point failed the self-check) and
// fault[1] (a workspace canary changed) -- see hsv_kernels.hip report_faults.
// Required (non-null) for the product variants.
hipError_t hsv_launch_verify(int variant, const uint8_t *pk, uint64_t pk_stride, const uint8_t *sig,
                             uint64_t sig_stride, const uint8_t *msg, uint64_t msg_stride,
                             uint32_t n, uint8_t *flags_out, uint32_t *strict_bits,
                             const uint32_t *comb_b, uint32_t *fault, hipStream_t stream);
// The same launch with a caller-provided workspace (ws, ws_cap bytes; the
// library pool is used when it is NULL or too small): a pipeline keeps one per
// stream instead of allocating per launch.  hsv_launch_ws_bytes(variant, n):
// the workspace a launch of n items needs (0 for variants without one).
hipError_t hsv_launch_verify_ws(int variant, const uint8_t *pk, uint64_t pk_stride, const uint8_t *sig,
                                uint64_t sig_stride, const uint8_t *msg, uint64_t msg_stride, uint32_t n,
                                uint8_t *flags_out, uint32_t *strict_bits, const uint32_t *comb_b, uint32_t *fault,
                                void *ws, size_t ws_cap, hipStream_t stream);
size_t hsv_launch_ws_bytes(int variant, uint32_t n);
// Fault injection (tests only; hsv_kernels.hip): the mode of the launches the
// calling thread issues (thread-scoped, so one test's injection never reaches
// another thread's calls); hsvi_set_inject returns the previous mode, or -1.
int hsvi_inject_mode(void);
int hsvi_set_inject(int mode);
// Lattice bound of the comb-path prepass (tests; 0 = default); returns the
// previous bound or -1.
int hsvi_set_lattice_bits(int bits);
// Row-form field arithmetic against the one-lane form (hsv_committee.hip).
int hsvi_lanesplit_check(const uint32_t *in, uint32_t rows, uint32_t *out);
// Read-and-clear of two device fault words in one atomic exchange each, on
// `stream`: out (device memory, 2 words) receives the old values.
hipError_t hsv_launch_fault_exchange(uint32_t *words, uint32_t *out, hipStream_t stream);
// digit width of the B comb table a variant reads: 8 (hsv_comb_table_bytes),
// 16 (the wide table, hsv_comb16_table_bytes) or 0 (none); comb_b must be
// that table for such variants
int hsv_variant_needs_comb(int variant);

// Time the v_mad_u64_u32 probe on the current device; MAC/s.
double hsv_launch_mad_peak(int device_cus);

#ifdef __cplusplus
}
#endif

// ---- committee key cache (hsv_committee.hip) -----------------------------
// Request block of the resident committee service (hsv_comb_resident_kernel,
// csrc/hsv_committee.hip), in coherent pinned host memory.  The request's
// payload (QcResidentBody, 144 words) travels in 48 chunks of 16 bytes, each
// {seq, three payload words}: the host writes a chunk's payload words, then
// its seq with a release store (x86 keeps stores in order), so a 16-byte
// read that finds the new seq in a chunk finds that chunk's new payload.  The
// kernel polls all 48 chunks with ONE vector load (one 16-byte read per lane)
// and takes the request once every chunk carries the same new seq -- the
// doorbell and the body in one PCIe round trip, no acquire fence.  It answers
// with two 8-byte stores {seq, flags} and {seq, fault bits}, each a single
// transaction, so the host needs no fence on its side either.
constexpr int kResidentVotes = 4;
struct QcResidentBody {                  // 144 words, offsets fixed (the kernel reads them raw)
  uint32_t m, nkeys, inject, msg_per_vote;  // votes (1..kResidentVotes), members, fault injection, 0/1
  const uint8_t *pks;                    // the committee view's device arrays
  const uint8_t *key_flags;
  const uint32_t *const *key_tables;
  const uint32_t *btable;
  uint32_t key_idx[kResidentVotes];      // word 12
  uint32_t sig[kResidentVotes][16];      // word 16: R || s per vote
  uint32_t msg[kResidentVotes][8];       // word 80: one digest per vote, or the shared digest in msg[0]
  uint32_t pk[kResidentVotes][8];        // word 112: each vote's key encoding (the member's, byte for byte)
};
constexpr int kResidentChunks = 48;      // 3 payload words each
static_assert(sizeof(QcResidentBody) == kResidentChunks * 3 * 4, "48 chunks of three words");
struct alignas(16) QcResidentChunk {
  uint32_t seq, w[3];
};
// answer bits besides the flags: bit 0 / 1 the self-check words of the
// launched form (curve check, canary), bit 2 the request header was refused
constexpr uint32_t kResidentFaultCurve = 1u, kResidentFaultCanary = 2u, kResidentBadRequest = 4u;
struct QcResidentReq {
  uint32_t stop, alive, pad0[14];        // host: stop word; kernel: set while it runs
  QcResidentChunk chunk[64];             // [0, kResidentChunks): the request
  uint64_t answer[2];                    // kernel: seq | flags << 32, seq | fault bits << 32
  uint32_t pad1[12];
};

#ifdef __cplusplus
extern "C" {
#endif
hipError_t hsv_launch_comb_resident(QcResidentReq *d_req, uint64_t idle_ticks, hipStream_t stream);
uint32_t hsv_comb_resident_votes(void);  // votes one request may hold (0: no service in this build)
hipError_t hsv_launch_comb_build(const uint8_t *encs, uint32_t nkeys, uint32_t negate, uint32_t *tables,
                                 uint32_t *tmp, uint8_t *key_flags, hipStream_t stream);
// key_tables[i]: device pointer to key i's comb table (hsv_comb_table_bytes)
hipError_t hsv_launch_comb_verify(const uint32_t *key_idx, const uint8_t *sig, uint64_t sig_stride,
                                  const uint8_t *msg, uint64_t msg_stride, uint32_t m, const uint8_t *pks,
                                  const uint8_t *key_flags, uint32_t nkeys, const uint32_t *const *key_tables,
                                  const uint32_t *btable, uint8_t *flags_out, uint32_t *fault, uint32_t *done,
                                  hipStream_t stream);
// Completion markers of the latency form (done != NULL above, m votes): one
// word per block, set to 1 by the block once its flags are released to the
// system; 0 when m is above the latency form's range (no markers).
uint32_t hsv_comb_marker_blocks(uint32_t m);
uint64_t hsv_comb_table_bytes(void);
uint64_t hsv_comb_tmp_bytes(uint32_t nkeys);
// wide (16-bit digit) comb table of B, hsv_comb.hpp
hipError_t hsv_launch_comb16_build(uint32_t *table, uint32_t *tmp, hipStream_t stream);
uint64_t hsv_comb16_table_bytes(void);
uint64_t hsv_comb16_tmp_bytes(void);
#ifdef __cplusplus
}
#endif

// ---- mempool transactions (hsv_mempool.hip) -------------------------------
#ifdef __cplusplus
extern "C" {
#endif
// 128-byte records pk || R || s || SHA-512(message)[..32] for n transactions
// (offsets[i]..offsets[i+1] of txs, or fixed tx_size when offsets is NULL).
hipError_t hsv_launch_tx_records(const uint8_t *txs, const uint64_t *offsets, uint64_t tx_size, uint32_t n,
                                 uint8_t *records, hipStream_t stream);
// The same records plus the point pass's scalar prepass on them (one read of
// each transaction): prep = the SoA prepass records (kPrepWords words per
// item, row stride n), items without a short lattice pair appended to fb_list
// through *fb_count.  Used by hsv_launch_verify_tx.
hipError_t hsv_launch_tx_prep(const uint8_t *txs, const uint64_t *offsets, uint64_t tx_size, uint32_t n,
                              uint8_t *records, uint32_t *prep, uint32_t *fb_count, uint32_t *fb_list,
                              int lat_bits, hipStream_t stream);
// Records, prepass and point pass in ONE persistent launch (hsv_mempool.hip,
// hsv_verify_tx_fused_kernel): grid = the point pass's persistent grid
// (hsv_tx_fused_blocks_per_cu blocks per CU), ctr = the zeroed HcCounters,
// ready = nbatch = ceil(n / 64) zeroed words, vt_ws / canary as
// hsv_verify_hp_kernel's.  n * 128 must stay below 2^32.
int hsv_tx_fused_blocks_per_cu(int device);
hipError_t hsv_launch_tx_fused(uint32_t grid, const uint8_t *txs, const uint64_t *offsets, uint64_t tx_size,
                               uint32_t n, uint8_t *records, uint32_t *rec, void *ctr, uint32_t *fb_list,
                               uint32_t *ready, int lat_bits, uint8_t *flags_out, uint32_t *strict_bits, void *vt_ws,
                               const uint32_t *comb_b, uint32_t *canary, uint32_t nonce, uint32_t inject,
                               uint32_t *fault, hipStream_t stream);
// Transactions end to end: records (128 B per item, caller's buffer) and
// verification, fused as above for large batches of the product variants;
// otherwise hsv_launch_tx_records + hsv_launch_verify.
hipError_t hsv_launch_verify_tx(int variant, const uint8_t *txs, const uint64_t *offsets, uint64_t tx_size,
                                uint32_t n, uint8_t *records, uint8_t *flags_out, uint32_t *strict_bits,
                                const uint32_t *comb_b, uint32_t *fault, hipStream_t stream);
// flags 0 (and STRICT_OK bit cleared) for transactions shorter than 96 bytes
hipError_t hsv_launch_tx_mask(const uint64_t *offsets, uint32_t n, uint8_t *flags, uint32_t *strict_bits,
                              hipStream_t stream);
#ifdef __cplusplus
}
#endif

// ---- error reporting shared by the C-ABI translation units -----------------
#ifdef __cplusplus
extern "C" {
#endif
// sets hsv_last_error() on the calling thread; returns code
int hsvi_set_error(int code, const char *msg);
// test hooks of hsv_capi.cpp (exported as hsv_set_* by libhsv_test.so only)
int hsvi_set_virtual_shards(int k);
int hsvi_set_pipe_nocopy(int on);  // hsv_test_pipe_nocopy (libhsv_test.so only)
int hsvi_set_pipe_schedule(const uint64_t *sizes, int count);  // hsv_test_pipe_schedule
int hsvi_set_variant(int v);
#ifdef __cplusplus
}
#endif
