// gfx950 kernels of the Ed25519 batch verifier.
//
//  hsv_verify_kernel   one verification per lane (see hsv_verify_core.hpp);
//                      the [1..256]B Niels table (24 KiB) is staged in LDS
//                      once per workgroup; inputs are read with 16-byte loads
//                      straight from the caller's layout (strided records).
//  hsv_mad_peak_kernel issue-rate probe of v_mad_u64_u32 for the roofline
//                      denominator (bench.py reports against it).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <type_traits>
#include <atomic>
#include <mutex>
#include <unordered_map>

#include "hsv_internal.h"
#include "hsv_verify_core.hpp"
#include "hsv_verify_hc.hpp"
#include "hsv_rowpoint.hpp"
#include "hsv_pointpass.hpp"

namespace hsv {

#ifdef HSV_PHASE_CLOCKS  // tools/phase_clock_probe.py only: 8 words per 64-item batch of the point pass
constexpr uint32_t kPhaseCap = 1u << 16;
__device__ uint64_t g_phase_clk[kPhaseCap * 8];
#endif

// Two-pass form (hsv_verify_hc.hpp, prep_scalars / verify_one_prepped).
// Pass 1: one lane per item, scalar work only; records to `rec` (SoA, row
// stride n), fallback items appended to fb_list.
template <int WA>
__global__ void __launch_bounds__(kBlock)
hsv_prep_kernel(const uint8_t *__restrict__ pk, uint64_t pk_stride, const uint8_t *__restrict__ sig,
                uint64_t sig_stride, const uint8_t *__restrict__ msg, uint64_t msg_stride, uint32_t n,
                uint32_t *__restrict__ rec, HcCounters *__restrict__ ctr, uint32_t *__restrict__ fb_list,
                int lat_bits) {
  // The prepass usually runs beside the previous batch's point pass (another
  // stream, or the previous chunk of a host pipeline), whose waves keep every
  // SIMD's VALU busy; this batch's point pass cannot start before the prepass
  // ends.  Highest wave priority: the SIMD issues the prepass's waves first.
  __builtin_amdgcn_s_setprio(3);
  const uint32_t idx = blockIdx.x * kBlock + threadIdx.x;
  if (idx >= n) return;
  uint32_t pkw[8], sigw[16], msgw[8];
  load_triple(pk, pk_stride, sig, sig_stride, msg, msg_stride, idx, pkw, sigw, msgw);
  if (prep_scalars<WA>(pkw, sigw, msgw, rec + idx, n, lat_bits)) fb_list[atomicAdd(&ctr->fb_count, 1u)] = idx;
}

// Pass 2: persistent grid, 64-item batches from ctr->next over a virtual
// range [fallback items | all items].  Fallback batches come first and run
// the full-length path; in the regular range a fallback item's lane computes
// nothing it stores.  strict_bits is zeroed before the launch and every
// batch ORs its bits in (a word can receive bits from both ranges).
template <int WA, int WAVES, int CB>
__global__ void __launch_bounds__(kBlock, WAVES)
hsv_verify_hp_kernel(const uint8_t *__restrict__ pk, uint64_t pk_stride, const uint8_t *__restrict__ sig,
                     uint64_t sig_stride, const uint8_t *__restrict__ msg, uint64_t msg_stride, uint32_t n,
                     uint8_t *__restrict__ flags_out, uint32_t *__restrict__ strict_bits,
                     uint4 *__restrict__ vt_ws, const uint32_t *__restrict__ comb_b,
                     const uint32_t *__restrict__ rec, HcCounters *__restrict__ ctr,
                     const uint32_t *__restrict__ fb_list, uint32_t *__restrict__ canary, uint32_t nonce,
                     uint32_t inject, uint32_t *__restrict__ fault) {
  constexpr int kEnt = (1 << (WA - 1)) + 1;
  const uint32_t slot = blockIdx.x * kBlock + threadIdx.x;
  GlobalVarTab<kEnt> vt{vt_ws + (uint64_t)slot * vt_lane_uint4<WA>(), inject};
  const uint32_t lane = threadIdx.x & 63u;
  canary[slot] = nonce;
  uint32_t bad = 0;
  const uint32_t nfb = __builtin_amdgcn_readfirstlane(ctr->fb_count);
  const uint32_t fb_end = (nfb + 63u) & ~63u;
  const uint32_t words = (n + 31u) / 32u;
#ifdef HSV_PHASE_CLOCKS
  uint32_t nbw = 0;  // batches this wave has taken
#endif
  for (;;) {
    uint32_t base = 0;
    if (lane == 0) base = atomicAdd(&ctr->next, 64u);
    base = __builtin_amdgcn_readfirstlane(__shfl(base, 0));
    if (base >= fb_end + n) break;
    if (inject == kInjectCanary) canary[slot] = ~nonce;
    if (base < fb_end) {
      const uint32_t j = base + lane;
      const bool valid = j < nfb;
      const uint32_t idx = fb_list[valid ? j : base];
      uint32_t pkw[8], sigw[16], msgw[8];
      load_triple(pk, pk_stride, sig, sig_stride, msg, msg_stride, idx, pkw, sigw, msgw);
      const uint32_t f = verify_one_full_comb<WA, false, CB>(pkw, sigw, msgw, comb_b, vt);
      bad |= ((f & kFault) ? 1u : 0u) | (canary[slot] != nonce ? 2u : 0u);
      if (valid) {
        if (flags_out) flags_out[idx] = (uint8_t)f;
        if (strict_bits && (f & kStrictOk)) atomicOr(&strict_bits[idx >> 5], 1u << (idx & 31u));
      }
      continue;
    }
    const uint32_t b0 = base - fb_end;
    const uint32_t idx = b0 + lane;
    const bool valid = idx < n;
    const uint32_t li = valid ? idx : n - 1u;
    uint32_t pkw[8], rw[8];
    {
      const uint4 *p = reinterpret_cast<const uint4 *>(pk + (uint64_t)li * pk_stride);
      const uint4 *r = reinterpret_cast<const uint4 *>(sig + (uint64_t)li * sig_stride);
      const uint4 p0 = p[0], p1 = p[1], r0 = r[0], r1 = r[1];
      pkw[0] = p0.x; pkw[1] = p0.y; pkw[2] = p0.z; pkw[3] = p0.w;
      pkw[4] = p1.x; pkw[5] = p1.y; pkw[6] = p1.z; pkw[7] = p1.w;
      rw[0] = r0.x; rw[1] = r0.y; rw[2] = r0.z; rw[3] = r0.w;
      rw[4] = r1.x; rw[5] = r1.y; rw[6] = r1.z; rw[7] = r1.w;
    }
    const uint32_t meta = rec[18ull * n + li];
    const bool own = valid && !(meta & kPrepFallback);
#ifdef HSV_PHASE_CLOCKS
    uint64_t clk[5];
    ++nbw;
    const uint64_t cyc0 = clock64();
    clk[0] = wall_clock64();
    const uint32_t f = verify_one_prepped<WA, CB>(pkw, rw, rec + li, n, meta, comb_b, vt, clk);
    clk[4] = wall_clock64();
    {  // lanes 0..7 store one word each (one store region keeps the work loop uniform)
      uint64_t v = 1;
      HSV_UNROLL
      for (int j = 0; j < 5; ++j) v = lane == (uint32_t)j ? clk[j] : v;
      v = lane == 5u ? (uint64_t)__builtin_amdgcn_s_getreg((31 << 11) | (0 << 6) | 4) : v;  // HW_ID
      v = lane == 6u ? ((uint64_t)blockIdx.x << 8 | nbw) : v;
      v = lane == 7u ? (0x100u | (uint64_t)__builtin_amdgcn_s_getreg((3 << 11) | (0 << 6) | 20) |  // XCC_ID
                        ((clock64() - cyc0) << 16))  // shader clocks over the batch
                     : v;
      if (lane < 8u && b0 / 64u < kPhaseCap) g_phase_clk[(uint64_t)(b0 / 64u) * 8u + lane] = v;
    }
#else
    const uint32_t f = verify_one_prepped<WA, CB>(pkw, rw, rec + li, n, meta, comb_b, vt);
#endif
    bad |= ((f & kFault) ? 1u : 0u) | (canary[slot] != nonce ? 2u : 0u);
    if (own && flags_out) flags_out[idx] = (uint8_t)f;
    if (strict_bits) {
      const uint64_t mask = __ballot(own && (f & kStrictOk));
      const uint32_t w = b0 / 32u + lane;
      const uint32_t part = lane ? (uint32_t)(mask >> 32) : (uint32_t)mask;
      if (lane < 2u && w < words && part) atomicOr(&strict_bits[w], part);
    }
  }
  report_faults(fault, bad);
}

// ---- streamed host batches (round 4) ---------------------------------------
// (Round 4 also had a streamed host form here: one persistent launch reading
// the records through the pinned staging's device mapping while the host was
// still packing them.  It measured slower than the chunked copy pipeline,
// 11.7 against 9.9 ms per 2^20 (profiles/r04d_host_api_ab.txt), and was
// removed from the library in round 5; it is in git history at 394d4d2.)

// ---- latency form for small batches: two lanes per item ------------------
// A lone wave issues one VALU instruction per 4 clocks whatever its lane
// count, so a QC of 67 or 667 votes costs one verification's instruction
// count end to end.  Here the even lane of a pair owns R and the odd lane A:
// each decompresses its own point, builds its own table, runs a one-scalar
// Straus loop (c1 for R, |c0| for A: 34 windows, 4 doublings + 1 addition)
// and half of the wide B comb (digits 0-7 / 8-15); the two partial sums meet
// through a lane swap and one addition.  Per lane that is one root chain
// instead of two and half the additions, with the same 136 doublings.

// q += sum of comb digits [8h, 8h + 8) of s (CB = 16) or [16h, 16h + 16) (CB = 8)
template <int CB>
__device__ __forceinline__ ge_ext comb_add_b_half(ge_ext q, const uint32_t s[8], const uint32_t *tb, uint32_t h) {
  constexpr int NP = 256 / CB, HALF = NP / 2;
  constexpr int ENT = 1 << (CB - 1);
  uint32_t sr[9];
  recode_add<9, CB, NP>(s, 8, sr);
  HSV_UNROLL
  for (int i = 0; i < 4; ++i) sr[i] = h ? sr[i + 4] : sr[i];  // the upper 128 bits for h = 1
  HSV_NOUNROLL
  for (int j = 0; j < HALF; ++j) {
    const uint32_t cb = sr[0] & ((1u << CB) - 1u);
    HSV_UNROLL
    for (int i = 0; i < 3; ++i) sr[i] = (sr[i] >> CB) | (sr[i + 1] << (32 - CB));
    sr[3] >>= CB;
    const CombPosTab tpb{tb + (uint64_t)(j + (int)h * HALF) * ENT * kCombEntryWords};
    q = ge_add_niels<true>(q, select_niels<CB>(tpb, cb));
  }
  return q;
}

__device__ __forceinline__ fe fe_swap_pair(const fe &a) {
  fe r;
  HSV_UNROLL
  for (int i = 0; i < kFeLimbs; ++i) r.v[i] = (uint32_t)__shfl_xor((int)a.v[i], 1, 64);
  return r;
}

// Pair-lane point pass of a prepped (non-fallback) item, in two phases; both
// lanes of the pair return the item's flag byte.  p = lane parity: 0 owns R,
// 1 owns A.  Phase 1 needs only the point: decompression and its table.
template <int WA, class VT>
__device__ __forceinline__ void pair_point_phase(uint32_t p, const uint32_t pk[8], const uint32_t rb[8], VT &vt,
                                                 uint32_t &ok, uint32_t &small) {
  constexpr int TS = 1 << (WA - 1);
  uint32_t pt[8];
  HSV_UNROLL
  for (int i = 0; i < 8; ++i) pt[i] = p ? pk[i] : rb[i];
  fe x, y;
  ok = ge_decompress(pt, x, y);
  small = ok & y_is_small_order(y);
  vt_build<TS>(vt, 0, fe_carry(fe_neg(x)), y);
}

// Phase 2: the scalars from the prepass record (word j of the item at
// rec[j * stride]), one-scalar Straus, half of the B comb, the lane swap.
template <int WA, int CB, class VT>
__device__ __forceinline__ uint32_t pair_scalar_phase(uint32_t p, uint32_t ok, uint32_t small, const uint32_t *rec,
                                                      uint64_t stride, uint32_t meta, const uint32_t *tb, VT &vt) {
  using G = HalfCombWindows<WA>;
  uint32_t d[1][5];
  HSV_UNROLL
  for (int i = 0; i < 5; ++i) d[0][i] = rec[(uint64_t)(i + 5 * (int)p) * stride];
  ge_ext q = straus_vt<WA, G::NW, 5, 1, false>(d, vt, (p && (meta & kPrepC0Neg)) ? 1u : 0u);
  uint32_t b[8];
  HSV_UNROLL
  for (int i = 0; i < 8; ++i) b[i] = rec[(10 + i) * stride];
  q = comb_add_b_half<CB>(q, b, tb, p);
  ge_ext o;
  o.X = fe_swap_pair(q.X);
  o.Y = fe_swap_pair(q.Y);
  o.Z = fe_swap_pair(q.Z);
  o.T = fe_swap_pair(q.T);
  q = ge_add_cached_rt(q, ge_to_cached(o), false);
  const uint32_t ok_o = (uint32_t)__shfl_xor((int)ok, 1, 64), small_o = (uint32_t)__shfl_xor((int)small, 1, 64);
  const uint32_t r_ok = p ? ok_o : ok, small_r = p ? small_o : small;
  const uint32_t a_ok = p ? ok : ok_o, small_a = p ? small : small_o;
  const uint32_t same = ge_is_neutral(q);
  return flags_byte(meta & kPrepSOk, a_ok, r_ok, small_a, small_r, same) | fault_bit(a_ok, r_ok, q);
}

template <int WA, int CB, class VT>
__device__ __forceinline__ uint32_t verify_pair_prepped(uint32_t p, const uint32_t pk[8], const uint32_t rb[8],
                                                        const uint32_t *rec, uint64_t stride, uint32_t meta,
                                                        const uint32_t *tb, VT &vt) {
  uint32_t ok, small;
  pair_point_phase<WA>(p, pk, rb, vt, ok, small);
  return pair_scalar_phase<WA, CB>(p, ok, small, rec, stride, meta, tb, vt);
}

// Pass 2 of the latency form: a plain grid of 2n lanes; lane t works on item
// t / 2.  Fallback items (no short lattice pair) run the full-length path on
// both lanes of their pair.
template <int WA, int CB>
__global__ void __launch_bounds__(kBlock)
hsv_verify_pair_kernel(const uint8_t *__restrict__ pk, uint64_t pk_stride, const uint8_t *__restrict__ sig,
                       uint64_t sig_stride, const uint8_t *__restrict__ msg, uint64_t msg_stride, uint32_t n,
                       uint8_t *__restrict__ flags_out, uint32_t *__restrict__ strict_bits,
                       uint4 *__restrict__ vt_ws, const uint32_t *__restrict__ comb_b,
                       const uint32_t *__restrict__ rec) {
  constexpr int kEnt = (1 << (WA - 1)) + 1;
  const uint32_t t = blockIdx.x * kBlock + threadIdx.x;
  GlobalVarTab<kEnt> vt{vt_ws + (uint64_t)t * vt_lane_uint4<WA>()};
  const uint32_t p = t & 1u, idx = t >> 1;
  const bool valid = idx < n;
  const uint32_t li = valid ? idx : n - 1u;
  const uint32_t meta = rec[18ull * n + li];
  uint32_t f;
  if (meta & kPrepFallback) {
    uint32_t pkw[8], sigw[16], msgw[8];
    load_triple(pk, pk_stride, sig, sig_stride, msg, msg_stride, li, pkw, sigw, msgw);
    f = verify_one_full_comb<WA, false, CB>(pkw, sigw, msgw, comb_b, vt);
  } else {
    uint32_t pkw[8], rw[8];
    const uint4 *pp = reinterpret_cast<const uint4 *>(pk + (uint64_t)li * pk_stride);
    const uint4 *rp = reinterpret_cast<const uint4 *>(sig + (uint64_t)li * sig_stride);
    const uint4 p0 = pp[0], p1 = pp[1], r0 = rp[0], r1 = rp[1];
    pkw[0] = p0.x; pkw[1] = p0.y; pkw[2] = p0.z; pkw[3] = p0.w;
    pkw[4] = p1.x; pkw[5] = p1.y; pkw[6] = p1.z; pkw[7] = p1.w;
    rw[0] = r0.x; rw[1] = r0.y; rw[2] = r0.z; rw[3] = r0.w;
    rw[4] = r1.x; rw[5] = r1.y; rw[6] = r1.z; rw[7] = r1.w;
    f = verify_pair_prepped<WA, CB>(p, pkw, rw, rec + li, n, meta, comb_b, vt);
  }
  if (valid && p == 0u) {
    if (flags_out) flags_out[idx] = (uint8_t)f;
    if (strict_bits && (f & kStrictOk)) atomicOr(&strict_bits[idx >> 5], 1u << (idx & 31u));
  }
}

// Latency form in ONE launch (default at <= kPairMax items): a block of three
// waves takes 64 items.  Waves 0 and 1 run the pair form's point phase (two
// lanes per item: decompress R or A, build its table) while wave 2 runs the
// scalar prepass of the same 64 items (SHA-512, k mod l, lattice reduction,
// recoding) into an LDS record.  The waves run on different SIMDs, so the
// prepass's latency hides behind the root chains; after the barrier the pair
// waves read their scalars from LDS.  Fallback items run the full-length path
// on both lanes of their pair.
constexpr int kFusedItems = 64;
template <int WA, int CB>
__global__ void __launch_bounds__(3 * 64)
hsv_verify_pair_fused_kernel(const uint8_t *__restrict__ pk, uint64_t pk_stride, const uint8_t *__restrict__ sig,
                             uint64_t sig_stride, const uint8_t *__restrict__ msg, uint64_t msg_stride, uint32_t n,
                             uint8_t *__restrict__ flags_out, uint32_t *__restrict__ strict_bits,
                             uint4 *__restrict__ vt_ws, const uint32_t *__restrict__ comb_b, int lat_bits,
                             uint32_t *__restrict__ canary, uint32_t nonce, uint32_t inject,
                             uint32_t *__restrict__ fault) {
  constexpr int kEnt = (1 << (WA - 1)) + 1;
  __shared__ uint32_t srec[kPrepWords * kFusedItems];
  const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63u;
  const uint32_t base = blockIdx.x * kFusedItems;
  const uint32_t t = threadIdx.x;  // pair lanes: t < 128
  const uint32_t p = t & 1u, item = base + (t >> 1);
  const uint32_t slot = blockIdx.x * 2u * kFusedItems + (t & 127u);
  GlobalVarTab<kEnt> vt{vt_ws + (uint64_t)slot * vt_lane_uint4<WA>(), inject};
  if (wave < 2) canary[slot] = inject == kInjectCanary ? ~nonce : nonce;
  uint32_t ok = 0, small = 0;
  if (wave == 2) {
    const uint32_t li = base + lane < n ? base + lane : n - 1u;
    uint32_t pkw[8], sigw[16], msgw[8];
    load_triple(pk, pk_stride, sig, sig_stride, msg, msg_stride, li, pkw, sigw, msgw);
    (void)prep_scalars<WA>(pkw, sigw, msgw, srec + lane, kFusedItems, lat_bits);
  } else {
    const uint32_t li = item < n ? item : n - 1u;
    uint32_t pkw[8], rw[8];
    const uint4 *pp = reinterpret_cast<const uint4 *>(pk + (uint64_t)li * pk_stride);
    const uint4 *rp = reinterpret_cast<const uint4 *>(sig + (uint64_t)li * sig_stride);
    const uint4 p0 = pp[0], p1 = pp[1], r0 = rp[0], r1 = rp[1];
    pkw[0] = p0.x; pkw[1] = p0.y; pkw[2] = p0.z; pkw[3] = p0.w;
    pkw[4] = p1.x; pkw[5] = p1.y; pkw[6] = p1.z; pkw[7] = p1.w;
    rw[0] = r0.x; rw[1] = r0.y; rw[2] = r0.z; rw[3] = r0.w;
    rw[4] = r1.x; rw[5] = r1.y; rw[6] = r1.z; rw[7] = r1.w;
    pair_point_phase<WA>(p, pkw, rw, vt, ok, small);
  }
  __syncthreads();
  if (wave == 2) return;
  const uint32_t il = t >> 1;
  const uint32_t meta = srec[(kPrepWords - 1) * kFusedItems + il];
  uint32_t f;
  const uint32_t li = item < n ? item : n - 1u;
  if (meta & kPrepFallback) {
    uint32_t pkw[8], sigw[16], msgw[8];
    load_triple(pk, pk_stride, sig, sig_stride, msg, msg_stride, li, pkw, sigw, msgw);
    f = verify_one_full_comb<WA, false, CB>(pkw, sigw, msgw, comb_b, vt);
  } else {
    f = pair_scalar_phase<WA, CB>(p, ok, small, srec + il, kFusedItems, meta, comb_b, vt);
  }
  report_faults(fault, ((f & kFault) ? 1u : 0u) | (canary[slot] != nonce ? 2u : 0u));
  if (item < n && p == 0u) {
    if (flags_out) flags_out[item] = (uint8_t)f;
    if (strict_bits && (f & kStrictOk)) atomicOr(&strict_bits[item >> 5], 1u << (item & 31u));
  }
}

// Row form of the latency kernel (default at <= kRowMax items): every field
// product of a verification spread over a 16-lane DPP row (hsv_rowpoint.hpp),
// two rows per item as the pair form's two lanes.  A block of four waves takes
// 6 items (RR = 1): waves 0-2 hold 12 rows (row 2i decompresses R of item i and
// builds [0..8](-R), row 2i + 1 the same for A, tables in LDS), wave 3 runs the
// scalar prepass of the block's items into an LDS record meanwhile.  After the
// barrier each row runs its one-scalar Straus (c1 for R, |c0| for A) and half
// of the B comb; the two rows of an item swap their sums (lane ^ 16) and add
// them.  Fallback items (no short lattice pair) run the full-length one-lane
// path on lane 0 of their R row.  Same flags, self-checks and canaries as the
// pair form.  RR = 2 (late round 3): every element over a pair of rows
// (RowLane2, hsv_fe16x16.hpp), so a block takes 3 items: rows 4i, 4i + 1 hold
// R of item i, rows 4i + 2, 4i + 3 hold A, and the R and A pairs swap their
// sums at lane ^ 32.
constexpr int kRowRows = 12;
template <int RR>
constexpr int kRowItemsOf = kRowRows / (2 * RR);
template <int WA, int CB, int RR>
__global__ void __launch_bounds__(4 * 64)
hsv_verify_row_kernel(const uint8_t *__restrict__ pk, uint64_t pk_stride, const uint8_t *__restrict__ sig,
                      uint64_t sig_stride, const uint8_t *__restrict__ msg, uint64_t msg_stride, uint32_t n,
                      uint8_t *__restrict__ flags_out, uint32_t *__restrict__ strict_bits,
                      uint4 *__restrict__ vt_ws, const uint32_t *__restrict__ comb_b, int lat_bits,
                      uint32_t *__restrict__ canary, uint32_t nonce, uint32_t inject, uint32_t *__restrict__ fault) {
  using G = HalfCombWindows<WA>;
  constexpr int TS = 1 << (WA - 1);
  constexpr int kEnt = TS + 1;
  constexpr int kRowItems = kRowItemsOf<RR>;
  __shared__ uint32_t srec[kPrepWords * kRowItems];
  __shared__ uint32_t stab[kRowRows * kEnt * 64];
  const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63u;
  const uint32_t base = blockIdx.x * kRowItems;
  if (wave == 3) {
    if (lane < (uint32_t)kRowItems) {
      const uint32_t li = base + lane < n ? base + lane : n - 1u;
      uint32_t pkw[8], sigw[16], msgw[8];
      load_triple(pk, pk_stride, sig, sig_stride, msg, msg_stride, li, pkw, sigw, msgw);
      (void)prep_scalars<WA>(pkw, sigw, msgw, srec + lane, kRowItems, lat_bits);
    }
    __syncthreads();
    return;
  }
  const std::conditional_t<RR == 2, RowLane2, RowLane> L;
  const uint32_t rb = wave * 4u + (lane >> 4);  // row of the block
  const uint32_t el = rb / RR;                  // element (row or row pair) of the block
  const uint32_t il = el >> 1, role = el & 1u;  // role 0: R, 1: A
  const bool lead = rb % RR == 0u;              // the row that reports (one of a pair)
  constexpr int kSwap = 16 * RR;
  const uint32_t item = base + il;
  const uint32_t li = item < n ? item : n - 1u;
  const uint32_t slot = blockIdx.x * (uint32_t)kRowRows + rb;
  canary[slot] = inject == kInjectCanary ? ~nonce : nonce;
  uint32_t ok, small, nc = 0;
  uint32_t *tab = stab + rb * (uint32_t)(kEnt * 64);
  {
    uint32_t enc[8];
    const uint4 *ep = reinterpret_cast<const uint4 *>(role ? pk + (uint64_t)li * pk_stride : sig + (uint64_t)li * sig_stride);
    const uint4 e0 = ep[0], e1 = ep[1];
    enc[0] = e0.x; enc[1] = e0.y; enc[2] = e0.z; enc[3] = e0.w;
    enc[4] = e1.x; enc[5] = e1.y; enc[6] = e1.z; enc[7] = e1.w;
    fe x, y;
    ok = ge_decompress_row(enc, x, y, small, nc, L);
    small &= ok;
    row_table_build<TS>(tab, x, y, L, inject, role == 0u);
  }
  __syncthreads();
  const uint32_t meta = srec[(kPrepWords - 1) * kRowItems + il];
  uint32_t f = 0, bad = 0;
  if (meta & kPrepFallback) {
    if (role == 0u && L.k == 0u && lead) {
      GlobalVarTab<kEnt> vt{vt_ws + (uint64_t)slot * vt_lane_uint4<WA>(), inject};
      uint32_t pkw[8], sigw[16], msgw[8];
      load_triple(pk, pk_stride, sig, sig_stride, msg, msg_stride, li, pkw, sigw, msgw);
      f = verify_one_full_comb<WA, false, CB>(pkw, sigw, msgw, comb_b, vt);
      bad = (f & kFault) ? 1u : 0u;
    }
  } else {
    uint32_t d[5];
    HSV_UNROLL
    for (int i = 0; i < 5; ++i) d[i] = srec[(i + 5 * (int)role) * kRowItems + il];
    rp_ext q = row_straus<WA, G::NW>(d, tab, (role && (meta & kPrepC0Neg)) ? 1u : 0u, L);
    uint32_t b[8];
    HSV_UNROLL
    for (int i = 0; i < 8; ++i) b[i] = srec[(10 + i) * kRowItems + il];
    q = row_comb_half<CB>(q, b, comb_b, role, L);
    // both rows of the item end with the whole sum Q
    q = rp_add_cached(q, rp_to_cached(rp_swap_rows(q, kSwap), fl_from_fe(fe_d2(), L), L), false, L);
    const uint32_t ok_o = (uint32_t)__shfl_xor((int)ok, kSwap, 64);
    const uint32_t small_o = (uint32_t)__shfl_xor((int)small, kSwap, 64);
    const uint32_t r_ok = role ? ok_o : ok, small_r = role ? small_o : small;
    const uint32_t a_ok = role ? ok : ok_o, small_a = role ? small : small_o;
    ge_ext qe;
    qe.X = fl_to_fe(q.X, L, nc);
    qe.Y = fl_to_fe(q.Y, L, nc);
    qe.Z = fl_to_fe(q.Z, L, nc);
    qe.T = qe.Z;
    uint32_t z_nonzero;
    const uint32_t sane = ge_is_sane_row(qe, z_nonzero);
    const uint32_t same = fe_is_zero(qe.X) & fe_eq(qe.Y, qe.Z) & z_nonzero;  // ge_is_neutral
    f = flags_byte(meta & kPrepSOk, a_ok, r_ok, small_a, small_r, same);
    bad = (a_ok & r_ok & (sane ^ 1u)) ? 1u : 0u;
  }
  report_faults(fault, bad | nc | (canary[slot] != nonce ? 2u : 0u));
  if (item < n && role == 0u && L.k == 0u && lead) {
    if (flags_out) flags_out[item] = (uint8_t)f;
    if (strict_bits && (f & kStrictOk)) atomicOr(&strict_bits[item >> 5], 1u << (item & 31u));
  }
}

// Quad form of the latency kernel (default at <= kQuadMax items, round 5):
// one item per block of four waves, one per SIMD.  Waves 0 and 1 hold R and
// A, each as one point per WAVE whose four rows compute the four independent
// products of every formula round at once (hsv_rowpoint.hpp q_*), so a
// doubling costs two row products instead of eight.  Each decompresses its
// point (the two-row chain, run by both row pairs) and builds [0..8](-P) in
// LDS while wave 2 runs the scalar prepass; then each runs its one-scalar
// Straus (c1 for R, |c0| for A) adding only the windows above the low
// kQuadLo.  The helper waves add those low windows over the same tables
// (wave 2 for c1, then the whole wide B comb; wave 3 for |c0|), and the R
// wave adds the three handed-over sums and checks.  Fallback items (no short
// lattice pair) run the full-length one-lane path on lane 0 of the R wave.
// Same flags, self-checks and canaries as the row form.  Kernel 84.4 us at one
// item (95.6 us without the helpers, profiles/r05y_kernel_trace/); phases in
// profiles/r05y_quadclk.txt.  The cut-over: one block per CU at <= 256 items;
// from 257 on some SIMDs would hold two of these lone-issue waves (0.169-0.173
// ms, profiles/r05k_cutover.txt), so larger batches take the joint form below
// (0.129-0.132 ms up to 768 items, profiles/r05x_cutover.txt).
#ifndef HSV_QUAD_MAX  // measurement builds may move the cut-over (tools/row_cutover_probe.py)
#define HSV_QUAD_MAX 256
#endif
constexpr uint32_t kQuadMax = HSV_QUAD_MAX;
// windows of each half-size scalar run by the helper waves (the low 80 bits):
// the point waves keep their 128 doublings but add only the high windows
constexpr int kQuadLo = 20;
#ifdef HSV_QUAD_CLOCKS
// Measurement builds only (tools/build_ab_libs.sh quadclk "-DHSV_QUAD_CLOCKS"):
// lane 0 of each wave of block 0 stamps the 100 MHz clock at fixed points
// (0 entry, 1 decompressed / prepass done, 2 table built, 3 past barrier 1,
// 4 Straus done, 5 wave 2's B comb done, 6 past barrier 2, 7 exit).
__device__ uint64_t g_quad_clk[4][9];  // slot 8: the wave's HW_ID (SIMD_ID in bits 5:4)
#define HSV_QUAD_CLK(w, slot)                                                  \
  do {                                                                         \
    if (blockIdx.x == 0u && (threadIdx.x & 63u) == 0u) {                       \
      g_quad_clk[w][slot] = wall_clock64();                                    \
      if (slot == 0) g_quad_clk[w][8] = __builtin_amdgcn_s_getreg((31 << 11) | 4); \
    }                                                                          \
  } while (0)
#else
#define HSV_QUAD_CLK(w, slot) \
  do {                        \
  } while (0)
#endif
template <int WA, int CB>
__global__ void __launch_bounds__(4 * 64)
hsv_verify_quad_kernel(const uint8_t *__restrict__ pk, uint64_t pk_stride, const uint8_t *__restrict__ sig,
                       uint64_t sig_stride, const uint8_t *__restrict__ msg, uint64_t msg_stride, uint32_t n,
                       uint8_t *__restrict__ flags_out, uint32_t *__restrict__ strict_bits,
                       uint4 *__restrict__ vt_ws, const uint32_t *__restrict__ comb_b, int lat_bits,
                       uint32_t *__restrict__ canary, uint32_t nonce, uint32_t inject, uint32_t *__restrict__ fault) {
  using G = HalfCombWindows<WA>;
  constexpr int TS = 1 << (WA - 1);
  constexpr int kEnt = TS + 1;
  __shared__ uint32_t srec[kPrepWords];
  __shared__ uint32_t stab[2][kEnt * 64];
  __shared__ uint32_t sq_a[4 * 16];     // the A wave's sum, cached form (component r on row r)
  __shared__ uint32_t sq_h[2][4 * 16];  // the helpers' sums: [c1_lo](-R) + [b]B, [c0_lo](-A)
  __shared__ uint32_t s_a[2];           // the A wave's ok, small
  const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63u;
  const uint32_t item = blockIdx.x;
  const uint32_t li = item < n ? item : n - 1u;
  HSV_QUAD_CLK(wave, 0);
  if (wave >= 2) {
    // helpers: wave 2 runs the scalar prepass on lane 0; after the tables
    // are built, each helper adds the low kQuadLo windows of one scalar over
    // its table (wave 2: c1 over -R, then the whole wide B comb over b; wave
    // 3: |c0| over -A) while the point waves run the high windows
    if (wave == 2u && lane == 0u) {
      uint32_t pkw[8], sigw[16], msgw[8];
      load_triple(pk, pk_stride, sig, sig_stride, msg, msg_stride, li, pkw, sigw, msgw);
      (void)prep_scalars<WA>(pkw, sigw, msgw, srec, 1, lat_bits);
    }
    HSV_QUAD_CLK(wave, 1);
    __syncthreads();
    HSV_QUAD_CLK(wave, 3);
    const uint32_t meta = srec[kPrepWords - 1];
    if (!(meta & kPrepFallback)) {
      const QuadLane L;
      const uint32_t h = wave - 2u;  // 0: R, 1: A
      uint32_t d[5];
      HSV_UNROLL
      for (int i = 0; i < 5; ++i) d[i] = srec[i + 5 * (int)h];
      qp_ext q = quad_straus_low<WA, G::NW, kQuadLo>(d, stab[h], (h && (meta & kPrepC0Neg)) ? 1u : 0u, L);
      HSV_QUAD_CLK(wave, 4);
      if (h == 0u) {
        uint32_t b[8];
        HSV_UNROLL
        for (int i = 0; i < 8; ++i) b[i] = srec[10 + i];
        HSV_NOUNROLL
        for (uint32_t half = 0; half < 2u; ++half) q = quad_comb_half<CB>(q, b, comb_b, half, L);
      }
      sq_h[h][L.r * 16u + L.k] = q_cached_component(q, fl_from_fe(fe_d2(), L), L);
    }
    HSV_QUAD_CLK(wave, 5);
    __syncthreads();
    HSV_QUAD_CLK(wave, 6);
    return;
  }
  const uint32_t role = wave;  // 0: R, 1: A
  const uint32_t slot = blockIdx.x * 2u + role;
  if (lane == 0u) canary[slot] = inject == kInjectCanary ? ~nonce : nonce;
  uint32_t ok, small, nc = 0;
  uint32_t *tab = stab[role];
  {
    const RowLane2 L2;
    uint32_t enc[8];
    const uint4 *ep = reinterpret_cast<const uint4 *>(role ? pk + (uint64_t)li * pk_stride : sig + (uint64_t)li * sig_stride);
    const uint4 e0 = ep[0], e1 = ep[1];
    enc[0] = e0.x; enc[1] = e0.y; enc[2] = e0.z; enc[3] = e0.w;
    enc[4] = e1.x; enc[5] = e1.y; enc[6] = e1.z; enc[7] = e1.w;
    fe x, y;
    ok = ge_decompress_row(enc, x, y, small, nc, L2);  // both row pairs, the same chain
    small &= ok;
    HSV_QUAD_CLK(role, 1);
    const QuadLane L;
    quad_table_build<TS>(tab, x, y, L, inject, role == 0u);
    HSV_QUAD_CLK(role, 2);
  }
  __syncthreads();
  HSV_QUAD_CLK(role, 3);
  const QuadLane L;
  const uint32_t meta = srec[kPrepWords - 1];
  uint32_t f = 0, bad = 0;
  qp_ext q{};
  if (!(meta & kPrepFallback)) {
    uint32_t d[5];
    HSV_UNROLL
    for (int i = 0; i < 5; ++i) d[i] = srec[i + 5 * (int)role];
    q = quad_straus<WA, G::NW, kQuadLo>(d, tab, (role && (meta & kPrepC0Neg)) ? 1u : 0u, L);
    HSV_QUAD_CLK(role, 4);
    if (role == 1u) {
      sq_a[L.r * 16u + L.k] = q_cached_component(q, fl_from_fe(fe_d2(), L), L);
      if (lane == 0u) {
        s_a[0] = ok;
        s_a[1] = small;
      }
    }
  }
  __syncthreads();
  HSV_QUAD_CLK(role, 6);
  if (role == 1u) {
    report_faults(fault, nc | (canary[slot] != nonce ? 2u : 0u));
    return;
  }
  if (meta & kPrepFallback) {
    if (lane == 0u) {
      GlobalVarTab<kEnt> vt{vt_ws + (uint64_t)slot * vt_lane_uint4<WA>(), inject};
      uint32_t pkw[8], sigw[16], msgw[8];
      load_triple(pk, pk_stride, sig, sig_stride, msg, msg_stride, li, pkw, sigw, msgw);
      f = verify_one_full_comb<WA, false, CB>(pkw, sigw, msgw, comb_b, vt);
      bad = (f & kFault) ? 1u : 0u;
    }
  } else {
    // Q = the R wave's sum + the A wave's + the helpers' (cached forms from LDS)
    q = q_add_op(q, q_op_of_cached(sq_a, L), L);
    q = q_add_op(q, q_op_of_cached(sq_h[0], L), L);
    q = q_add_op(q, q_op_of_cached(sq_h[1], L), L);
    const uint32_t a_ok = s_a[0], small_a = s_a[1];
    const RowLane &R = L;
    ge_ext qe;
    qe.X = fl_to_fe(q.X, R, nc);
    qe.Y = fl_to_fe(q.Y, R, nc);
    qe.Z = fl_to_fe(q.Z, R, nc);
    qe.T = qe.Z;
    uint32_t z_nonzero;
    const uint32_t sane = ge_is_sane_row(qe, z_nonzero);
    const uint32_t same = fe_is_zero(qe.X) & fe_eq(qe.Y, qe.Z) & z_nonzero;  // ge_is_neutral
    f = flags_byte(meta & kPrepSOk, a_ok, ok, small_a, small, same);
    bad = (a_ok & ok & (sane ^ 1u)) ? 1u : 0u;
  }
  report_faults(fault, bad | nc | (canary[slot] != nonce ? 2u : 0u));
  if (item < n && lane == 0u) {
    if (flags_out) flags_out[item] = (uint8_t)f;
    if (strict_bits && (f & kStrictOk)) atomicOr(&strict_bits[item >> 5], 1u << (item & 31u));
  }
  HSV_QUAD_CLK(0, 7);
}

// Joint quad form (variant 21 above kQuadMax, at <= kJointMax items): one
// item per WAVE, kJointItems point waves and one prepass wave per block, so
// 768 items still hold one block per CU and one wave per SIMD.  The point
// wave decompresses R on rows 0-1 and A on rows 2-3 at once (the two-row
// chain, each pair its own element), builds both tables [0..8](-R),
// [0..8](-A) in LDS with the quad formulas, then runs one two-scalar Straus
// (shared doublings, quad_straus2) over all but the low kJointLo windows; the
// prepass wave adds each item's low windows and its wide B comb meanwhile and
// hands the sum over in LDS.  Same flags, fallback, self-checks
// and canaries as the quad form.
constexpr uint32_t kJointItems = 3;
// windows of both scalars the prepass wave adds for each item after its
// prepasses (the low 28 bits): it finishes its three items' shares about when
// the point waves finish the rest
constexpr int kJointLo = 7;
#ifndef HSV_JOINT_MAX  // measurement builds may move the cut-over (tools/row_cutover_probe.py)
#define HSV_JOINT_MAX 768
#endif
constexpr uint32_t kJointMax = HSV_JOINT_MAX;
template <int WA, int CB>
__global__ void __launch_bounds__((kJointItems + 1) * 64)
hsv_verify_joint_kernel(const uint8_t *__restrict__ pk, uint64_t pk_stride, const uint8_t *__restrict__ sig,
                        uint64_t sig_stride, const uint8_t *__restrict__ msg, uint64_t msg_stride, uint32_t n,
                        uint8_t *__restrict__ flags_out, uint32_t *__restrict__ strict_bits,
                        uint4 *__restrict__ vt_ws, const uint32_t *__restrict__ comb_b, int lat_bits,
                        uint32_t *__restrict__ canary, uint32_t nonce, uint32_t inject, uint32_t *__restrict__ fault) {
  using G = HalfCombWindows<WA>;
  constexpr int TS = 1 << (WA - 1);
  constexpr int kEnt = TS + 1;
  constexpr uint32_t K = kJointItems;
  __shared__ uint32_t srec[kPrepWords * K];
  __shared__ uint32_t stab[K][2][kEnt * 64];
  __shared__ uint32_t sq_b[K][4 * 16];  // each item's low windows + [b]B, cached form (component r on row r)
  const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63u;
  const uint32_t base = blockIdx.x * K;
  if (wave == K) {
    // the items' scalar prepasses on lanes 0..K-1, then each item's whole
    // wide B comb (16 additions) while the point waves run their Straus loops
    if (lane < K) {
      const uint32_t li = base + lane < n ? base + lane : n - 1u;
      uint32_t pkw[8], sigw[16], msgw[8];
      load_triple(pk, pk_stride, sig, sig_stride, msg, msg_stride, li, pkw, sigw, msgw);
      (void)prep_scalars<WA>(pkw, sigw, msgw, srec + lane, K, lat_bits);
    }
    __syncthreads();
    const QuadLane L;
    const uint32_t d2 = fl_from_fe(fe_d2(), L);
    HSV_NOUNROLL
    for (uint32_t t = 0; t < K; ++t) {
      const uint32_t meta_t = srec[(kPrepWords - 1) * K + t];
      if (meta_t & kPrepFallback) continue;
      // the low kJointLo windows of the item's two scalars over its tables,
      // then its whole wide B comb onto that sum
      uint32_t d1[5], d0[5], b[8];
      HSV_UNROLL
      for (int i = 0; i < 5; ++i) {
        d1[i] = srec[i * K + t];
        d0[i] = srec[(5 + i) * K + t];
      }
      HSV_UNROLL
      for (int i = 0; i < 8; ++i) b[i] = srec[(10 + i) * K + t];
      qp_ext qb = quad_straus2_low<WA, G::NW, kJointLo>(d1, d0, stab[t][0], stab[t][1],
                                                         (meta_t & kPrepC0Neg) ? 1u : 0u, L);
      HSV_NOUNROLL
      for (uint32_t h = 0; h < 2u; ++h) qb = quad_comb_half<CB>(qb, b, comb_b, h, L);
      sq_b[t][L.r * 16u + L.k] = q_cached_component(qb, d2, L);
    }
    __syncthreads();
    return;
  }
  const uint32_t item = base + wave;
  const uint32_t li = item < n ? item : n - 1u;
  const uint32_t slot = blockIdx.x * K + wave;
  if (lane == 0u) canary[slot] = inject == kInjectCanary ? ~nonce : nonce;
  uint32_t ok, small, nc = 0;  // rows 0-1: R's, rows 2-3: A's
  uint32_t *tab_r = stab[wave][0], *tab_a = stab[wave][1];
  {
    const RowLane2 L2;
    const uint32_t role = lane >> 5;  // 0: R, 1: A
    uint32_t enc[8];
    const uint4 *ep = reinterpret_cast<const uint4 *>(role ? pk + (uint64_t)li * pk_stride : sig + (uint64_t)li * sig_stride);
    const uint4 e0 = ep[0], e1 = ep[1];
    enc[0] = e0.x; enc[1] = e0.y; enc[2] = e0.z; enc[3] = e0.w;
    enc[4] = e1.x; enc[5] = e1.y; enc[6] = e1.z; enc[7] = e1.w;
    fe x, y;
    ok = ge_decompress_row(enc, x, y, small, nc, L2);  // each row pair its own element
    small &= ok;
    const QuadLane L;
    HSV_NOUNROLL
    for (uint32_t t = 0; t < 2u; ++t) {
      // element t (rows 2t, 2t + 1) on every row: v_permlane32_swap puts the
      // lower half's value in result 0 and the upper half's in result 1
      fe xt, yt;
      HSV_UNROLL
      for (int l = 0; l < kFeLimbs; ++l) {
        const auto px = __builtin_amdgcn_permlane32_swap(x.v[l], x.v[l], false, false);
        const auto py = __builtin_amdgcn_permlane32_swap(y.v[l], y.v[l], false, false);
        xt.v[l] = t ? px[1] : px[0];
        yt.v[l] = t ? py[1] : py[0];
      }
      quad_table_build<TS>(t ? tab_a : tab_r, xt, yt, L, inject, t == 0u);
    }
  }
  __syncthreads();
  const QuadLane L;
  const uint32_t meta = srec[(kPrepWords - 1) * K + wave];
  const uint32_t r_ok = __builtin_amdgcn_readlane(ok, 0), small_r = __builtin_amdgcn_readlane(small, 0);
  const uint32_t a_ok = __builtin_amdgcn_readlane(ok, 32), small_a = __builtin_amdgcn_readlane(small, 32);
  uint32_t f = 0, bad = 0;
  qp_ext q{};
  if (!(meta & kPrepFallback)) {
    uint32_t d1[5], d0[5];
    HSV_UNROLL
    for (int i = 0; i < 5; ++i) {
      d1[i] = srec[i * K + wave];
      d0[i] = srec[(5 + i) * K + wave];
    }
    q = quad_straus2<WA, G::NW, kJointLo>(d1, d0, tab_r, tab_a, (meta & kPrepC0Neg) ? 1u : 0u, L);
  }
  __syncthreads();  // the prepass wave's [b]B
  if (meta & kPrepFallback) {
    if (lane == 0u) {
      GlobalVarTab<kEnt> vt{vt_ws + (uint64_t)slot * vt_lane_uint4<WA>(), inject};
      uint32_t pkw[8], sigw[16], msgw[8];
      load_triple(pk, pk_stride, sig, sig_stride, msg, msg_stride, li, pkw, sigw, msgw);
      f = verify_one_full_comb<WA, false, CB>(pkw, sigw, msgw, comb_b, vt);
      bad = (f & kFault) ? 1u : 0u;
    }
  } else {
    q = q_add_op(q, q_op_of_cached(sq_b[wave], L), L);
    const RowLane &R = L;
    ge_ext qe;
    qe.X = fl_to_fe(q.X, R, nc);
    qe.Y = fl_to_fe(q.Y, R, nc);
    qe.Z = fl_to_fe(q.Z, R, nc);
    qe.T = qe.Z;
    uint32_t z_nonzero;
    const uint32_t sane = ge_is_sane_row(qe, z_nonzero);
    const uint32_t same = fe_is_zero(qe.X) & fe_eq(qe.Y, qe.Z) & z_nonzero;  // ge_is_neutral
    f = flags_byte(meta & kPrepSOk, a_ok, r_ok, small_a, small_r, same);
    bad = (a_ok & r_ok & (sane ^ 1u)) ? 1u : 0u;
  }
  report_faults(fault, bad | nc | (canary[slot] != nonce ? 2u : 0u));
  if (item < n && lane == 0u) {
    if (flags_out) flags_out[item] = (uint8_t)f;
    if (strict_bits && (f & kStrictOk)) atomicOr(&strict_bits[item >> 5], 1u << (item & 31u));
  }
}


// ---- v_mad_u64_u32 issue-rate probe -------------------------------------
// 8 independent accumulation chains, 16 mads per asm statement (the compiler
// puts an s_nop after every asm statement that writes an SGPR, so one mad per
// statement would measure mad + s_nop).
constexpr int kPeakIters = 2048;

#define HSV_PEAK_MAD(c) "v_mad_u64_u32 %" #c ", s[40:41], %8, %9, %" #c "\n\t"
__global__ void __launch_bounds__(256) hsv_mad_peak_kernel(uint32_t *sink, uint32_t seed) {
  const uint32_t t = threadIdx.x + blockIdx.x * blockDim.x + seed;
  uint64_t x0 = t, x1 = t + 1, x2 = t + 2, x3 = t + 3, x4 = t + 4, x5 = t + 5, x6 = t + 6, x7 = t + 7;
  const uint32_t a = t | 1u, b = t * 3u + 7u;
  for (int it = 0; it < kPeakIters; ++it)
    asm volatile(HSV_PEAK_MAD(0) HSV_PEAK_MAD(1) HSV_PEAK_MAD(2) HSV_PEAK_MAD(3) HSV_PEAK_MAD(4) HSV_PEAK_MAD(5)
                 HSV_PEAK_MAD(6) HSV_PEAK_MAD(7) HSV_PEAK_MAD(0) HSV_PEAK_MAD(1) HSV_PEAK_MAD(2) HSV_PEAK_MAD(3)
                 HSV_PEAK_MAD(4) HSV_PEAK_MAD(5) HSV_PEAK_MAD(6) HSV_PEAK_MAD(7)
                 : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3), "+v"(x4), "+v"(x5), "+v"(x6), "+v"(x7)
                 : "v"(a), "v"(b)
                 : "s40", "s41");
  const uint64_t r = x0 ^ x1 ^ x2 ^ x3 ^ x4 ^ x5 ^ x6 ^ x7;
  if ((uint32_t)(r ^ (r >> 32)) == 0x9e3779b9u) sink[0] = 1u;
}
#undef HSV_PEAK_MAD

}  // namespace hsv

// Kernel variant ids (hsv_set_variant, test library).  The library builds two
// (kVariantIds below):
//  19: two passes -- scalar prepass (hsv_prep_kernel), then the persistent
//      point pass with the fallback items dealt out first (WA 4, 3 waves/SIMD,
//      wide comb of B)
//  21: the default: 19's kernels above 2^13 items; at or below, the latency
//      forms (quad / joint / row / pair)
// Ids 0-18, 20 and 22 were rounds 1-4's measured alternatives; they left the
// source in round 5 (git history before that cleanup).  The id space stays
// [0, 22) so old measurement records keep their meaning.
extern "C" int hsvi_num_variants(void) { return 22; }

namespace {
struct WsPools {
  std::mutex mu;
  std::unordered_map<int, hipMemPool_t> pools;  // device -> the library's workspace pool
};
WsPools &ws_pools() {
  static WsPools p;
  return p;
}
}  // namespace

// hsv_shutdown: return the pools' free blocks to the driver (blocks still in
// use by enqueued work stay)
extern "C" void hsv_ws_trim(void) {
  WsPools &wp = ws_pools();
  std::lock_guard<std::mutex> lk(wp.mu);
  for (auto &kv : wp.pools) (void)hipMemPoolTrimTo(kv.second, 0);
}

// Free memory the pool keeps between calls (HSV_WS_POOL_KEEP_MB, default 4096
// MiB; 0 returns every block at each synchronisation): a freed block is reused
// only by later launches on the same stream, so an application that spreads
// batches over many streams would otherwise keep one workspace per stream
// (about 0.5 GB for a 2^20-item batch) out of its own allocator's reach.  Above
// the threshold the pool hands idle blocks back to the driver whenever a
// stream or event synchronisation observes their frees.
static uint64_t ws_pool_keep_bytes() {
  static const uint64_t b = [] {
    long long mb = 4096;
    if (const char *v = std::getenv("HSV_WS_POOL_KEEP_MB")) mb = std::atoll(v);
    if (mb < 0) mb = 0;
    return (uint64_t)mb << 20;
  }();
  return b;
}

extern "C" hipError_t hsv_ws_malloc(void **p, size_t bytes, hipStream_t stream) {
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  WsPools &wp = ws_pools();
  hipMemPool_t pool = nullptr;
  {
    std::lock_guard<std::mutex> lk(wp.mu);
    auto &pools = wp.pools;
    auto it = pools.find(dev);
    if (it == pools.end()) {
      hipMemPoolProps props = {};
      props.allocType = hipMemAllocationTypePinned;
      props.handleTypes = hipMemHandleTypeNone;
      props.location.type = hipMemLocationTypeDevice;
      props.location.id = dev;
      e = hipMemPoolCreate(&pool, &props);
      if (e != hipSuccess) return e;
      uint64_t keep = ws_pool_keep_bytes();
      e = hipMemPoolSetAttribute(pool, hipMemPoolAttrReleaseThreshold, &keep);
      if (e != hipSuccess) return e;
      // A block is reused only on the stream that freed it (stream order
      // alone makes that safe).  No cross-stream reuse of any kind:
      // - internal dependencies would make a new launch wait for another
      //   stream, and launches on different streams (consecutive batches,
      //   pipelined chunks) must be free to overlap;
      // - with event-dependency and opportunistic reuse, a launch on a
      //   stream that had waited (through a third stream) on an event of the
      //   freeing stream got a block still in use by a running launch there:
      //   two point passes shared one work counter and prepass records and
      //   returned wrong flags (round 5, tools/mempool_split_probe.py,
      //   tests/test_device_model.py::test_batches_behind_cross_stream_event_chains).
      int no = 0;
      for (hipMemPoolAttr a : {hipMemPoolReuseAllowInternalDependencies, hipMemPoolReuseFollowEventDependencies,
                               hipMemPoolReuseAllowOpportunistic}) {
        e = hipMemPoolSetAttribute(pool, a, &no);
        if (e != hipSuccess) return e;
      }
#ifdef HSV_WS_POOL_PROBE
      // Measurement builds only (tools/build_ab_libs.sh): one
      // cross-stream reuse policy back on -- 1 event dependencies, 2
      // opportunistic -- to pin which one handed a running launch's block on.
      {
        int yes = 1;
        e = hipMemPoolSetAttribute(pool, HSV_WS_POOL_PROBE == 1 ? hipMemPoolReuseFollowEventDependencies
                                                                : hipMemPoolReuseAllowOpportunistic, &yes);
        if (e != hipSuccess) return e;
      }
#endif
      it = pools.emplace(dev, pool).first;
    }
    pool = it->second;
  }
  e = hipMallocFromPoolAsync(p, bytes, pool, stream);
  if (e == hipErrorOutOfMemory) {
    // Blocks freed on other streams are never reused here.  When the device
    // runs out: wait for the calling stream (its own frees complete), hand
    // every idle block of the pool back to the driver -- blocks freed on
    // idle or destroyed streams among them -- and try once more; otherwise
    // the caller gets the out-of-memory error.  No device-wide wait: that
    // would stall every stream of the application, and blocks still held by
    // launches running on other streams stay theirs.
    (void)hipGetLastError();
    hsvi_resident_pause(1);
    if (hipStreamSynchronize(stream) == hipSuccess && hipMemPoolTrimTo(pool, 0) == hipSuccess)
      e = hipMallocFromPoolAsync(p, bytes, pool, stream);
    hsvi_resident_pause(0);
    if (e == hipSuccess) (void)hipGetLastError();
  }
  return e;
}

namespace {

// Lattice bound of the comb-path prepass (hsvi_set_lattice_bits; tests lower
// it to 133 so the lattice-fallback fixtures take the full-length path).
std::atomic<int> g_lat_bits{hsv::kLatCombBits};

// Fault injection mode of the launches the calling thread issues
// (hsvi_set_inject; only libhsv_test.so exports a setter).  Thread-scoped: a
// test that injects on one thread leaves every other thread's calls alone.
thread_local uint32_t t_inject = hsv::kInjectNone;

// HSV_TX_FUSED=0: transactions as the record kernel + point pass pair (the
// round-5 form), for A/B runs; read once per process.
bool tx_fused_enabled() {
  static const bool on = [] {
    const char *v = std::getenv("HSV_TX_FUSED");
    return !(v && v[0] == '0');
  }();
  return on;
}

// Per-launch canary nonce: odd, so never 0 (zeroed memory) or all-ones.
uint32_t next_nonce() {
  static std::atomic<uint32_t> ctr{0x9e3779b9u};
  return (ctr.fetch_add(0x61c88646u) * 2654435761u) | 1u;
}



// Two-pass launch (variants 19/20): prepass over all items, then the
// persistent point pass.  Workspace: per-lane tables | counters (256 B) |
// fallback list (4 B per item) | prep records (kPrepWords x 4 B per item).
// Transactions whose records the prepass writes itself (hsv_launch_tx_prep):
// the point pass then reads pk / R (and, for fallback items, s and the
// digest) from `records` at stride 128.
struct TxPrep {
  const uint8_t *txs;
  const uint64_t *offsets;
  uint64_t tx_size;
  uint8_t *records;
};

template <int WA, int WAVES, int CB>
hipError_t launch_hp(const uint8_t *pk, uint64_t pk_stride, const uint8_t *sig, uint64_t sig_stride,
                     const uint8_t *msg, uint64_t msg_stride, uint32_t n, uint8_t *flags_out,
                     uint32_t *strict_bits, const uint32_t *comb_b, uint32_t *fault, hipStream_t stream,
                     const TxPrep *tx = nullptr, void *ws_in = nullptr, size_t ws_cap = 0,
                     size_t *ws_need = nullptr) {
  const void *kern = reinterpret_cast<const void *>(hsv::hsv_verify_hp_kernel<WA, WAVES, CB>);
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  static std::mutex mu;
  static std::unordered_map<int, std::pair<int, int>> slots_per_dev;  // device -> (blocks per CU, CUs)
  int bpc = 1, cus = 1;
  {
    std::lock_guard<std::mutex> lk(mu);
    auto it = slots_per_dev.find(dev);
    if (it == slots_per_dev.end()) {
      int b = 0, c = 0;
      e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, kern, hsv::kBlock, 0);
      if (e != hipSuccess) return e;
      e = hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev);
      if (e != hipSuccess) return e;
      it = slots_per_dev.emplace(dev, std::make_pair(std::max(1, b), std::max(1, c))).first;
    }
    bpc = it->second.first;
    cus = it->second.second;
  }
  // A persistent grid must fit the device at once: its blocks leave when the
  // work counter runs out, and a block still waiting for a place would hold
  // the launch open.  Once the resident latency service has run in this
  // process its block may sit on one CU (and a request from another thread
  // may relaunch it while this grid is dispatched), so the grid then leaves
  // one CU's worth of blocks out (1/256 of the slots).
  // Transactions of the product form run as ONE fused launch (records,
  // prepass and point pass; hsv_mempool.hip) unless HSV_TX_FUSED=0 selects
  // the record kernel + point pass pair; its grid follows its own occupancy.
  const bool fused = tx && WA == 4 && WAVES == HSV_HP_WAVES && CB == 16 && tx_fused_enabled() &&
                     (uint64_t)n * 128u <= 0xffffffffull && hsv_tx_fused_blocks_per_cu(dev) > 0;
  if (fused) bpc = std::min(bpc, hsv_tx_fused_blocks_per_cu(dev));
  const int resident = bpc * (hsvi_resident_started() && cus > 1 ? cus - 1 : cus);
  const uint32_t blocks_needed = (n + hsv::kBlock - 1) / hsv::kBlock;
  const uint32_t grid = std::min<uint32_t>(blocks_needed, (uint32_t)resident);
  const size_t ws_bytes = (size_t)grid * hsv::kBlock * hsv::vt_lane_uint4<WA>() * sizeof(uint4);
  const size_t canary_bytes = ((size_t)grid * hsv::kBlock * sizeof(uint32_t) + 255) & ~(size_t)255;
  const size_t fb_bytes = (size_t)n * sizeof(uint32_t);
  const size_t rec_bytes = (size_t)n * hsv::kPrepWords * sizeof(uint32_t);
  const size_t ready_bytes = fused ? (((size_t)(n + 63u) / 64u) * sizeof(uint32_t) + 255) & ~(size_t)255 : 0;
  const size_t need = ws_bytes + 256 + canary_bytes + fb_bytes + rec_bytes + ready_bytes;
  if (ws_need) {  // size query only
    *ws_need = need;
    return hipSuccess;
  }
  // the caller's workspace when it is large enough (a pipeline that keeps one
  // per stream), else one from the library pool, freed on the stream
  void *ws = ws_in && ws_cap >= need ? ws_in : nullptr;
  const bool own = ws == nullptr;
  if (own) e = hsv_ws_malloc(&ws, need, stream);
  if (e != hipSuccess) return e;
  uint8_t *ws8 = static_cast<uint8_t *>(ws);
  uint4 *vt_ws = reinterpret_cast<uint4 *>(ws);
  hsv::HcCounters *ctr = reinterpret_cast<hsv::HcCounters *>(ws8 + ws_bytes);
  uint32_t *canary = reinterpret_cast<uint32_t *>(ws8 + ws_bytes + 256);
  uint32_t *fb_list = reinterpret_cast<uint32_t *>(ws8 + ws_bytes + 256 + canary_bytes);
  uint32_t *rec = reinterpret_cast<uint32_t *>(ws8 + ws_bytes + 256 + canary_bytes + fb_bytes);
  uint32_t *ready = reinterpret_cast<uint32_t *>(ws8 + ws_bytes + 256 + canary_bytes + fb_bytes + rec_bytes);
  e = hipMemsetAsync(ctr, 0, sizeof(hsv::HcCounters), stream);
  if (e == hipSuccess && strict_bits) e = hipMemsetAsync(strict_bits, 0, (size_t)((n + 31u) / 32u) * 4u, stream);
  if (e == hipSuccess && fused) {
    e = hipMemsetAsync(ready, 0, ready_bytes, stream);
    if (e == hipSuccess)
      e = hsv_launch_tx_fused(grid, tx->txs, tx->offsets, tx->tx_size, n, tx->records, rec, ctr, fb_list, ready,
                              g_lat_bits.load(), flags_out, strict_bits, vt_ws, comb_b, canary, next_nonce(), t_inject,
                              fault, stream);
    const hipError_t ef = own ? hipFreeAsync(ws, stream) : hipSuccess;
    return e != hipSuccess ? e : ef;
  }
  if (e == hipSuccess && tx) {
    static_assert(WA == 4, "hsv_launch_tx_prep writes the WA = 4 prepass record");
    e = hsv_launch_tx_prep(tx->txs, tx->offsets, tx->tx_size, n, tx->records, rec, &ctr->fb_count, fb_list,
                           g_lat_bits.load(), stream);
    pk = tx->records;
    sig = tx->records + 32;
    msg = tx->records + 96;
    pk_stride = sig_stride = msg_stride = 128;
  } else if (e == hipSuccess) {
    hipLaunchKernelGGL((hsv::hsv_prep_kernel<WA>), dim3(blocks_needed), dim3(hsv::kBlock), 0, stream, pk, pk_stride,
                       sig, sig_stride, msg, msg_stride, n, rec, ctr, fb_list, g_lat_bits.load());
    e = hipGetLastError();
  }
  if (e == hipSuccess) {
    {
      hipLaunchKernelGGL((hsv::hsv_verify_hp_kernel<WA, WAVES, CB>), dim3(grid), dim3(hsv::kBlock), 0, stream, pk,
                         pk_stride, sig, sig_stride, msg, msg_stride, n, flags_out, strict_bits, vt_ws, comb_b, rec,
                         ctr, fb_list, canary, next_nonce(), t_inject, fault);
    }
    e = hipGetLastError();
  }
  const hipError_t ef = own ? hipFreeAsync(ws, stream) : hipSuccess;
  return e != hipSuccess ? e : ef;
}

// Latency form (variant 21 below kPairMax items): one launch of the fused
// kernel (prepass wave + two pair waves per 64 items).  Workspace: the pair
// lanes' tables.  Round 1 ran the prepass and hsv_verify_pair_kernel as two
// launches; at 2^12 items the pair form is 27 % faster end to end than the
// point pass, at 2^15 7 % slower (profiles/r01o_qc_latency.json).
constexpr uint32_t kPairMax = 1u << 13;
// The row form at or below this many items.  p50 of a generic call, row /
// pair form (tools/row_cutover_probe.py, profiles/r03zp_row_cutover.txt):
// 0.216 / 0.450 ms at 64 items, 0.226 / 0.466 at 1024, 0.230 / 0.467 at 1536
// (256 blocks of four waves: one block per CU), 0.422 / 0.470 at 2048, 0.427 /
// 0.477 at 3072, 0.626 / 0.487 at 4096.
constexpr uint32_t kRowMaxDefault = 3072;

template <int WA, int CB>
hipError_t launch_pair(const uint8_t *pk, uint64_t pk_stride, const uint8_t *sig, uint64_t sig_stride,
                       const uint8_t *msg, uint64_t msg_stride, uint32_t n, uint8_t *flags_out,
                       uint32_t *strict_bits, const uint32_t *comb_b, uint32_t *fault, hipStream_t stream,
                       void *ws_in = nullptr, size_t ws_cap = 0, size_t *ws_need = nullptr) {
  const uint32_t grid = (n + hsv::kFusedItems - 1) / hsv::kFusedItems;
  const size_t slots = (size_t)grid * 2u * hsv::kFusedItems;
  const size_t ws_bytes = slots * hsv::vt_lane_uint4<WA>() * sizeof(uint4);
  const size_t need = ws_bytes + slots * sizeof(uint32_t);
  if (ws_need) {
    *ws_need = need;
    return hipSuccess;
  }
  void *ws = ws_in && ws_cap >= need ? ws_in : nullptr;
  const bool own = ws == nullptr;
  hipError_t e = own ? hsv_ws_malloc(&ws, need, stream) : hipSuccess;
  if (e != hipSuccess) return e;
  if (strict_bits) e = hipMemsetAsync(strict_bits, 0, (size_t)((n + 31u) / 32u) * 4u, stream);
  if (e == hipSuccess) {
    hipLaunchKernelGGL((hsv::hsv_verify_pair_fused_kernel<WA, CB>), dim3(grid), dim3(3 * 64), 0, stream, pk,
                       pk_stride, sig, sig_stride, msg, msg_stride, n, flags_out, strict_bits,
                       static_cast<uint4 *>(ws), comb_b, g_lat_bits.load(),
                       reinterpret_cast<uint32_t *>(static_cast<uint8_t *>(ws) + ws_bytes), next_nonce(),
                       t_inject, fault);
    e = hipGetLastError();
  }
  const hipError_t ef = own ? hipFreeAsync(ws, stream) : hipSuccess;
  return e != hipSuccess ? e : ef;
}

// Row form (variant 21 above kJointMax, at <= row_max() items): kRowItemsOf<1>
// items per block of four waves.  The workspace holds one full-length table
// and one canary per row (the fallback path's tables; the row tables live in
// LDS).  The two-rows-per-element form (RR = 2, round 3's default up to 768
// items, 0.178-0.182 ms) gave way to the joint quad form there (0.130-0.134
// ms, profiles/r05l_cutover.txt); the kernel template still takes RR, and
// only RR = 1 is instantiated.
constexpr uint32_t row_max() { return kRowMaxDefault; }

template <int WA, int CB>
hipError_t launch_row(const uint8_t *pk, uint64_t pk_stride, const uint8_t *sig, uint64_t sig_stride,
                      const uint8_t *msg, uint64_t msg_stride, uint32_t n, uint8_t *flags_out,
                      uint32_t *strict_bits, const uint32_t *comb_b, uint32_t *fault, hipStream_t stream,
                      void *ws_in = nullptr, size_t ws_cap = 0, size_t *ws_need = nullptr) {
  const uint32_t items = hsv::kRowItemsOf<1>;
  const uint32_t grid = (n + items - 1) / items;
  const size_t slots = (size_t)grid * hsv::kRowRows;
  const size_t ws_bytes = slots * hsv::vt_lane_uint4<WA>() * sizeof(uint4);
  const size_t need = ws_bytes + slots * sizeof(uint32_t);
  if (ws_need) {
    *ws_need = need;
    return hipSuccess;
  }
  void *ws = ws_in && ws_cap >= need ? ws_in : nullptr;
  const bool own = ws == nullptr;
  hipError_t e = own ? hsv_ws_malloc(&ws, need, stream) : hipSuccess;
  if (e != hipSuccess) return e;
  if (strict_bits) e = hipMemsetAsync(strict_bits, 0, (size_t)((n + 31u) / 32u) * 4u, stream);
  if (e == hipSuccess) {
    hipLaunchKernelGGL((hsv::hsv_verify_row_kernel<WA, CB, 1>), dim3(grid), dim3(4 * 64), 0, stream, pk, pk_stride, sig, sig_stride, msg, msg_stride,
                       n, flags_out, strict_bits, static_cast<uint4 *>(ws), comb_b, g_lat_bits.load(),
                       reinterpret_cast<uint32_t *>(static_cast<uint8_t *>(ws) + ws_bytes), next_nonce(),
                       t_inject, fault);
    e = hipGetLastError();
  }
  const hipError_t ef = own ? hipFreeAsync(ws, stream) : hipSuccess;
  return e != hipSuccess ? e : ef;
}

// Quad form (variant 21 at <= kQuadMax items): one item per block of three
// waves.  The workspace holds one full-length table and one canary per point
// wave (the fallback path's tables; the quad tables live in LDS).
template <int WA, int CB>
hipError_t launch_quad(const uint8_t *pk, uint64_t pk_stride, const uint8_t *sig, uint64_t sig_stride,
                       const uint8_t *msg, uint64_t msg_stride, uint32_t n, uint8_t *flags_out,
                       uint32_t *strict_bits, const uint32_t *comb_b, uint32_t *fault, hipStream_t stream,
                       void *ws_in = nullptr, size_t ws_cap = 0, size_t *ws_need = nullptr) {
  const uint32_t grid = n;
  const size_t slots = (size_t)grid * 2u;
  const size_t ws_bytes = slots * hsv::vt_lane_uint4<WA>() * sizeof(uint4);
  const size_t need = ws_bytes + slots * sizeof(uint32_t);
  if (ws_need) {
    *ws_need = need;
    return hipSuccess;
  }
  void *ws = ws_in && ws_cap >= need ? ws_in : nullptr;
  const bool own = ws == nullptr;
  hipError_t e = own ? hsv_ws_malloc(&ws, need, stream) : hipSuccess;
  if (e != hipSuccess) return e;
  if (strict_bits) e = hipMemsetAsync(strict_bits, 0, (size_t)((n + 31u) / 32u) * 4u, stream);
  if (e == hipSuccess) {
    hipLaunchKernelGGL((hsv::hsv_verify_quad_kernel<WA, CB>), dim3(grid), dim3(4 * 64), 0, stream, pk, pk_stride,
                       sig, sig_stride, msg, msg_stride, n, flags_out, strict_bits, static_cast<uint4 *>(ws), comb_b,
                       g_lat_bits.load(), reinterpret_cast<uint32_t *>(static_cast<uint8_t *>(ws) + ws_bytes),
                       next_nonce(), t_inject, fault);
    e = hipGetLastError();
  }
  const hipError_t ef = own ? hipFreeAsync(ws, stream) : hipSuccess;
  return e != hipSuccess ? e : ef;
}

// Joint quad form (variant 21 above kQuadMax, at <= kJointMax items):
// kJointItems items per block; one full-length table and one canary per
// point wave in the workspace.
template <int WA, int CB>
hipError_t launch_joint(const uint8_t *pk, uint64_t pk_stride, const uint8_t *sig, uint64_t sig_stride,
                        const uint8_t *msg, uint64_t msg_stride, uint32_t n, uint8_t *flags_out,
                        uint32_t *strict_bits, const uint32_t *comb_b, uint32_t *fault, hipStream_t stream,
                        void *ws_in = nullptr, size_t ws_cap = 0, size_t *ws_need = nullptr) {
  const uint32_t grid = (n + hsv::kJointItems - 1) / hsv::kJointItems;
  const size_t slots = (size_t)grid * hsv::kJointItems;
  const size_t ws_bytes = slots * hsv::vt_lane_uint4<WA>() * sizeof(uint4);
  const size_t need = ws_bytes + slots * sizeof(uint32_t);
  if (ws_need) {
    *ws_need = need;
    return hipSuccess;
  }
  void *ws = ws_in && ws_cap >= need ? ws_in : nullptr;
  const bool own = ws == nullptr;
  hipError_t e = own ? hsv_ws_malloc(&ws, need, stream) : hipSuccess;
  if (e != hipSuccess) return e;
  if (strict_bits) e = hipMemsetAsync(strict_bits, 0, (size_t)((n + 31u) / 32u) * 4u, stream);
  if (e == hipSuccess) {
    hipLaunchKernelGGL((hsv::hsv_verify_joint_kernel<WA, CB>), dim3(grid), dim3((hsv::kJointItems + 1) * 64), 0,
                       stream, pk, pk_stride, sig, sig_stride, msg, msg_stride, n, flags_out, strict_bits,
                       static_cast<uint4 *>(ws), comb_b, g_lat_bits.load(),
                       reinterpret_cast<uint32_t *>(static_cast<uint8_t *>(ws) + ws_bytes), next_nonce(), t_inject,
                       fault);
    e = hipGetLastError();
  }
  const hipError_t ef = own ? hipFreeAsync(ws, stream) : hipSuccess;
  return e != hipSuccess ? e : ef;
}

}  // namespace

extern "C" hipError_t hsv_launch_verify_ws(int variant, const uint8_t *pk, uint64_t pk_stride, const uint8_t *sig,
                                           uint64_t sig_stride, const uint8_t *msg, uint64_t msg_stride, uint32_t n,
                                           uint8_t *flags_out, uint32_t *strict_bits, const uint32_t *comb_b,
                                           uint32_t *fault, void *ws, size_t ws_cap, hipStream_t stream) {
  if (n == 0) return hipSuccess;
  if (variant != 19 && variant != 21)
    return hsv_launch_verify(variant, pk, pk_stride, sig, sig_stride, msg, msg_stride, n, flags_out, strict_bits,
                             comb_b, fault, stream);
  if (!comb_b || !fault) return hipErrorInvalidValue;
  if (variant == 21 && n <= hsv::kQuadMax)
    return launch_quad<4, 16>(pk, pk_stride, sig, sig_stride, msg, msg_stride, n, flags_out, strict_bits, comb_b,
                              fault, stream, ws, ws_cap);
  if (variant == 21 && n <= hsv::kJointMax)
    return launch_joint<4, 16>(pk, pk_stride, sig, sig_stride, msg, msg_stride, n, flags_out, strict_bits, comb_b,
                               fault, stream, ws, ws_cap);
  if (variant == 21 && n <= row_max())
    return launch_row<4, 16>(pk, pk_stride, sig, sig_stride, msg, msg_stride, n, flags_out, strict_bits, comb_b,
                             fault, stream, ws, ws_cap);
  if (variant == 21 && n <= kPairMax)
    return launch_pair<4, 16>(pk, pk_stride, sig, sig_stride, msg, msg_stride, n, flags_out, strict_bits, comb_b,
                              fault, stream, ws, ws_cap);
  return launch_hp<4, HSV_HP_WAVES, 16>(pk, pk_stride, sig, sig_stride, msg, msg_stride, n, flags_out, strict_bits,
                                        comb_b, fault, stream, nullptr, ws, ws_cap);
}

extern "C" size_t hsv_launch_ws_bytes(int variant, uint32_t n) {
  size_t need = 0;
  if (variant == 21 && n <= hsv::kQuadMax)
    (void)launch_quad<4, 16>(nullptr, 0, nullptr, 0, nullptr, 0, n, nullptr, nullptr, nullptr, nullptr, nullptr,
                             nullptr, 0, &need);
  else if (variant == 21 && n <= hsv::kJointMax)
    (void)launch_joint<4, 16>(nullptr, 0, nullptr, 0, nullptr, 0, n, nullptr, nullptr, nullptr, nullptr, nullptr,
                              nullptr, 0, &need);
  else if (variant == 21 && n <= row_max())
    (void)launch_row<4, 16>(nullptr, 0, nullptr, 0, nullptr, 0, n, nullptr, nullptr, nullptr, nullptr, nullptr,
                            nullptr, 0, &need);
  else if (variant == 21 && n <= kPairMax)
    (void)launch_pair<4, 16>(nullptr, 0, nullptr, 0, nullptr, 0, n, nullptr, nullptr, nullptr, nullptr, nullptr,
                             nullptr, 0, &need);
  else if (variant == 19 || variant == 21)
    (void)launch_hp<4, HSV_HP_WAVES, 16>(nullptr, 0, nullptr, 0, nullptr, 0, n, nullptr, nullptr, nullptr, nullptr,
                                         nullptr, nullptr, nullptr, 0, &need);
  return need;
}

extern "C" hipError_t hsv_launch_verify(int variant, const uint8_t *pk, uint64_t pk_stride,
                                        const uint8_t *sig, uint64_t sig_stride,
                                        const uint8_t *msg, uint64_t msg_stride, uint32_t n,
                                        uint8_t *flags_out, uint32_t *strict_bits,
                                        const uint32_t *comb_b, uint32_t *fault, hipStream_t stream) {
  if (n == 0) return hipSuccess;
  if (hsv_variant_needs_comb(variant) && !comb_b) return hipErrorInvalidValue;
  if (!fault && variant >= 19) return hipErrorInvalidValue;
  switch (variant) {
    case 19:
      return launch_hp<4, 3, 16>(pk, pk_stride, sig, sig_stride, msg, msg_stride, n, flags_out, strict_bits, comb_b,
                                 fault, stream);
    case 21:
      if (n <= hsv::kQuadMax)
        return launch_quad<4, 16>(pk, pk_stride, sig, sig_stride, msg, msg_stride, n, flags_out, strict_bits, comb_b,
                                  fault, stream);
      if (n <= hsv::kJointMax)
        return launch_joint<4, 16>(pk, pk_stride, sig, sig_stride, msg, msg_stride, n, flags_out, strict_bits, comb_b,
                                   fault, stream);
      if (n <= row_max())
        return launch_row<4, 16>(pk, pk_stride, sig, sig_stride, msg, msg_stride, n, flags_out, strict_bits, comb_b,
                                 fault, stream);
      if (n <= kPairMax)
        return launch_pair<4, 16>(pk, pk_stride, sig, sig_stride, msg, msg_stride, n, flags_out, strict_bits, comb_b,
                                  fault, stream);
      return launch_hp<4, HSV_HP_WAVES, 16>(pk, pk_stride, sig, sig_stride, msg, msg_stride, n, flags_out, strict_bits,
                                            comb_b, fault, stream);
    default: return hipErrorInvalidValue;
  }
}

extern "C" hipError_t hsv_launch_verify_tx(int variant, const uint8_t *txs, const uint64_t *offsets,
                                           uint64_t tx_size, uint32_t n, uint8_t *records, uint8_t *flags_out,
                                           uint32_t *strict_bits, const uint32_t *comb_b, uint32_t *fault,
                                           hipStream_t stream) {
  if (n == 0) return hipSuccess;
  if ((variant == 19 || variant == 21) && n > kPairMax) {
    if (!comb_b || !fault) return hipErrorInvalidValue;
    const TxPrep tx{txs, offsets, tx_size, records};
    return launch_hp<4, HSV_HP_WAVES, 16>(nullptr, 0, nullptr, 0, nullptr, 0, n, flags_out, strict_bits, comb_b,
                                          fault, stream, &tx);
  }
  hipError_t e = hsv_launch_tx_records(txs, offsets, tx_size, n, records, stream);
  if (e != hipSuccess) return e;
  return hsv_launch_verify(variant, records, 128, records + 32, 128, records + 96, 128, n, flags_out, strict_bits,
                           comb_b, fault, stream);
}

// Variant ids compiled into this library.  The product build carries the
// default (21: variant 19's two-pass kernels above 2^13 items, the pair-lane
// latency form at or below) and 19 itself.  The other ids of earlier rounds
// are measurement history (git history before round 5's cleanup).
static const int kVariantIds[] = {19, 21};

extern "C" int hsvi_variant_list(int *out, int cap) {
  const int n = (int)(sizeof(kVariantIds) / sizeof(kVariantIds[0]));
  for (int i = 0; out && i < n && i < cap; ++i) out[i] = kVariantIds[i];
  return n;
}

extern "C" int hsvi_variant_available(int variant) {
  for (int v : kVariantIds)
    if (v == variant) return 1;
  return 0;
}

extern "C" double hsv_launch_mad_peak(int device_cus) {
  // device-wide waits and a free below: the resident service is paused
  struct Pause {
    Pause() { hsvi_resident_pause(1); }
    ~Pause() { hsvi_resident_pause(0); }
  } pause;
  uint32_t *sink = nullptr;
  if (hipMalloc(&sink, 64) != hipSuccess) return -1.0;
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const int grid = device_cus * 8;
  hipLaunchKernelGGL(hsv::hsv_mad_peak_kernel, dim3(grid), dim3(256), 0, 0, sink, 1u);
  (void)hipDeviceSynchronize();
  (void)hipEventRecord(e0, 0);
  const int reps = 5;
  for (int r = 0; r < reps; ++r)
    hipLaunchKernelGGL(hsv::hsv_mad_peak_kernel, dim3(grid), dim3(256), 0, 0, sink, (uint32_t)r);
  (void)hipEventRecord(e1, 0);
  (void)hipEventSynchronize(e1);
  float ms = 0.f;
  (void)hipEventElapsedTime(&ms, e0, e1);
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  (void)hipFree(sink);
  const double macs = (double)reps * grid * 256.0 * hsv::kPeakIters * 16.0;
  return ms > 0.f ? macs / (ms * 1e-3) : -1.0;
}

// The lattice bound of the comb-path prepass (tests): 0 restores the default
// (kLatCombBits); otherwise 128..kLatCombBits.  Returns the previous bound, or
// -1 for an out-of-range value.
extern "C" int hsvi_set_lattice_bits(int bits) {
  if (bits == 0) bits = hsv::kLatCombBits;
  if (bits < 128 || bits > hsv::kLatCombBits) return -1;
  return g_lat_bits.exchange(bits);
}

// Fault injection mode of the calling thread's following launches (kInject*:
// 1 zeroed tables, 2 overwritten canary, 3 flipped table bits, 4 a record
// batch of the fused transaction launch never published; 0 = off).
// Returns the previous mode, or -1 for an unknown one.
extern "C" int hsvi_set_inject(int mode) {
  if (mode < 0 || mode > (int)hsv::kInjectNoPublish) return -1;
  const int prev = (int)t_inject;
  t_inject = (uint32_t)mode;
  return prev;
}
extern "C" int hsvi_inject_mode(void) { return (int)t_inject; }

namespace {
__global__ void hsv_fault_exchange_kernel(uint32_t *words, uint32_t *out) {
  if (threadIdx.x < 2) out[threadIdx.x] = atomicExch(&words[threadIdx.x], 0u);
}
}  // namespace

extern "C" hipError_t hsv_launch_fault_exchange(uint32_t *words, uint32_t *out, hipStream_t stream) {
  hipLaunchKernelGGL(hsv_fault_exchange_kernel, dim3(1), dim3(64), 0, stream, words, out);
  return hipGetLastError();
}

extern "C" int hsv_variant_needs_comb(int variant) {
  if (variant >= 10 && variant <= 14) return 8;
  if (variant >= 15 && variant <= 22) return 16;
  return 0;
}

#ifdef HSV_PHASE_CLOCKS
extern "C" __attribute__((visibility("default"))) int hsv_phase_clocks_read(uint64_t *dst, size_t words, int clear) {
  const size_t nw = std::min<size_t>(words, (size_t)hsv::kPhaseCap * 8);
  if (hipMemcpyFromSymbol(dst, HIP_SYMBOL(hsv::g_phase_clk), nw * sizeof(uint64_t)) != hipSuccess) return -1;
  if (clear) {
    void *p = nullptr;
    if (hipGetSymbolAddress(&p, HIP_SYMBOL(hsv::g_phase_clk)) != hipSuccess) return -1;
    if (hipMemset(p, 0, (size_t)hsv::kPhaseCap * 8 * sizeof(uint64_t)) != hipSuccess) return -1;
  }
  return 0;
}
#endif

#ifdef HSV_QUAD_CLOCKS
// Measurement builds only: block 0's stamps of the last quad-form launch (3
// waves x 8 u64, 100 MHz); 0 or -1 on a HIP error.
extern "C" __attribute__((visibility("default"))) int hsv_quad_clocks(uint64_t *out) {
  if (hipDeviceSynchronize() != hipSuccess) return -1;
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(hsv::g_quad_clk), sizeof(hsv::g_quad_clk)) == hipSuccess ? 0 : -1;
}
#endif
