// Committee key cache kernels, see hsv_comb.hpp.
//
//  hsv_comb_build_kernel   one lane per (key, position j): [2^(8j)](+/-P) by
//                          8j doublings (j is wave-uniform: keys are padded to
//                          a multiple of 64 per position), 127 additions, one
//                          batched inversion -> 128 affine Niels entries.
//  hsv_comb_verify_kernel  one verification per lane against a cached key
//                          (key i's table at key_tables[i], so a cache can
//                          grow by appending table blocks without moving them):
//                          64 mixed additions from the key's table and the B
//                          table, then R decompression and the projective
//                          comparison.  Same flag byte as hsv_verify_kernel.
//  hsv_comb_verify_quad_fused_kernel  the same check for batches of at most
//                          2^12 votes (QC latency): four lanes per vote for
//                          the additions, R decompressed by a second wave.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <type_traits>

#include "hsv_comb.hpp"
#include "hsv_fe16x16.hpp"
#include "hsv_internal.h"

namespace hsv {

__global__ void __launch_bounds__(256)
hsv_comb_build_kernel(const uint8_t *__restrict__ encs, uint32_t nkeys, uint32_t npad, uint32_t negate,
                      uint32_t *__restrict__ tables, uint32_t *__restrict__ tmp,
                      uint8_t *__restrict__ key_flags) {
  const uint32_t id = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t j = id / npad, key = id % npad;
  if (j >= (uint32_t)kCombPos || key >= nkeys) return;
  uint32_t w[8];
  const uint4 *p = reinterpret_cast<const uint4 *>(encs + (uint64_t)key * 32);
  const uint4 p0 = p[0], p1 = p[1];
  w[0] = p0.x; w[1] = p0.y; w[2] = p0.z; w[3] = p0.w;
  w[4] = p1.x; w[5] = p1.y; w[6] = p1.z; w[7] = p1.w;
  fe x, y;
  const uint32_t ok = ge_decompress(w, x, y);
  if (j == 0 && key_flags) key_flags[key] = (uint8_t)((ok ? kKeyAOk : 0u) | (ok && y_is_small_order(y) ? kKeySmallA : 0u));
  const ge_ext base = comb_position_base(x, y, negate, (int)j);
  comb_build_position(base, tables + (uint64_t)key * kCombTableWords + (uint64_t)j * kCombEnt * kCombEntryWords,
                      tmp + (uint64_t)id * kCombEnt * 8);
}

__global__ void __launch_bounds__(256, 2)
hsv_comb_verify_kernel(const uint32_t *__restrict__ key_idx, const uint8_t *__restrict__ sig,
                       uint64_t sig_stride, const uint8_t *__restrict__ msg, uint64_t msg_stride,
                       uint32_t m, const uint8_t *__restrict__ pks, const uint8_t *__restrict__ key_flags,
                       uint32_t nkeys, const uint32_t *const *__restrict__ key_tables,
                       const uint32_t *__restrict__ btable, uint8_t *__restrict__ flags_out, uint32_t inject,
                       uint32_t *__restrict__ fault) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= m) return;
  const uint32_t kidx = key_idx[i];
  const bool kvalid = kidx < nkeys;
  const uint32_t kk = kvalid ? kidx : 0u;
  uint32_t pkw[8], sigw[16], msgw[8];
  {
    const uint4 *p = reinterpret_cast<const uint4 *>(pks + (uint64_t)kk * 32);
    const uint4 *s = reinterpret_cast<const uint4 *>(sig + (uint64_t)i * sig_stride);
    const uint4 *g = reinterpret_cast<const uint4 *>(msg + (uint64_t)i * msg_stride);
    const uint4 p0 = p[0], p1 = p[1];
    const uint4 s0 = s[0], s1 = s[1], s2 = s[2], s3 = s[3];
    const uint4 m0 = g[0], m1 = g[1];
    pkw[0] = p0.x; pkw[1] = p0.y; pkw[2] = p0.z; pkw[3] = p0.w;
    pkw[4] = p1.x; pkw[5] = p1.y; pkw[6] = p1.z; pkw[7] = p1.w;
    sigw[0] = s0.x; sigw[1] = s0.y; sigw[2] = s0.z; sigw[3] = s0.w;
    sigw[4] = s1.x; sigw[5] = s1.y; sigw[6] = s1.z; sigw[7] = s1.w;
    sigw[8] = s2.x; sigw[9] = s2.y; sigw[10] = s2.z; sigw[11] = s2.w;
    sigw[12] = s3.x; sigw[13] = s3.y; sigw[14] = s3.z; sigw[15] = s3.w;
    msgw[0] = m0.x; msgw[1] = m0.y; msgw[2] = m0.z; msgw[3] = m0.w;
    msgw[4] = m1.x; msgw[5] = m1.y; msgw[6] = m1.z; msgw[7] = m1.w;
  }
  const uint32_t f = verify_one_comb(pkw, key_flags[kk], sigw, msgw, key_tables[kk], btable, inject);
  if (f & kFault) fault[0] = 1u;  // device self-check (hsv_kernels.hip report_faults)
  flags_out[i] = kvalid ? (uint8_t)f : (uint8_t)0;
}

// Latency form of hsv_comb_verify_kernel for small batches (a QC is 67 or
// 667 votes): L = 16 lanes per vote, one DPP row.  Lane g of a
// vote's group adds the comb entries of positions [g P, (g+1) P), P = 32 / L,
// for both k (the key's table) and s (the B table): 2P mixed additions on the
// critical lane instead of 64; the group's partial sums meet through log2(L)
// lane-swap + addition rounds (16 lanes: 4 + 4 additions in sequence, 4 lanes:
// 16 + 2).  Every lane of the group hashes the vote (same instruction stream,
// no extra latency); flags come out of lane 0 exactly as verify_one_comb
// computes them.  With R decompressed on one lane (round 2) its root chain was
// the critical path and 16 lanes measured 4-7 % slower than 4
// (profiles/r02w_qc_ab.txt).  With the lane-split R waves the additions are
// the longer piece at 4 lanes per vote, and a block of 4 lanes per vote needs
// 5 waves, which then share SIMDs: C1 / C3 p50 0.099 / 0.105 ms at 4 lanes,
// 0.057 / 0.062 at 8 (3 waves), 0.055 / 0.062 at 16 (2 waves), against
// 0.082 / 0.088 ms for round 2's form (profiles/r03z_qc_ab.txt).  (The
// lane-count switch and the other closed latency-form experiments of rounds
// 3-4 -- one-lane R, one row per R, the hash on the comb wave or on every
// lane, one-lane final checks, compact root-chain and SHA-512 bodies -- were
// removed in round 5; they are in git history at 5c186e7.)
constexpr int kCombLanes = 16;
constexpr int kCombPosPerLane = kCombPos / kCombLanes;

// Checks of a vote's final sum spread over its 16-lane row: after the swap
// rounds every lane of the vote's row holds Q, and the row is a DPP row, so
// the self-check and the equation run as rounds of one field operation per
// lane (ge_is_sane_row, ge_eq_affine_row in hsv_fe16x16.hpp).

__device__ __forceinline__ ge_ext ge_swap_xor(const ge_ext &p, int m) {
  ge_ext r;
  HSV_UNROLL
  for (int i = 0; i < kFeLimbs; ++i) {
    r.X.v[i] = (uint32_t)__shfl_xor((int)p.X.v[i], m, 64);
    r.Y.v[i] = (uint32_t)__shfl_xor((int)p.Y.v[i], m, 64);
    r.Z.v[i] = (uint32_t)__shfl_xor((int)p.Z.v[i], m, 64);
    r.T.v[i] = (uint32_t)__shfl_xor((int)p.T.v[i], m, 64);
  }
  return r;
}

// The latency form in specialised waves (at <= kCombQuadMax votes): a block
// takes 64 / L votes.  Wave 0 computes each vote's combined sum
// Q = [s]B - [k]A over L lanes; the R waves decompress the votes' R at the
// same time on other SIMDs and leave (x, y, flags) in LDS.  R's root chain,
// the longest single piece, runs beside the hash and the comb additions: the
// vote costs max(hash + comb, root chain) + the final comparison.  The R
// waves hold one vote per 16-lane row with the products spread over the row
// (ge_decompress_row, hsv_fe16x16.hpp: 32 us for the root chain on a lone
// wave against 57 us on one lane, profiles/r03z_ubench_lanesplit.txt), four
// votes per wave.  Each vote takes two rows (RowLane2: a product's 16 steps
// split 8 + 8 between the rows, 25.4 against 32.2 us for the root chain,
// profiles/r03zz_ubench_lanesplit2.txt), two votes per wave.
constexpr int kRRows = 2;
using RLane = RowLane2;
constexpr int kRVotesPerWave = 4 / kRRows;
constexpr int kFusedVotes = 64 / kCombLanes;
constexpr int kFusedRWaves = (kFusedVotes + kRVotesPerWave - 1) / kRVotesPerWave;
// A hash wave (the last of the block) computes k = H(R || A || M) mod l and
// its comb digits for the block's votes while the comb wave adds the s half
// (the B table needs no hash), and hands the digits over in LDS: the comb
// wave's path becomes max(hash, s additions) + k additions + swap rounds
// instead of their sum.  A one-body SHA-512 (half the code fetched cold at
// each launch) measured no faster: 10.2 against 9.7 us at C1, 13.5 against
// 13.2 us at C3 (profiles/r04t_qcclk_*.txt).
constexpr uint32_t kHashWaveIdx = 1 + kFusedRWaves;
constexpr int kFusedThreads = 64 * (2 + kFusedRWaves);

#ifdef HSV_QC_WAVE_CLOCKS
// Measurement builds only (tools/qc_wave_clocks.py): lane 0 of every wave
// stamps the 100 MHz constant clock at fixed points of its path -- 0 entry,
// 1 past the entry barrier, 2 its own work done (comb: the s half), 3 the
// comb wave past the k handover (R and hash waves: their first loads
// landed), 4 at the final barrier, 5 exit; slot 6 holds the wave's place
// (XCC_ID << 32 | HW_ID: SIMD, CU, SH, SE), 7 / 8 the shader clock
// (s_memtime) at entry / exit, so the tool can tell a slower clock from
// shared SIMDs.
constexpr uint32_t kQcClkWaves = 4096;
constexpr int kQcClkSlots = 10;  // slot 9: HSV_QC_WAVE_CLOCKS_TWICE
__device__ uint64_t g_qc_clk[kQcClkWaves][kQcClkSlots];
#define HSV_QC_CLK(slot)                                                       \
  do {                                                                         \
    const uint32_t wi_ = blockIdx.x * (uint32_t)(kFusedThreads / 64) + wave;   \
    if (lane == 0u && wi_ < kQcClkWaves) {                                     \
      g_qc_clk[wi_][slot] = wall_clock64();                                    \
      if (slot == 0) {                                                         \
        g_qc_clk[wi_][7] = clock64();                                          \
        g_qc_clk[wi_][6] = ((uint64_t)__builtin_amdgcn_s_getreg((15 << 11) | 20) << 32) | \
                           (uint64_t)__builtin_amdgcn_s_getreg((31 << 11) | 4); \
      }                                                                        \
      if (slot == 5) g_qc_clk[wi_][8] = clock64();                             \
    }                                                                          \
  } while (0)
// slot 3 of the R and hash waves: once the wave's first loads have landed
#define HSV_QC_CLK_LOADED(slot)        \
  do {                                 \
    __builtin_amdgcn_s_waitcnt(0);     \
    HSV_QC_CLK(slot);                  \
  } while (0)
#else
#define HSV_QC_CLK(slot) \
  do {                   \
  } while (0)
#define HSV_QC_CLK_LOADED(slot) \
  do {                          \
  } while (0)
#endif

// Reading each block's inputs once into LDS before the entry barrier
// (instead of each wave reading its own vote words from the pinned staging)
// was measured and dropped in round 4: per-wave stamps put every role of the
// C3 kernel 4.4-4.6 us behind C1 either way, and the barrier ahead of every
// wave cost C1 3.5 us (profiles/r04i_qc_ab_stage.txt).  The resident service
// does stage its request in LDS, read in one load by wave 0 (below).

// one vote's words: the key A, the signature (R, s) and the message digest M
// (p / sp / gp: the vote's key encoding, signature and digest, in global
// memory or LDS)
__device__ __forceinline__ void load_vote_words(const uint4 *p, const uint4 *sp, const uint4 *gp, uint32_t pkw[8],
                                                uint32_t sigw[16], uint32_t msgw[8]) {
  const uint4 p0 = p[0], p1 = p[1];
  const uint4 s0 = sp[0], s1 = sp[1], s2 = sp[2], s3 = sp[3];
  const uint4 m0 = gp[0], m1 = gp[1];
  pkw[0] = p0.x; pkw[1] = p0.y; pkw[2] = p0.z; pkw[3] = p0.w;
  pkw[4] = p1.x; pkw[5] = p1.y; pkw[6] = p1.z; pkw[7] = p1.w;
  sigw[0] = s0.x; sigw[1] = s0.y; sigw[2] = s0.z; sigw[3] = s0.w;
  sigw[4] = s1.x; sigw[5] = s1.y; sigw[6] = s1.z; sigw[7] = s1.w;
  sigw[8] = s2.x; sigw[9] = s2.y; sigw[10] = s2.z; sigw[11] = s2.w;
  sigw[12] = s3.x; sigw[13] = s3.y; sigw[14] = s3.z; sigw[15] = s3.w;
  msgw[0] = m0.x; msgw[1] = m0.y; msgw[2] = m0.z; msgw[3] = m0.w;
  msgw[4] = m1.x; msgw[5] = m1.y; msgw[6] = m1.z; msgw[7] = m1.w;
}

// lane g's 8 P digit bits of a recoded scalar, starting at bit 8 g P
__device__ __forceinline__ uint64_t lane_digits(const uint32_t r[9], uint32_t g) {
  constexpr int kBits = 8 * kCombPosPerLane;
  uint64_t d = 0;
  HSV_UNROLL
  for (int q = 0; q < kCombLanes; ++q) {
    const int w = (q * kBits) / 32, sh = (q * kBits) % 32;
    const uint64_t v = ((((uint64_t)r[w + 1] << 32) | r[w]) >> sh) & (kBits == 64 ? ~0ull : ((1ull << kBits) - 1));
    d = g == (uint32_t)q ? v : d;
  }
  return d;
}

// One block's votes [blk * kFusedVotes, ...) of the latency form; the
// launched kernel below runs it for its blockIdx, the resident service
// (hsv_comb_resident_kernel) for block 0 of each request.
__device__ __forceinline__ void comb_quad_block(const uint32_t *__restrict__ key_idx, const uint8_t *__restrict__ sig,
                                                uint64_t sig_stride, const uint8_t *__restrict__ msg,
                                                uint64_t msg_stride, uint32_t m, const uint8_t *__restrict__ pks,
                                                const uint8_t *__restrict__ key_flags, uint32_t nkeys,
                                                const uint32_t *const *__restrict__ key_tables,
                                                const uint32_t *__restrict__ btable, uint8_t *__restrict__ flags_out,
                                                uint32_t inject, uint32_t *__restrict__ fault,
                                                uint32_t *__restrict__ done, uint32_t blk,
                                                const uint8_t *__restrict__ vote_pks = nullptr) {
  __shared__ uint32_t r_x[kFusedVotes][kFeLimbs], r_y[kFusedVotes][kFeLimbs], r_fl[kFusedVotes];
  __shared__ uint32_t k_rec[kFusedVotes][9], k_ready;
  const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63u;
  const uint32_t base = blk * kFusedVotes;
  HSV_QC_CLK(0);
#ifdef HSV_QC_WAVE_CLOCKS
  const uint64_t call_t0 = wall_clock64(), call_s0 = clock64();  // block entry, for hsv_qc_call_stamps
#endif
  // vote v of the block reads vote min(base + v, m - 1): the last block's
  // spare slots repeat the batch's last vote and write no flag
  auto vote_of = [&](uint32_t v) { return base + v < m ? base + v : m - 1u; };
  // LDS keeps the last block's flag: cleared before any wave can look
  if (threadIdx.x == 0) k_ready = 0u;
  __syncthreads();
  HSV_QC_CLK(1);
  // (the resident service passes key_idx / sig / msg pointing into its LDS copy of the request)
  auto vote_sig = [&](uint32_t v) { return reinterpret_cast<const uint4 *>(sig + (uint64_t)vote_of(v) * sig_stride); };
  auto vote_msg = [&](uint32_t v) { return reinterpret_cast<const uint4 *>(msg + (uint64_t)vote_of(v) * msg_stride); };
  auto vote_kidx = [&](uint32_t v) -> uint32_t { return key_idx[vote_of(v)]; };
  // the key's encoding: the committee's copy in HBM, or (resident service)
  // the request's copy in LDS -- the same bytes, the host found the member
  // index by comparing all 32 of them
  auto vote_pk = [&](uint32_t v, uint32_t kk) {
    return reinterpret_cast<const uint4 *>(vote_pks ? vote_pks + 32ull * vote_of(v) : pks + (uint64_t)kk * 32);
  };
  if (wave == kHashWaveIdx) {
    // one lane per vote hashes (lanes 0..kFusedVotes-1); the rest of the
    // wave stays masked off
    const uint32_t vl = lane;
    if (vl < (uint32_t)kFusedVotes) {
      const uint32_t kidx = vote_kidx(vl);
      const uint32_t kk = kidx < nkeys ? kidx : 0u;
      uint32_t pkw[8], sigw[16], msgw[8], h[16], kr[9];
      load_vote_words(vote_pk(vl, kk), vote_sig(vl), vote_msg(vl), pkw, sigw, msgw);
      HSV_QC_CLK_LOADED(3);
      sha512_96(sigw, pkw, msgw, h);
      const sc k = sc_reduce512(h);
      recode_add<9, 8, kCombPos>(k.v, 8, kr);
      HSV_UNROLL
      for (int w = 0; w < 9; ++w) k_rec[vl][w] = kr[w];
    }
    HSV_QC_CLK(2);
    __hip_atomic_store(&k_ready, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    HSV_QC_CLK(4);
    __syncthreads();
    HSV_QC_CLK(5);
    return;
  }
  if (wave >= 1) {
    const RLane L;
    const uint32_t row = lane >> 4;
    const uint32_t vr = (wave - 1u) * kRVotesPerWave + row / kRRows;  // this row's vote in the block
    if (vr < (uint32_t)kFusedVotes) {
      const uint4 *sp = vote_sig(vr);
      const uint4 s0 = sp[0], s1 = sp[1];
      HSV_QC_CLK_LOADED(3);
      const uint32_t rw[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
      fe rx, ry;
#ifdef HSV_TIMING_STUB_RWAVE  // tools/qc_phase_probe.py only: wrong flags, the quad path's time alone
      rx = fe_small(0);
      ry = fe_from_words_masked(rw);
      const uint32_t r_ok = 1u, small = 0u, nc = 0u;
#else
      uint32_t small, nc = 0;
#ifdef HSV_QC_WAVE_CLOCKS_TWICE  // measurement builds only: a second, warm-cache decompression
      {
        fe x2, y2;
        uint32_t small2, nc2 = 0;
        const uint32_t ok2 = ge_decompress_row(rw, x2, y2, small2, nc2, L);
        HSV_QC_CLK(9);
        nc |= (ok2 ^ ok2) | (x2.v[0] & 0u) | (small2 & 0u);  // keeps the first pass alive
        asm volatile("" ::"v"(x2.v[0]), "v"(y2.v[0]), "v"(ok2), "v"(nc2));
      }
#endif
      const uint32_t r_ok = ge_decompress_row(rw, rx, ry, small, nc, L);
#endif
      const uint32_t small_r = r_ok & small;
      if (L.k == 0u && row % kRRows == 0u) {
        HSV_UNROLL
        for (int l = 0; l < kFeLimbs; ++l) {
          r_x[vr][l] = rx.v[l];
          r_y[vr][l] = ry.v[l];
        }
        r_fl[vr] = r_ok | (small_r << 1) | (nc << 2);  // bit 2: self-check (fl_to_fe)
      }
    }
    HSV_QC_CLK(2);
    HSV_QC_CLK(4);
    __syncthreads();
    HSV_QC_CLK(5);
    return;
  }
  const uint32_t vl = lane / kCombLanes, g = lane % kCombLanes;
  const uint32_t i0 = base + vl;
  const bool valid = i0 < m;
  const uint32_t kidx = vote_kidx(vl);
  const bool kvalid = kidx < nkeys;
  const uint32_t kk = kvalid ? kidx : 0u;
  uint32_t pkw[8], sigw[16], msgw[8];
  load_vote_words(vote_pk(vl, kk), vote_sig(vl), vote_msg(vl), pkw, sigw, msgw);
  const uint32_t s_ok = sc_is_canonical(sigw + 8);
  // the key's flags now: read after the final barrier, this load's latency sat
  // on the call's critical path
  const uint32_t kf = key_flags[kk];
#ifdef HSV_TIMING_STUB_QUADPATH  // tools/qc_phase_probe.py only: wrong flags, the R waves' time alone
  ge_ext q = ge_identity();
  const uint32_t *ta = key_tables[kk];
  (void)ta;
#else
  const uint32_t *ta = key_tables[kk];
  ge_ext q = ge_identity();
  uint32_t sr[9];
  recode_add<9, 8, kCombPos>(sigw + 8, 8, sr);
  uint64_t sd = lane_digits(sr, g), kd;
  // the s half first, while the hash wave works on k
  HSV_NOUNROLL
  for (int jj = 0; jj < kCombPosPerLane; ++jj) {
    const uint32_t j = g * kCombPosPerLane + (uint32_t)jj;
    const CombPosTab tpb{btable + (uint64_t)j * kCombEnt * kCombEntryWords};
    q = ge_add_niels<true>(q, select_niels<8>(tpb, (uint32_t)sd & 0xffu));
    sd >>= 8;
  }
  HSV_QC_CLK(2);
  while (__hip_atomic_load(&k_ready, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) == 0u)
    __builtin_amdgcn_s_sleep(1);
  HSV_QC_CLK(3);
  {
    uint32_t kr[9];
    HSV_UNROLL
    for (int w = 0; w < 9; ++w) kr[w] = k_rec[vl][w];
    kd = lane_digits(kr, g);
  }
  HSV_NOUNROLL
  for (int jj = 0; jj < kCombPosPerLane; ++jj) {
    const uint32_t j = g * kCombPosPerLane + (uint32_t)jj;
    const CombPosTab tpa{ta + (uint64_t)j * kCombEnt * kCombEntryWords};
    ge_niels na = select_niels<8>(tpa, (uint32_t)kd & 0xffu);
    kd >>= 8;
    if (inject != kInjectNone && jj == 0) na = niels_injected(na, inject);
    q = ge_add_niels<true>(q, na);
  }
  HSV_UNROLL
  for (int mask = 1; mask < kCombLanes; mask <<= 1)
    q = ge_add_cached_rt(q, ge_to_cached(ge_swap_xor(q, mask)), mask < kCombLanes / 2);
#endif
  // the self-check of Q needs nothing from the R waves: before the barrier
  uint32_t z_nonzero = 0;
  const uint32_t sane = ge_is_sane_row(q, z_nonzero);
  HSV_QC_CLK(4);
  __syncthreads();
  fe rx, ry;
  HSV_UNROLL
  for (int l = 0; l < kFeLimbs; ++l) {
    rx.v[l] = r_x[vl][l];
    ry.v[l] = r_y[vl][l];
  }
  const uint32_t rf = r_fl[vl];
  const uint32_t r_ok = rf & 1u, small_r = (rf >> 1) & 1u;
  const uint32_t same = ge_eq_affine_row(q, rx, ry, z_nonzero);
  const uint32_t a_ok = (kf & kKeyAOk) ? 1u : 0u;
  const uint32_t small_a = a_ok & ((kf & kKeySmallA) ? 1u : 0u);
  const uint32_t parse_ok = s_ok & a_ok & r_ok;
  const uint32_t eq_ok = parse_ok & same;
  const uint32_t strict_ok = eq_ok & (small_a ^ 1u) & (small_r ^ 1u);
  const uint32_t f = (strict_ok ? kStrictOk : 0u) | (eq_ok ? kEqOk : 0u) | (parse_ok ? kParseOk : 0u) |
                     (small_a ? kSmallA : 0u) | (small_r ? kSmallR : 0u) | (s_ok ? kSOk : 0u) |
                     (a_ok ? kAOk : 0u) | (r_ok ? kROk : 0u);
  const uint32_t fb = a_ok & r_ok & (sane ^ 1u);
  if (fb | ((rf >> 2) & 1u)) fault[0] = 1u;  // device self-check (hsv_kernels.hip report_faults)
  if (valid && g == 0u) flags_out[i0] = kvalid ? (uint8_t)f : (uint8_t)0;
  HSV_QC_CLK(5);
#ifdef HSV_QC_WAVE_CLOCKS
  // measurement builds: block 0's entry and end (100 MHz constant clock) and
  // shader clock, next to the call's self-check words in pinned memory, so
  // the host reads them after each call without a device-wide sync
  // (tools/qc_tail_clocks.py); released with the flags below
  if (blk == 0u && lane == 0u && done) {
    uint64_t *st = reinterpret_cast<uint64_t *>(fault + 4);
    st[0] = call_t0;
    st[1] = wall_clock64();
    st[2] = call_s0;
    st[3] = clock64();
  }
#endif
  if (done) {
    // completion marker (HSV_QC_SYNC=marker): every wave of the block is past
    // its reads (the R and hash waves before the barrier / k_ready), and this
    // wave's flag and fault stores are released to the system before lane 0
    // marks the block done, so the host may read the flags off pinned memory
    // without waiting for the kernel's completion signal
    __atomic_thread_fence(__ATOMIC_RELEASE);
    if (lane == 0u) __hip_atomic_store(&done[blk], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

__global__ void __launch_bounds__(kFusedThreads)
hsv_comb_verify_quad_fused_kernel(const uint32_t *__restrict__ key_idx, const uint8_t *__restrict__ sig,
                                  uint64_t sig_stride, const uint8_t *__restrict__ msg, uint64_t msg_stride,
                                  uint32_t m, const uint8_t *__restrict__ pks, const uint8_t *__restrict__ key_flags,
                                  uint32_t nkeys, const uint32_t *const *__restrict__ key_tables,
                                  const uint32_t *__restrict__ btable, uint8_t *__restrict__ flags_out,
                                  uint32_t inject, uint32_t *__restrict__ fault, uint32_t *__restrict__ done) {
  comb_quad_block(key_idx, sig, sig_stride, msg, msg_stride, m, pks, key_flags, nkeys, key_tables, btable, flags_out,
                  inject, fault, done, blockIdx.x);
}

// The resident latency service (HSV_QC_RESIDENT=1, csrc/hsv_committee_api.cpp):
// one block that stays on its CU and answers requests of at most
// kResidentVotes votes posted in coherent pinned memory (QcResidentReq,
// hsv_internal.h), instead of a launch per request: a block of this shape
// answers a doorbell in 2.2 us against 5.8 us for a launch with marker sync
// (profiles/r05a_aql_latency.txt, tools/resident_latency.hip).  Per request:
//   * wave 0 polls the request itself: lanes 0..47 each read their 16-byte
//     chunk {seq, 3 payload words} with one uncached vector load (sc0 sc1, so
//     no cache can answer with an older copy), s_sleep between polls.  Once
//     every chunk carries the same new seq the whole request has arrived --
//     the host writes each chunk's payload before its seq, and x86 keeps
//     stores in order -- so the doorbell and the body take ONE PCIe round
//     trip.  (Round 4's form read eight header words one by one with
//     dependent LDS stores between them, ~10 us; the round-5 form before this
//     one took a doorbell read, a system-scope acquire and a body read.)
//   * the block validates the header before it dereferences anything: 1 <= m
//     <= kResidentVotes, non-null committee arrays, 1 <= nkeys <= 2^20.  An
//     invalid request is answered with kResidentBadRequest and no
//     verification (HSV_ERR_DEVICE_FAULT on the host), never with a memory
//     access;
//   * comb_quad_block reads the votes' key indices, key encodings, signatures
//     and digests from the LDS copy and writes its flags and self-check word
//     into LDS; thread 0 answers with two 8-byte system-scope stores {seq,
//     flags} and {seq, fault bits} -- each one transaction, so no release
//     fence (and no L2 write-back) is needed before them.
// It leaves on the stop word or after idle_ticks (100 MHz) without a request,
// and clears `alive` as it goes, so no grid outlives its process; the host
// relaunches it on the next request.
__device__ __forceinline__ uint4 load16_uncached(const void *p) {
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
  u32x4 r;
  asm volatile("global_load_dwordx4 %0, %1, off sc0 sc1\n\ts_waitcnt vmcnt(0)" : "=v"(r) : "v"(p) : "memory");
  return make_uint4(r.x, r.y, r.z, r.w);
}

constexpr uint32_t kResidentMaxKeys = 1u << 20;  // hsv_committee_create's bound and above the auto cache's

__global__ void __launch_bounds__(kFusedThreads) hsv_comb_resident_kernel(QcResidentReq *req, uint64_t idle_ticks) {
  __shared__ uint32_t payload[kResidentChunks * 3 + 4];  // QcResidentBody, word for word
  __shared__ uint32_t cmd_seq, cmd_stop, res_fault;
  __shared__ uint8_t res_flags[kResidentVotes];
  const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63u;
  const bool chunk_lane = lane < (uint32_t)kResidentChunks;
  uint32_t last = 0;
  if (wave == 0u) {
    last = __builtin_amdgcn_readfirstlane(load16_uncached(&req->chunk[0]).x);
    if (lane == 0u) __hip_atomic_store(&req->alive, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  for (;;) {
    if (wave == 0u) {
      const uint64_t t0 = wall_clock64();
      uint32_t sq = last, stop = 0;
      uint4 c = make_uint4(0, 0, 0, 0);
      for (;;) {
        if (chunk_lane) c = load16_uncached(&req->chunk[lane]);
        stop = __builtin_amdgcn_readfirstlane(__hip_atomic_load(&req->stop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM));
        sq = __builtin_amdgcn_readfirstlane(c.x);
        // the request is complete when every chunk carries chunk 0's seq and it is new
        const bool same = !chunk_lane || c.x == sq;
        if (stop || (sq != last && __all(same))) break;
        if (wall_clock64() - t0 > idle_ticks) {
          stop = 1u;
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
      last = sq;
      if (!stop && chunk_lane) {
        payload[3u * lane] = c.y;
        payload[3u * lane + 1u] = c.z;
        payload[3u * lane + 2u] = c.w;
      }
      if (lane == 0u) {
        cmd_seq = sq;
        cmd_stop = stop;
        res_fault = 0u;
      }
      if (lane < (uint32_t)kResidentVotes) res_flags[lane] = 0u;  // an unwritten flag reads as a rejection
    }
    __syncthreads();
    if (cmd_stop) break;
    const uint32_t sq = cmd_seq;
    const QcResidentBody &b = *reinterpret_cast<const QcResidentBody *>(payload);
    const uint32_t m = b.m, nkeys = b.nkeys;
    const bool valid = m >= 1u && m <= (uint32_t)kResidentVotes && m <= (uint32_t)kFusedVotes && nkeys >= 1u &&
                       nkeys <= kResidentMaxKeys && b.pks && b.key_flags && b.key_tables && b.btable;
    if (valid) {  // block-uniform: every wave takes the same branch
      comb_quad_block(b.key_idx, reinterpret_cast<const uint8_t *>(b.sig), 64,
                      reinterpret_cast<const uint8_t *>(b.msg), b.msg_per_vote ? 32 : 0, m, b.pks, b.key_flags,
                      nkeys, b.key_tables, b.btable, res_flags, b.inject, &res_fault, nullptr, 0u,
                      reinterpret_cast<const uint8_t *>(b.pk));
    }
    __syncthreads();  // every wave past its reads of this request and its LDS flag stores
    if (threadIdx.x == 0) {
      uint32_t fl = 0;
      for (int i = 0; i < kResidentVotes; ++i) fl |= (uint32_t)res_flags[i] << (8 * i);
      const uint32_t fb = (res_fault ? kResidentFaultCurve : 0u) | (valid ? 0u : kResidentBadRequest);
      __hip_atomic_store(&req->answer[0], (uint64_t)sq | ((uint64_t)fl << 32), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_SYSTEM);
      __hip_atomic_store(&req->answer[1], (uint64_t)sq | ((uint64_t)fb << 32), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
  if (threadIdx.x == 0) __hip_atomic_store(&req->alive, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Test hook (tests/test_lanesplit.py): the row forms of hsv_fe16x16.hpp
// against the one-lane form, one input of 16 words (a | b, 8 little-endian
// words each) per element: one 16-lane row (RowLane) or two (RowLane2).
// Bits (shifted by 3 for the two-row form): bit 0 a * b differs, bit 1
// a^((p-5)/8) differs, bit 2 ge_decompress_row(a) differs from
// ge_decompress(a) in its flag or, for a decodable a, in (x, y).
template <class Lane, int kRows>
__global__ void __launch_bounds__(64) hsv_lanesplit_check_kernel(const uint32_t *__restrict__ in, uint32_t rows,
                                                                 uint32_t *__restrict__ out) {
  const Lane L;
  constexpr uint32_t kPerWave = 4u / kRows, kShift = kRows == 1 ? 0u : 3u;
  const uint32_t r = blockIdx.x * kPerWave + (threadIdx.x >> 4) / kRows;
  const uint32_t rr = r < rows ? r : rows - 1u;
  uint32_t aw[8], bw[8];
  HSV_UNROLL
  for (int i = 0; i < 8; ++i) {
    aw[i] = in[16u * rr + i];
    bw[i] = in[16u * rr + 8u + i];
  }
  const fe a = fe_from_words_masked(aw), b = fe_from_words_masked(bw);
  uint32_t bad = 0;
  bad |= fe_eq(fe_mul(a, b), fl_to_fe(fl_mul(fl_from_fe(a, L), fl_from_fe(b, L), L), L)) ? 0u : 1u;
  bad |= fe_eq(fe_pow22523(a), fl_to_fe(fl_pow22523(fl_from_fe(a, L), L), L)) ? 0u : 2u;
  fe x0, y0, x1, y1;
  uint32_t small1;
  const uint32_t ok0 = ge_decompress(aw, x0, y0);
  uint32_t nc1 = 0;
  const uint32_t ok1 = ge_decompress_row(aw, x1, y1, small1, nc1, L);
  bad |= (ok0 == ok1 && nc1 == 0u && (!ok0 || (fe_eq(x0, x1) && fe_eq(y0, y1) && y_is_small_order(y0) == small1)))
             ? 0u
             : 4u;
  // the odd row of a pair checks its own copy too
  if constexpr (kRows == 2) bad |= __shfl_xor(bad, 16);
  if (r < rows && (threadIdx.x & (16u * kRows - 1u)) == 0u) out[r] |= bad << kShift;
}

// one lane per (position j, chunk c) of the wide B table; j is wave-uniform
// (256 chunks per position)
__global__ void __launch_bounds__(256) hsv_comb16_build_kernel(uint32_t *__restrict__ table,
                                                             uint32_t *__restrict__ tmp) {
  const uint32_t id = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t j = id / (uint32_t)kComb16ChunksPerPos, c = id % (uint32_t)kComb16ChunksPerPos;
  if (j >= (uint32_t)kComb16Pos) return;
  const uint32_t bw[8] = {0x66666658u, 0x66666666u, 0x66666666u, 0x66666666u,
                          0x66666666u, 0x66666666u, 0x66666666u, 0x66666666u};
  fe x, y;
  (void)ge_decompress(bw, x, y);
  comb16_build_chunk(x, y, (int)j, c, table, tmp + (uint64_t)id * kComb16Chunk * 8);
}

}  // namespace hsv

extern "C" hipError_t hsv_launch_comb16_build(uint32_t *table, uint32_t *tmp, hipStream_t stream) {
  const uint32_t lanes = (uint32_t)(hsv::kComb16Pos * hsv::kComb16ChunksPerPos);
  hipLaunchKernelGGL(hsv::hsv_comb16_build_kernel, dim3(lanes / 256u), dim3(256), 0, stream, table, tmp);
  return hipGetLastError();
}

// Test hook, not in hsv.h: runs hsv_lanesplit_check_kernel on the current
// device over `rows` host inputs of 16 words; 0 or a hipError_t.
extern "C" int hsvi_lanesplit_check(const uint32_t *in, uint32_t rows, uint32_t *out) {
  if (rows == 0) return 0;
  struct Pause {  // a device-wide wait and frees below
    Pause() { hsvi_resident_pause(1); }
    ~Pause() { hsvi_resident_pause(0); }
  } pause;
  uint32_t *d_in = nullptr, *d_out = nullptr;
  hipError_t e = hipMalloc(&d_in, (size_t)rows * 64);
  if (e == hipSuccess) e = hipMalloc(&d_out, (size_t)rows * 4);
  if (e == hipSuccess) e = hipMemcpy(d_in, in, (size_t)rows * 64, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemset(d_out, 0, (size_t)rows * 4);
  if (e == hipSuccess) {
    hipLaunchKernelGGL((hsv::hsv_lanesplit_check_kernel<hsv::RowLane, 1>), dim3((rows + 3) / 4), dim3(64), 0, 0,
                       d_in, rows, d_out);
    e = hipGetLastError();
  }
  if (e == hipSuccess) {
    hipLaunchKernelGGL((hsv::hsv_lanesplit_check_kernel<hsv::RowLane2, 2>), dim3((rows + 1) / 2), dim3(64), 0, 0,
                       d_in, rows, d_out);
    e = hipGetLastError();
  }
  if (e == hipSuccess) e = hipDeviceSynchronize();
  if (e == hipSuccess) e = hipMemcpy(out, d_out, (size_t)rows * 4, hipMemcpyDeviceToHost);
  if (d_in) (void)hipFree(d_in);
  if (d_out) (void)hipFree(d_out);
  return (int)e;
}

extern "C" uint64_t hsv_comb16_table_bytes(void) { return hsv::kComb16TableWords * 4ull; }
extern "C" uint64_t hsv_comb16_tmp_bytes(void) {
  return (uint64_t)hsv::kComb16Pos * hsv::kComb16ChunksPerPos * hsv::kComb16Chunk * 8ull * 4ull;
}

extern "C" hipError_t hsv_launch_comb_build(const uint8_t *encs, uint32_t nkeys, uint32_t negate,
                                            uint32_t *tables, uint32_t *tmp, uint8_t *key_flags,
                                            hipStream_t stream) {
  if (nkeys == 0) return hipSuccess;
  const uint32_t npad = (nkeys + 63u) / 64u * 64u;
  const uint32_t lanes = npad * (uint32_t)hsv::kCombPos;
  hipLaunchKernelGGL(hsv::hsv_comb_build_kernel, dim3((lanes + 255u) / 256u), dim3(256), 0, stream, encs,
                     nkeys, npad, negate, tables, tmp, key_flags);
  return hipGetLastError();
}

// batches up to this many votes take the four-lanes-per-vote form
static constexpr uint32_t kCombQuadMax = 1u << 12;

#ifdef HSV_QC_WAVE_CLOCKS
static thread_local uint32_t *t_last_fault = nullptr;  // the calling thread's last latency-form launch
#endif

extern "C" hipError_t hsv_launch_comb_verify(const uint32_t *key_idx, const uint8_t *sig, uint64_t sig_stride,
                                             const uint8_t *msg, uint64_t msg_stride, uint32_t m,
                                             const uint8_t *pks, const uint8_t *key_flags, uint32_t nkeys,
                                             const uint32_t *const *key_tables, const uint32_t *btable,
                                             uint8_t *flags_out, uint32_t *fault, uint32_t *done,
                                             hipStream_t stream) {
  if (m == 0) return hipSuccess;
  if (!fault) return hipErrorInvalidValue;
#ifdef HSV_QC_WAVE_CLOCKS
  t_last_fault = done ? fault : nullptr;
#endif
  const uint32_t inject = (uint32_t)hsvi_inject_mode();
  if (m <= kCombQuadMax) {  // latency form: four lanes per vote, R decompressed by the R waves
    hipLaunchKernelGGL(hsv::hsv_comb_verify_quad_fused_kernel, dim3((m + hsv::kFusedVotes - 1) / hsv::kFusedVotes),
                       dim3(hsv::kFusedThreads), 0, stream, key_idx, sig, sig_stride, msg, msg_stride, m, pks, key_flags, nkeys,
                       key_tables, btable, flags_out, inject, fault, done);
    return hipGetLastError();
  }
  if (done) return hipErrorInvalidValue;  // markers: latency form only
  hipLaunchKernelGGL(hsv::hsv_comb_verify_kernel, dim3((m + 255u) / 256u), dim3(256), 0, stream, key_idx, sig,
                     sig_stride, msg, msg_stride, m, pks, key_flags, nkeys, key_tables, btable, flags_out, inject,
                     fault);
  return hipGetLastError();
}

extern "C" hipError_t hsv_launch_comb_resident(QcResidentReq *d_req, uint64_t idle_ticks, hipStream_t stream) {
  if (!d_req) return hipErrorInvalidValue;
  hipLaunchKernelGGL(hsv::hsv_comb_resident_kernel, dim3(1), dim3(hsv::kFusedThreads), 0, stream, d_req, idle_ticks);
  return hipGetLastError();
}

extern "C" uint32_t hsv_comb_resident_votes(void) {
  return (uint32_t)std::min<int>(hsv::kFusedVotes, kResidentVotes);
}

extern "C" uint32_t hsv_comb_marker_blocks(uint32_t m) {
  return m <= kCombQuadMax ? (m + hsv::kFusedVotes - 1) / hsv::kFusedVotes : 0u;
}

extern "C" uint64_t hsv_comb_table_bytes(void) { return hsv::kCombTableWords * 4ull; }
extern "C" uint64_t hsv_comb_tmp_bytes(uint32_t nkeys) {
  const uint64_t npad = (nkeys + 63u) / 64u * 64u;
  return npad * (uint64_t)hsv::kCombPos * hsv::kCombEnt * 8ull * 4ull;
}

#ifdef HSV_QC_WAVE_CLOCKS
// Measurement builds only: copies the wave stamps of the last latency-form
// launches (waves x 10 u64: six 100 MHz stamps, place, shader clock, one
// spare stamp) to `out` and clears them; returns the
// waves per block, or -1 on a HIP error.
extern "C" __attribute__((visibility("default"))) int hsv_qc_wave_clocks(uint64_t *out, size_t waves) {
  const size_t n = std::min<size_t>(waves, hsv::kQcClkWaves) * hsv::kQcClkSlots * sizeof(uint64_t);
  if (hipDeviceSynchronize() != hipSuccess) return -1;
  if (out && hipMemcpyFromSymbol(out, HIP_SYMBOL(hsv::g_qc_clk), n) != hipSuccess) return -1;
  void *p = nullptr;
  if (hipGetSymbolAddress(&p, HIP_SYMBOL(hsv::g_qc_clk)) != hipSuccess) return -1;
  if (hipMemset(p, 0, sizeof(hsv::g_qc_clk)) != hipSuccess || hipDeviceSynchronize() != hipSuccess) return -1;
  return hsv::kFusedThreads / 64;
}

// Block 0's stamps of the calling thread's last marker-synced committee call
// (entry and end on the 100 MHz clock, shader clock at both): 4 words, read
// from the call's pinned sync region.  0, or -1 when there was no such call.
extern "C" __attribute__((visibility("default"))) int hsv_qc_call_stamps(uint64_t *out) {
  if (!t_last_fault || !out) return -1;
  hipPointerAttribute_t a;
  if (hipPointerGetAttributes(&a, t_last_fault) != hipSuccess || !a.hostPointer) return -1;
  std::memcpy(out, static_cast<const uint32_t *>(a.hostPointer) + 4, 4 * sizeof(uint64_t));
  return 0;
}

// The same without synchronising the device (a resident block keeps running):
// copies on a stream of its own, no clearing.
extern "C" __attribute__((visibility("default"))) int hsv_qc_wave_clocks_nosync(uint64_t *out, size_t waves) {
  const size_t n = std::min<size_t>(waves, hsv::kQcClkWaves) * hsv::kQcClkSlots * sizeof(uint64_t);
  hipStream_t st = nullptr;
  if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess) return -1;
  hipError_t e = hipMemcpyFromSymbolAsync(out, HIP_SYMBOL(hsv::g_qc_clk), n, 0, hipMemcpyDeviceToHost, st);
  if (e == hipSuccess) e = hipStreamSynchronize(st);
  (void)hipStreamDestroy(st);
  return e == hipSuccess ? hsv::kFusedThreads / 64 : -1;
}
#endif
