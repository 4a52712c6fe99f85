// The point pass's shared pieces (hsv_kernels.hip: hsv_verify_hp_kernel and
// the latency forms; hsv_mempool.hip: the fused transaction launch): the
// per-lane table store, record loads, work counters and the device
// self-check words.
#pragma once
#include <hip/hip_runtime.h>

#include "hsv_verify_core.hpp"

#ifndef HSV_HP_WAVES
#define HSV_HP_WAVES 3  // waves per SIMD of the point pass (launch bounds: 168 VGPRs)
#endif

namespace hsv {

constexpr int kBlock = 256;


// Per-lane variable-base tables in global memory (hsv_verify_core.hpp, VT):
// lane region = 2 tables x (ENT - 1) entries x 128 B, entry = 8 x uint4.
// Entry 0 of every table is the identity: it is not stored per lane; a zero
// digit reads this one shared line (L2-resident) instead.  Loose encoding of
// (Y+X, Y-X, 2Z, 2dT) = (1, 1, 2, 0).
__device__ const uint4 kVtIdentity[8] = {{1u, 0u, 0u, 0u}, {0u, 0u, 0u, 0u}, {1u, 0u, 0u, 0u}, {0u, 0u, 0u, 0u},
                                         {2u, 0u, 0u, 0u}, {0u, 0u, 0u, 0u}, {0u, 0u, 0u, 0u}, {0u, 0u, 0u, 0u}};

// Fault injection (hsv_test_inject_fault, tests only; uniform kernel argument,
// kInject* in hsv_verify_core.hpp): the table stores of every lane are
// replaced, between the table build and the window loop, by what a corrupted
// workspace would hold.
template <int ENT>
struct GlobalVarTab {
  static constexpr int kStored = ENT - 1;  // entries 1 .. ENT-1 per table
  uint4 *base;
  uint32_t inject = kInjectNone;
  __device__ __forceinline__ void put(int t, int m, const uint32_t w[32]) const {
    if (m == 0) return;
    uint4 *e = base + (t * kStored + m - 1) * 8;
    if (__builtin_expect(inject == kInjectZeroTables || (inject == kInjectFlipTables && t == 0), 0)) {
      HSV_UNROLL
      for (int q = 0; q < 8; ++q)
        e[q] = inject == kInjectZeroTables ? make_uint4(0u, 0u, 0u, 0u)
                                           : make_uint4(w[4 * q] ^ (q == 0 ? 1u : 0u), w[4 * q + 1], w[4 * q + 2],
                                                        w[4 * q + 3]);
      return;
    }
    HSV_UNROLL
    for (int q = 0; q < 8; ++q) {
#ifdef HSV_TIMING_STUB_TABLE_STORES  // timing probe only: entries computed, never stored
      asm volatile("" ::"v"(w[4 * q]), "v"(w[4 * q + 1]), "v"(w[4 * q + 2]), "v"(w[4 * q + 3]));
#else
      e[q] = make_uint4(w[4 * q], w[4 * q + 1], w[4 * q + 2], w[4 * q + 3]);
#endif
    }
  }
  __device__ __forceinline__ void get(int t, uint32_t m, uint32_t w[32]) const {
    const uint4 *e = m ? base + (t * kStored + (int)m - 1) * 8 : kVtIdentity;
    HSV_UNROLL
    for (int q = 0; q < 8; ++q) {
      const uint4 v = e[q];
      w[4 * q] = v.x; w[4 * q + 1] = v.y; w[4 * q + 2] = v.z; w[4 * q + 3] = v.w;
    }
  }
};

template <int WA>
constexpr int vt_lane_uint4() { return 2 * (1 << (WA - 1)) * 8; }


// one (pk, sig, msg) record into words
__device__ __forceinline__ void load_triple(const uint8_t *pk, uint64_t pk_stride, const uint8_t *sig,
                                            uint64_t sig_stride, const uint8_t *msg, uint64_t msg_stride,
                                            uint64_t i, uint32_t pkw[8], uint32_t sigw[16], uint32_t msgw[8]) {
  const uint4 *p = reinterpret_cast<const uint4 *>(pk + i * pk_stride);
  const uint4 *s = reinterpret_cast<const uint4 *>(sig + i * sig_stride);
  const uint4 *m = reinterpret_cast<const uint4 *>(msg + i * msg_stride);
  const uint4 p0 = p[0], p1 = p[1];
  const uint4 s0 = s[0], s1 = s[1], s2 = s[2], s3 = s[3];
  const uint4 m0 = m[0], m1 = m[1];
  pkw[0] = p0.x; pkw[1] = p0.y; pkw[2] = p0.z; pkw[3] = p0.w;
  pkw[4] = p1.x; pkw[5] = p1.y; pkw[6] = p1.z; pkw[7] = p1.w;
  sigw[0] = s0.x; sigw[1] = s0.y; sigw[2] = s0.z; sigw[3] = s0.w;
  sigw[4] = s1.x; sigw[5] = s1.y; sigw[6] = s1.z; sigw[7] = s1.w;
  sigw[8] = s2.x; sigw[9] = s2.y; sigw[10] = s2.z; sigw[11] = s2.w;
  sigw[12] = s3.x; sigw[13] = s3.y; sigw[14] = s3.z; sigw[15] = s3.w;
  msgw[0] = m0.x; msgw[1] = m0.y; msgw[2] = m0.z; msgw[3] = m0.w;
  msgw[4] = m1.x; msgw[5] = m1.y; msgw[6] = m1.z; msgw[7] = m1.w;
}

// Work counters of the comb kernels, zeroed before the launch (32 bytes).
struct HcCounters {
  uint32_t next;      // main pass: next item handed out
  uint32_t fb_count;  // deferred full-length items appended to fb_list
  uint32_t fb_next;   // fallback pass: next fb_list entry handed out
  uint32_t pad;
  uint32_t rnext;     // fused transaction launch: next 64-transaction record batch handed out
  uint32_t rdone;     // fused transaction launch: record batches published
  uint32_t pad2[2];
};

// Device self-checks of the product kernels (a device failure must
// never become a silent reject).  Each launch gets
//   fault[2]  two words the host zeroed: fault[0] <- 1 when an item's final
//             point fails ge_is_sane (kFault), fault[1] <- 1 when a lane's
//             canary changed; written with plain stores once the work loop
//             is done (no atomics, so the words may live in pinned host memory);
//   canary    one word per lane slot of the workspace, set to the launch's
//             nonce when the lane starts and compared after every batch.
// The host turns a non-zero word into HSV_ERR_DEVICE_FAULT.
__device__ __forceinline__ void report_faults(uint32_t *fault, uint32_t bad) {
  if (bad & 1u) fault[0] = 1u;
  if (bad & 2u) fault[1] = 1u;
}

}  // namespace hsv
