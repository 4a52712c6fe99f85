// Internal interfaces between the C-ABI layer (hsv_capi.cpp) and the kernels.
#pragma once
#include <hip/hip_runtime_api.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

// Enqueue one verification launch on `stream` (no synchronisation).
int hsv_num_variants(void);
hipError_t hsv_launch_verify(int variant, const uint8_t *pk, uint64_t pk_stride, const uint8_t *sig,
                             uint64_t sig_stride, const uint8_t *msg, uint64_t msg_stride,
                             uint32_t n, uint8_t *flags_out, uint32_t *strict_bits,
                             hipStream_t stream);

// Time the v_mad_u64_u32 probe on the current device; MAC/s.
double hsv_launch_mad_peak(int device_cus);

#ifdef __cplusplus
}
#endif
