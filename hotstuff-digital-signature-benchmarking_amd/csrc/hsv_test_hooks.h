/*
 * hsv_test_hooks.h -- test and measurement hooks of libhsv_test.so.
 *
 * libhsv_test.so is libhsv.so's object files plus csrc/hsv_test_hooks.cpp:
 * the same kernels and host code, and in addition the hooks below.  The
 * product library exports none of them (tests/test_capi.py checks its
 * dynamic symbols against include/hsv.h), so no stray call can change the
 * behaviour of a deployed process.  tests/ and tools/ load libhsv_test.so
 * for the cases that need a hook (hsverify/_testing.py).
 */
#ifndef HSV_TEST_HOOKS_H_
#define HSV_TEST_HOOKS_H_

#include "hsv.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Fault injection for the launches the CALLING THREAD issues from now on
 * (csrc/hsv_verify_core.hpp kInject*: 1 zeroed tables, 2 overwritten
 * workspace canary, 3 one flipped table bit; 0 = off).  Other threads' calls
 * are unaffected.  Returns the previous mode, or -1 for an unknown one. */
HSV_API int hsv_test_inject_fault(int mode);
HSV_API int hsv_test_inject_mode(void);
/* Zero the tables of the automatic committee cache in HBM (a real
 * corruption, for the cached path's self-check); returns the number of
 * cached keys, 0 when there is no cache, < 0 on error. */
HSV_API int hsv_test_corrupt_auto_committee(void);
/* Row-form field arithmetic against the one-lane form (tests/test_lanesplit.py). */
HSV_API int hsv_test_lanesplit_check(const uint32_t *in, uint32_t rows, uint32_t *out);
/* Lattice bound of the comb-path prepass (0 = default 138; 133 sends the
 * lattice-fallback fixtures down the full-length path); previous bound or -1. */
HSV_API int hsv_set_lattice_bits(int bits);
/* Kernel variant of the following calls (the ids hsv_variant_list reports). */
HSV_API int hsv_set_variant(int variant);
HSV_API int hsv_variant_list(int *out, int cap);
HSV_API int hsv_variant_available(int variant);
HSV_API int hsv_num_variants(void);
/* Split host batches of >= 2^16 items into k shards on the bound device
 * (the multi-device gather path on a one-GPU box); 0 restores the default. */
HSV_API int hsv_set_virtual_shards(int k);
/* Measurement only (tools/host_api_ab.py): a pipelined host call of the same
 * size as the slot's previous one skips the pack and the copies and verifies
 * what that call left in HBM -- the chunk schedule's GPU time alone.  Its
 * flags are the previous inputs' flags, so it never belongs in a product
 * library.  Returns the previous setting. */
HSV_API int hsv_test_pipe_nocopy(int on);
/* Measurement only (tools/host_sched_ab.py): the launch-chunk sizes of the
 * pipelined host call (items; the last size repeats; count 0 restores the
 * default schedule).  Returns HSV_OK or HSV_ERR_INVALID_ARG. */
HSV_API int hsv_test_pipe_schedule(const uint64_t *sizes, int count);
/* Host placement plan (csrc/hsv_numa.cpp) for the PCI functions in bdfs_csv
 * ("0000:0d:00.0,...") under a sysfs tree at sysfs_root, within the CPUs of
 * allowed_cpulist ("0-7"): per function its NUMA node (-1 unknown), the
 * number of that node's allowed CPUs its threads are pinned to, and its
 * pack-pool size.  Returns the number of functions or HSV_ERR_INVALID_ARG. */
HSV_API int hsv_test_numa_plan(const char *sysfs_root, const char *bdfs_csv, const char *allowed_cpulist,
                               int pack_default, int *node_out, int *ncpus_out, int *pack_out, int cap);
/* A thread pinned the way the library pins its shard workers and pack
 * helpers, to the CPUs of `cpulist`: the affinity it then reports (count, CPUs
 * written to cpus_out), or HSV_ERR_INVALID_ARG. */
HSV_API int hsv_test_pinned_thread_cpus(const char *cpulist, int *cpus_out, int cap);
/* The resident latency service (HSV_QC_RESIDENT=1): requests posted to it and
 * answered by it in this process so far (either pointer may be NULL). */
HSV_API void hsv_test_resident_counts(uint64_t *posted, uint64_t *answered);
/* Post one resident request whose header claims m votes (0, or above the
 * service's limit): the kernel must refuse it, so the call returns
 * HSV_ERR_DEVICE_FAULT without reading through the header. */
HSV_API int hsv_test_resident_post_bad(uint32_t m);
/* Measurement only (tools/mempool_split_probe.py): the 128-byte records
 * pk || R || s || SHA-512(message)[..32] of n transactions, enqueued on
 * `stream` (the record kernel of hsv_verify_transactions_device's small-batch
 * form, without the verification). */
HSV_API int hsv_test_tx_records(const uint8_t *d_txs, const uint64_t *d_offsets, size_t tx_size, size_t n,
                                uint8_t *d_records, void *stream);

#ifdef __cplusplus
}
#endif

#endif /* HSV_TEST_HOOKS_H_ */
