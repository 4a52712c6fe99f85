// The exported test and measurement hooks of libhsv_test.so (declared in
// csrc/hsv_test_hooks.h).  Each forwards to an internal, hidden function of
// the shared objects; libhsv.so is linked without this file.
#include "hsv_test_hooks.h"

#include <string>
#include <thread>
#include <vector>

#include "hsv_host.h"
#include "hsv_internal.h"

extern "C" {

int hsv_test_inject_fault(int mode) { return hsvi_set_inject(mode); }
int hsv_test_inject_mode(void) { return hsvi_inject_mode(); }
int hsv_test_corrupt_auto_committee(void) { return hsvh::auto_committee_corrupt_tables(); }
int hsv_test_lanesplit_check(const uint32_t *in, uint32_t rows, uint32_t *out) {
  return hsvi_lanesplit_check(in, rows, out);
}
int hsv_set_lattice_bits(int bits) { return hsvi_set_lattice_bits(bits); }
int hsv_set_variant(int variant) { return hsvi_set_variant(variant); }
int hsv_variant_list(int *out, int cap) { return hsvi_variant_list(out, cap); }
int hsv_variant_available(int variant) { return hsvi_variant_available(variant); }
int hsv_num_variants(void) { return hsvi_num_variants(); }
int hsv_set_virtual_shards(int k) { return hsvi_set_virtual_shards(k); }
int hsv_test_pipe_nocopy(int on) { return hsvi_set_pipe_nocopy(on); }
int hsv_test_pipe_schedule(const uint64_t *sizes, int count) { return hsvi_set_pipe_schedule(sizes, count); }

int hsv_test_numa_plan(const char *sysfs_root, const char *bdfs_csv, const char *allowed_cpulist, int pack_default,
                       int *node_out, int *ncpus_out, int *pack_out, int cap) {
  if (!sysfs_root || !bdfs_csv || !allowed_cpulist) return HSV_ERR_INVALID_ARG;
  std::vector<std::string> bdfs;
  std::string cur;
  for (const char *p = bdfs_csv;; ++p) {
    if (*p == ',' || *p == '\0') {
      bdfs.push_back(cur);
      cur.clear();
      if (*p == '\0') break;
    } else {
      cur += *p;
    }
  }
  std::vector<int> allowed;
  if (!hsvh::parse_cpulist(allowed_cpulist, allowed)) return HSV_ERR_INVALID_ARG;
  const std::vector<hsvh::HostPlace> pl = hsvh::plan_host_places(sysfs_root, bdfs, allowed, pack_default);
  for (int i = 0; i < (int)pl.size() && i < cap; ++i) {
    if (node_out) node_out[i] = pl[i].node;
    if (ncpus_out) ncpus_out[i] = (int)pl[i].cpus.size();
    if (pack_out) pack_out[i] = pl[i].pack_threads;
  }
  return (int)pl.size();
}

int hsv_test_pinned_thread_cpus(const char *cpulist, int *cpus_out, int cap) {
  std::vector<int> want;
  if (!cpulist || !hsvh::parse_cpulist(cpulist, want)) return HSV_ERR_INVALID_ARG;
  std::vector<int> got;
  bool ok = false;
  std::thread t([&] {
    ok = hsvh::pin_current_thread(want);
    got = hsvh::current_affinity();
  });
  t.join();
  if (!ok) return HSV_ERR_INVALID_ARG;
  for (int i = 0; i < (int)got.size() && i < cap; ++i) cpus_out[i] = got[i];
  return (int)got.size();
}
void hsv_test_resident_counts(uint64_t *posted, uint64_t *answered) { hsvh::resident_counts(posted, answered); }
int hsv_test_resident_post_bad(uint32_t m) { return hsvh::resident_post_bad(m); }
int hsv_test_tx_records(const uint8_t *d_txs, const uint64_t *d_offsets, size_t tx_size, size_t n,
                        uint8_t *d_records, void *stream) {
  if (n > UINT32_MAX) return HSV_ERR_INVALID_ARG;
  const hipError_t e = hsv_launch_tx_records(d_txs, d_offsets, tx_size, (uint32_t)n, d_records,
                                             reinterpret_cast<hipStream_t>(stream));
  return e == hipSuccess ? HSV_OK : HSV_ERR_HIP;
}

}  // extern "C"
