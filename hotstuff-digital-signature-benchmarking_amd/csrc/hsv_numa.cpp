// Host placement of the library's own threads (DESIGN.md
// section 7): each GPU's NUMA node, read from sysfs, and the CPUs of that
// node the process may run on.  The shard workers of a multi-GPU host batch
// and the helpers of each device's pack pool run there, and they allocate and
// first touch that device's pinned staging, so the pack writes and the DMA
// reads of a shard stay on the GPU's own socket.  The library never moves the
// application's threads; it only places the threads it starts.
#include <hip/hip_runtime_api.h>
#include <sched.h>

#include <algorithm>
#include <cctype>
#include <cstdlib>
#include <fstream>
#include <map>
#include <mutex>
#include <sstream>
#include <string>
#include <thread>
#include <vector>

#include "hsv_host.h"

namespace hsvh {

// "0-3,8,10-11" -> {0,1,2,3,8,10,11}; false on a malformed list
bool parse_cpulist(const std::string &text, std::vector<int> &out) {
  out.clear();
  std::stringstream ss(text);
  std::string part;
  while (std::getline(ss, part, ',')) {
    part.erase(std::remove_if(part.begin(), part.end(), [](unsigned char c) { return std::isspace(c); }), part.end());
    if (part.empty()) continue;
    const size_t dash = part.find('-');
    char *end = nullptr;
    const long lo = std::strtol(part.c_str(), &end, 10);
    if (end == part.c_str() || lo < 0) return false;
    long hi = lo;
    if (dash != std::string::npos) {
      const char *h = part.c_str() + dash + 1;
      hi = std::strtol(h, &end, 10);
      if (end == h || hi < lo) return false;
    } else if (*end != '\0') {
      return false;
    }
    if (hi - lo > 65536) return false;
    for (long c = lo; c <= hi; ++c) out.push_back((int)c);
  }
  std::sort(out.begin(), out.end());
  out.erase(std::unique(out.begin(), out.end()), out.end());
  return true;
}

namespace {

bool read_file(const std::string &path, std::string &out) {
  std::ifstream f(path);
  if (!f) return false;
  std::stringstream ss;
  ss << f.rdbuf();
  out = ss.str();
  return true;
}

std::string lower(std::string s) {
  for (char &c : s) c = (char)std::tolower((unsigned char)c);
  return s;
}

}  // namespace

std::vector<int> current_affinity() {
  std::vector<int> cpus;
  cpu_set_t set;
  CPU_ZERO(&set);
  if (sched_getaffinity(0, sizeof(set), &set) != 0) return cpus;
  for (int c = 0; c < CPU_SETSIZE; ++c)
    if (CPU_ISSET(c, &set)) cpus.push_back(c);
  return cpus;
}

bool pin_current_thread(const std::vector<int> &cpus) {
  if (cpus.empty()) return false;
  cpu_set_t set;
  CPU_ZERO(&set);
  for (int c : cpus)
    if (c >= 0 && c < CPU_SETSIZE) CPU_SET(c, &set);
  return sched_setaffinity(0, sizeof(set), &set) == 0;
}

int default_pack_threads() {
  // 11 helpers + the caller, capped by the CPUs this process may run on (the
  // GPU box's cgroup gives a job 16); at 12 copying threads the pack of 2^20
  // triples takes ~1.1-1.4 ms (tools/host_pipeline_probe.py, BENCH r05/r06)
  int n = std::min(11, (int)std::thread::hardware_concurrency() - 1);
  if (const char *v = std::getenv("HSV_PACK_THREADS")) n = std::atoi(v);
  return std::max(0, std::min(n, 32));
}

std::vector<HostPlace> plan_host_places(const std::string &root, const std::vector<std::string> &bdfs,
                                        const std::vector<int> &allowed, int pack_default) {
  std::vector<HostPlace> places(bdfs.size());
  std::map<int, int> devs_on_node;
  for (size_t i = 0; i < bdfs.size(); ++i) {
    HostPlace &p = places[i];
    std::string text;
    if (bdfs[i].empty() || !read_file(root + "/bus/pci/devices/" + lower(bdfs[i]) + "/numa_node", text)) continue;
    char *end = nullptr;
    const long node = std::strtol(text.c_str(), &end, 10);
    if (end == text.c_str() || node < 0) continue;  // -1: a single-node host or no NUMA information
    std::vector<int> cpus;
    if (!read_file(root + "/devices/system/node/node" + std::to_string(node) + "/cpulist", text) ||
        !parse_cpulist(text, cpus))
      continue;
    p.node = (int)node;
    // only the CPUs the process may use (a cgroup or the application's own
    // binding may exclude the node: then the threads stay unpinned)
    std::vector<int> both;
    std::set_intersection(cpus.begin(), cpus.end(), allowed.begin(), allowed.end(), std::back_inserter(both));
    p.cpus = both;
    if (!both.empty()) ++devs_on_node[p.node];
  }
  for (HostPlace &p : places) {
    p.pack_threads = pack_default;
    if (p.cpus.empty()) continue;
    // the node's CPUs shared among the pack pools of its GPUs, one CPU of
    // each share left for that GPU's shard worker
    const int share = (int)p.cpus.size() / std::max(1, devs_on_node[p.node]);
    p.pack_threads = std::max(0, std::min(pack_default, share - 1));
  }
  return places;
}

const HostPlace &device_place(int device) {
  static std::mutex mu;
  static std::vector<HostPlace> places;
  static bool done = false;
  static const HostPlace none{-1, {}, default_pack_threads()};
  std::lock_guard<std::mutex> lk(mu);
  if (!done) {
    done = true;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
    (void)hipGetLastError();
    std::vector<std::string> bdfs(n);
    for (int d = 0; d < n; ++d) {
      char buf[64] = {0};
      if (hipDeviceGetPCIBusId(buf, sizeof(buf), d) == hipSuccess) bdfs[d] = buf;
      (void)hipGetLastError();
    }
    std::vector<int> allowed = current_affinity();
    std::sort(allowed.begin(), allowed.end());
    places = plan_host_places("/sys", bdfs, allowed, default_pack_threads());
  }
  return device >= 0 && device < (int)places.size() ? places[device] : none;
}

}  // namespace hsvh
