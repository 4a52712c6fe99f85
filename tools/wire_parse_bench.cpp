// Host-side cost of the bincode parsers (tools/, not built by default):
//   g++ -O3 -std=c++17 -Ihotstuff-digital-signature-benchmarking_amd/csrc -Iinclude tools/wire_parse_bench.cpp \
//       hotstuff-digital-signature-benchmarking_amd/csrc/hsv_wire_parse.cpp -o tools/wire_parse_bench
// with /tmp/tc.bin and /tmp/qc.bin written by tools/wire_samples.py (a C3 TC and QC).
#include "hsv_wire_parse.h"
#include <chrono>
#include <cstdio>
#include <fstream>
#include <iterator>
#include <vector>
#include <algorithm>
int main() {
  std::ifstream f("/tmp/tc.bin", std::ios::binary); std::vector<uint8_t> tc((std::istreambuf_iterator<char>(f)), {});
  std::ifstream g("/tmp/qc.bin", std::ios::binary); std::vector<uint8_t> qc((std::istreambuf_iterator<char>(g)), {});
  hsvw::TcParsed t; hsvw::QcParsed q; std::string err;
  for (int k = 0; k < 2; ++k) {
    std::vector<double> a, b;
    for (int i = 0; i < 2000; ++i) {
      auto t0 = std::chrono::steady_clock::now();
      bool ok = hsvw::parse_tc(tc.data(), tc.size(), t, err);
      auto t1 = std::chrono::steady_clock::now();
      bool ok2 = hsvw::parse_qc(qc.data(), qc.size(), q, err);
      auto t2 = std::chrono::steady_clock::now();
      if (!ok || !ok2) { printf("fail %s\n", err.c_str()); return 1; }
      a.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count());
      b.push_back(std::chrono::duration<double, std::micro>(t2 - t1).count());
    }
    std::sort(a.begin(), a.end()); std::sort(b.begin(), b.end());
    printf("tc parse p50 %.2f us, qc parse p50 %.2f us\n", a[1000], b[1000]);
  }
}
