// Host staging-pack probe (CPU side of the drop-in path).
// Packs 2^20 (pk 32 | sig 64 | digest 32) items from three pageable arrays
// into pinned staging, 16 MiB chunk by chunk, in several forms, on T threads,
// optionally while the DMA engine copies the other staging buffer to the GPU
// (as in the pipelined call).  Prints GB/s of packed bytes per form.
//
//   hipcc -O3 -std=c++17 -mavx2 -o tools/pack_probe tools/pack_probe.cpp -lpthread
//   tools/pack_probe [threads...]
#include <hip/hip_runtime.h>
#include <immintrin.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <thread>
#include <vector>

namespace {

constexpr size_t kN = size_t(1) << 20, kChunk = size_t(1) << 17, kRec = 128;

double now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// fn(part) over nparts parts on T threads (fresh threads per chunk would cost
// more than the pool's wake-up; a spin barrier pool keeps the probe simple)
struct Pool {
  explicit Pool(int t) : t_(t) {
    for (int i = 1; i < t; ++i) th_.emplace_back([this, i] { loop(i); });
  }
  ~Pool() {
    stop_ = true;
    gen_.fetch_add(1);
    for (auto &t : th_) t.join();
  }
  void run(int nparts, const std::function<void(int)> &fn) {
    fn_ = &fn;
    nparts_ = nparts;
    next_.store(0);
    done_.store(0);
    gen_.fetch_add(1, std::memory_order_release);
    work();
    while (done_.load(std::memory_order_acquire) < t_) _mm_pause();
  }

 private:
  void work() {
    for (int p; (p = next_.fetch_add(1)) < nparts_;) (*fn_)(p);
    done_.fetch_add(1, std::memory_order_release);
  }
  void loop(int) {
    uint64_t seen = 0;  // the generation at construction (a late start must not skip a run)
    for (;;) {
      uint64_t g;
      while ((g = gen_.load(std::memory_order_acquire)) == seen) _mm_pause();
      seen = g;
      if (stop_) return;
      work();
    }
  }
  int t_;
  std::vector<std::thread> th_;
  std::atomic<uint64_t> gen_{0};
  std::atomic<int> next_{0}, done_{0};
  const std::function<void(int)> *fn_ = nullptr;
  int nparts_ = 0;
  std::atomic<bool> stop_{false};
};

inline void nt_copy32(uint8_t *d, const uint8_t *s) {
  _mm256_stream_si256(reinterpret_cast<__m256i *>(d), _mm256_loadu_si256(reinterpret_cast<const __m256i *>(s)));
}

}  // namespace

int main(int argc, char **argv) {
  std::vector<int> threads;
  for (int i = 1; i < argc; ++i) threads.push_back(std::atoi(argv[i]));
  if (threads.empty()) threads = {1, 4, 8, 12, 16};
  std::vector<uint8_t> pk(kN * 32), sig(kN * 64), msg(kN * 32);
  for (size_t i = 0; i < pk.size(); ++i) pk[i] = uint8_t(i * 7);
  for (size_t i = 0; i < sig.size(); ++i) sig[i] = uint8_t(i * 13);
  for (size_t i = 0; i < msg.size(); ++i) msg[i] = uint8_t(i * 3);
  uint8_t *h = nullptr, *d = nullptr;
  const size_t stage = kChunk * kRec;
  if (hipHostMalloc(&h, 2 * stage, hipHostMallocDefault) != hipSuccess || hipMalloc(&d, 2 * stage) != hipSuccess) {
    std::fprintf(stderr, "allocation failed\n");
    return 1;
  }
  std::memset(h, 0, 2 * stage);
  hipStream_t cs;
  (void)hipStreamCreateWithFlags(&cs, hipStreamNonBlocking);

  const char *forms[] = {"records_memcpy", "records_nt", "soa_memcpy", "soa_nt"};
  for (int t : threads) {
    Pool pool(t);
    for (int form = 0; form < 4; ++form) {
      for (int dma = 0; dma < 2; ++dma) {
        std::vector<double> runs;
        for (int rep = 0; rep < 9; ++rep) {
          double packed = 0;
          for (size_t base = 0, k = 0; base < kN; base += kChunk, ++k) {
            uint8_t *st = h + (k & 1) * stage;
            if (dma) {  // the DMA engine reads the other buffer meanwhile
              (void)hipStreamSynchronize(cs);
              (void)hipMemcpyAsync(d, h + ((k + 1) & 1) * stage, stage, hipMemcpyHostToDevice, cs);
            }
            const int nparts = 16;
            const double t0 = now_ms();
            pool.run(nparts, [&](int p) {
              const size_t lo = kChunk * p / nparts, hi = kChunk * (p + 1) / nparts;
              if (form == 0) {
                for (size_t i = lo; i < hi; ++i) {
                  uint8_t *r = st + kRec * i;
                  std::memcpy(r, &pk[(base + i) * 32], 32);
                  std::memcpy(r + 32, &sig[(base + i) * 64], 64);
                  std::memcpy(r + 96, &msg[(base + i) * 32], 32);
                }
              } else if (form == 1) {
                for (size_t i = lo; i < hi; ++i) {
                  uint8_t *r = st + kRec * i;
                  nt_copy32(r, &pk[(base + i) * 32]);
                  nt_copy32(r + 32, &sig[(base + i) * 64]);
                  nt_copy32(r + 64, &sig[(base + i) * 64 + 32]);
                  nt_copy32(r + 96, &msg[(base + i) * 32]);
                }
                _mm_sfence();
              } else if (form == 2) {
                std::memcpy(st + lo * 32, &pk[(base + lo) * 32], (hi - lo) * 32);
                std::memcpy(st + kChunk * 32 + lo * 64, &sig[(base + lo) * 64], (hi - lo) * 64);
                std::memcpy(st + kChunk * 96 + lo * 32, &msg[(base + lo) * 32], (hi - lo) * 32);
              } else {
                auto nt = [](uint8_t *dst, const uint8_t *src, size_t bytes) {
                  for (size_t o = 0; o < bytes; o += 32) nt_copy32(dst + o, src + o);
                };
                nt(st + lo * 32, &pk[(base + lo) * 32], (hi - lo) * 32);
                nt(st + kChunk * 32 + lo * 64, &sig[(base + lo) * 64], (hi - lo) * 64);
                nt(st + kChunk * 96 + lo * 32, &msg[(base + lo) * 32], (hi - lo) * 32);
                _mm_sfence();
              }
            });
            packed += now_ms() - t0;
          }
          (void)hipStreamSynchronize(cs);
          runs.push_back(packed);
        }
        std::sort(runs.begin(), runs.end());
        const double med = runs[runs.size() / 2];
        std::printf("{\"threads\": %d, \"form\": \"%s\", \"concurrent_h2d\": %d, \"median_ms\": %.3f, \"min_ms\": %.3f, "
                    "\"max_ms\": %.3f, \"GBps\": %.1f}\n",
                    t, forms[form], dma, med, runs.front(), runs.back(), kN * kRec / (med * 1e-3) / 1e9);
        std::fflush(stdout);
      }
    }
  }
  return 0;
}
