// Diagnostic (not a test, not product code): the host side of the copying
// to_tensor_fn path on the GPU box. Reports the box's topology (affinity,
// cgroup quota/throttling, NUMA nodes, the GPU's NUMA node from its PCI bus
// id, where hipHostMalloc's pages land) and measures, for 17 MB (one c2
// batch of cells):
//   - host memcpy into a pinned slot: glibc memcpy vs non-temporal AVX2
//     stores, 1..8 threads, threads unbound / bound to the GPU's node / bound
//     to another node;
//   - H2D DMA from the pinned slot (whole and 2 MB chunks);
//   - copy + chunked DMA together (what ldt_abi.cpp's CopyPool does).
// build: hipcc -O2 -mavx2 --offload-arch=gfx950 tools/probes/host_bw.cpp -o tools/probes/host_bw -lpthread
#include <hip/hip_runtime.h>
#include <immintrin.h>
#include <sched.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <fstream>
#include <sstream>
#include <string>
#include <thread>
#include <vector>

static double now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static std::vector<int> parse_list(const std::string &s) {
  std::vector<int> v;
  std::stringstream ss(s);
  std::string part;
  while (std::getline(ss, part, ',')) {
    if (part.empty()) continue;
    size_t d = part.find('-');
    int a = atoi(part.c_str()), b = d == std::string::npos ? a : atoi(part.c_str() + d + 1);
    for (int x = a; x <= b; ++x) v.push_back(x);
  }
  return v;
}

static std::string slurp(const std::string &p) {
  std::ifstream f(p);
  std::stringstream ss;
  ss << f.rdbuf();
  std::string s = ss.str();
  while (!s.empty() && (s.back() == '\n' || s.back() == ' ')) s.pop_back();
  return s;
}

static int page_node(void *p) {
  void *pages[1] = {(void *)((uintptr_t)p & ~(uintptr_t)4095)};
  int status[1] = {-99};
  long r = syscall(SYS_move_pages, 0, 1, pages, nullptr, status, 0);
  return r == 0 ? status[0] : -100;
}

static void bind_cpus(const std::vector<int> &cpus) {
  if (cpus.empty()) return;
  cpu_set_t cs;
  CPU_ZERO(&cs);
  for (int c : cpus) CPU_SET(c, &cs);
  sched_setaffinity(0, sizeof(cs), &cs);
}

__attribute__((target("avx2"))) static void copy_nt(uint8_t *dst, const uint8_t *src, size_t n) {
  size_t i = 0;
  // dst is 4 KB aligned per chunk; src may be anything
  for (; i + 128 <= n; i += 128) {
    __m256i a = _mm256_loadu_si256((const __m256i *)(src + i));
    __m256i b = _mm256_loadu_si256((const __m256i *)(src + i + 32));
    __m256i c = _mm256_loadu_si256((const __m256i *)(src + i + 64));
    __m256i d = _mm256_loadu_si256((const __m256i *)(src + i + 96));
    _mm256_stream_si256((__m256i *)(dst + i), a);
    _mm256_stream_si256((__m256i *)(dst + i + 32), b);
    _mm256_stream_si256((__m256i *)(dst + i + 64), c);
    _mm256_stream_si256((__m256i *)(dst + i + 96), d);
  }
  _mm_sfence();
  if (i < n) memcpy(dst + i, src + i, n - i);
}

struct Cfg {
  int threads;
  bool nt;
  std::vector<int> cpus; // empty: unbound
};

// one timed copy of n bytes split into equal parts over cfg.threads threads
// (threads started once, spin on a generation counter)
static double copy_rate(uint8_t *dst, const uint8_t *src, size_t n, const Cfg &cfg, int reps) {
  std::atomic<int> gen{0}, done{0};
  std::atomic<bool> stop{false};
  const int T = cfg.threads;
  std::vector<std::thread> th;
  for (int t = 0; t < T; ++t)
    th.emplace_back([&, t] {
      if (!cfg.cpus.empty()) bind_cpus({cfg.cpus[(size_t)t % cfg.cpus.size()]});
      int seen = 0;
      for (;;) {
        int g;
        while ((g = gen.load(std::memory_order_acquire)) == seen && !stop.load()) _mm_pause();
        if (stop.load()) return;
        seen = g;
        size_t per = ((n + T - 1) / T + 4095) & ~(size_t)4095;
        size_t lo = std::min(n, (size_t)t * per), hi = std::min(n, lo + per);
        if (cfg.nt) copy_nt(dst + lo, src + lo, hi - lo);
        else memcpy(dst + lo, src + lo, hi - lo);
        done.fetch_add(1, std::memory_order_acq_rel);
      }
    });
  double best = 1e30, sum = 0;
  for (int r = 0; r < reps + 2; ++r) {
    done.store(0);
    double t0 = now();
    gen.fetch_add(1, std::memory_order_acq_rel);
    while (done.load(std::memory_order_acquire) < T) _mm_pause();
    double dt = now() - t0;
    if (r >= 2) {
      best = std::min(best, dt);
      sum += dt;
    }
  }
  stop.store(true);
  for (auto &x : th) x.join();
  (void)best;
  return n / (sum / reps) / 1e9;
}

int main(int argc, char **argv) {
  const size_t n = (size_t)(argc > 1 ? atof(argv[1]) : 17.2) * 1000000;
  const int reps = argc > 2 ? atoi(argv[2]) : 30;
  cpu_set_t cs;
  sched_getaffinity(0, sizeof(cs), &cs);
  std::vector<int> aff;
  for (int c = 0; c < CPU_SETSIZE; ++c)
    if (CPU_ISSET(c, &cs)) aff.push_back(c);
  printf("affinity_cpus %zu\n", aff.size());
  printf("cgroup cpu.max: %s\n", slurp("/sys/fs/cgroup/cpu.max").c_str());
  std::string st0 = slurp("/sys/fs/cgroup/cpu.stat");
  printf("cgroup cpu.stat (start): %s\n", st0.c_str());
  printf("cpuset.cpus.effective: %s\n", slurp("/sys/fs/cgroup/cpuset.cpus.effective").c_str());
  printf("cpuset.mems.effective: %s\n", slurp("/sys/fs/cgroup/cpuset.mems.effective").c_str());
  std::vector<std::vector<int>> node_cpus;
  for (int nd = 0; nd < 64; ++nd) {
    std::string cl = slurp("/sys/devices/system/node/node" + std::to_string(nd) + "/cpulist");
    if (cl.empty()) break;
    std::vector<int> all = parse_list(cl), mine;
    for (int c : all)
      if (CPU_ISSET(c, &cs)) mine.push_back(c);
    node_cpus.push_back(mine);
    printf("node%d cpulist %s (in affinity: %zu)  meminfo: %s\n", nd, cl.c_str(), mine.size(),
           slurp("/sys/devices/system/node/node" + std::to_string(nd) + "/meminfo").substr(0, 80).c_str());
  }
  int ndev = 0;
  int gpu_node = -1;
  if (hipGetDeviceCount(&ndev) == hipSuccess && ndev > 0) {
    char bus[64] = {0};
    hipDeviceGetPCIBusId(bus, sizeof(bus), 0);
    std::string b = bus;
    for (auto &ch : b) ch = (char)tolower(ch);
    std::string nn = slurp("/sys/bus/pci/devices/" + b + "/numa_node");
    gpu_node = nn.empty() ? -1 : atoi(nn.c_str());
    printf("gpu0 pci %s numa_node %s local_cpulist %s\n", b.c_str(), nn.c_str(),
           slurp("/sys/bus/pci/devices/" + b + "/local_cpulist").c_str());
  }
  printf("main thread on cpu %d\n", sched_getcpu());

  // source: malloc'd and first-touched by the main thread (as pyarrow does)
  uint8_t *src = (uint8_t *)aligned_alloc(64, n + 4096) + 17; // Arrow cells are not aligned
  memset(src, 1, n);
  printf("src page node %d\n", page_node(src));
  uint8_t *dst = nullptr;
  bool pinned = ndev > 0 && hipHostMalloc((void **)&dst, n + 4096, hipHostMallocDefault) == hipSuccess;
  if (!pinned) dst = (uint8_t *)aligned_alloc(4096, n + 4096);
  memset(dst, 0, n);
  printf("dst (%s) page nodes: first %d mid %d last %d\n", pinned ? "hipHostMalloc" : "malloc", page_node(dst),
         page_node(dst + n / 2), page_node(dst + n - 1));
  uint8_t *dst2 = nullptr;
  if (pinned && hipHostMalloc((void **)&dst2, n + 4096, hipHostMallocNumaUser) == hipSuccess) {
    memset(dst2, 0, n);
    printf("dst2 (hipHostMallocNumaUser) page node %d\n", page_node(dst2));
  }

  std::vector<std::pair<std::string, std::vector<int>>> binds = {{"unbound", {}}};
  if (gpu_node >= 0 && gpu_node < (int)node_cpus.size() && !node_cpus[gpu_node].empty())
    binds.push_back({"gpu_node", node_cpus[gpu_node]});
  for (int nd = 0; nd < (int)node_cpus.size(); ++nd)
    if (nd != gpu_node && !node_cpus[nd].empty()) {
      binds.push_back({"node" + std::to_string(nd), node_cpus[nd]});
      break;
    }
  for (auto &b : binds)
    for (int nt = 0; nt < 2; ++nt)
      for (int T : {1, 2, 4, 6, 8}) {
        Cfg cfg{T, nt == 1, b.second};
        double r = copy_rate(dst, src, n, cfg, reps);
        printf("copy %-8s %-7s threads %d: %6.2f GB/s  (%.0f us per %.1f MB)\n", b.first.c_str(),
               nt ? "nt-avx2" : "memcpy", T, r, n / r / 1e3, n / 1e6);
        fflush(stdout);
      }
  if (pinned) {
    void *d = nullptr;
    hipMalloc(&d, n + 4096);
    hipStream_t s;
    hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    for (size_t chunk : {n, (size_t)2 << 20, (size_t)4 << 20}) {
      for (uint8_t *hb : {dst, dst2}) {
        if (!hb) continue;
        double sum = 0;
        for (int r = 0; r < reps + 2; ++r) {
          double t0 = now();
          for (size_t lo = 0; lo < n; lo += chunk)
            hipMemcpyAsync((uint8_t *)d + lo, hb + lo, std::min(chunk, n - lo), hipMemcpyHostToDevice, s);
          hipStreamSynchronize(s);
          if (r >= 2) sum += now() - t0;
        }
        printf("h2d %s chunk %zu KB: %.2f GB/s (%.0f us)\n", hb == dst ? "default" : "numauser", chunk >> 10,
               n / (sum / reps) / 1e9, sum / reps * 1e6);
      }
    }
    // copy + chunked DMA together (CopyPool-like): 6 threads, 2 MB chunks
    for (int bnd = 0; bnd < (int)binds.size(); ++bnd)
      for (int nt = 0; nt < 2; ++nt) {
        const int T = 6;
        const size_t chunk = (size_t)2 << 20;
        const size_t nch = (n + chunk - 1) / chunk;
        double sum = 0;
        for (int r = 0; r < reps + 2; ++r) {
          std::atomic<size_t> next{0};
          double t0 = now();
          std::vector<std::thread> th;
          for (int t = 0; t < T; ++t)
            th.emplace_back([&, t] {
              if (!binds[bnd].second.empty()) bind_cpus({binds[bnd].second[(size_t)t % binds[bnd].second.size()]});
              for (;;) {
                size_t i = next.fetch_add(1);
                if (i >= nch) return;
                size_t lo = i * chunk, len = std::min(chunk, n - lo);
                if (nt) copy_nt(dst + lo, src + lo, len);
                else memcpy(dst + lo, src + lo, len);
                hipMemcpyAsync((uint8_t *)d + lo, dst + lo, len, hipMemcpyHostToDevice, s);
              }
            });
          for (auto &x : th) x.join();
          hipStreamSynchronize(s);
          if (r >= 2) sum += now() - t0;
        }
        printf("copy+h2d %-8s %-7s 6 threads 2MB chunks: %.0f us per batch (incl. thread start)\n",
               binds[bnd].first.c_str(), nt ? "nt-avx2" : "memcpy", sum / reps * 1e6);
      }
  }
  printf("cgroup cpu.stat (end): %s\n", slurp("/sys/fs/cgroup/cpu.stat").c_str());
  return 0;
}
