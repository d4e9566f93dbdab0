// ldt_hostcopy.cpp — copy pool and its placement (ldt_hostcopy.hpp). HIP-free:
// the pool only moves host bytes; the DMA is enqueued by ldt_abi.cpp.
#include "ldt_hostcopy.hpp"

#include <immintrin.h>
#include <pthread.h>
#include <sched.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <map>

namespace ldt {

namespace {

int64_t now_ns() {
  return std::chrono::duration_cast<std::chrono::nanoseconds>(
             std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

std::string read_line(const std::string &path) {
  FILE *f = fopen(path.c_str(), "r");
  if (!f) return "";
  char buf[4096];
  std::string s;
  if (fgets(buf, sizeof(buf), f)) s = buf;
  fclose(f);
  while (!s.empty() && (s.back() == '\n' || s.back() == ' ')) s.pop_back();
  return s;
}

// "0-3,8,10-11" -> {0,1,2,3,8,10,11}
std::vector<int> parse_cpulist(const std::string &s) {
  std::vector<int> v;
  size_t i = 0;
  while (i < s.size()) {
    size_t j = s.find(',', i);
    if (j == std::string::npos) j = s.size();
    const std::string part = s.substr(i, j - i);
    if (!part.empty()) {
      const size_t d = part.find('-');
      const int a = atoi(part.c_str());
      const int b = d == std::string::npos ? a : atoi(part.c_str() + d + 1);
      for (int x = a; x <= b && x - a < 1 << 16; ++x) v.push_back(x);
    }
    i = j + 1;
  }
  return v;
}

// cgroup v2 cpu.max, else v1 cfs quota; 0 when unlimited / unknown
double cgroup_quota() {
  const std::string m = read_line("/sys/fs/cgroup/cpu.max");
  if (!m.empty()) {
    if (m.compare(0, 3, "max") == 0) return 0;
    double q = 0, p = 0;
    if (sscanf(m.c_str(), "%lf %lf", &q, &p) == 2 && p > 0) return q / p;
    return 0;
  }
  const std::string q = read_line("/sys/fs/cgroup/cpu/cpu.cfs_quota_us");
  const std::string p = read_line("/sys/fs/cgroup/cpu/cpu.cfs_period_us");
  if (!q.empty() && !p.empty() && atof(q.c_str()) > 0 && atof(p.c_str()) > 0)
    return atof(q.c_str()) / atof(p.c_str());
  return 0;
}

int env_int(const char *name, int dflt) {
  const char *v = getenv(name);
  return v && *v ? atoi(v) : dflt;
}

__attribute__((target("avx2"))) void copy_nt_avx2(uint8_t *dst, const uint8_t *src, size_t n) {
  size_t i = 0;
  // align the destination to 32 bytes for the streaming stores
  const size_t head = std::min(n, (size_t)((32 - ((uintptr_t)dst & 31)) & 31));
  if (head) memcpy(dst, src, head);
  i = head;
  for (; i + 128 <= n; i += 128) {
    const __m256i a = _mm256_loadu_si256((const __m256i *)(src + i));
    const __m256i b = _mm256_loadu_si256((const __m256i *)(src + i + 32));
    const __m256i c = _mm256_loadu_si256((const __m256i *)(src + i + 64));
    const __m256i d = _mm256_loadu_si256((const __m256i *)(src + i + 96));
    _mm256_stream_si256((__m256i *)(dst + i), a);
    _mm256_stream_si256((__m256i *)(dst + i + 32), b);
    _mm256_stream_si256((__m256i *)(dst + i + 64), c);
    _mm256_stream_si256((__m256i *)(dst + i + 96), d);
  }
  _mm_sfence();
  if (i < n) memcpy(dst + i, src + i, n - i);
}

bool have_avx2() {
  static const bool v = __builtin_cpu_supports("avx2");
  return v;
}

} // namespace

void copy_bytes(void *dst, const void *src, size_t n, bool nt) {
  if (nt && have_avx2() && n >= 4096)
    copy_nt_avx2(static_cast<uint8_t *>(dst), static_cast<const uint8_t *>(src), n);
  else
    memcpy(dst, src, n);
}

CopyPlacement copy_placement(const char *pci_bus_id, int nthreads, bool bind) {
  CopyPlacement P;
  P.quota_cpus = cgroup_quota();
  P.local_rank = std::max(0, env_int("LOCAL_RANK", 0));
  P.local_world = std::max(1, env_int("LOCAL_WORLD_SIZE", 1));
  cpu_set_t cs;
  CPU_ZERO(&cs);
  std::vector<int> aff;
  if (sched_getaffinity(0, sizeof(cs), &cs) == 0)
    for (int c = 0; c < CPU_SETSIZE; ++c)
      if (CPU_ISSET(c, &cs)) aff.push_back(c);
  // the GPU's local CPUs (sysfs), inside the affinity set
  std::vector<int> local;
  if (pci_bus_id && *pci_bus_id) {
    std::string b = pci_bus_id;
    for (auto &ch : b) ch = (char)tolower((unsigned char)ch);
    const std::string dir = "/sys/bus/pci/devices/" + b;
    const std::string nn = read_line(dir + "/numa_node");
    if (!nn.empty()) P.gpu_numa = atoi(nn.c_str());
    P.local_cpulist = read_line(dir + "/local_cpulist");
    const std::vector<int> lc = parse_cpulist(P.local_cpulist);
    for (int c : lc)
      if (std::binary_search(aff.begin(), aff.end(), c)) local.push_back(c);
  }
  if (local.empty()) local = aff;
  // one CPU per physical core (the first of its SMT siblings), grouped by L3
  std::map<std::string, std::vector<int>> by_l3;
  for (int c : local) {
    const std::string cpu = "/sys/devices/system/cpu/cpu" + std::to_string(c);
    const std::vector<int> sib = parse_cpulist(read_line(cpu + "/topology/thread_siblings_list"));
    if (!sib.empty() && sib.front() != c && std::binary_search(local.begin(), local.end(), sib.front()))
      continue;
    std::string l3 = read_line(cpu + "/cache/index3/id");
    if (l3.empty()) l3 = read_line(cpu + "/cache/index3/shared_cpu_list");
    by_l3[l3].push_back(c);
  }
  // cores round-robin over the L3 domains: a rank's consecutive threads land
  // in different domains (each domain's link to memory is the copy limit)
  std::vector<int> order;
  for (size_t k = 0;; ++k) {
    bool any = false;
    for (auto &g : by_l3)
      if (k < g.second.size()) {
        order.push_back(g.second[k]);
        any = true;
      }
    if (!any) break;
  }
  P.l3_domains = (int)by_l3.size();
  P.candidates = (int)order.size();
  if (nthreads < 0) {
    // the CPU budget of one rank: the cgroup quota (or the GPU-local cores)
    // shared by the node's ranks, minus the caller and one more thread
    const double budget = (P.quota_cpus > 0 ? P.quota_cpus : (double)order.size()) / P.local_world;
    nthreads = std::max(0, std::min(6, (int)budget - 2));
  }
  nthreads = std::min(nthreads, 31);
  const size_t base = (size_t)P.local_rank * (size_t)std::max(nthreads, 1);
  for (int t = 0; t < nthreads; ++t)
    P.cpus.push_back(bind && !order.empty() ? order[(base + (size_t)t) % order.size()] : -1);
  return P;
}

CopyPool::CopyPool(const std::vector<int> &cpus, bool nt, bool l3) : nt_(nt) {
  for (int cpu : cpus) th_.emplace_back([this, cpu, l3] { run(cpu, l3); });
}

CopyPool::~CopyPool() {
  {
    std::lock_guard<std::mutex> g(m_);
    stop_ = true;
    ++gen_;
  }
  cv_.notify_all();
  for (auto &t : th_) t.join();
}

void CopyPool::start(void *dst, const void *src, size_t n) {
  t_start_ = now_ns();
  if (th_.empty() || n < ((size_t)1 << 20)) {
    copy_bytes(dst, src, n, nt_);
    sync_done_ = true;
    wake_us_ = 0;
    span_us_ = (now_ns() - t_start_) * 1e-3;
    return;
  }
  sync_done_ = false;
  {
    std::lock_guard<std::mutex> g(m_);
    dst_ = static_cast<uint8_t *>(dst);
    src_ = static_cast<const uint8_t *>(src);
    n_ = n;
    // ~4 chunks per thread (the caller joins late), at least 256 KB, whole pages
    const size_t parts = 4 * (th_.size() + 1);
    chunk_ = std::max<size_t>(((n + parts - 1) / parts + 4095) & ~(size_t)4095, (size_t)1 << 18);
    nchunks_ = (uint32_t)((n + chunk_ - 1) / chunk_);
    done_ = 0;
    t_first_.store(0, std::memory_order_relaxed);
    ++gen_;
    ticket_.store((uint64_t)(uint32_t)gen_ << 32, std::memory_order_release);
  }
  cv_.notify_all();
}

void CopyPool::finish() {
  if (sync_done_) return;
  uint32_t g;
  {
    std::lock_guard<std::mutex> l(m_);
    g = (uint32_t)gen_;
  }
  work(g, false);
  std::unique_lock<std::mutex> lk(m_);
  done_cv_.wait(lk, [this] { return done_ == nchunks_; });
  sync_done_ = true;
  const int64_t tf = t_first_.load(std::memory_order_relaxed);
  wake_us_ = tf ? (tf - t_start_) * 1e-3 : -1.0;
  span_us_ = (now_ns() - t_start_) * 1e-3;
}

void CopyPool::work(uint32_t g, bool pool_thread) {
  for (;;) {
    // claim chunk i of generation g only (a fetch_add could consume a chunk
    // of a newer copy that this thread then would not do)
    uint64_t t = ticket_.load(std::memory_order_acquire);
    do {
      if ((uint32_t)(t >> 32) != g || (uint32_t)t >= nchunks_) return;
    } while (!ticket_.compare_exchange_weak(t, t + 1, std::memory_order_acq_rel, std::memory_order_acquire));
    if (pool_thread) {
      int64_t z = 0;
      t_first_.compare_exchange_strong(z, now_ns(), std::memory_order_relaxed);
    }
    const uint32_t i = (uint32_t)t;
    const size_t lo = (size_t)i * chunk_, hi = std::min(n_, lo + chunk_);
    copy_bytes(dst_ + lo, src_ + lo, hi - lo, nt_);
    std::lock_guard<std::mutex> l(m_);
    if (++done_ == nchunks_) done_cv_.notify_all();
  }
}

void CopyPool::run(int cpu, bool l3) {
  if (cpu >= 0) {
    cpu_set_t cs;
    CPU_ZERO(&cs);
    CPU_SET(cpu, &cs);
    if (l3) {
      // the core's L3 domain (SMT siblings included) within the affinity the
      // thread inherited: a busy core does not hold the thread's wake-up
      cpu_set_t inh;
      CPU_ZERO(&inh);
      if (pthread_getaffinity_np(pthread_self(), sizeof(inh), &inh) == 0)
        for (int c : parse_cpulist(read_line("/sys/devices/system/cpu/cpu" + std::to_string(cpu) +
                                             "/cache/index3/shared_cpu_list")))
          if (c >= 0 && c < CPU_SETSIZE && CPU_ISSET(c, &inh)) CPU_SET(c, &cs);
    }
    (void)pthread_setaffinity_np(pthread_self(), sizeof(cs), &cs); // best effort
  }
  uint64_t seen = 0;
  for (;;) {
    uint32_t g;
    {
      std::unique_lock<std::mutex> lk(m_);
      cv_.wait(lk, [&] { return gen_ != seen; });
      seen = gen_;
      if (stop_) return;
      g = (uint32_t)gen_;
    }
    work(g, true);
  }
}

} // namespace ldt
