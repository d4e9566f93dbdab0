// ldt_hostcopy.hpp — the host half of the copying to_tensor_fn path: a small
// persistent thread pool per context that moves a batch's Arrow cells into
// the context's pinned slot while the calling thread walks the JPEG headers,
// and where its threads run.
//
// Round-4 measurements on the MI355X box (tools/probes/host_bw.cpp,
// tools/probes/hip_api_cost.cpp):
//   - an H2D hipMemcpyAsync of 1 MB issued on an idle stream costs ~184 us of
//     host time (the runtime copies it synchronously); one 17 MB transfer is
//     enqueued in ~1 us. So the pool only copies host memory; the batch goes
//     to HBM in one DMA that the calling thread enqueues (ldt_abi.cpp).
//   - memcpy into the pinned slot saturates at ~85 GB/s when all threads sit
//     in one L3 domain (one CCD) and at ~48 GB/s from the GPU's remote NUMA
//     node; threads spread over the CCDs of the GPU's node scale past that.
//     So each thread is bound to one physical core of the GPU-local node,
//     cores taken round-robin over the L3 domains, the rank's block of them
//     chosen by LOCAL_RANK.
//   - the pool's size follows the cgroup CPU quota shared by the node's ranks
//     (LOCAL_WORLD_SIZE), not sched_getaffinity (which shows every host CPU).
#pragma once
#include <stddef.h>
#include <stdint.h>

#include <atomic>
#include <condition_variable>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

namespace ldt {

// Where the copy threads of device `device` run, and how many there are.
struct CopyPlacement {
  std::vector<int> cpus;  // one CPU per thread (-1: unbound)
  int gpu_numa = -1;      // the GPU's NUMA node (sysfs), -1 unknown
  double quota_cpus = 0;  // cgroup CPU quota (0: none)
  int local_rank = 0, local_world = 1;
  int l3_domains = 0;     // L3 domains the candidate CPUs span
  int candidates = 0;     // physical cores considered (GPU-local, in affinity)
  std::string local_cpulist; // the GPU's local CPUs (sysfs local_cpulist), "" unknown
};

// nthreads < 0: size from the quota (budget per rank - 2, at most 6).
// pci_bus_id: hipDeviceGetPCIBusId's string ("" if unknown). bind = false:
// threads unbound (cpus all -1).
CopyPlacement copy_placement(const char *pci_bus_id, int nthreads, bool bind);

// Copies n bytes src -> dst in chunks; the caller joins in at finish().
// Chunks are claimed with one 64-bit ticket (generation in the high half), so
// a thread still looping over an old copy can never take a chunk of the next
// one. nt: non-temporal AVX2 stores (when the CPU has AVX2).
class CopyPool {
public:
  // l3: each thread may run on any CPU of its core's L3 domain (inside the
  // process affinity) instead of on that core alone
  CopyPool(const std::vector<int> &cpus, bool nt, bool l3 = false);
  ~CopyPool();
  int threads() const { return (int)th_.size(); }
  void start(void *dst, const void *src, size_t n);
  void finish();
  // diagnostics of the last finished copy, microseconds: from start() to the
  // first chunk a pool thread claimed, and to the last chunk done
  double last_wake_us() const { return wake_us_; }
  double last_span_us() const { return span_us_; }

private:
  void work(uint32_t g, bool pool_thread);
  void run(int cpu, bool l3);
  std::vector<std::thread> th_;
  std::mutex m_;
  std::condition_variable cv_, done_cv_;
  uint64_t gen_ = 0;
  std::atomic<uint64_t> ticket_{0};
  bool stop_ = false, sync_done_ = true, nt_ = false;
  uint8_t *dst_ = nullptr;
  const uint8_t *src_ = nullptr;
  size_t n_ = 0, chunk_ = 0;
  uint32_t nchunks_ = 0, done_ = 0;
  int64_t t_start_ = 0;
  std::atomic<int64_t> t_first_{0};
  double wake_us_ = 0, span_us_ = 0;
};

// memcpy with non-temporal stores when `nt` and the CPU has AVX2.
void copy_bytes(void *dst, const void *src, size_t n, bool nt);

} // namespace ldt
