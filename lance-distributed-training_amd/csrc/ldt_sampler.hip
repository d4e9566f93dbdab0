// ldt_sampler.hip — map-style DistributedSampler index computation on gfx950.
//
// Replaces the index path of torch.utils.data.DistributedSampler as the
// reference uses it for its map-style loader (lance_map_style.py:58 ->
// torch/utils/data/distributed.py:107-141, torch 2.10):
//   perm    = torch.randperm(n, generator=manual_seed(seed + epoch))   :110-112
//   padded  = perm[p % n] for p < total_size (drop_last: p < total_size <= n) :116-127
//   indices = padded[rank : total_size : num_replicas]                   :134
// torch.randperm on CPU (n < 2^32/20) is a forward Fisher-Yates over MT19937:
//   for i in [0, n-1): z = mt() % (n - i); swap(r[i], r[i + z])
// Kernels, bit-exact with that sequence:
//   k_mt_targets   one workgroup: MT19937 (seed = low 32 bits of the 64-bit
//                  torch seed), each 624-word twist computed in 3 dependency
//                  phases by up to 227 lanes; raw words out.
//   k_link_targets all lanes: temper, swap target H[i] = i + mt_i % (n - i),
//                  bucket the i by H[i] (linked lists by atomicExch).
//   k_dist_chain   one lane per output index: the final content of position
//                  (rank + k*W) % n follows from a short backward chain through
//                  the buckets, so no swap is ever executed and a rank computes
//                  only its own n/W positions.
// (An earlier version ran the swaps in parallel rounds of deterministic
// reservations, Shun et al. SODA 2015, in one workgroup: 1.6 ms at n = 75,750,
// latency-bound on ~40 dependent rounds. The chain form has no rounds.)
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "ldt_kernels.hpp"

namespace ldt {

namespace {
constexpr int kMtN = 624;
constexpr int kMtM = 397;
constexpr uint32_t kMtMatrix = 0x9908b0dfu;

__device__ __forceinline__ uint32_t mt_twist(uint32_t cur, uint32_t next, uint32_t far) {
  const uint32_t y = (cur & 0x80000000u) | (next & 0x7fffffffu);
  return far ^ (y >> 1) ^ ((y & 1u) ? kMtMatrix : 0u);
}

__device__ __forceinline__ uint32_t mt_temper(uint32_t y) {
  y ^= y >> 11;
  y ^= (y << 7) & 0x9d2c5680u;
  y ^= (y << 15) & 0xefc60000u;
  y ^= y >> 18;
  return y;
}
} // namespace

// Raw MT19937 state words for outputs [0, n-1) into H (tempered later). One
// workgroup of 256 lanes.
__global__ void __launch_bounds__(256) k_mt_targets(uint32_t seed, int32_t n, int32_t *H) {
  __shared__ uint32_t st[2][kMtN];
  const int tid = threadIdx.x;
  if (tid == 0) {
    uint32_t v = seed;
    st[0][0] = v;
    for (int j = 1; j < kMtN; ++j) {
      v = 1812433253u * (v ^ (v >> 30)) + (uint32_t)j;
      st[0][j] = v;
    }
  }
  __syncthreads();
  const int64_t count = (int64_t)n - 1;
  int cur = 0;
  for (int64_t base = 0; base < count; base += kMtN) {
    const uint32_t *O = st[cur];
    uint32_t *N = st[cur ^ 1];
    // phase A: k in [0, 227) reads only the old state
    if (tid < kMtN - kMtM) N[tid] = mt_twist(O[tid], O[tid + 1], O[tid + kMtM]);
    __syncthreads();
    // phase B: k in [227, 454) reads new[k - 227]
    {
      const int k = tid + (kMtN - kMtM);
      if (tid < kMtN - kMtM) N[k] = mt_twist(O[k], O[k + 1], N[k - (kMtN - kMtM)]);
    }
    __syncthreads();
    // phase C: k in [454, 624); k = 623 wraps to new[0]
    {
      const int k = tid + 2 * (kMtN - kMtM);
      if (k < kMtN) {
        const uint32_t nxt = k + 1 < kMtN ? O[k + 1] : N[0];
        N[k] = mt_twist(O[k], nxt, N[k - (kMtN - kMtM)]);
      }
    }
    __syncthreads();
    // raw (untempered) words out; tempering and the modulo run in the
    // all-lanes link kernel, keeping this serial loop to the three phases
    for (int k = tid; k < kMtN; k += 256) {
      const int64_t i = base + k;
      if (i < count) H[i] = (int32_t)N[k];
    }
    // no barrier here: the next phase A writes the buffer that was O, read
    // last before the barrier that ended phase C; N is only read from now on
    cur ^= 1;
  }
}

// Bucket the swap targets by value: one singly linked list per value v of the
// i with H[i] == v (arbitrary order; buckets hold ~1 entry on average,
// at most ~ln n). head[] is pre-filled with -1.
// Also turns the raw word into the swap target H[i] = i + mt_i % (n - i).
__global__ void k_link_targets(int32_t *H, int32_t n, int32_t *head, int32_t *nxt) {
  const int32_t i = (int32_t)(blockIdx.x * blockDim.x + threadIdx.x);
  if (i >= n - 1) return;
  const int32_t h = i + (int32_t)(mt_temper((uint32_t)H[i]) % (uint32_t)(n - i));
  H[i] = h;
  nxt[i] = atomicExch(&head[h], i);
}

// The rank's indices straight from the swap targets, no swaps executed.
// Position p's final value, tracing the transpositions (i, H[i]) backwards
// (H[i] >= i): step p moves p to v = H[p] (position n-1 has no step); after
// that only an earlier step i with H[i] == v moves it, to v = i. So
//   v = H[p], b = p;  while (i = max{i < b : H[i] == v}) exists: v = b = i
// and perm[p] = v. Chains average ~1 step (max ~17 at n = 75,750).
__global__ void k_dist_chain(const int32_t *H, const int32_t *head, const int32_t *nxt, int64_t n,
                             int rank, int world, int64_t num_samples, int64_t *out) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= num_samples) return;
  const int32_t p = (int32_t)(((int64_t)rank + k * world) % n);
  int32_t v = p < n - 1 ? H[p] : p;
  int32_t b = p;
  while (n > 1) {  // n == 1: no steps, head/nxt unused
    int32_t best = -1;
    for (int32_t e = head[v]; e >= 0; e = nxt[e])
      if (e < b && e > best) best = e;
    if (best < 0) break;
    v = b = best;
  }
  out[k] = v;
}

// out[k] = perm[(rank + k*W) % n] (perm == nullptr: identity, shuffle=False).
__global__ void k_dist_select(const int32_t *perm, int64_t n, int rank, int world,
                              int64_t num_samples, int64_t *out) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= num_samples) return;
  const int64_t p = ((int64_t)rank + k * world) % n;
  out[k] = perm ? (int64_t)perm[p] : p;
}

hipError_t launch_dist_shuffled(uint32_t seed, int64_t n, int rank, int world,
                                int64_t num_samples, int32_t *H, int32_t *head, int32_t *nxt,
                                int64_t *out, hipStream_t s) {
  if (num_samples <= 0) return hipSuccess;
  if (n > 1) {
    hipLaunchKernelGGL(k_mt_targets, dim3(1), dim3(256), 0, s, seed, (int32_t)n, H);
    hipError_t e = hipMemsetAsync(head, 0xff, (size_t)n * sizeof(int32_t), s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_link_targets, dim3((unsigned)((n - 1 + 255) / 256)), dim3(256), 0, s, H,
                       (int32_t)n, head, nxt);
  }
  hipLaunchKernelGGL(k_dist_chain, dim3((unsigned)((num_samples + 255) / 256)), dim3(256), 0, s,
                     H, head, nxt, n, rank, world, num_samples, out);
  return hipGetLastError();
}

hipError_t launch_dist_select(const int32_t *perm, int64_t n, int rank, int world,
                              int64_t num_samples, int64_t *out, hipStream_t s) {
  if (num_samples <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_dist_select, dim3((unsigned)((num_samples + 255) / 256)), dim3(256), 0, s,
                     perm, n, rank, world, num_samples, out);
  return hipGetLastError();
}

} // namespace ldt
