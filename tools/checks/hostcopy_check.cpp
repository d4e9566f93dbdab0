// Host check of the copy pool and its placement (csrc/ldt_hostcopy.cpp, which
// is HIP-free): built with g++ (+ ASan/UBSan) by tests/test_hostcopy.py.
//   copy     random sizes and source/destination misalignments through
//            copy_bytes (memcpy / non-temporal AVX2) and through CopyPool with
//            0..7 threads, repeated on one pool (generations), byte-exact.
//   place    copy_placement("", n, bind) under LOCAL_RANK / LOCAL_WORLD_SIZE:
//            distinct cores within a rank, disjoint between ranks while the
//            cores last, quota-derived thread count; prints one JSON line.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <random>
#include <set>
#include <vector>

#include "../../lance-distributed-training_amd/csrc/ldt_hostcopy.hpp"

using namespace ldt;

static int check_copy() {
  std::mt19937_64 rng(7);
  std::vector<uint8_t> src(5 << 20), dst(5 << 20);
  for (auto &b : src) b = (uint8_t)rng();
  for (int nt = 0; nt < 2; ++nt)
    for (int threads : {0, 1, 3, 7}) {
      std::vector<int> cpus(threads, -1);
      CopyPool pool(cpus, nt == 1);
      for (int rep = 0; rep < 12; ++rep) {
        const size_t so = rng() % 61, doff = rng() % 37;
        const size_t n = rep % 3 == 0 ? rng() % 5000 : (rng() % ((4u << 20) - 64)) + 1;
        memset(dst.data(), 0xAB, dst.size());
        if (rep & 1) {
          pool.start(dst.data() + doff, src.data() + so, n);
          pool.finish();
        } else {
          copy_bytes(dst.data() + doff, src.data() + so, n, nt == 1);
        }
        if (memcmp(dst.data() + doff, src.data() + so, n) != 0) {
          fprintf(stderr, "copy mismatch nt=%d threads=%d n=%zu so=%zu do=%zu\n", nt, threads, n, so, doff);
          return 1;
        }
        if ((doff && dst[doff - 1] != 0xAB) || dst[doff + n] != 0xAB) {
          fprintf(stderr, "copy wrote outside [dst, dst+n) nt=%d n=%zu\n", nt, n);
          return 1;
        }
      }
    }
  printf("copy ok\n");
  return 0;
}

static int check_place(int nthreads, int bind) {
  const CopyPlacement P = copy_placement("", nthreads, bind != 0);
  std::set<int> seen;
  for (int c : P.cpus) {
    if (bind && c < 0) {
      fprintf(stderr, "unbound thread with bind\n");
      return 1;
    }
    if (c >= 0 && !seen.insert(c).second && (int)P.cpus.size() <= P.candidates) {
      fprintf(stderr, "cpu %d twice\n", c);
      return 1;
    }
  }
  printf("{\"threads\": %zu, \"cpus\": [", P.cpus.size());
  for (size_t i = 0; i < P.cpus.size(); ++i) printf("%s%d", i ? ", " : "", P.cpus[i]);
  printf("], \"candidates\": %d, \"l3_domains\": %d, \"quota\": %.2f, \"local_rank\": %d, \"local_world\": %d}\n",
         P.candidates, P.l3_domains, P.quota_cpus, P.local_rank, P.local_world);
  return 0;
}

int main(int argc, char **argv) {
  if (argc > 1 && !strcmp(argv[1], "copy")) return check_copy();
  if (argc > 3 && !strcmp(argv[1], "place")) return check_place(atoi(argv[2]), atoi(argv[3]));
  fprintf(stderr, "usage: hostcopy_check copy | place <threads> <bind>\n");
  return 2;
}
