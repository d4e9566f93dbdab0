// Host check: the 0xFF-driven destuff classification (ds_classify16_ff, the
// fused destuff of k_huff_image) equals the per-byte rules (ds_classify16,
// the k_destuff_* kernels) on random 0xFF/marker-heavy words, positions and
// lengths. Built with hipcc as host code (no GPU); tests/test_host_logic.py.
#include "ldt_device.hpp"
#include <cstdio>
#include <random>
#include <cstdlib>
using namespace ldt;
int main(int argc, char **argv) {
  const long iters = argc > 1 ? atol(argv[1]) : 20000000;
  std::mt19937_64 g(1);
  const uint8_t pool[] = {0xFF, 0x00, 0xD0, 0xD7, 0xD8, 0xD9, 0xC4, 0x12, 0xFE, 0xCF, 0x80, 0x7F};
  long bad = 0, n = 0;
  for (int it = 0; it < iters; ++it) {
    uint32_t wv[6];
    for (int i = 0; i < 6; ++i) {
      uint32_t w = 0;
      for (int b = 0; b < 4; ++b) {
        uint32_t v = (g() % 3 == 0) ? (uint32_t)(g() & 255) : pool[g() % sizeof(pool)];
        w |= v << (8 * b);
      }
      wv[i] = w;
    }
    int64_t p0 = (int64_t)(g() % 64) - 24;
    int64_t L = (int64_t)(g() % 48);
    uint32_t k1, r1, k2, r2; int e1, e2;
    ds_classify16(wv, p0, L, k1, r1, e1);
    ds_classify16_ff(wv, p0, L, k2, r2, e2);
    ++n;
    if (k1 != k2 || r1 != r2 || e1 != e2) { if (bad++ < 5) printf("mismatch p0=%ld L=%ld k %x %x r %x %x e %d %d\n", (long)p0, (long)L, k1, k2, r1, r2, e1, e2); }
  }
  printf("%ld cases, %ld mismatches\n", n, bad);
  return bad != 0;
}
