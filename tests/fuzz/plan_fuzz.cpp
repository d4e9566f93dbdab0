// Fuzz driver for libldt's host JPEG header planner (csrc/ldt_plan.cpp), built
// for the CPU with -fsanitize=address,undefined by tests/test_plan_fuzz.py.
// Input on stdin: records of [uint32 little-endian length][bytes]. Each cell is
// copied into a heap buffer of exactly its length, so any read past the cell
// is an ASan report. Output: one line per cell, the LDT_IMG_* status the
// planner gives it (walk_markers, then plan_progressive for SOF2 or the
// Huffman table derivation for baseline files, as ldt_abi.cpp decode_core does).
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/ldt.h"
#include "../../lance-distributed-training_amd/csrc/ldt_plan.hpp"

using namespace ldt;

static bool g_print_scans = false; // PLAN_SCANS=1: also print each scan's (offset, length)

static int plan_one(const uint8_t *cell, int64_t len) {
  Header H;
  int st = walk_markers(cell, len, H);
  if (st != LDT_IMG_OK) return st;
  if (H.width > LDT_MAX_DIM || H.height > LDT_MAX_DIM) return LDT_IMG_TOO_LARGE;
  if (H.progressive) {
    ProgPlan P;
    st = plan_progressive(cell, len, H, P);
    if (st != LDT_IMG_OK) return st;
    if (g_print_scans)
      for (const auto &sc : P.scans) printf("%lld:%lld ", (long long)sc.data_off, (long long)sc.data_len);
    for (const auto &t : P.tabs) {
      ProgTab pt;
      if (!build_prog_tab(t.first, t.second, pt)) return LDT_IMG_NOT_JPEG;
    }
    return LDT_IMG_OK;
  }
  for (int k = 0; k < H.ncomp; ++k) {
    if (!H.qpresent[H.tq[k]] || !H.dc[H.td[k]].present || !H.ac[H.ta[k]].present) return LDT_IMG_NOT_JPEG;
    HuffTab t;
    if (!build_huff(H.dc[H.td[k]], true, t) || !build_huff(H.ac[H.ta[k]], false, t)) return LDT_IMG_NOT_JPEG;
    (void)huff_key(H.ac[H.ta[k]], false);
  }
  return LDT_IMG_OK;
}

int main() {
  g_print_scans = getenv("PLAN_SCANS") != nullptr;
  uint32_t n;
  while (fread(&n, 4, 1, stdin) == 1) {
    uint8_t *cell = (uint8_t *)malloc(n ? n : 1);
    if (n && fread(cell, 1, n, stdin) != n) return 2;
    printf("%d\n", plan_one(cell, n));
    free(cell);
  }
  return 0;
}
