// Host planner timing (diagnostic): walk_markers, plan_progressive and
// build_prog_tab over a batch of cells read from stdin ([uint32 length][bytes]
// records, e.g. a c2p batch), repeated; prints microseconds per batch per phase.
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <chrono>
#include <vector>

#include "../../include/ldt.h"
#include "../../lance-distributed-training_amd/csrc/ldt_plan.hpp"

using namespace ldt;
using clk = std::chrono::steady_clock;

int main(int argc, char **argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 20;
  std::vector<std::vector<uint8_t>> cells;
  uint32_t n;
  while (fread(&n, 4, 1, stdin) == 1) {
    cells.emplace_back(n);
    if (n && fread(cells.back().data(), 1, n, stdin) != n) return 2;
  }
  double t_walk = 0, t_prog = 0, t_tab = 0;
  long ok = 0;
  for (int r = 0; r < reps; ++r)
    for (auto &c : cells) {
      Header H;
      auto a = clk::now();
      int st = walk_markers(c.data(), (int64_t)c.size(), H);
      auto b = clk::now();
      t_walk += std::chrono::duration<double, std::micro>(b - a).count();
      if (st != LDT_IMG_OK || !H.progressive) continue;
      ProgPlan P;
      st = plan_progressive(c.data(), (int64_t)c.size(), H, P);
      auto d = clk::now();
      t_prog += std::chrono::duration<double, std::micro>(d - b).count();
      for (const auto &t : P.tabs) {
        ProgTab pt;
        ok += build_prog_tab(t.first, t.second, pt);
      }
      t_tab += std::chrono::duration<double, std::micro>(clk::now() - d).count();
    }
  printf("cells %zu: walk %.1f us, plan_progressive %.1f us, build_prog_tab %.1f us per batch (%ld tables)\n",
         cells.size(), t_walk / reps, t_prog / reps, t_tab / reps, ok / reps);
  return 0;
}
