// ldt_plan.hpp — the host-side JPEG header planner of libldt.so: marker
// walk (SOI..SOS), Huffman table derivation and the progressive scan walk.
// It parses untrusted bytes, so it lives in its own HIP-free translation unit
// (ldt_plan.cpp) that tests/test_plan_fuzz.py also builds for the CPU with
// AddressSanitizer + UBSan and fuzzes (tests/fuzz/plan_fuzz.cpp).
#pragma once
#include <stdint.h>

#include <string>
#include <utility>
#include <vector>

#include "ldt_types.hpp"

namespace ldt {

// ---------------------------------------------------------------------------
// Marker walk (ITU T.81 B.2; libjpeg jdmarker.c semantics for the subset).
// ---------------------------------------------------------------------------
struct RawHuff {
  uint8_t counts[16];
  uint8_t syms[256];
  int nsym;
  bool present;
};

struct Header {
  int width = 0, height = 0, ncomp = 0;
  int cid[4], h[4], v[4], tq[4], td[4], ta[4];
  uint16_t q[4][64]; // natural order
  bool qpresent[4] = {false, false, false, false};
  RawHuff dc[4], ac[4];
  int restart = 0;
  bool jfif = false, adobe = false;
  int adobe_transform = -1;
  int64_t scan_pos = 0; // offset of entropy-coded data within the cell
                        // (progressive: of the first SOS marker)
  bool progressive = false;
};

struct ProgPlan {
  std::vector<ProgScan> scans;                // tab[]: indices into tabs
  std::vector<std::pair<RawHuff, bool>> tabs; // (table, is_dc)
  uint16_t q[4][64];                          // latched quant tables, natural order
};

// Returns an LDT_IMG_* code (include/ldt.h).
int walk_markers(const uint8_t *cell, int64_t len, Header &H);
// jdhuff.c jpeg_make_d_derived_tbl into the device layout; false = bad table.
bool build_huff(const RawHuff &r, bool is_dc, HuffTab &t);
std::string huff_key(const RawHuff &r, bool dc);
bool build_prog_tab(const RawHuff &r, bool is_dc, ProgTab &t);
// Returns an LDT_IMG_* code.
int plan_progressive(const uint8_t *cell, int64_t len, const Header &H0, ProgPlan &P);

} // namespace ldt
