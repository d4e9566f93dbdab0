// ldt_abi.cpp — host side of libldt.so: the C-ABI declared in include/ldt.h.
//
// Per batch the host does planning only: it walks each cell's JPEG marker
// segments (SOI..SOS, a few hundred bytes; the entropy-coded data is never
// touched on the host), dedupes Huffman/quantisation tables, lays out the
// device workspace and writes one compact plan blob (descriptors, segments,
// tables, the ToTensor/Normalize LUT, labels, per-image status) into a pinned
// ring slot. One H2D copy moves the plan, one moves the cells (unless they are
// already resident), then five kernels run on the caller's stream.
//
// Replaces, per batch: lance_iterable.py:41-49 (to_pylist, PIL open/convert,
// Resize, ToTensor, stack, label tensor) and lance_map_style.py:34-44.
#include <hip/hip_runtime.h>
#include <sched.h>
#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <memory>
#include <chrono>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "../../include/ldt.h"
#include "ldt_hostcopy.hpp"
#include "ldt_kernels.hpp"
#include "ldt_plan.hpp"

using namespace ldt;

namespace {

inline int64_t align_up(int64_t v, int64_t a) { return (v + a - 1) / a * a; }

} // namespace

// ---------------------------------------------------------------------------
// Context.
// ---------------------------------------------------------------------------
struct DevBuf {
  void *p = nullptr;
  size_t cap = 0;
};

struct PinBuf {
  void *p = nullptr;
  size_t cap = 0;
};

// Host phases of decode_core (LDT_OPT_HOST_TIMING; read with ldt_host_times).
enum HostPhase {
  kHpSlot = 0, // waiting for the pinned slot, starting the cell copy
  kHpParse,    // header walk + per-image plans (overlaps the cell copy)
  kHpPlan,     // plan blob, device workspace sizing
  kHpCopy,     // waiting for the cell copy to finish, H2D enqueue
  kHpLaunch,   // kernel launches
  kHpStatus,   // status copy, return
  // not phases of the calling thread: the copy pool's wake-up (copy start to
  // the first chunk a pool thread took) and span (copy start to its end)
  kHpCopyWake,
  kHpCopySpan,
  kHpCount
};

#ifndef LDT_FUSE_DEFAULT
#define LDT_FUSE_DEFAULT true // experiment builds: -DLDT_FUSE_DEFAULT=false
#endif

struct ldt_ctx {
  int device = 0;
  std::string err;
  bool sync_status = true;
  int huff_mode = 0;
  int resize_impl = 0;
  int warm_pct = 0;
  int subseq_bits = 256; // minimum S of the parallel decoder
  int resize_waves_pct = 100;
  int resize_wpg = 0;
  bool fuse_destuff = LDT_FUSE_DEFAULT; // LDT_OPT_FUSED_DESTUFF
  int copy_threads = -1; // -1: default (from the cgroup quota per local rank, <= 6)
  int copy_bind = 2;      // LDT_OPT_COPY_BIND: pool threads on GPU-local cores' L3 domains (1: the cores)
  bool copy_nt = true;    // LDT_OPT_COPY_NT: non-temporal stores into the slot
  int copy_mode = 0;      // LDT_OPT_COPY_MODE: 0 DMA on the device's copy stream, 1 on the caller's
  hipStream_t copy_stream = nullptr; // ldt_set_copy_stream: replaces the device's copy stream (mode 0)
  bool host_timing = false;
  bool debug_counters = false; // LDT_OPT_DEBUG_COUNTERS
  int64_t win_cap = -1;        // LDT_OPT_HUFF_WINDOW: cap on k_huff_image's LDS window (bytes; -1 none)
  CopyPlacement placement; // of the current pool
  static constexpr int kSlots = 2;
  // device cells, one buffer per pinned slot: a copy-stream DMA into one may
  // run while the kernels of the slot's previous batch still read the other
  DevBuf d_data[kSlots];
  hipEvent_t data_free_ev[kSlots] = {nullptr, nullptr}; // its last reader (Huffman stage) done
  hipEvent_t h2d_ev[kSlots] = {nullptr, nullptr};       // its DMA done (copy stream)
  bool data_used[kSlots] = {false, false};
  DevBuf d_plan, d_dstuf, d_coef, d_brec, d_bcarry, d_pcoef, d_dcv, d_planes, d_raw, d_dscnt;
  DevBuf d_perm; // DistributedSampler scratch: 3 int32 arrays of dataset_len
  std::unique_ptr<CopyPool> copier; // host -> pinned copies (created on first use)
  PinBuf h_data[kSlots], h_plan[kSlots];
  hipEvent_t slot_ev[kSlots] = {nullptr, nullptr};
  bool slot_used[kSlots] = {false, false};
  int slot = 0;
  // per-image status of the last decode on each pinned slot (device part,
  // copied back at the end of the batch): ticket = the call's number, event
  // = recorded after the copy, so a status can be read `kSlots` calls later
  // without waiting for the newer batches (ldt_fetch_status_ticket)
  int32_t *h_status[kSlots] = {nullptr, nullptr}; // pinned
  size_t h_status_cap[kSlots] = {0, 0};
  hipEvent_t st_ev[kSlots] = {nullptr, nullptr};
  int64_t st_ticket[kSlots] = {-1, -1};
  int64_t st_n[kSlots] = {0, 0};
  int64_t tickets = 0; // decode calls that enqueued work
  int last_sl = 0;     // slot of the most recent decode
  int64_t last_n = 0;
  hipEvent_t done_ev = nullptr;
  hipStream_t last_stream = nullptr;
  bool have_last = false;
  // the progressive coefficient buffer must be all zero between batches
  // (k_idct restores it); set while k_prog output may be in it without a
  // k_idct launched after it, so the next call clears it
  bool coef_dirty = false;
  std::unordered_map<std::string, int> hmap;
  std::vector<HuffTab> htabs;
  // stage profiling: one event per stage boundary, sets recycled once read
  bool profile = false;
  struct EvSet {
    hipEvent_t ev[LDT_NUM_STAGES + 1];
    int first_stage, last_stage; // stages [first, last) were recorded
  };
  std::vector<EvSet> ev_free, ev_pending;
  double stage_ms[LDT_NUM_STAGES] = {0, 0, 0, 0, 0};
  int64_t stage_cnt[LDT_NUM_STAGES] = {0, 0, 0, 0, 0};
  EvSet *cur_ev = nullptr;
  int64_t last_off_redo = -1; // debug counters of the last batch (plan blob offset)
  int last_resize_wpg = -1;   // k_resize4 waves per workgroup of the last JPEG batch (0: streaming kernel)
  uint8_t *last_plan_dev = nullptr; // that batch's plan blob on the device
  double host_us[kHpCount] = {};
  int64_t host_calls = 0;
};

namespace {

// Host phase times of decode_core (LDT_OPT_HOST_TIMING = 1), accumulated per
// context and read with ldt_host_times. Diagnostic only.
struct HostTimer {
  ldt_ctx *c;
  bool on;
  std::chrono::steady_clock::time_point t;
  explicit HostTimer(ldt_ctx *cc) : c(cc), on(cc->host_timing) {
    if (on) t = std::chrono::steady_clock::now();
  }
  void mark(int k) {
    if (!on) return;
    const auto n = std::chrono::steady_clock::now();
    c->host_us[k] += std::chrono::duration<double, std::micro>(n - t).count();
    t = n;
    if (k == kHpStatus) ++c->host_calls;
  }
};

struct DeviceGuard {
  int prev = -1;
  explicit DeviceGuard(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (prev != dev) (void)hipSetDevice(dev);
  }
  ~DeviceGuard() {
    int cur = -1;
    if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
  }
};

int set_err(ldt_ctx *c, int code, const char *fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  if (c) c->err = buf;
  return code;
}

#define HIPCHK(ctx, expr)                                                                      \
  do {                                                                                         \
    hipError_t e_ = (expr);                                                                    \
    if (e_ != hipSuccess)                                                                      \
      return set_err(ctx, LDT_ERR_HIP, "%s failed: %s", #expr, hipGetErrorString(e_));         \
  } while (0)

// Grow a device buffer; contents are not preserved (a new allocation is
// zero-filled on `s` when `zero`). Synchronises `s` first so no in-flight work
// still references the old allocation.
int ensure_dev(ldt_ctx *c, DevBuf &b, size_t need, hipStream_t s, bool zero = false) {
  if (b.cap >= need) return LDT_OK;
  size_t cap = need + need / 4 + 4096;
  if (b.p) {
    HIPCHK(c, hipStreamSynchronize(s));
    HIPCHK(c, hipDeviceSynchronize());
    // the last batch's plan blob (ldt_debug_counters) may live in this buffer
    const uintptr_t lo = (uintptr_t)b.p, lp = (uintptr_t)c->last_plan_dev;
    if (lp >= lo && lp < lo + b.cap) {
      c->last_plan_dev = nullptr;
      c->last_off_redo = -1;
    }
    HIPCHK(c, hipFree(b.p));
    b.p = nullptr;
    b.cap = 0;
  }
  if (hipMalloc(&b.p, cap) != hipSuccess)
    return set_err(c, LDT_ERR_NOMEM, "hipMalloc(%zu) failed", cap);
  b.cap = cap;
  if (zero) HIPCHK(c, hipMemsetAsync(b.p, 0, cap, s));
  return LDT_OK;
}

// Host ranges page-locked in place (ldt_register_host), for all contexts. A
// decode that DMAs from a range holds it (inflight) until its copy is
// enqueued and marks the device it used; ldt_unregister_host drops the range,
// waits for the holders, then synchronises every device that used it before
// unpinning.
struct HostRange {
  uintptr_t lo, hi;
  int inflight = 0;
  uint64_t devmask = 0;
};
std::mutex g_host_m;
std::condition_variable g_host_cv;
std::vector<std::shared_ptr<HostRange>> g_host_ranges;

std::shared_ptr<HostRange> host_acquire(const void *p, size_t n, int dev) {
  const uintptr_t lo = (uintptr_t)p, hi = lo + n;
  std::lock_guard<std::mutex> l(g_host_m);
  for (auto &r : g_host_ranges)
    if (lo >= r->lo && hi <= r->hi) {
      ++r->inflight;
      r->devmask |= 1ull << (dev & 63);
      return r;
    }
  return nullptr;
}

void host_release(std::shared_ptr<HostRange> &r) {
  if (!r) return;
  {
    std::lock_guard<std::mutex> l(g_host_m);
    --r->inflight;
  }
  g_host_cv.notify_all();
  r.reset();
}

bool host_registered(const void *p, size_t n) {
  const uintptr_t lo = (uintptr_t)p, hi = lo + n;
  std::lock_guard<std::mutex> l(g_host_m);
  for (const auto &r : g_host_ranges)
    if (lo >= r->lo && hi <= r->hi) return true;
  return false;
}

CopyPool &copier(ldt_ctx *c) {
  if (!c->copier) {
    char bus[64] = {0};
    if (hipDeviceGetPCIBusId(bus, sizeof(bus), c->device) != hipSuccess) {
      (void)hipGetLastError();
      bus[0] = 0;
    }
    c->placement = copy_placement(bus, c->copy_threads, c->copy_bind != 0);
    c->copier.reset(new CopyPool(c->placement.cpus, c->copy_nt, c->copy_bind == 2));
  }
  return *c->copier;
}

void pinned_copy(ldt_ctx *c, void *dst, const void *src, size_t n) {
  CopyPool &p = copier(c);
  p.start(dst, src, n);
  p.finish();
}

// One non-blocking stream per device for the cells' H2D DMA (LDT_OPT_COPY_MODE
// 0), shared by the process's contexts: the transfer of a batch then runs
// while the kernels of the batches before it still occupy the contexts'
// streams (one more HIP stream per process; the copy engine does the work).
hipStream_t copy_stream(int device) {
  static std::mutex m;
  static hipStream_t streams[64] = {};
  std::lock_guard<std::mutex> l(m);
  if (device < 0 || device >= 64) return nullptr;
  if (!streams[device] && hipStreamCreateWithFlags(&streams[device], hipStreamNonBlocking) != hipSuccess) {
    (void)hipGetLastError();
    streams[device] = nullptr;
  }
  return streams[device];
}

// Joins an asynchronous cell copy on every exit path of decode_core: the
// caller's host buffer is borrowed only for the duration of the call.
struct CopyJoin {
  CopyPool *p = nullptr;
  void wait() {
    if (p) p->finish();
    p = nullptr;
  }
  ~CopyJoin() { wait(); }
};

int ensure_pin(ldt_ctx *c, PinBuf &b, size_t need) {
  if (b.cap >= need) return LDT_OK;
  size_t cap = need + need / 4 + 4096;
  if (b.p) {
    HIPCHK(c, hipHostFree(b.p));
    b.p = nullptr;
    b.cap = 0;
  }
  if (hipHostMalloc(&b.p, cap, hipHostMallocDefault) != hipSuccess)
    return set_err(c, LDT_ERR_NOMEM, "hipHostMalloc(%zu) failed", cap);
  b.cap = cap;
  return LDT_OK;
}

// Grow pinned slot `sl`'s buffer (`which` = h_data or h_plan) and, while it
// is idle, the other slot's to the same size: a pinned allocation costs
// milliseconds, so it should not wait for the first call on the other slot.
int ensure_pin_slots(ldt_ctx *c, PinBuf (&bufs)[ldt_ctx::kSlots], int sl, size_t need) {
  int rc;
  if ((rc = ensure_pin(c, bufs[sl], need))) return rc;
  for (int k = 0; k < ldt_ctx::kSlots; ++k) {
    if (k == sl || bufs[k].cap >= need) continue;
    if (c->slot_used[k] && hipEventQuery(c->slot_ev[k]) != hipSuccess) continue;
    (void)hipGetLastError();
    if ((rc = ensure_pin(c, bufs[k], need))) return rc;
  }
  return LDT_OK;
}

// Wait until the pinned slot's previous H2D copies have completed.
int acquire_slot(ldt_ctx *c) {
  c->slot = (c->slot + 1) % ldt_ctx::kSlots;
  if (c->slot_used[c->slot]) HIPCHK(c, hipEventSynchronize(c->slot_ev[c->slot]));
  return LDT_OK;
}

// Order this call after the previous one when the caller switches streams.
int order_streams(ldt_ctx *c, hipStream_t s) {
  if (c->have_last && c->last_stream != s) HIPCHK(c, hipStreamWaitEvent(s, c->done_ev, 0));
  return LDT_OK;
}

int finish_call(ldt_ctx *c, hipStream_t s) {
  HIPCHK(c, hipEventRecord(c->done_ev, s));
  c->last_stream = s;
  c->have_last = true;
  return LDT_OK;
}

// ---- stage profiling helpers ----
void prof_begin(ldt_ctx *c, int first_stage, hipStream_t s) {
  c->cur_ev = nullptr;
  if (!c->profile) return;
  ldt_ctx::EvSet es;
  if (!c->ev_free.empty()) {
    es = c->ev_free.back();
    c->ev_free.pop_back();
  } else {
    for (int k = 0; k <= LDT_NUM_STAGES; ++k)
      if (hipEventCreate(&es.ev[k]) != hipSuccess) return;
  }
  es.first_stage = es.last_stage = first_stage;
  c->ev_pending.push_back(es);
  c->cur_ev = &c->ev_pending.back();
  (void)hipEventRecord(c->cur_ev->ev[first_stage], s);
}

// Marks the end of `stage` (events for stages must be recorded in order).
void prof_mark(ldt_ctx *c, int stage, hipStream_t s) {
  if (!c->cur_ev) return;
  (void)hipEventRecord(c->cur_ev->ev[stage + 1], s);
  c->cur_ev->last_stage = stage + 1;
}

void build_lut(const ldt_norm *norm, float *lut) {
  // torchvision to_tensor: float32(v) / 255 (IEEE single), then Normalize:
  // (x - mean) / std in float32 (tensor.sub_(mean).div_(std)).
  for (int c = 0; c < 3; ++c)
    for (int v = 0; v < 256; ++v) {
      volatile float x = (float)v / 255.0f;
      if (norm) {
        volatile float t = x - norm->mean[c];
        x = t / norm->std[c];
      }
      lut[c * 256 + v] = x;
    }
}

// The batch's cells (pinned slot or registered pages) -> the slot's device
// buffer. LDT_OPT_COPY_MODE 0: one DMA on the device's copy stream, after the
// kernels that last read that buffer; `s` waits for it. Mode 1 (or no copy
// stream): on `s` itself, behind the previous batch's kernels.
int enqueue_cells(ldt_ctx *c, int sl, const void *src, size_t n, hipStream_t s) {
  hipStream_t cs = c->copy_mode != 0 ? nullptr : (c->copy_stream ? c->copy_stream : copy_stream(c->device));
  if (!cs) {
    HIPCHK(c, hipMemcpyAsync(c->d_data[sl].p, src, n, hipMemcpyHostToDevice, s));
    return LDT_OK;
  }
  if (c->data_used[sl]) HIPCHK(c, hipStreamWaitEvent(cs, c->data_free_ev[sl], 0));
  HIPCHK(c, hipMemcpyAsync(c->d_data[sl].p, src, n, hipMemcpyHostToDevice, cs));
  HIPCHK(c, hipEventRecord(c->h2d_ev[sl], cs));
  HIPCHK(c, hipStreamWaitEvent(s, c->h2d_ev[sl], 0));
  return LDT_OK;
}

struct ImgPlan {
  Header H;
  int status = LDT_IMG_OK;
  int64_t cell_off = 0, cell_len = 0;
};

// Core of every JPEG decode entry point.
//   data_host: cells (host); cell i = [off(i) - base, off(i+1) - base)
//   data_dev : if non-null, the cells already live in HBM at the same offsets.
template <typename OffT>
int decode_core(ldt_ctx *c, const uint8_t *data_host, const uint8_t *data_dev, const OffT *offsets,
                int64_t arr_offset, int64_t n, const uint8_t *validity, const int64_t *labels,
                int64_t label_offset, float *out_img, int64_t *out_lbl, const ldt_norm *norm,
                hipStream_t s, int32_t *status_out) {
  if (!c) return LDT_ERR_ARG;
  if (n < 0 || (n > 0 && (!data_host || !offsets || !out_img || !status_out)))
    return set_err(c, LDT_ERR_ARG, "bad argument (n=%lld)", (long long)n);
  if (n == 0) return LDT_OK;
  if (labels && !out_lbl) return set_err(c, LDT_ERR_ARG, "labels given without out_lbl");
  DeviceGuard g(c->device);
  int rc;
  if ((rc = order_streams(c, s))) return rc;
  HostTimer ht(c);
  const int64_t base = (int64_t)offsets[arr_offset];
  const int64_t total_bytes = (int64_t)offsets[arr_offset + n] - base;
  if (total_bytes < 0) return set_err(c, LDT_ERR_ARG, "offsets not monotonic");
  const uint8_t *cells_host = data_host + base; // cell i at cells_host + (offsets[i] - base)
  if (c->coef_dirty) {
    // an earlier call failed between the Huffman and IDCT launches
    if (c->d_pcoef.p) HIPCHK(c, hipMemsetAsync(c->d_pcoef.p, 0, c->d_pcoef.cap, s));
    c->coef_dirty = false;
  }

  // ---- pinned slot, then the cells' way to HBM, which the header walk below
  // overlaps: the pool threads copy them into the slot (a registered range is
  // DMAed from the caller's pages at once). The copy is joined after the
  // header walk and the batch goes to HBM in one DMA (enqueue_cells). ----
  if ((rc = acquire_slot(c))) return rc;
  const int sl = c->slot;
  std::shared_ptr<HostRange> reg; // registered range the H2D reads from
  CopyJoin cj;
  prof_begin(c, LDT_STAGE_H2D, s);
  if (!data_dev && total_bytes > 0) {
    if ((rc = ensure_dev(c, c->d_data[sl], (size_t)total_bytes + 16, s))) return rc;
    reg = host_acquire(cells_host, (size_t)total_bytes, c->device);
    if (reg) {
      if ((rc = enqueue_cells(c, sl, cells_host, (size_t)total_bytes, s))) return rc;
    } else {
      // room for the plan blob after the cells (plan_with_cells below)
      const size_t room = (size_t)total_bytes + 16 + std::max<size_t>((size_t)total_bytes / 8, (size_t)1 << 18);
      if ((rc = ensure_pin_slots(c, c->h_data, sl, room))) return rc;
      CopyPool &pool = copier(c);
      pool.start(c->h_data[sl].p, cells_host, (size_t)total_bytes);
      cj.p = &pool;
    }
  }
  struct RegRelease {
    std::shared_ptr<HostRange> &r;
    ~RegRelease() { host_release(r); }
  } reg_release{reg};
  ht.mark(kHpSlot);

  // ---- parse headers ----
  std::vector<ImgPlan> P((size_t)n);
  std::vector<ImgDesc> D((size_t)n);
  std::vector<Segment> S;
  std::vector<int32_t> st((size_t)n, 0);
  std::vector<std::vector<uint16_t>> qtabs;
  std::unordered_map<std::string, int> qmap;
  std::vector<int> batch_htab_ids; // ctx table id -> index in this batch
  std::unordered_map<int, int> hid_to_batch;
  std::vector<HuffTab> batch_htabs;
  int64_t dst_total = 0, coef_blocks = 0, pcoef_blocks = 0, plane_total = 0, max_blocks = 0;
  const bool parallel = c->huff_mode != 1;
  const int SB = c->subseq_bits;
  std::vector<int32_t> par_img; // images on the parallel decoder (one workgroup each)
  int n_serial = 0;
  int64_t max_window = 0;       // largest LDS window a parallel image needs
  int32_t n_chunks = 0;          // destuff chunks (kDsChunk bytes of scan data each)
  std::vector<int32_t> chunk_img;
  int max_w = 1, max_h = 1, max_ks_h = 3, max_ks_v = 3, max_tabs = 1, n_fast420 = 0;
  std::vector<ProgScan> pscans;  // progressive images' scans (k_prog)
  std::vector<ProgTab> ptabs;
  std::unordered_map<std::string, int> ptab_map;
  std::vector<int32_t> prog_img;
  bool any_bad = false;
  // The tables of the previous image (per component): images of one dataset
  // mostly share their DQT/DHT bytes, so a byte compare against the last
  // match skips the key strings and hash lookups of the dedupe below.
  struct LastQ {
    uint16_t q[64];
    int idx = -1;
  } last_q[3];
  struct LastH {
    RawHuff r;
    int bidx = -1;
  } last_h[3][2];
  auto same_huff = [](const RawHuff &a, const RawHuff &b) {
    return a.nsym == b.nsym && memcmp(a.counts, b.counts, 16) == 0 && memcmp(a.syms, b.syms, (size_t)a.nsym) == 0;
  };
  for (int64_t i = 0; i < n; ++i) {
    ImgPlan &ip = P[(size_t)i];
    ImgDesc &d = D[(size_t)i];
    memset(&d, 0, sizeof(d));
    const int64_t r = arr_offset + i;
    ip.cell_off = (int64_t)offsets[r] - base;
    ip.cell_len = (int64_t)offsets[r + 1] - (int64_t)offsets[r];
    d.seg_base = (int32_t)S.size();
    if (validity && !((validity[r >> 3] >> (r & 7)) & 1)) {
      ip.status = LDT_IMG_NULL;
    } else if (ip.cell_len < 0) {
      ip.status = LDT_IMG_NOT_JPEG;
    } else {
      ip.status = walk_markers(cells_host + ip.cell_off, ip.cell_len, ip.H);
    }
    Header &H = ip.H;
    if (ip.status == LDT_IMG_OK && (H.width > LDT_MAX_DIM || H.height > LDT_MAX_DIM))
      ip.status = LDT_IMG_TOO_LARGE;
    int hmax = 1, vmax = 1;
    if (ip.status == LDT_IMG_OK) {
      for (int k = 0; k < H.ncomp; ++k) {
        if (!H.progressive &&
            (!H.qpresent[H.tq[k]] || !H.dc[H.td[k]].present || !H.ac[H.ta[k]].present)) {
          ip.status = LDT_IMG_NOT_JPEG;
          break;
        }
        hmax = H.h[k] > hmax ? H.h[k] : hmax;
        vmax = H.v[k] > vmax ? H.v[k] : vmax;
      }
    }
    if (ip.status == LDT_IMG_OK && H.ncomp == 3) {
      // supported upsampling: every component factor divides the max, <= 2
      int bpm = 0;
      if (H.h[0] != hmax || H.v[0] != vmax) ip.status = LDT_IMG_UNSUPPORTED; // subsampled luma
      for (int k = 0; k < 3; ++k) {
        if (hmax % H.h[k] || vmax % H.v[k]) ip.status = LDT_IMG_UNSUPPORTED;
        bpm += H.h[k] * H.v[k];
      }
      if (bpm > kMaxBlocksPerMcu) ip.status = LDT_IMG_UNSUPPORTED;
    }
    if (ip.status != LDT_IMG_OK) {
      st[(size_t)i] = ip.status;
      any_bad = true;
      d.width = d.height = 1;
      d.nseg = 0;
      continue;
    }
    d.width = H.width;
    d.height = H.height;
    d.ncomp = H.ncomp;
    if (H.ncomp == 1) {
      d.color = 2;
      d.mcux = (H.width + 7) / 8;
      d.mcuy = (H.height + 7) / 8;
      d.bpm = 1;
      d.bcomp[0] = 0;
      d.ch[0] = d.cv[0] = 1;
      d.hf[0] = d.vf[0] = 1;
    } else {
      // jdapimin.c default_decompress_parms: JFIF -> YCbCr; Adobe transform 0 -> RGB;
      // otherwise component ids 'R','G','B' -> RGB; else YCbCr.
      bool rgb;
      if (H.jfif) rgb = false;
      else if (H.adobe) rgb = (H.adobe_transform == 0);
      else rgb = (H.cid[0] == 82 && H.cid[1] == 71 && H.cid[2] == 66);
      d.color = rgb ? 1 : 0;
      d.mcux = (H.width + 8 * hmax - 1) / (8 * hmax);
      d.mcuy = (H.height + 8 * vmax - 1) / (8 * vmax);
      int b = 0;
      for (int k = 0; k < 3; ++k) {
        d.ch[k] = H.h[k];
        d.cv[k] = H.v[k];
        d.hf[k] = hmax / H.h[k];
        d.vf[k] = vmax / H.v[k];
        for (int yy = 0; yy < H.v[k]; ++yy)
          for (int xx = 0; xx < H.h[k]; ++xx) {
            d.bcomp[b] = (uint8_t)k;
            d.bdx[b] = (uint8_t)xx;
            d.bdy[b] = (uint8_t)yy;
            ++b;
          }
      }
      d.bpm = b;
    }
    ProgPlan PP;
    if (H.progressive) {
      ip.status = plan_progressive(cells_host + ip.cell_off, ip.cell_len, H, PP);
      if (ip.status != LDT_IMG_OK) {
        st[(size_t)i] = ip.status;
        any_bad = true;
        d.width = d.height = 1;
        d.nseg = 0;
        continue;
      }
    }
    int64_t pl = plane_total;
    for (int k = 0; k < H.ncomp; ++k) {
      const int bw = d.mcux * d.ch[k], bh = d.mcuy * d.cv[k];
      d.plane_stride[k] = bw * 8;
      d.plane_off[k] = pl;
      pl += align_up((int64_t)bw * 8 * bh * 8, 256);
      d.cdw[k] = (int)(((int64_t)H.width * d.ch[k] + hmax - 1) / hmax);
      d.cdh[k] = (int)(((int64_t)H.height * d.cv[k] + vmax - 1) / vmax);
      if (H.ncomp == 1) {
        d.cdw[k] = H.width;
        d.cdh[k] = H.height;
      }
      // quant table (progressive: latched at the component's first scan)
      const uint16_t *qsrc = H.progressive ? PP.q[k] : H.q[H.tq[k]];
      if (last_q[k].idx >= 0 && memcmp(last_q[k].q, qsrc, 128) == 0) {
        d.qt[k] = last_q[k].idx;
      } else {
        std::string qk(reinterpret_cast<const char *>(qsrc), 128);
        auto qi = qmap.find(qk);
        if (qi == qmap.end()) {
          qi = qmap.emplace(qk, (int)qtabs.size()).first;
          qtabs.emplace_back(qsrc, qsrc + 64);
        }
        d.qt[k] = qi->second;
        memcpy(last_q[k].q, qsrc, 128);
        last_q[k].idx = d.qt[k];
      }
      // Huffman tables (deduped across the context's lifetime)
      for (int pass = 0; pass < 2 && !H.progressive; ++pass) {
        const RawHuff &rh = pass == 0 ? H.dc[H.td[k]] : H.ac[H.ta[k]];
        LastH &lh = last_h[k][pass];
        if (lh.bidx >= 0 && same_huff(lh.r, rh)) {
          if (pass == 0) d.dct[k] = lh.bidx;
          else d.act[k] = lh.bidx;
          continue;
        }
        std::string key = huff_key(rh, pass == 0);
        auto it = c->hmap.find(key);
        int cid;
        if (it == c->hmap.end()) {
          HuffTab t;
          if (!build_huff(rh, pass == 0, t)) {
            ip.status = LDT_IMG_NOT_JPEG;
            break;
          }
          cid = (int)c->htabs.size();
          c->htabs.push_back(t);
          c->hmap.emplace(std::move(key), cid);
        } else {
          cid = it->second;
        }
        auto bi = hid_to_batch.find(cid);
        int bidx;
        if (bi == hid_to_batch.end()) {
          bidx = (int)batch_htabs.size();
          batch_htabs.push_back(c->htabs[(size_t)cid]);
          hid_to_batch.emplace(cid, bidx);
        } else {
          bidx = bi->second;
        }
        if (pass == 0) d.dct[k] = bidx;
        else d.act[k] = bidx;
        lh.r = rh;
        lh.bidx = bidx;
      }
    }
    if (ip.status != LDT_IMG_OK) {
      st[(size_t)i] = ip.status;
      any_bad = true;
      d.nseg = 0;
      d.width = d.height = 1;
      continue;
    }
    if (H.progressive) {
      // k_prog decodes it: no baseline segments, destuff chunks or decoder
      // workgroups; its scans join the batch's scan table
      plane_total = pl;
      d.restart = 0;
      d.nseg = 0;
      d.ds_first = n_chunks;
      d.dst_off = dst_total;
      d.prog_first = (int32_t)pscans.size();
      d.prog_count = (int32_t)PP.scans.size();
      for (ProgScan sc : PP.scans) {
        sc.data_off += ip.cell_off;
        for (int k = 0; k < 4; ++k) {
          if (sc.tab[k] < 0) continue;
          const auto &rt = PP.tabs[(size_t)sc.tab[k]];
          std::string key = huff_key(rt.first, rt.second);
          auto it = ptab_map.find(key);
          if (it == ptab_map.end()) {
            ProgTab t;
            if (!build_prog_tab(rt.first, rt.second, t)) {
              ip.status = LDT_IMG_NOT_JPEG;
              break;
            }
            it = ptab_map.emplace(std::move(key), (int)ptabs.size()).first;
            ptabs.push_back(t);
          }
          sc.tab[k] = it->second;
        }
        pscans.push_back(sc);
      }
      if (ip.status != LDT_IMG_OK) {
        pscans.resize((size_t)d.prog_first);
        st[(size_t)i] = ip.status;
        any_bad = true;
        d.nseg = 0;
        d.prog_count = 0;
        d.width = d.height = 1;
        continue;
      }
      prog_img.push_back((int32_t)i);
    }
    if (!H.progressive) {
      // distinct tables over the image's (component, DC/AC) contexts
      int ids[6], nd = 0;
      for (int x = 0; x < 6; ++x) {
        const int cc = (x >> 1) < d.ncomp ? (x >> 1) : 0;
        const int tix = (x & 1) ? d.act[cc] : d.dct[cc];
        bool seen = false;
        for (int q = 0; q < nd; ++q) seen = seen || ids[q] == tix;
        if (!seen) ids[nd++] = tix;
      }
      if (nd > max_tabs) max_tabs = nd;
    }
    const int64_t nmcu = (int64_t)d.mcux * d.mcuy;
    if (!H.progressive) {
    plane_total = pl;
    d.restart = H.restart;
    d.nseg = H.restart ? (int32_t)((nmcu + H.restart - 1) / H.restart) : 1;
    for (int sidx = 0; sidx < d.nseg; ++sidx) {
      Segment sg;
      memset(&sg, 0, sizeof(sg));
      sg.img = (int32_t)i;
      sg.mcu_first = H.restart ? sidx * H.restart : 0;
      sg.mcu_count = H.restart ? (int32_t)std::min<int64_t>(H.restart, nmcu - sg.mcu_first)
                               : (int32_t)nmcu;
      S.push_back(sg);
    }
    d.src_off = ip.cell_off + H.scan_pos;
    d.src_len = ip.cell_len - H.scan_pos;
    const int64_t par_room = kHuffThreads - (int64_t)d.nseg;
    const int64_t par_s = (d.src_len * 8 + par_room - 1) / std::max<int64_t>(par_room, 1);
    if (parallel && d.nseg <= kMaxParSegs && par_s <= kMaxParS - 64) {
      // k_huff_image: all of the image's slots in one workgroup. Slots are
      // sum over segments of ceil(bits_s / S) <= bits / S + nseg, so
      // S >= bits / (kHuffThreads - nseg) fits; the option is a lower bound.
      const int64_t bits = d.src_len * 8;
      const int64_t room = kHuffThreads - d.nseg;
      int64_t sbits = std::max<int64_t>((bits + room - 1) / room, std::max(SB, 64));
      sbits = (sbits + 31) & ~(int64_t)31;
      // an odd number of 32-bit words per range: lanes' LDS window reads start
      // in distinct banks
      if (((sbits >> 5) & 1) == 0) sbits += 32;
      d.sub_bits = (int32_t)sbits;
      par_img.push_back((int32_t)i);
      max_window = std::max<int64_t>(max_window, destuff_region_bytes(d.src_len, d.nseg) + 16);
    } else {
      d.sub_bits = 0;
      ++n_serial;
    }
    // destuff chunks over the scan bytes from the 4-aligned word before them
    d.ds_first = n_chunks;
    d.ds_count = (int32_t)((d.src_len + 3 + kDsChunkBytes - 1) / kDsChunkBytes);
    for (int q = 0; q < d.ds_count; ++q) chunk_img.push_back((int32_t)i);
    n_chunks += d.ds_count;
    d.dst_off = dst_total;
    dst_total += destuff_region_bytes(d.src_len, d.nseg);
    } // !progressive
    // each image's coefficients: room for 8 packed units per block (baseline),
    // and for progressive images also eight dense group planes of npad blocks
    // (coef_piece) in the progressive buffer (ldt_kernels.hpp)
    d.coef_off = coef_blocks;
    const int64_t nblk = nmcu * d.bpm;
    const int64_t npad = (nblk + kCoefAlign - 1) & ~(int64_t)(kCoefAlign - 1);
    coef_blocks += npad;
    d.pcoef_off = pcoef_blocks;
    if (H.progressive) pcoef_blocks += npad;
    if (nblk > max_blocks) max_blocks = nblk;
    if (resize_fast420(d)) ++n_fast420;
    if (H.width > max_w) max_w = H.width;
    if (H.height > max_h) max_h = H.height;
    int kh = resample_ksize_host(H.width, kOut), kv = resample_ksize_host(H.height, kOut);
    if (kh > max_ks_h) max_ks_h = kh;
    if (kv > max_ks_v) max_ks_v = kv;
  }

  // Fused destuff: a k_huff_image workgroup whose image's destuffed stream
  // fits its LDS window destuffs the scan bytes itself (ldt_huffman.hip
  // destuff_into_window); those images get no destuff chunks (ds_count 0)
  int n_ds_img = 0; // baseline images left to k_destuff_*
  {
    int64_t cap = kHuffLdsMax - kHuffStaticLds - huff_tab_lds_image(max_tabs);
    if (c->win_cap >= 0) cap = std::min<int64_t>(cap, c->win_cap);
    const int64_t winb = std::min<int64_t>(max_window, cap) & ~(int64_t)15;
    chunk_img.clear();
    n_chunks = 0;
    for (int64_t i = 0; i < n; ++i) {
      ImgDesc &d = D[(size_t)i];
      d.ds_first = n_chunks;
      if (st[(size_t)i] != LDT_IMG_OK || d.nseg == 0) {
        d.ds_count = 0;
        continue;
      }
      const bool fused = c->fuse_destuff && d.sub_bits > 0 &&
                         destuff_region_bytes(d.src_len, d.nseg) + 16 <= winb;
      d.ds_count = fused ? 0 : (int32_t)((d.src_len + 3 + kDsChunkBytes - 1) / kDsChunkBytes);
      for (int q = 0; q < d.ds_count; ++q) chunk_img.push_back((int32_t)i);
      n_chunks += d.ds_count;
      n_ds_img += fused ? 0 : 1;
    }
  }

  ht.mark(kHpParse); // headers parsed, per-image plans built
  // ---- plan blob layout ----
  PlanHdr ph;
  memset(&ph, 0, sizeof(ph));
  ph.n = (int32_t)n;
  ph.nseg = (int32_t)S.size();
  ph.nhuff = (int32_t)batch_htabs.size();
  ph.nquant = (int32_t)qtabs.size();
  int64_t off = align_up(sizeof(PlanHdr), 64);
  ph.off_desc = off;
  off = align_up(off + (int64_t)sizeof(ImgDesc) * n, 64);
  ph.off_seg = off;
  off = align_up(off + (int64_t)sizeof(Segment) * (int64_t)S.size(), 64);
  ph.off_huff = off;
  off = align_up(off + (int64_t)sizeof(HuffTab) * (int64_t)batch_htabs.size(), 64);
  ph.off_quant = off;
  off = align_up(off + 128 * (int64_t)qtabs.size(), 64);
  ph.off_lut = off;
  off = align_up(off + 3 * 256 * 4, 64);
  ph.off_labels = off;
  off = align_up(off + (labels ? 8 * n : 0), 64);
  const int64_t off_status = off;
  off = align_up(off + 4 * n, 64);
  const int64_t off_wg = off;
  off = align_up(off + 4 * (int64_t)par_img.size(), 64);
  const int64_t off_chunk = off;
  off = align_up(off + 4 * (int64_t)n_chunks, 64);
  const int64_t off_redo = off;
  off = align_up(off + 64, 64);
  const int64_t off_pscan = off;
  off = align_up(off + (int64_t)sizeof(ProgScan) * (int64_t)pscans.size(), 64);
  const int64_t off_ptab = off;
  off = align_up(off + (int64_t)sizeof(ProgTab) * (int64_t)ptabs.size(), 64);
  const int64_t off_pimg = off;
  off = align_up(off + 4 * (int64_t)prog_img.size(), 64);
  const int64_t plan_bytes = off;
  ph.has_labels = labels ? 1 : 0;
  ph.max_ks_h = max_ks_h;
  ph.max_ks_v = max_ks_v;
  ph.max_w = max_w;
  ph.max_blocks = max_blocks;
  ph.total_blocks = coef_blocks;

  // Host cells copied into the pinned slot: the plan blob follows them in the
  // slot and reaches HBM in the same DMA (a separate small H2D copy would be
  // enqueued behind the stream's wait for that DMA, and the runtime may
  // perform small copies synchronously). Otherwise its own pinned buffer and
  // copy on `s`.
  const int64_t plan_off = align_up(total_bytes + 16, 256);
  const bool plan_with_cells = cj.p != nullptr && (int64_t)c->h_data[sl].cap >= plan_off + plan_bytes;
  uint8_t *hp;
  if (plan_with_cells) {
    hp = static_cast<uint8_t *>(c->h_data[sl].p) + plan_off;
  } else {
    if ((rc = ensure_pin_slots(c, c->h_plan, sl, (size_t)plan_bytes))) return rc;
    hp = static_cast<uint8_t *>(c->h_plan[sl].p);
  }
  memcpy(hp, &ph, sizeof(ph));
  memcpy(hp + ph.off_desc, D.data(), sizeof(ImgDesc) * (size_t)n);
  if (!S.empty()) memcpy(hp + ph.off_seg, S.data(), sizeof(Segment) * S.size());
  if (!batch_htabs.empty())
    memcpy(hp + ph.off_huff, batch_htabs.data(), sizeof(HuffTab) * batch_htabs.size());
  for (size_t q = 0; q < qtabs.size(); ++q) memcpy(hp + ph.off_quant + 128 * q, qtabs[q].data(), 128);
  build_lut(norm, reinterpret_cast<float *>(hp + ph.off_lut));
  if (labels) memcpy(hp + ph.off_labels, labels + label_offset, 8 * (size_t)n);
  memcpy(hp + off_status, st.data(), 4 * (size_t)n);
  if (!par_img.empty()) memcpy(hp + off_wg, par_img.data(), 4 * par_img.size());
  if (n_chunks) memcpy(hp + off_chunk, chunk_img.data(), 4 * (size_t)n_chunks);
  memset(hp + off_redo, 0, 64);
  if (!pscans.empty()) memcpy(hp + off_pscan, pscans.data(), sizeof(ProgScan) * pscans.size());
  if (!ptabs.empty()) memcpy(hp + off_ptab, ptabs.data(), sizeof(ProgTab) * ptabs.size());
  if (!prog_img.empty()) memcpy(hp + off_pimg, prog_img.data(), 4 * prog_img.size());

  // ---- device workspace ----
  if (plan_with_cells) {
    if ((rc = ensure_dev(c, c->d_data[sl], (size_t)(plan_off + plan_bytes), s))) return rc;
  } else if ((rc = ensure_dev(c, c->d_plan, (size_t)plan_bytes, s))) {
    return rc;
  }
  // slack: a decoder finishing its last block may read a few hundred bytes
  // past an image's region
  if ((rc = ensure_dev(c, c->d_dstuf, (size_t)dst_total + 1024, s))) return rc;
  // packed coefficients and block records: written before they are read in
  // every batch; the progressive planes: all zero between batches (k_idct
  // clears what it reads), so they are zeroed only when allocated
  if ((rc = ensure_dev(c, c->d_coef, (size_t)coef_blocks * 128 + 256, s))) return rc;
  if ((rc = ensure_dev(c, c->d_brec, (size_t)coef_blocks * 4 + 64, s))) return rc;
  if ((rc = ensure_dev(c, c->d_bcarry, (size_t)coef_blocks / 16 + 64, s))) return rc;
  if (pcoef_blocks > 0 && (rc = ensure_dev(c, c->d_pcoef, (size_t)pcoef_blocks * 128 + 64, s, true))) return rc;
  if ((rc = ensure_dev(c, c->d_dcv, (size_t)coef_blocks * 2 + 64, s))) return rc;
  if ((rc = ensure_dev(c, c->d_planes, (size_t)plane_total + 64, s))) return rc;
  if ((rc = ensure_dev(c, c->d_dscnt, 16 * (size_t)(n_chunks + 1), s))) return rc;
  ht.mark(kHpPlan); // plan blob written, buffers sized
  const uint8_t *dev_cells = data_dev;
  if (!data_dev) {
    if (cj.p) {
      // every chunk copied into the slot: one DMA of the batch
      CopyPool *pool = cj.p;
      cj.wait();
      if (c->host_timing) {
        c->host_us[kHpCopyWake] += std::max(0.0, pool->last_wake_us());
        c->host_us[kHpCopySpan] += pool->last_span_us();
      }
      const size_t nb = (size_t)(plan_with_cells ? plan_off + plan_bytes : total_bytes);
      if ((rc = enqueue_cells(c, sl, c->h_data[sl].p, nb, s))) return rc;
    }
    host_release(reg);
    dev_cells = static_cast<const uint8_t *>(c->d_data[sl].p);
  }
  if (!plan_with_cells) HIPCHK(c, hipMemcpyAsync(c->d_plan.p, hp, (size_t)plan_bytes, hipMemcpyHostToDevice, s));
  HIPCHK(c, hipEventRecord(c->slot_ev[sl], s));
  c->slot_used[sl] = true;
  prof_mark(c, LDT_STAGE_H2D, s);
  ht.mark(kHpCopy);

  uint8_t *dp = plan_with_cells ? static_cast<uint8_t *>(c->d_data[sl].p) + plan_off
                                : static_cast<uint8_t *>(c->d_plan.p);
  DevPlan p;
  p.descs = reinterpret_cast<const ImgDesc *>(dp + ph.off_desc);
  p.segs = reinterpret_cast<Segment *>(dp + ph.off_seg);
  p.htabs = reinterpret_cast<const HuffTab *>(dp + ph.off_huff);
  p.qtabs = reinterpret_cast<const uint16_t *>(dp + ph.off_quant);
  p.lut = reinterpret_cast<const float *>(dp + ph.off_lut);
  p.labels = labels ? reinterpret_cast<const int64_t *>(dp + ph.off_labels) : nullptr;
  p.n = (int)n;
  p.nseg = (int)S.size();
  p.max_ks_h = max_ks_h;
  p.max_ks_v = max_ks_v;
  p.max_w = max_w;
  p.max_h = max_h;
  p.max_blocks = max_blocks;
  p.n_par = (int)par_img.size();
  p.par_img = reinterpret_cast<const int32_t *>(dp + off_wg);
  p.n_serial = n_serial;
  {
    // LDS window of k_huff_image: the largest image's stream, capped by what
    // is left of the CU's LDS after the tables (bigger streams read global)
    int64_t cap = kHuffLdsMax - kHuffStaticLds - huff_tab_lds_image(max_tabs);
    if (c->win_cap >= 0) cap = std::min<int64_t>(cap, c->win_cap);
    p.win_bytes = (int)(std::min<int64_t>(max_window, cap) & ~(int64_t)15);
  }
  p.warm_pct = c->warm_pct;
  p.resize_waves_pct = c->resize_waves_pct;
  p.resize_wpg = c->resize_wpg;
  // 4:2:0 sources <= 512 px: 0 the packed 16-bit staging (k_resize4<5>),
  // 1 the 32-bit staging (k_resize4<0>)
  p.resize420 = c->resize_impl == 1 ? 0 : 3;
  p.n_chunks = n_chunks;
  p.n_ds_img = n_ds_img;
  p.chunk_img = reinterpret_cast<const int32_t *>(dp + off_chunk);
  // diagnostic counters only on request: their atomics cost the kernels time
  p.redo = c->debug_counters ? reinterpret_cast<int32_t *>(dp + off_redo) : nullptr;
  p.max_tabs = max_tabs;
  p.n_fast420 = n_fast420;
  p.n_prog = (int)prog_img.size();
  p.prog_img = reinterpret_cast<const int32_t *>(dp + off_pimg);
  p.pscans = reinterpret_cast<const ProgScan *>(dp + off_pscan);
  p.ptabs = reinterpret_cast<const ProgTab *>(dp + off_ptab);
  c->last_off_redo = c->debug_counters ? off_redo : -1;
  c->last_plan_dev = dp;
  DevWork w;
  w.data = dev_cells;
  w.dstuf = static_cast<uint8_t *>(c->d_dstuf.p);
  w.coef = static_cast<int16_t *>(c->d_coef.p);
  w.brec = static_cast<uint32_t *>(c->d_brec.p);
  w.bcarry = static_cast<uint32_t *>(c->d_bcarry.p);
  w.pcoef = static_cast<int16_t *>(c->d_pcoef.p);
  w.dcv = static_cast<int16_t *>(c->d_dcv.p);
  w.planes = static_cast<uint8_t *>(c->d_planes.p);
  w.status = reinterpret_cast<int32_t *>(dp + off_status);
  w.ds_cnt = static_cast<int4 *>(c->d_dscnt.p);

  HIPCHK(c, launch_destuff(p, w, s));
  prof_mark(c, LDT_STAGE_DESTUFF, s);
  c->coef_dirty = p.n_prog > 0; // until k_idct is enqueued behind k_prog's output
  HIPCHK(c, launch_huff_parallel(p, w, s));
  HIPCHK(c, launch_huff_serial(p, w, s));
  HIPCHK(c, launch_prog(p, w, s));
  HIPCHK(c, launch_dc_scan(p, w, s));
  if (!data_dev && !plan_with_cells) {
    // the cells' last readers are enqueued: a later DMA into this slot's
    // device buffer waits for them (copy stream). With the plan blob in the
    // same buffer, its readers (k_idct, the resize, the status copy) come
    // later: the event is recorded after the status copy below.
    HIPCHK(c, hipEventRecord(c->data_free_ev[sl], s));
    c->data_used[sl] = true;
  }
  prof_mark(c, LDT_STAGE_HUFFMAN, s);
  HIPCHK(c, launch_idct(p, w, s));
  c->coef_dirty = false;
  prof_mark(c, LDT_STAGE_IDCT, s);
  {
    // k_resize4 writes the failed images itself; the streaming fallback does not
    hipError_t rerr = hipSuccess;
    int wpg = 0;
    const bool r4 = c->resize_impl != 2 &&
                    launch_resize4_jpeg(p, w, out_img, labels ? out_lbl : nullptr, s, &rerr, &wpg);
    c->last_resize_wpg = r4 ? wpg : 0;
    if (!r4) rerr = launch_resize_jpeg(p, w, out_img, labels ? out_lbl : nullptr, s);
    HIPCHK(c, rerr);
    if (!r4) HIPCHK(c, launch_fill_failed(p, w, out_img, labels ? out_lbl : nullptr, s));
  }
  prof_mark(c, LDT_STAGE_RESIZE, s);
  c->cur_ev = nullptr;

  ht.mark(kHpLaunch); // kernels launched
  // ---- per-image status back to the host, into this slot's buffer ----
  if ((size_t)n > c->h_status_cap[sl]) {
    if (c->h_status[sl]) {
      HIPCHK(c, hipEventSynchronize(c->st_ev[sl])); // its last copy has landed
      HIPCHK(c, hipHostFree(c->h_status[sl]));
    }
    c->h_status[sl] = nullptr;
    c->h_status_cap[sl] = 0;
    c->st_ticket[sl] = -1;
    if (hipHostMalloc((void **)&c->h_status[sl], 4 * (size_t)n, hipHostMallocDefault) != hipSuccess)
      return set_err(c, LDT_ERR_NOMEM, "hipHostMalloc(status) failed");
    c->h_status_cap[sl] = (size_t)n;
  }
  HIPCHK(c, hipMemcpyAsync(c->h_status[sl], w.status, 4 * (size_t)n, hipMemcpyDeviceToHost, s));
  HIPCHK(c, hipEventRecord(c->st_ev[sl], s));
  if (plan_with_cells) {
    // every reader of the slot's device buffer (cells and plan blob) is
    // enqueued: a later DMA into it waits for the status copy
    HIPCHK(c, hipEventRecord(c->data_free_ev[sl], s));
    c->data_used[sl] = true;
  }
  c->st_ticket[sl] = ++c->tickets;
  c->st_n[sl] = n;
  c->last_sl = sl;
  c->last_n = n;
  if ((rc = finish_call(c, s))) return rc;
  ht.mark(kHpStatus); // status copy enqueued
  memcpy(status_out, st.data(), 4 * (size_t)n);
  if (c->sync_status) {
    HIPCHK(c, hipStreamSynchronize(s));
    bool bad = false;
    for (int64_t i = 0; i < n; ++i) {
      if (status_out[i] == 0) status_out[i] = c->h_status[sl][i];
      if (status_out[i]) bad = true;
    }
    if (bad) return set_err(c, LDT_ERR_IMAGE, "one or more images failed to decode");
  } else if (any_bad) {
    return set_err(c, LDT_ERR_IMAGE, "one or more images failed to parse");
  }
  return LDT_OK;
}

} // namespace

// ---------------------------------------------------------------------------
// C-ABI.
// ---------------------------------------------------------------------------
extern "C" {

const char *ldt_version(void) { return "ldt 0.1.0 gfx950"; }

ldt_ctx *ldt_create(int device, size_t max_batch_bytes, int max_n) {
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev) return nullptr;
  ldt_ctx *c = new (std::nothrow) ldt_ctx();
  if (!c) return nullptr;
  c->device = device;
  DeviceGuard g(device);
  for (int k = 0; k < ldt_ctx::kSlots; ++k)
    if (hipEventCreateWithFlags(&c->slot_ev[k], hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&c->st_ev[k], hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&c->data_free_ev[k], hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&c->h2d_ev[k], hipEventDisableTiming) != hipSuccess) {
      delete c;
      return nullptr;
    }
  if (hipEventCreateWithFlags(&c->done_ev, hipEventDisableTiming) != hipSuccess) {
    delete c;
    return nullptr;
  }
  if (max_batch_bytes > 0) {
    for (int k = 0; k < ldt_ctx::kSlots; ++k) (void)ensure_dev(c, c->d_data[k], max_batch_bytes, nullptr);
    for (int k = 0; k < ldt_ctx::kSlots; ++k) (void)ensure_pin(c, c->h_data[k], max_batch_bytes);
  }
  (void)max_n;
  return c;
}

void ldt_destroy(ldt_ctx *c) {
  if (!c) return;
  DeviceGuard g(c->device);
  (void)hipDeviceSynchronize();
  DevBuf *dbs[] = {&c->d_data[0], &c->d_data[1], &c->d_plan, &c->d_dstuf, &c->d_coef, &c->d_brec, &c->d_bcarry, &c->d_pcoef, &c->d_dcv,
                    &c->d_planes, &c->d_raw, &c->d_dscnt};
  for (DevBuf *b : dbs)
    if (b->p) (void)hipFree(b->p);
  for (int k = 0; k < ldt_ctx::kSlots; ++k) {
    if (c->h_data[k].p) (void)hipHostFree(c->h_data[k].p);
    if (c->h_plan[k].p) (void)hipHostFree(c->h_plan[k].p);
    if (c->slot_ev[k]) (void)hipEventDestroy(c->slot_ev[k]);
    if (c->st_ev[k]) (void)hipEventDestroy(c->st_ev[k]);
    if (c->data_free_ev[k]) (void)hipEventDestroy(c->data_free_ev[k]);
    if (c->h2d_ev[k]) (void)hipEventDestroy(c->h2d_ev[k]);
    if (c->h_status[k]) (void)hipHostFree(c->h_status[k]);
  }
  if (c->done_ev) (void)hipEventDestroy(c->done_ev);
  delete c;
}

const char *ldt_last_error(ldt_ctx *c) { return c ? c->err.c_str() : "null context"; }

int ldt_register_host(ldt_ctx *c, const void *ptr, size_t len) {
  if (!c || !ptr || len == 0) return c ? set_err(c, LDT_ERR_ARG, "register: empty range") : LDT_ERR_ARG;
  DeviceGuard g(c->device);
  if (host_registered(ptr, len)) return LDT_OK;
  hipError_t e = hipHostRegister(const_cast<void *>(ptr), len, hipHostRegisterDefault);
  if (e != hipSuccess) { // e.g. a read-only mapping
    (void)hipGetLastError();
    e = hipHostRegister(const_cast<void *>(ptr), len, hipHostRegisterReadOnly);
  }
  if (e != hipSuccess) {
    (void)hipGetLastError();
    return set_err(c, LDT_ERR_HIP, "hipHostRegister(%zu bytes): %s", len, hipGetErrorString(e));
  }
  auto r = std::make_shared<HostRange>();
  r->lo = (uintptr_t)ptr;
  r->hi = (uintptr_t)ptr + len;
  std::lock_guard<std::mutex> l(g_host_m);
  g_host_ranges.push_back(std::move(r));
  return LDT_OK;
}

int ldt_unregister_host(ldt_ctx *c, const void *ptr) {
  if (!c) return LDT_ERR_ARG;
  DeviceGuard g(c->device);
  uint64_t devmask;
  {
    // no new decode picks the range up once it is out of the list; wait for
    // the ones that did until they have enqueued their copies
    std::unique_lock<std::mutex> l(g_host_m);
    auto it = std::find_if(g_host_ranges.begin(), g_host_ranges.end(),
                           [&](const std::shared_ptr<HostRange> &r) { return r->lo == (uintptr_t)ptr; });
    if (it == g_host_ranges.end()) return set_err(c, LDT_ERR_ARG, "unregister: range not registered");
    std::shared_ptr<HostRange> r = *it;
    g_host_ranges.erase(it);
    g_host_cv.wait(l, [&] { return r->inflight == 0; });
    devmask = r->devmask;
  }
  // every device that copied from the range has finished doing so
  for (int d = 0; d < 64; ++d) {
    if (!((devmask >> d) & 1)) continue;
    DeviceGuard gd(d);
    HIPCHK(c, hipDeviceSynchronize());
  }
  HIPCHK(c, hipHostUnregister(const_cast<void *>(ptr)));
  return LDT_OK;
}

// The stream a context's cells go to HBM on in LDT_OPT_COPY_MODE 0 (NULL:
// the device's own copy stream). A caller that owns its streams lends one
// here, so that the DMAs do not add a fifth stream to the process's four
// hardware queues (DecodePipeline's adaptive mode, transforms.py).
int ldt_set_copy_stream(ldt_ctx *c, void *stream) {
  if (!c) return LDT_ERR_ARG;
  c->copy_stream = (hipStream_t)stream;
  return LDT_OK;
}

int ldt_set_option(ldt_ctx *c, int option, int64_t value) {
  if (!c) return LDT_ERR_ARG;
  switch (option) {
  case LDT_OPT_SYNC_STATUS:
    c->sync_status = value != 0;
    return LDT_OK;
  case LDT_OPT_HUFF_MODE:
    if (value < 0 || value > 2) return set_err(c, LDT_ERR_ARG, "huff mode %lld", (long long)value);
    c->huff_mode = (int)value;
    return LDT_OK;
  case LDT_OPT_PROFILE:
    c->profile = value != 0;
    return LDT_OK;
  case LDT_OPT_SYNC_WARM:
    if (value < 0 || value > 200) return set_err(c, LDT_ERR_ARG, "sync warm-up %lld", (long long)value);
    c->warm_pct = (int)value;
    return LDT_OK;
  case LDT_OPT_HUFF_WINDOW:
    if (value < -1 || value > kHuffLdsMax) return set_err(c, LDT_ERR_ARG, "window cap %lld", (long long)value);
    c->win_cap = value;
    return LDT_OK;
  case LDT_OPT_DEBUG_COUNTERS:
    c->debug_counters = value != 0;
    return LDT_OK;
  case LDT_OPT_RESIZE_IMPL:
    if (value < 0 || value > 2) return set_err(c, LDT_ERR_ARG, "resize impl %lld", (long long)value);
    c->resize_impl = (int)value;
    return LDT_OK;
  case LDT_OPT_SUBSEQ_BITS:
    if (value < 64 || value > 8192 || (value & 31))
      return set_err(c, LDT_ERR_ARG, "subsequence bits %lld", (long long)value);
    c->subseq_bits = (int)value;
    return LDT_OK;
  case LDT_OPT_COPY_THREADS:
    if (value < -1 || value > 31) return set_err(c, LDT_ERR_ARG, "copy threads %lld", (long long)value);
    if ((int)value != c->copy_threads) {
      c->copy_threads = (int)value;
      c->copier.reset(); // rebuilt with the new size on the next copy
    }
    return LDT_OK;
  case LDT_OPT_HOST_TIMING:
    c->host_timing = value != 0;
    return LDT_OK;
  case LDT_OPT_RESIZE_WAVES_PCT:
    if (value < 10 || value > 1000) return set_err(c, LDT_ERR_ARG, "resize waves %lld%%", (long long)value);
    c->resize_waves_pct = (int)value;
    return LDT_OK;
  case LDT_OPT_RESIZE_WG_WAVES:
    if (value != 0 && value != 1 && value != 2 && value != 4)
      return set_err(c, LDT_ERR_ARG, "resize waves per workgroup %lld", (long long)value);
    c->resize_wpg = (int)value;
    return LDT_OK;
  case LDT_OPT_FUSED_DESTUFF:
    c->fuse_destuff = value != 0;
    return LDT_OK;
  case LDT_OPT_COPY_MODE:
    if (value < 0 || value > 1) return set_err(c, LDT_ERR_ARG, "copy mode %lld", (long long)value);
    c->copy_mode = (int)value;
    return LDT_OK;
  case LDT_OPT_COPY_BIND:
    if (value < 0 || value > 2) return set_err(c, LDT_ERR_ARG, "copy bind %lld", (long long)value);
    if ((int)value != c->copy_bind) {
      c->copy_bind = (int)value;
      c->copier.reset();
    }
    return LDT_OK;
  case LDT_OPT_COPY_NT:
    if ((value != 0) != c->copy_nt) {
      c->copy_nt = value != 0;
      c->copier.reset();
    }
    return LDT_OK;
  default:
    return set_err(c, LDT_ERR_ARG, "unknown option %d", option);
  }
}

int ldt_decode_batch(ldt_ctx *c, const uint8_t *data, const int32_t *offsets, int64_t arr_offset,
                     int64_t n, const uint8_t *validity, const int64_t *labels,
                     int64_t label_offset, float *out_img_dev, int64_t *out_lbl_dev,
                     const ldt_norm *norm, void *stream, int32_t *per_image_status) {
  return decode_core<int32_t>(c, data, nullptr, offsets, arr_offset, n, validity, labels,
                              label_offset, out_img_dev, out_lbl_dev, norm, (hipStream_t)stream,
                              per_image_status);
}

int ldt_decode_batch_large(ldt_ctx *c, const uint8_t *data, const int64_t *offsets,
                           int64_t arr_offset, int64_t n, const uint8_t *validity,
                           const int64_t *labels, int64_t label_offset, float *out_img_dev,
                           int64_t *out_lbl_dev, const ldt_norm *norm, void *stream,
                           int32_t *per_image_status) {
  return decode_core<int64_t>(c, data, nullptr, offsets, arr_offset, n, validity, labels,
                              label_offset, out_img_dev, out_lbl_dev, norm, (hipStream_t)stream,
                              per_image_status);
}

int ldt_decode_batch_resident(ldt_ctx *c, const uint8_t *data_host, const uint8_t *data_dev,
                              const int64_t *offsets, int64_t n, const int64_t *labels,
                              float *out_img_dev, int64_t *out_lbl_dev, const ldt_norm *norm,
                              void *stream, int32_t *per_image_status) {
  if (!data_dev) return set_err(c, LDT_ERR_ARG, "data_dev is null");
  if (c && n > 0 && offsets[0] != 0)
    return set_err(c, LDT_ERR_ARG, "resident offsets must start at 0");
  return decode_core<int64_t>(c, data_host, data_dev, offsets, 0, n, nullptr, labels, 0,
                              out_img_dev, out_lbl_dev, norm, (hipStream_t)stream,
                              per_image_status);
}

int ldt_host_info(ldt_ctx *c, char *buf, size_t len) {
  if (!c || !buf || len == 0) return LDT_ERR_ARG;
  DeviceGuard g(c->device);
  (void)copier(c); // placement of the pool the next copy uses
  const CopyPlacement &P = c->placement;
  std::string cpus;
  for (size_t i = 0; i < P.cpus.size(); ++i) cpus += (i ? "," : "") + std::to_string(P.cpus[i]);
  const int w = snprintf(buf, len,
                         "{\"copy_threads\": %d, \"copy_cpus\": [%s], \"gpu_numa\": %d, \"quota_cpus\": %.2f, "
                         "\"local_rank\": %d, \"local_world\": %d, \"l3_domains\": %d, \"candidate_cores\": %d, "
                         "\"copy_bind\": %d, \"copy_nt\": %d, \"copy_mode\": %d, \"local_cpulist\": \"%s\"}",
                         (int)P.cpus.size(), cpus.c_str(), P.gpu_numa, P.quota_cpus, P.local_rank, P.local_world,
                         P.l3_domains, P.candidates, c->copy_bind, c->copy_nt ? 1 : 0, c->copy_mode,
                         P.local_cpulist.c_str());
  return w >= 0 && (size_t)w < len ? LDT_OK : set_err(c, LDT_ERR_ARG, "host info: buffer of %zu bytes too small", len);
}

int ldt_host_times(ldt_ctx *c, double *us_out, int64_t *calls_out, int reset) {
  if (!c) return LDT_ERR_ARG;
  for (int k = 0; k < kHpCount; ++k) {
    if (us_out) us_out[k] = c->host_us[k];
    if (reset) c->host_us[k] = 0;
  }
  if (calls_out) *calls_out = c->host_calls;
  if (reset) c->host_calls = 0;
  return LDT_OK;
}

int ldt_stage_times(ldt_ctx *c, double *ms_out, int64_t *count_out, int reset) {
  if (!c) return LDT_ERR_ARG;
  DeviceGuard g(c->device);
  for (auto &es : c->ev_pending) {
    HIPCHK(c, hipEventSynchronize(es.ev[es.last_stage]));
    for (int k = es.first_stage; k < es.last_stage; ++k) {
      float ms = 0.f;
      HIPCHK(c, hipEventElapsedTime(&ms, es.ev[k], es.ev[k + 1]));
      c->stage_ms[k] += ms;
      c->stage_cnt[k] += 1;
    }
    c->ev_free.push_back(es);
  }
  c->ev_pending.clear();
  for (int k = 0; k < LDT_NUM_STAGES; ++k) {
    if (ms_out) ms_out[k] = c->stage_ms[k];
    if (count_out) count_out[k] = c->stage_cnt[k];
    if (reset) {
      c->stage_ms[k] = 0;
      c->stage_cnt[k] = 0;
    }
  }
  return LDT_OK;
}

namespace {
int merge_status(ldt_ctx *c, int sl, int32_t *st, int64_t n) {
  if (n > c->st_n[sl]) return set_err(c, LDT_ERR_ARG, "n exceeds that batch");
  bool bad = false;
  for (int64_t i = 0; i < n; ++i) {
    if (st[i] == 0) st[i] = c->h_status[sl][i];
    if (st[i]) bad = true;
  }
  return bad ? set_err(c, LDT_ERR_IMAGE, "one or more images failed to decode") : LDT_OK;
}
} // namespace

int ldt_fetch_status(ldt_ctx *c, void *stream, int32_t *st, int64_t n) {
  if (!c || !st) return LDT_ERR_ARG;
  DeviceGuard g(c->device);
  HIPCHK(c, hipStreamSynchronize((hipStream_t)stream));
  if (c->tickets == 0) return n == 0 ? LDT_OK : set_err(c, LDT_ERR_ARG, "no decode yet");
  return merge_status(c, c->last_sl, st, n);
}

int64_t ldt_last_ticket(ldt_ctx *c) { return c ? c->tickets : -1; }

int ldt_fetch_status_ticket(ldt_ctx *c, int64_t ticket, int32_t *st, int64_t n) {
  if (!c || !st) return LDT_ERR_ARG;
  DeviceGuard g(c->device);
  for (int k = 0; k < ldt_ctx::kSlots; ++k)
    if (c->st_ticket[k] == ticket && ticket > 0) {
      HIPCHK(c, hipEventSynchronize(c->st_ev[k]));
      return merge_status(c, k, st, n);
    }
  return set_err(c, LDT_ERR_ARG, "status of call %lld is no longer held (last %lld)", (long long)ticket,
                 (long long)c->tickets);
}

int ldt_resize_raw(ldt_ctx *c, const uint8_t *hwc, int hwc_is_device, int64_t n, int h, int w,
                   int64_t cell_stride, float *out_img_dev, const ldt_norm *norm, void *stream) {
  if (!c) return LDT_ERR_ARG;
  if (n < 0 || h <= 0 || w <= 0 || h > LDT_MAX_DIM || w > LDT_MAX_DIM || !out_img_dev ||
      (n > 0 && !hwc) || cell_stride < (int64_t)h * w * 3)
    return set_err(c, LDT_ERR_ARG, "bad raw resize arguments");
  if (n == 0) return LDT_OK;
  DeviceGuard g(c->device);
  hipStream_t s = (hipStream_t)stream;
  int rc;
  if ((rc = order_streams(c, s))) return rc;
  if ((rc = acquire_slot(c))) return rc;
  const int sl = c->slot;
  if ((rc = ensure_pin(c, c->h_plan[sl], 3 * 256 * 4))) return rc;
  float *hl = static_cast<float *>(c->h_plan[sl].p);
  build_lut(norm, hl);
  if ((rc = ensure_dev(c, c->d_plan, 3 * 256 * 4, s))) return rc;
  const uint8_t *src = hwc;
  if (!hwc_is_device) {
    const size_t bytes = (size_t)(cell_stride * (n - 1) + (int64_t)h * w * 3);
    if ((rc = ensure_pin(c, c->h_data[sl], bytes))) return rc;
    if ((rc = ensure_dev(c, c->d_raw, bytes, s))) return rc;
    pinned_copy(c, c->h_data[sl].p, hwc, bytes);
    HIPCHK(c, hipMemcpyAsync(c->d_raw.p, c->h_data[sl].p, bytes, hipMemcpyHostToDevice, s));
    src = static_cast<const uint8_t *>(c->d_raw.p);
  }
  HIPCHK(c, hipMemcpyAsync(c->d_plan.p, hl, 3 * 256 * 4, hipMemcpyHostToDevice, s));
  HIPCHK(c, hipEventRecord(c->slot_ev[sl], s));
  c->slot_used[sl] = true;
  prof_begin(c, LDT_STAGE_RESIZE, s);
  {
    hipError_t rerr = hipSuccess;
    if (!(c->resize_impl != 2 &&
          launch_resize4_raw(src, cell_stride, (int)n, h, w, static_cast<const float *>(c->d_plan.p),
                             out_img_dev, s, &rerr)))
      rerr = launch_resize_raw(src, cell_stride, (int)n, h, w,
                               static_cast<const float *>(c->d_plan.p), out_img_dev, s);
    HIPCHK(c, rerr);
  }
  prof_mark(c, LDT_STAGE_RESIZE, s);
  c->cur_ev = nullptr;
  if ((rc = finish_call(c, s))) return rc;
  if (c->sync_status) HIPCHK(c, hipStreamSynchronize(s));
  return LDT_OK;
}

int ldt_shard_ranges(ldt_ctx *c, int64_t num_rows, int64_t batch_size, int rank, int world_size,
                     int64_t *out_ranges_dev, int64_t capacity, int64_t *out_count_dev,
                     void *stream) {
  if (!c) return LDT_ERR_ARG;
  if (num_rows < 0 || batch_size <= 0 || world_size <= 0 || rank < 0 || rank >= world_size ||
      !out_count_dev || (capacity > 0 && !out_ranges_dev))
    return set_err(c, LDT_ERR_ARG, "bad shard_ranges arguments");
  DeviceGuard g(c->device);
  HIPCHK(c, launch_shard_ranges(num_rows, batch_size, rank, world_size, out_ranges_dev, capacity,
                                out_count_dev, (hipStream_t)stream));
  return LDT_OK;
}

int ldt_shard_fragments(ldt_ctx *c, const int64_t *fragment_rows_dev, int nfrag,
                        int64_t batch_size, int rank, int world_size, int64_t pad_to,
                        int64_t *out_dev, int64_t capacity, int64_t *out_count_dev,
                        int64_t *out_local_count_dev, void *stream) {
  if (!c) return LDT_ERR_ARG;
  if (nfrag < 0 || batch_size <= 0 || world_size <= 0 || rank < 0 || rank >= world_size ||
      !out_count_dev || !out_local_count_dev || (nfrag > 0 && !fragment_rows_dev) ||
      (capacity > 0 && !out_dev))
    return set_err(c, LDT_ERR_ARG, "bad shard_fragments arguments");
  DeviceGuard g(c->device);
  HIPCHK(c, launch_shard_fragments(fragment_rows_dev, nfrag, batch_size, rank, world_size, pad_to,
                                   out_dev, capacity, out_count_dev, out_local_count_dev,
                                   (hipStream_t)stream));
  return LDT_OK;
}

// torch.utils.data.DistributedSampler.__iter__ (distributed.py:107-141) on
// device: randperm (n < 2^32/20, torch's MT19937 Fisher-Yates branch), pad by
// wrapping or truncate (drop_last), stride by rank. num_samples as :94-103.
int ldt_distributed_indices(ldt_ctx *c, int64_t dataset_len, int num_replicas, int rank,
                            int shuffle, uint64_t seed, int drop_last, int64_t *out_dev,
                            int64_t capacity, int64_t *num_samples_out, void *stream) {
  if (!c) return LDT_ERR_ARG;
  if (dataset_len < 0 || num_replicas <= 0 || rank < 0 || rank >= num_replicas ||
      (capacity > 0 && !out_dev))
    return set_err(c, LDT_ERR_ARG, "bad distributed_indices arguments");
  if (dataset_len >= (int64_t)(UINT32_MAX / 20))
    return set_err(c, LDT_ERR_ARG,
                   "dataset_len %lld >= 2^32/20: torch.randperm switches to 64-bit draws",
                   (long long)dataset_len);
  const int64_t n = dataset_len, W = num_replicas;
  int64_t num_samples;
  if (drop_last && n % W != 0) {
    // math.ceil((n - W) / W) with true division (n - W may be negative)
    const int64_t a = n - W;
    num_samples = a >= 0 ? (a + W - 1) / W : -((-a) / W);
  } else {
    num_samples = (n + W - 1) / W;
  }
  if (num_samples < 0) num_samples = 0;
  if (num_samples_out) *num_samples_out = num_samples;
  if (num_samples == 0) return LDT_OK;
  if (capacity < num_samples)
    return set_err(c, LDT_ERR_ARG, "capacity %lld < num_samples %lld", (long long)capacity,
                   (long long)num_samples);
  DeviceGuard g(c->device);
  hipStream_t s = (hipStream_t)stream;
  if (shuffle) {
    int rc;
    if ((rc = ensure_dev(c, c->d_perm, (size_t)n * 4 * 3 + 64, s))) return rc;
    int32_t *base = static_cast<int32_t *>(c->d_perm.p);
    HIPCHK(c, launch_dist_shuffled((uint32_t)(seed & 0xffffffffu), n, rank, num_replicas,
                                   num_samples, base, base + n, base + 2 * n, out_dev, s));
  } else {
    HIPCHK(c, launch_dist_select(nullptr, n, rank, num_replicas, num_samples, out_dev, s));
  }
  return LDT_OK;
}

// Debug hook (LDT_OPT_DEBUG_COUNTERS = 1): the parallel Huffman decoder's
// counters of the last batch, 16 int32 summed over its k_huff_image
// workgroups (ldt_huffman.hip): [0] unused, [1] workgroups (images), [2]
// convergence rounds (sum), [3] rounds (max), [4] memo adoptions, [5]
// write-pass symbols (sum over lanes), [6] write-pass symbols of each wave's
// slowest lane (sum), [7] unused, [8] setup, [9] phase 1, [10] rounds, [11]
// block-count scan, [12] write pass + DC scan (10 ns s_memrealtime ticks),
// [13] needy slots and [14] waves they ran on (summed over rounds), [15]
// unused. Without the option the kernels get no counter pointer and this
// returns LDT_ERR_ARG.
int ldt_debug_counters(ldt_ctx *c, int32_t *out16, void *stream) {
  if (!c || !out16) return LDT_ERR_ARG;
  DeviceGuard g(c->device);
  if (c->last_off_redo < 0)
    return set_err(c, LDT_ERR_ARG, "no batch decoded with LDT_OPT_DEBUG_COUNTERS = 1 yet");
  HIPCHK(c, hipStreamSynchronize((hipStream_t)stream));
  HIPCHK(c, hipMemcpy(out16, c->last_plan_dev + c->last_off_redo, 64,
                      hipMemcpyDeviceToHost));
  return LDT_OK;
}

// Test hook (not part of ldt.h's stable surface): which resize kernel the last
// JPEG batch took: k_resize4's waves per workgroup (1, 2 or 4), 0 for the
// streaming kernel, -1 before any batch.
int ldt_debug_last_resize(ldt_ctx *c) { return c ? c->last_resize_wpg : LDT_ERR_ARG; }

// Test hook (not part of ldt.h's stable surface): Pillow resample coefficient
// tables computed on the device, for parity tests against the oracle.
int ldt_debug_resample_coeffs(ldt_ctx *c, int in_size, int out_size, int32_t *bounds_dev,
                              int32_t *kk_dev, void *stream) {
  if (!c) return LDT_ERR_ARG;
  DeviceGuard g(c->device);
  HIPCHK(c, launch_resample_coeffs(in_size, out_size, resample_ksize_host(in_size, out_size),
                                   bounds_dev, kk_dev, (hipStream_t)stream));
  return LDT_OK;
}

} // extern "C"
