// rgc_abi.cpp — host orchestration of the batched get_cliques pipeline + the C-ABI
// (include/repic_gc.h).
//
// rgc_run:
//   1. size-class every micrograph by its box count; each class is one launch of the fused
//      per-micrograph kernel (rgc_fused.hip) with an LDS image sized for the class;
//   2. one sync: read per-micrograph stats and the clique reservation cursor; if the output
//      arrays were too small, grow them and re-run the fused launches (first calls only);
//   3. micrographs too large for LDS (or whose edges overflowed the class's LDS edge
//      capacity) are gathered into a compact sub-batch and run through the multi-kernel
//      pipeline (rgc_kernels.hip), writing after the fused outputs.
// One context per device/stream; device workspace is a grow-only arena.
#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <climits>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <map>
#include <mutex>
#include <thread>
#include <tuple>
#include <vector>

#include "../../include/repic_gc.h"
#include "pyset.h"
#include "rgc_kernels.h"

using namespace rgc;

static thread_local std::string g_err;

static int fail(const std::string& msg) {
  g_err = msg;
  return -1;
}
#define HIPCHK(expr)                                                                   \
  do {                                                                                 \
    hipError_t e_ = (expr);                                                            \
    if (e_ != hipSuccess)                                                              \
      return fail(std::string(#expr) + ": " + hipGetErrorString(e_));                   \
  } while (0)
#define TRY(expr)           \
  do {                      \
    int r_ = (expr);        \
    if (r_ != 0) return r_; \
  } while (0)

namespace {

enum DevBufId {
  // fused path / whole batch
  D_FBOXOFF, D_FIDBASE, D_MGLIST, D_MGOUT, D_CURSOR, D_X, D_Y, D_S,
  // outputs
  D_ROWS, D_W, D_CONF, D_CONS, D_MEMBERS, D_ORDER,
  // multi-kernel path (sub-batch)
  D_SUBMG, D_SUBX, D_SUBY, D_SUBS, D_ORIG, D_STAMPS,
  D_BOXOFF, D_CELLOFF, D_P0OFF, D_IDBASE, D_GRID, D_CELLSTART, D_SX, D_SY, D_SBOX, D_SPICK, D_SMG, D_BMG,
  D_BPICK, D_FWDCNT, D_FWDOFF, D_TILES, D_TOTAL, D_EDST, D_EJI, D_PARENT, D_HASEDGE, D_CSIZE,
  D_STAT, D_INSKEY, D_COMPMIN, D_CCOUNT, D_COFF, D_INCL, D_VLIST, D_VSORT, D_VROW, D_BOFF, D_RLO, D_ADJG, D_RBOUND, D_RFLAG, D_DFSMG, D_ROOTBOX, D_EXLIST,
  D_LCNT, D_LOFF, D_LROOT0, D_LROOT1, D_LM0, D_LM1, D_LP0, D_LP1, D_PK,
  // HBM level-tree slots of the 1024-thread fused launches (K >= 4)
  D_QG, D_QGSLOT,
  // set-order tie entries of the fused launches (k_fused_ties)
  D_TIES,
  // RGC_F_EDGES test hook
  D_EU, D_EV, D_EJIOUT,
  // score_detections raster
  D_SC_BOX, D_SC_GOFF, D_SC_POFF, D_SC_TP, D_SC_TR, D_SC_TW, D_SC_CNT,
  // run_ilp set packing
  D_IL_CPTR, D_IL_ROW, D_IL_W, D_IL_REP, D_IL_PAR, D_IL_ROOT, D_IL_CSIZE, D_IL_RCNT, D_IL_RCUR,
  D_IL_RPTR, D_IL_RCOLS, D_IL_CID, D_IL_CN, D_IL_COFF, D_IL_CCUR, D_IL_MEM, D_IL_LOC, D_IL_SCR,
  D_IL_BIG, D_IL_NBIG, D_IL_WSCR, D_IL_X, D_IL_EX, D_IL_RLOC, D_IL_CERT, D_IL_KEY, D_IL_ST,
  D_IL_RMAX, D_IL_OWN, D_IL_LAM, D_IL_GRAD, D_IL_CS, D_IL_CNT, D_IL_GAP, D_IL_STSAVE,
  D_IL_FS, D_IL_FSCNT, D_IL_FSKEEP, D_LBUCKET, D_WIDELIST,
  D_COUNT
};
enum HostBufId {
  H_FSTAGE, H_STAGE, H_TOTAL, H_MGOUT, H_STAT, H_MGOFF, H_ROWS, H_W, H_CONF, H_CONS, H_MEMBERS,
  H_ORDER, H_EU, H_EV, H_EJIOUT, H_COUNT
};

struct Buf {
  void* p = nullptr;
  size_t cap = 0;
};

// LDS is allocated in 1280-byte blocks, 128 per CU (gfx950, measured with
// tools/probe/lds_occ.hip: 3 workgroups per CU up to 53760 B, 2 above it; the HIP occupancy
// API over-reports 3 up to 54613 B, so it is not used).
constexpr int LDS_BLOCK = 1280;
#ifdef RGC_STAMPS
constexpr int LDS_BLOCKS = 127;   // (diagnostic build: the fused kernel's static LDS counters)
#else
constexpr int LDS_BLOCKS = 128;
#endif
// Micrographs above this many boxes go straight to the large-micrograph route.  Above 2048
// boxes the fused layout uses 2 n grid cells and u16 parents (29 B per box + 2 B per edge),
// so a 4096-box micrograph (C3: ~4k boxes, ~15k edges) runs in one workgroup per CU with room
// for 22k edges; at 4608 boxes ~13k edges still fit.
constexpr int64_t FUSED_MAX_BOXES = 4608;
// device cursors after the per-micrograph block: [0] clique reservation, [1] edges of finished
// micrographs, [2] edge-dump reservation (RGC_F_EDGES), [3] spare
// [0] cliques [1] edges [2] edge dump [4] deferrals; [CUR_TIES] ties, on its own 64-B line
// (its per-wave atomics would queue behind the reservations on cursor[0]'s line)
constexpr size_t CUR_BYTES = 128;
// D_MGOUT / H_MGOUT = per-micrograph SoA block, then two cursor slots of CUR_BYTES: a run
// uses slot cur_slot and its kernel zeroes the other one for the next run (no memset packet)
static int lds_blocks(int bytes) { return (bytes + LDS_BLOCK - 1) / LDS_BLOCK; }

// One fused launch configuration: micrographs of <= nmax boxes, forward-edge capacity ecap,
// dynamic LDS bytes, coordinate width, workgroup size.
struct FusedPlan {
  int nmax = 0, ecap = 0, lds = 0, wg = 0;   // wg: workgroups per CU
  int nt = 512;                              // threads per workgroup
  bool wide = false;
};

// Workgroups per CU the VGPRs of the nt-thread kernel allow (nt / 64 waves per workgroup over
// 4 SIMDs of 512 VGPRs, at most 8 waves per SIMD).
static int vgpr_wg_cap(int k, bool wide, int nt) {
  static int cache[2][MAX_K + 1][5] = {};
  const int slot = nt == 256 ? 0 : nt == 384 ? 1 : nt == 512 ? 2 : nt == 768 ? 3 : 4;
  int& v = cache[wide][k][slot];
  if (!v) {
    const int r = fused_vgprs(k, wide, nt);
    const int waves = r > 0 ? std::min(8, 512 / (((r + 7) / 8) * 8)) : 0;
    v = 1 + waves * 4 / (nt / 64);   // stored + 1 (0 = not computed)
  }
  return v - 1;
}

// The most workgroups per CU that LDS (with ecap >= nmax) and VGPRs allow, then the largest
// edge capacity at that occupancy (free LDS up to the next allocation boundary).  Among the
// compiled workgroup sizes the one with the most resident waves per CU wins (ties: the
// smallest): where LDS admits only one or two workgroups per CU, 768 / 1024 threads put the
// idle SIMD slots to work.  max_wg = 1: the whole 160 KiB (largest ecap).
// RGC_DIAG_NT (experiments only) forces one workgroup size when it is compiled for k.
static bool plan_fused(int k, bool wide, int nmax, int max_wg, FusedPlan* p) {
  const int base = fused_lds_bytes(nmax, 0, wide);
  const int need = lds_blocks(fused_lds_bytes(nmax, nmax, wide));
  if (need > LDS_BLOCKS) return false;
  static const int diag_nt = [] {
    const char* e = getenv("RGC_DIAG_NT");
    return e ? atoi(e) : 0;
  }();
  int w = 0, nt = 512, best_waves = 0;
  for (int cand : {256, 384, 512, 768, 1024}) {
    if (!fused_nt_ok(k, cand) || (diag_nt && fused_nt_ok(k, diag_nt) && cand != diag_nt)) continue;
    const int wc = std::min(std::min(max_wg, vgpr_wg_cap(k, wide, cand)), LDS_BLOCKS / need);
    if (wc < 1) continue;
    if (wc * cand / 64 > best_waves) { best_waves = wc * cand / 64; w = wc; nt = cand; }
  }
  if (w < 1) return false;
  const int budget = (LDS_BLOCKS / w) * LDS_BLOCK;
  int ecap = std::min(65535, (budget - base) / 2);
  while (ecap > nmax && fused_lds_bytes(nmax, ecap, wide) > budget) ecap -= 8;
  p->nmax = nmax;
  p->ecap = ecap;
  p->wide = wide;
  p->wg = w;
  p->nt = nt;
  p->lds = fused_lds_bytes(nmax, ecap, wide);
  return p->lds <= budget;
}

// size class of a micrograph of n boxes (64-box steps to 1024, then 128, then 256)
static int fused_class(int64_t n) {
  if (n <= 1024) return (int)std::max<int64_t>(64, (n + 63) / 64 * 64);
  if (n <= 2048) return (int)((n + 127) / 128 * 128);
  return (int)((n + 255) / 256 * 256);
}

// plan_fused memoised per (k, pass, class); nmax = 0 marks "does not fit"
static const FusedPlan& cached_plan(int k, int pass, int nmax) {
  static std::map<std::tuple<int, int, int>, FusedPlan> memo;
  static std::mutex mu;
  std::lock_guard<std::mutex> lk(mu);
  auto it = memo.find({k, pass, nmax});
  if (it != memo.end()) return it->second;
  FusedPlan p;
  // RGC_DIAG_MAX_WG: occupancy experiments only (caps workgroups per CU; outputs unchanged)
  static const int diag_wg = [] {
    const char* e = getenv("RGC_DIAG_MAX_WG");
    return e ? std::max(1, atoi(e)) : LDS_BLOCKS;
  }();
  if (!plan_fused(k, pass > 0, nmax, pass == 2 ? 1 : diag_wg, &p)) p = FusedPlan();
  return memo.emplace(std::make_tuple(k, pass, nmax), p).first->second;
}

}  // namespace

// one side copy stream per device for the whole process (created on first use, kept for the
// process's lifetime)
static int shared_copy_stream(int device, hipStream_t* out) {
  static std::mutex mu;
  static std::vector<hipStream_t> streams;
  std::lock_guard<std::mutex> lk(mu);
  if ((int)streams.size() <= device) streams.resize(device + 1, nullptr);
  if (!streams[device]) HIPCHK(hipStreamCreateWithFlags(&streams[device], hipStreamNonBlocking));
  *out = streams[device];
  return 0;
}

struct rgc_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  bool own_stream = false;
  Buf d[D_COUNT];
  Buf h[H_COUNT];
  std::vector<hipEvent_t> events;
  std::vector<const char*> ev_names;
  int n_ev = 0;
  bool timing = false;
  std::vector<float> times;
  std::vector<const char*> time_names;
  int64_t cap_cliques = 0;   // capacity of the per-clique output arrays
  int64_t cap_edges = 0;     // RGC_F_EDGES: capacity of the edge dump
  int64_t n_edge_dump = 0;   // RGC_F_EDGES: edges of the last run (host copies in H_EU..)
  int cur_slot = 0;          // device cursor slot of the next run (the other one is zeroed)
  void* slots_at = nullptr;  // D_MGOUT address whose cursor slots are known to be zeroed
  size_t slots_off = 0;      // ... at this offset
  int pend_slot = 0;         // cursor slot of the submitted run
  int lazy_n_mg = -1;        // micrographs of the last lazy-stats run not yet fetched
  hipEvent_t ev_tail = nullptr;    // timing: recorded after each fused pass's stats copy   // fused cursor already cleared on the stream for next run
  std::vector<uint64_t> stamps;   // diagnostic build only
  // rgc_submit / rgc_wait: one run in flight per context
  bool pend = false;       // a submitted run awaits rgc_wait
  bool pend_fast = false;  // it is the single fused launch (else it already ran: pend_rc/out)
  int pend_rc = 0;
  rgc_batch_in pin{};      // the submitted batch (caller keeps its arrays alive until rgc_wait)
  rgc_batch_out pend_out{};
  hipEvent_t ev_sub = nullptr;   // after the submitted run's stats copy
  int qg_nslots = 0;             // HBM level-tree slots allocated (ensure_qg)
  // rgc_submit: stream of the per-micrograph stats copy (non-lazy runs).  Unless the caller
  // names one (rgc_ctx_set_copy_stream, ABI 9), the process-wide copy stream of the device,
  // shared by every context: streams beyond GPU_MAX_HW_QUEUES (4) share hardware queues
  bool copy_set = false;
  hipStream_t copy_stream = nullptr;
  bool wide_hint = false;   // rgc_submit: the last batch had micrographs for the f64 layout
  hipEvent_t ev_k = nullptr;           // rgc_submit: after the fused launch
  uint64_t tiles_epoch = 0;      // scan_epoch_count() when D_TILES was last zeroed
  // rgc_submit's general path (host syncs per clique level) runs here; rgc_wait joins it
  std::thread worker;
  std::string pend_err;          // the worker's error message (g_err is per thread)
};

static int ensure_dev(rgc_ctx* c, int id, size_t bytes, size_t keep = 0) {
  Buf& b = c->d[id];
  if (bytes == 0) bytes = 16;
  if (b.cap >= bytes) return 0;
  size_t cap = std::max(bytes, b.cap + b.cap / 2);
  cap = (cap + 255) & ~(size_t)255;
  void* p = nullptr;
  HIPCHK(hipMalloc(&p, cap));
  if (b.p && keep) {
    HIPCHK(hipMemcpyAsync(p, b.p, std::min(keep, b.cap), hipMemcpyDeviceToDevice, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
  }
  if (b.p) HIPCHK(hipFree(b.p));
  b.p = p;
  b.cap = cap;
  // the scan tile buffer: word 0 is the one-pass scan's claim counter (every scan leaves it
  // zero), the rest per-tile states tagged with a launch epoch; a new buffer starts all zero
  // (no state of a reused allocation can match a later epoch)
  if (id == D_TILES) {
    HIPCHK(hipMemsetAsync(p, 0, cap, c->stream));
    c->tiles_epoch = scan_epoch_count();
  }
  return 0;
}

// Before a run that scans: launch epochs repeat after 2^22 - 1 scans process-wide, so a tile
// buffer whose states may date from SCAN_EPOCH_REFRESH scans ago is zeroed first.
static int tiles_refresh(rgc_ctx* c) {
  Buf& b = c->d[D_TILES];
  if (!b.p || scan_epoch_count() - c->tiles_epoch < SCAN_EPOCH_REFRESH) return 0;
  HIPCHK(hipMemsetAsync(b.p, 0, b.cap, c->stream));
  c->tiles_epoch = scan_epoch_count();
  return 0;
}

// HBM level-tree slots of the 1024-thread fused launches (K = 4, rgc_fused.hip P4): twice as
// many as the CUs (LDS admits one such workgroup per CU), QG_BYTES each; the slot bitmap is
// zeroed once and every workgroup clears its bit again before it ends.
constexpr int QG_BYTES = 1 << 20;
static int ensure_qg(rgc_ctx* c, FusedArgs& A, int k, int nt) {
  A.qg_base = nullptr;
  A.qg_slots = nullptr;
  A.qg_nslots = 0;
  A.qg_bytes = 0;
  if (nt != 1024 || k != 4) return 0;
  if (!c->qg_nslots) {
    int ncu = 0;
    HIPCHK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, c->device));
    const int ns = (2 * std::max(ncu, 1) + 31) / 32 * 32;
    TRY(ensure_dev(c, D_QG, (size_t)ns * QG_BYTES));
    TRY(ensure_dev(c, D_QGSLOT, (size_t)ns / 8));
    HIPCHK(hipMemsetAsync(c->d[D_QGSLOT].p, 0, (size_t)ns / 8, c->stream));
    c->qg_nslots = ns;
  }
  A.qg_base = static_cast<char*>(c->d[D_QG].p);
  A.qg_slots = static_cast<uint32_t*>(c->d[D_QGSLOT].p);
  A.qg_nslots = c->qg_nslots;
  A.qg_bytes = QG_BYTES;
  return 0;
}

static int ensure_host(rgc_ctx* c, int id, size_t bytes) {
  Buf& b = c->h[id];
  if (bytes == 0) bytes = 16;
  if (b.cap >= bytes) return 0;
  if (b.p) HIPCHK(hipHostFree(b.p));
  size_t cap = std::max(bytes, b.cap + b.cap / 2);
  b.p = nullptr;
  b.cap = 0;
  HIPCHK(hipHostMalloc(&b.p, cap, hipHostMallocDefault));
  b.cap = cap;
  return 0;
}

template <typename T>
static T* D(rgc_ctx* c, int id) { return reinterpret_cast<T*>(c->d[id].p); }
template <typename T>
static T* H(rgc_ctx* c, int id) { return reinterpret_cast<T*>(c->h[id].p); }

static int mark(rgc_ctx* c, const char* name) {
  if (!c->timing) return 0;
  if (c->n_ev >= (int)c->events.size()) {
    hipEvent_t e;
    HIPCHK(hipEventCreate(&e));
    c->events.push_back(e);
    c->ev_names.push_back(nullptr);
  }
  c->ev_names[c->n_ev] = name;
  HIPCHK(hipEventRecord(c->events[c->n_ev], c->stream));
  ++c->n_ev;
  return 0;
}

// Grow the per-clique output arrays to `need` cliques, keeping the first `keep` cliques.
static int ensure_outputs(rgc_ctx* c, int64_t need, int64_t keep, int k, bool members,
                          bool multi) {
  TRY(ensure_dev(c, D_ROWS, need * k * 4, keep * k * 4));
  TRY(ensure_dev(c, D_W, need * 4, keep * 4));
  TRY(ensure_dev(c, D_CONF, need * 4, keep * 4));
  TRY(ensure_dev(c, D_CONS, need * 4, keep * 4));
  TRY(ensure_dev(c, D_TIES, need * (4 + k) * 4));   // <= one entry per clique
  if (members) TRY(ensure_dev(c, D_MEMBERS, need * k * 4, keep * k * 4));
  if (multi) TRY(ensure_dev(c, D_ORDER, need * k, keep * k));
  return 0;
}

// Grow the RGC_F_EDGES dump arrays to `need` edges, keeping the first `keep`.
static int ensure_edges(rgc_ctx* c, int64_t need, int64_t keep) {
  TRY(ensure_dev(c, D_EU, need * 4, keep * 4));
  TRY(ensure_dev(c, D_EV, need * 4, keep * 4));
  TRY(ensure_dev(c, D_EJIOUT, need * 8, keep * 8));
  return 0;
}

// Cursor pointers of a fused run (see DCUR_BYTES) and the per-micrograph stats, which the
// kernel writes straight into host-mapped pinned memory: no copy or memset packet per run.
struct FusedIo {
  unsigned long long *cur, *clear;
  const unsigned long long* h_cur;   // host copy of cur (after the stats copy)
  int slot;
  MgOut o;
};
static int fused_io(rgc_ctx* c, int n_mg, size_t cur_off, FusedIo* io) {
  TRY(ensure_host(c, H_MGOUT, cur_off + 2 * CUR_BYTES));
  TRY(ensure_dev(c, D_MGOUT, cur_off + 2 * CUR_BYTES));
  char* d = D<char>(c, D_MGOUT);
  if (c->slots_at != d || c->slots_off != cur_off) {   // new buffer or layout: zero both slots
    HIPCHK(hipMemsetAsync(d + cur_off, 0, 2 * CUR_BYTES, c->stream));
    c->slots_at = d;
    c->slots_off = cur_off;
    c->cur_slot = 0;
  }
  const int sl = c->cur_slot;
  io->slot = sl;
  io->cur = reinterpret_cast<unsigned long long*>(d + cur_off + sl * CUR_BYTES);
  io->clear = reinterpret_cast<unsigned long long*>(d + cur_off + (1 - sl) * CUR_BYTES);
  io->h_cur = reinterpret_cast<const unsigned long long*>(H<char>(c, H_MGOUT) + cur_off +
                                                           sl * CUR_BYTES);
  io->o = mgout_bind(d, n_mg);
  return 0;
}

// ---------------------------------------------------------------------------- multi-kernel path
// Runs the multi-kernel pipeline on a (sub-)batch whose x/y/score are device arrays, writing
// per-clique outputs at [out_base, out_base + C).  Fills st_out[n_mg] (clique_base/cnt set).
static int run_multi(rgc_ctx* c, int n_mg, int k, double B, double two_b2, int get_cc, int multi,
                     bool want_members, bool want_ji, const int64_t* box_off, const int64_t* id_base, const double* x,
                     const double* y, const double* sc, int64_t out_base,
                     std::vector<MgStat>& st_out, int64_t* C_out, int64_t* E_out) {
  const int64_t N = box_off[(int64_t)n_mg * k];
  const size_t nbo = (size_t)n_mg * k + 1;
  std::vector<int32_t> cell_off(n_mg + 1);
  int64_t cells = 0;
  bool bin_wide = false;   // k1_bin's u32 counters: a micrograph of more than 65535 boxes
  int max_n = 0;           // largest micrograph (k1_bin's LDS; LDS union-find when it fits)
  for (int m = 0; m < n_mg; ++m) {
    const int64_t nm = box_off[(int64_t)(m + 1) * k] - box_off[(int64_t)m * k];
    bin_wide |= nm > 65535;
    max_n = std::max<int>(max_n, (int)std::min<int64_t>(nm, INT32_MAX));
  }
  for (int m = 0; m < n_mg; ++m) {
    cell_off[m] = (int32_t)cells;
    const int64_t nm = box_off[(int64_t)(m + 1) * k] - box_off[(int64_t)m * k];
    cells += bin_budget(nm, bin_wide) + 2;
  }
  cell_off[n_mg] = (int32_t)cells;
  if (cells >= (1LL << 31)) return fail("too many grid cells in one batch");
  const size_t stage_bytes = nbo * 4 + 2 * (n_mg + 1) * 4 + n_mg * 8 + 64;
  TRY(ensure_host(c, H_STAGE, stage_bytes));
  int32_t* st_bo = H<int32_t>(c, H_STAGE);
  int32_t* st_co = st_bo + nbo;
  int32_t* st_p0 = st_co + n_mg + 1;   // picker-0 prefix: wavefront -> clique root
  int64_t* st_id = reinterpret_cast<int64_t*>(
      (reinterpret_cast<uintptr_t>(st_p0 + n_mg + 1) + 7) & ~(uintptr_t)7);
  for (size_t i = 0; i < nbo; ++i) st_bo[i] = (int32_t)box_off[i];
  std::memcpy(st_co, cell_off.data(), (n_mg + 1) * 4);
  std::memcpy(st_id, id_base, n_mg * 8);
  int64_t n_roots = 0;
  for (int m = 0; m < n_mg; ++m) {
    st_p0[m] = (int32_t)n_roots;
    n_roots += box_off[(int64_t)m * k + 1] - box_off[(int64_t)m * k];
  }
  st_p0[n_mg] = (int32_t)n_roots;

  // the per-micrograph metadata (box offsets, cell offsets, picker-0 prefix, id bases) go up
  // in ONE copy of the host staging block; the device block has the same layout
  const size_t meta_bytes = (size_t)(reinterpret_cast<char*>(st_id + n_mg) -
                                     reinterpret_cast<char*>(st_bo));
  TRY(ensure_dev(c, D_BOXOFF, meta_bytes));
  TRY(ensure_dev(c, D_GRID, n_mg * sizeof(MgGrid)));
  TRY(ensure_dev(c, D_CELLSTART, cells * 4));
  TRY(ensure_dev(c, D_SX, N * 8));
  TRY(ensure_dev(c, D_SY, N * 8));
  TRY(ensure_dev(c, D_SBOX, N * 4));
  TRY(ensure_dev(c, D_SPICK, N));
  TRY(ensure_dev(c, D_SMG, N * 4));
  TRY(ensure_dev(c, D_BMG, N * 4));
  TRY(ensure_dev(c, D_BPICK, N));
  TRY(ensure_dev(c, D_FWDCNT, N * 4));
  TRY(ensure_dev(c, D_FWDOFF, (N + 1) * 8));
  TRY(ensure_dev(c, D_TILES, scan_tiles_needed(N + 1) * 8));
  TRY(ensure_dev(c, D_TOTAL, 32));
  TRY(ensure_dev(c, D_PARENT, N * 4));
  TRY(ensure_dev(c, D_HASEDGE, N));
  TRY(ensure_dev(c, D_CSIZE, N * 4));
  TRY(ensure_dev(c, D_STAT, n_mg * sizeof(MgStat)));
  TRY(ensure_dev(c, D_INSKEY, N * 8));
  if (get_cc) TRY(ensure_dev(c, D_COMPMIN, N * 8));
  TRY(ensure_dev(c, D_CCOUNT, N * 4));
  TRY(ensure_dev(c, D_COFF, (N + 1) * 8));
  TRY(ensure_dev(c, D_INCL, N));
  TRY(ensure_dev(c, D_VLIST, N * 4));
  TRY(ensure_dev(c, D_VSORT, N * 4));
  TRY(ensure_dev(c, D_VROW, N * 4));
  TRY(ensure_dev(c, D_BOFF, (N + 1) * 8));
  TRY(ensure_dev(c, D_RLO, 2 * (size_t)n_mg * 8 + 8));
  TRY(ensure_host(c, H_TOTAL, 32));
  TRY(ensure_host(c, H_STAT, n_mg * sizeof(MgStat)));
  TRY(ensure_host(c, H_MGOFF, 2 * (size_t)n_mg * 8 + 8));
  TRY(ensure_dev(c, D_RBOUND, N * 8));
  TRY(ensure_dev(c, D_RFLAG, N));
  TRY(ensure_dev(c, D_ROOTBOX, n_roots * 4));
  TRY(ensure_dev(c, D_DFSMG, n_mg));

  hipStream_t s = c->stream;
  TRY(mark(c, "h2d_meta"));
  HIPCHK(hipMemcpyAsync(D<void>(c, D_BOXOFF), st_bo, meta_bytes, hipMemcpyHostToDevice, s));
  const int32_t* d_co = D<int32_t>(c, D_BOXOFF) + (st_co - st_bo);
  const int32_t* d_p0 = D<int32_t>(c, D_BOXOFF) + (st_p0 - st_bo);
  const int64_t* d_id = reinterpret_cast<const int64_t*>(
      D<char>(c, D_BOXOFF) + (reinterpret_cast<char*>(st_id) - reinterpret_cast<char*>(st_bo)));
  TRY(mark(c, "memset"));
  // the level loop's first count array (non-roots stay 0) is zeroed with the others
  TRY(ensure_dev(c, D_LCNT, N * 4));
  {
    rgc::FillSegs F{};
    F.add(D<void>(c, D_HASEDGE), N, 0);
    F.add(D<void>(c, D_CSIZE), N * 4, 0);
    F.add(D<void>(c, D_INCL), N, 0);
    F.add(D<void>(c, D_CCOUNT), N * 4, 0);
    F.add(D<void>(c, D_VLIST), N * 4, 0);   // row-rank bucket counters
    F.add(D<void>(c, D_RFLAG), N, 0);
    F.add(D<void>(c, D_DFSMG), n_mg, 0);
    F.add(D<void>(c, D_INSKEY), N * 8, 0xff);
    F.add(D<void>(c, D_LCNT), N * 4, 0);
    if (get_cc) F.add(D<void>(c, D_COMPMIN), N * 8, 0xff);
    rgc::launch_fill_multi(s, F);
  }

  const int32_t* bo = D<int32_t>(c, D_BOXOFF);
  TRY(mark(c, "k1_bin"));
  launch_bin(s, n_mg, k, B, bo, d_co, x, y, D<MgGrid>(c, D_GRID),
             D<int32_t>(c, D_CELLSTART), D<double>(c, D_SX), D<double>(c, D_SY),
             D<int32_t>(c, D_SBOX), D<uint8_t>(c, D_SPICK), D<int32_t>(c, D_SMG),
             D<int32_t>(c, D_BMG), D<uint8_t>(c, D_BPICK), bin_wide, max_n);
  TRY(mark(c, "k2_pairs_count"));
  launch_pairs(s, false, (int)N, k, B, two_b2, bo, d_co, D<MgGrid>(c, D_GRID),
               D<int32_t>(c, D_CELLSTART), D<double>(c, D_SX), D<double>(c, D_SY),
               D<int32_t>(c, D_SBOX), D<uint8_t>(c, D_SPICK), D<int32_t>(c, D_SMG),
               D<int32_t>(c, D_FWDCNT), nullptr, nullptr, nullptr);
  TRY(mark(c, "scan_edges"));
  launch_scan(s, N, D<int32_t>(c, D_FWDCNT), D<int64_t>(c, D_FWDOFF), D<int64_t>(c, D_TILES),
              D<int64_t>(c, D_TOTAL));
  HIPCHK(hipMemcpyAsync(H<int64_t>(c, H_TOTAL), D<int64_t>(c, D_TOTAL), 8,
                        hipMemcpyDeviceToHost, s));
  HIPCHK(hipGetLastError());
  HIPCHK(hipStreamSynchronize(s));
  const int64_t E = H<int64_t>(c, H_TOTAL)[0];
  if (E < 0) return fail("edge scan: look-back guard exhausted (stale tile buffer)");
  *E_out = E;
  TRY(ensure_dev(c, D_EDST, E * 4));
  TRY(ensure_dev(c, D_ADJG, E * 8));
  if (want_ji) TRY(ensure_dev(c, D_EJI, E * 8));   // (the edge JIs feed the RGC_F_EDGES dump only)
  TRY(mark(c, "k2_pairs_fill"));
  launch_pairs(s, true, (int)N, k, B, two_b2, bo, d_co, D<MgGrid>(c, D_GRID),
               D<int32_t>(c, D_CELLSTART), D<double>(c, D_SX), D<double>(c, D_SY),
               D<int32_t>(c, D_SBOX), D<uint8_t>(c, D_SPICK), D<int32_t>(c, D_SMG),
               D<int32_t>(c, D_FWDCNT), D<int64_t>(c, D_FWDOFF), D<int32_t>(c, D_EDST),
               want_ji ? D<double>(c, D_EJI) : nullptr);

  static const char* cc_names[7] = {"k4_init",     "k4_union",    "k4_compress", "k4_stats",
                                    "k4_ins_keys", "k4_comp_min", "k4_target"};
  for (int phase = 0; phase < 7; ++phase) {
    if ((phase == 5 || phase == 6) && !get_cc) continue;
    TRY(mark(c, cc_names[phase]));
    launch_cc(s, phase, (int)N, n_mg, k, get_cc, bo, D<int32_t>(c, D_BMG), D<uint8_t>(c, D_BPICK),
              D<int64_t>(c, D_FWDOFF), D<int32_t>(c, D_EDST), D<int32_t>(c, D_PARENT),
              D<uint8_t>(c, D_HASEDGE), D<int32_t>(c, D_CSIZE), D<MgStat>(c, D_STAT),
              D<unsigned long long>(c, D_INSKEY), D<unsigned long long>(c, D_COMPMIN), max_n);
  }

  CliqueArgs A;
  A.k = k; A.flags = get_cc | (multi << 1); A.n_mg = n_mg; A.n_roots = n_roots; A.C = 0;
  A.B = B; A.two_b2 = two_b2;
  A.box_off = bo; A.p0off = d_p0; A.id_base = d_id;
  A.x = x; A.y = y; A.score = sc; A.bmg = D<int32_t>(c, D_BMG); A.bpick = D<uint8_t>(c, D_BPICK);
  A.fwd_off = D<int64_t>(c, D_FWDOFF); A.e_dst = D<int32_t>(c, D_EDST);
  A.parent = D<int32_t>(c, D_PARENT); A.st = D<MgStat>(c, D_STAT);
  A.ins_key = D<unsigned long long>(c, D_INSKEY); A.clique_off = D<int64_t>(c, D_COFF);
  A.vrow = D<int32_t>(c, D_VROW);
  A.pk = nullptr;
  A.ccount = D<int32_t>(c, D_CCOUNT); A.in_clique = D<uint8_t>(c, D_INCL);
  A.adjg = D<uint64_t>(c, D_ADJG); A.rbound = D<uint64_t>(c, D_RBOUND);
  A.rflag = D<uint8_t>(c, D_RFLAG); A.dfs_mg = D<uint8_t>(c, D_DFSMG); A.dfs_base = 0;
  A.root_box = D<int32_t>(c, D_ROOTBOX);
  A.exmask = nullptr; A.exlist = nullptr; A.excount = nullptr;
  A.members = nullptr; A.rows = nullptr; A.w = nullptr; A.conf = nullptr; A.consensus = nullptr;
  A.order = nullptr;
  int64_t* d_tot = D<int64_t>(c, D_TOTAL);   // [0] edges, [1] DFS cliques, [2] level, [3] rank
  int64_t* h_tot = H<int64_t>(c, H_TOTAL);
  TRY(mark(c, "k5_setup"));   // DFS routing, neighbourhood bitmaps
  launch_clique_setup(s, (int)N, A);
  TRY(mark(c, "k5_dfs_count"));   // (micrographs with a root of > RB_W neighbours only)
  if (launch_cliques_dfs(s, false, (int)N, A) != 0) return fail("unsupported k");
  launch_scan(s, N, D<int32_t>(c, D_CCOUNT), D<int64_t>(c, D_COFF), D<int64_t>(c, D_TILES),
              d_tot + 1);
  // prefix levels: count -> scan -> (host reads the size) -> fill, ping-pong item buffers
  LevelArgs L;
  L.D = 0; L.n_items = N; L.in_root = nullptr; L.in_M = nullptr; L.in_P = nullptr;
  L.cnt = nullptr; L.off = nullptr; L.out_root = nullptr; L.out_M = nullptr; L.out_P = nullptr;
  L.next_cnt = nullptr;
  int cur = 0;
  int64_t C1 = 0, C2 = 0;
  // k >= 3 without members in the outputs: the leaf level's cliques are generated inside their
  // epilogue (k5_leaf_epi), their members never written (the exact pass's excepted)
  const bool leaf_epi = !want_members && !multi && k >= 3;
  for (int lv = 0; lv <= k - 2; ++lv) {
    const bool first = lv == 0, leaf = lv == k - 2;
    L.D = lv;
    TRY(ensure_dev(c, D_LCNT, L.n_items * 4));
    TRY(ensure_dev(c, D_LOFF, (L.n_items + 1) * 8));
    TRY(ensure_dev(c, D_TILES, scan_tiles_needed(L.n_items + 1) * 8));
    L.cnt = D<int32_t>(c, D_LCNT);
    L.off = D<int64_t>(c, D_LOFF);
    // (the leaf level of k >= 3: its counts and marks came from the last fill, next_cnt)
    if (!(leaf && k >= 3)) {
      TRY(mark(c, leaf ? "k5_leaf_count" : "k5_level_count"));
      // (first level: L.cnt was zeroed with the per-box arrays; non-roots stay 0)
      if (launch_clique_level(s, first, leaf, false, A, L) != 0) return fail("unsupported k");
    }
    // (the leaf level of the fused leaf epilogue: its scan also records the prefix holding
    // each wave's first clique; C1 <= 64 n_items, so at most n_items / 2 + 1 waves)
    int32_t* lbucket = nullptr;
    if (leaf && leaf_epi) {
      TRY(ensure_dev(c, D_LBUCKET, ((size_t)L.n_items / 2 + 2) * 4));
      lbucket = D<int32_t>(c, D_LBUCKET);
    }
    launch_scan(s, L.n_items, L.cnt, D<int64_t>(c, D_LOFF), D<int64_t>(c, D_TILES), d_tot + 2,
                lbucket, LEAF_Q);
    HIPCHK(hipMemcpyAsync(h_tot + 1, d_tot + 1, 16, hipMemcpyDeviceToHost, s));
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(s));
    const int64_t nn = h_tot[2];
    C2 = h_tot[1];
    if (nn < 0 || C2 < 0) return fail("clique scan: look-back guard exhausted (stale tile buffer)");
    if (leaf) {
      C1 = nn;
      break;
    }
    const int o = cur ^ 1;
    TRY(ensure_dev(c, D_LROOT0 + o, nn * 4));
    TRY(ensure_dev(c, D_LM0 + o, nn * 8));
    TRY(ensure_dev(c, D_LP0 + o, nn * 8));
    L.out_root = D<int32_t>(c, D_LROOT0 + o);
    L.out_M = D<uint64_t>(c, D_LM0 + o);
    L.out_P = D<uint64_t>(c, D_LP0 + o);
    // the last fill's children are the leaf prefixes: it writes their leaf counts into the
    // count buffer (this level's counts are dead after the scan; sized here so the leaf
    // iteration's ensure_dev keeps it) and marks the clique vertices
    L.next_cnt = nullptr;
    if (lv == k - 3) {
      TRY(ensure_dev(c, D_LCNT, nn * 4));
      L.next_cnt = D<int32_t>(c, D_LCNT);
    }
    TRY(mark(c, "k5_level_fill"));
    launch_clique_level(s, first, false, true, A, L);
    L.next_cnt = nullptr;
    L.in_root = L.out_root; L.in_M = L.out_M; L.in_P = L.out_P;
    L.n_items = nn;
    cur = o;
  }
  // row ranks need only the clique-vertex flags of the count passes (bucket counters in
  // D_VLIST, slots in D_CSIZE: the CC sizes are dead by now; buckets in D_FWDCNT, dead since
  // the edge scan)
  TRY(mark(c, "k7_rank"));
  launch_rank(s, (int)N, n_mg, k, bo, D<int32_t>(c, D_BMG), D<MgGrid>(c, D_GRID), x, y,
              D<uint8_t>(c, D_INCL), D<int32_t>(c, D_VLIST), D<int32_t>(c, D_CSIZE),
              D<int32_t>(c, D_FWDCNT), D<int64_t>(c, D_BOFF), D<int64_t>(c, D_TILES), d_tot + 3,
              D<int32_t>(c, D_VSORT), D<int32_t>(c, D_VROW), D<MgStat>(c, D_STAT));
  const int64_t C = C1 + C2;
  *C_out = C;
  TRY(ensure_outputs(c, out_base + C, out_base, k, true, multi != 0));
  A.C = C;
  A.dfs_base = C1;
  A.members = D<int32_t>(c, D_MEMBERS) + out_base * k;
  A.rows = D<int32_t>(c, D_ROWS) + out_base * k;
  A.w = D<float>(c, D_W) + out_base;
  A.conf = D<float>(c, D_CONF) + out_base;
  A.consensus = D<int32_t>(c, D_CONS) + out_base;
  A.order = multi ? D<uint8_t>(c, D_ORDER) + out_base * k : nullptr;
  if (!leaf_epi) {
    TRY(mark(c, "k5_leaf_fill"));
    launch_clique_level(s, k == 2, true, true, A, L);
  }
  TRY(mark(c, "k5_dfs_fill"));
  launch_cliques_dfs(s, true, (int)N, A);
  // exact list [C], ballot words [ceil(C / 64)], per compaction wave: offsets and counts
  const int64_t exw = (C + 63) / 64, exnw = (exw + 63) / 64;
  TRY(ensure_dev(c, D_EXLIST, (C + exw + exnw + 1) * 8 + exnw * 4 + 16));
  TRY(ensure_dev(c, D_TILES, scan_tiles_needed(exnw + 1) * 8));
  A.exlist = D<int64_t>(c, D_EXLIST);
  A.exmask = reinterpret_cast<uint64_t*>(A.exlist + C);
  A.exwoff = reinterpret_cast<int64_t*>(A.exmask + exw);
  A.exwtot = reinterpret_cast<int32_t*>(A.exwoff + exnw + 1);
  A.tiles = D<int64_t>(c, D_TILES);
  // the exact list's length: the compaction scan's total (the rank scan's total is dead)
  A.excount = reinterpret_cast<unsigned long long*>(d_tot + 3);
  TRY(ensure_dev(c, D_PK, (size_t)N * 16));
  A.pk = D<double>(c, D_PK);
  // the epilogues set one bit per clique for the exact pass in these words
  HIPCHK(hipMemsetAsync(A.exmask, 0, exw * 8, s));
  TRY(mark(c, "k5_pack"));
  launch_clique_pack(s, (int)N, A);
  A.epi_lo = 0;
  if (leaf_epi) {
    TRY(mark(c, "k5_leaf_epi"));
    // (the prefix holding each wave's first clique: written by the leaf level's scan)
    if (launch_clique_leaf_epi(s, A, L, D<int32_t>(c, D_LBUCKET), C1) != 0)
      return fail("unsupported k");
    A.epi_lo = C1;   // k5_epilogue: the DFS route's cliques only
  }
  TRY(mark(c, "k5_epilogue"));
  launch_clique_epilogue(s, false, A);
  TRY(mark(c, "k5_epi_exact"));
  launch_clique_epilogue(s, true, A);
  TRY(mark(c, "k5_ranges"));
  launch_clique_ranges(s, A, C1, D<int64_t>(c, D_RLO), D<int64_t>(c, D_RLO) + n_mg,
                       leaf_epi ? L.in_root : nullptr, leaf_epi ? L.off : nullptr,
                       leaf_epi ? L.n_items : 0);
  HIPCHK(hipMemcpyAsync(H<void>(c, H_STAT), D<void>(c, D_STAT), n_mg * sizeof(MgStat),
                        hipMemcpyDeviceToHost, s));
  HIPCHK(hipMemcpyAsync(H<void>(c, H_MGOFF), D<void>(c, D_RLO), 2 * (size_t)n_mg * 8,
                        hipMemcpyDeviceToHost, s));
  HIPCHK(hipGetLastError());
  HIPCHK(hipStreamSynchronize(s));
  const MgStat* st = H<MgStat>(c, H_STAT);
  const int64_t* rlo = H<int64_t>(c, H_MGOFF);
  const int64_t* rhi = rlo + n_mg;
  st_out.assign(st, st + n_mg);
  for (int m = 0; m < n_mg; ++m) {
    st_out[m].clique_base = out_base + rlo[m];
    st_out[m].clique_cnt = rhi[m] - rlo[m];
    if (st_out[m].status == RGC_OK && st_out[m].clique_cnt == 0) st_out[m].status = RGC_NO_CLIQUES;
  }
  return 0;
}

// ---------------------------------------------------------------------------- rgc_run
static int run_impl(rgc_ctx* c, const rgc_batch_in* in, rgc_batch_out* out) {
  const int n_mg = in->n_mg, k = in->k;
  const uint32_t flags = in->flags;
  if (n_mg < 0) return fail("n_mg < 0");
  if (k < 1 || k > MAX_K) return fail("k (number of pickers) must be in 1..8");
  if (in->box_size > (1LL << 26)) return fail("box_size too large (> 2^26)");
  const int64_t N = n_mg ? in->box_off[(int64_t)n_mg * k] : 0;
  if (N >= (1LL << 31) - 1) return fail("too many boxes in one batch (>= 2^31)");
  const int get_cc = (flags & RGC_F_GET_CC) ? 1 : 0;
  const int multi = (flags & RGC_F_MULTI_OUT) ? 1 : 0;
  const bool want_members = (flags & (RGC_F_MEMBERS | RGC_F_MULTI_OUT)) != 0;
  const bool want_edges = (flags & RGC_F_EDGES) != 0;
  c->n_edge_dump = 0;
  TRY(tiles_refresh(c));
  const double B = (double)in->box_size;
  const double two_b2 = (double)(2 * in->box_size * in->box_size);
  c->timing = (flags & RGC_F_TIMING) != 0;
  c->n_ev = 0;

  // per-micrograph outputs: pinned SoA block, filled by one copy of the device mirror
  // the fused kernels' reservation cursor (16 B) sits right after the per-micrograph block,
  // so one copy returns both
  const size_t cur_off = (mgout_bytes(n_mg) + 15) & ~(size_t)15;
  TRY(ensure_host(c, H_MGOUT, cur_off + 2 * CUR_BYTES));
  const MgOut ho = mgout_bind(H<void>(c, H_MGOUT), n_mg);
  std::memset(out, 0, sizeof(*out));
  out->status = ho.status;
  out->cc_max = ho.cc_max;
  out->cc_cnt = ho.cc_cnt;
  out->n_nodes = ho.n_nodes;
  out->n_vert = ho.n_vert;
  out->n_edges_mg = ho.n_edges;
  out->clique_base = ho.clique_base;
  out->clique_cnt = ho.clique_cnt;
  out->n_boxes = N;
  if (n_mg == 0) return 0;
  if (k == 1) {  // no picker pairs -> no edges -> reference ValueError on every micrograph
    std::memset(H<void>(c, H_MGOUT), 0, mgout_bytes(n_mg));
    std::fill(ho.status, ho.status + n_mg, RGC_NO_EDGES);
    return 0;
  }
  hipStream_t s = c->stream;

  // ---- inputs on device
  const bool no_fused = (flags & RGC_F_NO_FUSED) != 0;
  const double *x = in->x, *y = in->y, *sc = in->score;
  const size_t nbo = (size_t)n_mg * k + 1;
  const size_t fstage = nbo * 4 + n_mg * 8 + 3 * (size_t)n_mg * 4 + 64;   // 3 passes of lists
  TRY(ensure_host(c, H_FSTAGE, fstage));
  int32_t* f_bo = H<int32_t>(c, H_FSTAGE);
  int64_t* f_id = reinterpret_cast<int64_t*>(
      (reinterpret_cast<uintptr_t>(f_bo + nbo) + 7) & ~(uintptr_t)7);
  int32_t* f_ml = reinterpret_cast<int32_t*>(f_id + n_mg);
  // per-micrograph offsets on the device: the caller's HBM-resident copies, or an upload
  const bool dev_meta = (flags & RGC_F_DEVICE_META) != 0;
  if (dev_meta && (!in->dev_box_off || !in->dev_id_base))
    return fail("RGC_F_DEVICE_META needs dev_box_off and dev_id_base");
  TRY(ensure_dev(c, D_MGLIST, 3 * (size_t)n_mg * 4 + 4));
  const unsigned long long* h_cur = nullptr;   // host copy of the fused run's cursor slot
  const int32_t* d_bo = in->dev_box_off;
  const int64_t* d_id = in->dev_id_base;
  if (!dev_meta) {
    for (size_t i = 0; i < nbo; ++i) f_bo[i] = (int32_t)in->box_off[i];
    std::memcpy(f_id, in->id_base, n_mg * 8);
    TRY(ensure_dev(c, D_FBOXOFF, nbo * 4));
    TRY(ensure_dev(c, D_FIDBASE, n_mg * 8));
    TRY(mark(c, "h2d_meta"));
    HIPCHK(hipMemcpyAsync(D<void>(c, D_FBOXOFF), f_bo, nbo * 4, hipMemcpyHostToDevice, s));
    HIPCHK(hipMemcpyAsync(D<void>(c, D_FIDBASE), f_id, n_mg * 8, hipMemcpyHostToDevice, s));
    d_bo = D<int32_t>(c, D_FBOXOFF);
    d_id = D<int64_t>(c, D_FIDBASE);
  }
  if (!(flags & RGC_F_DEVICE_INPUTS)) {
    TRY(ensure_dev(c, D_X, N * 8));
    TRY(ensure_dev(c, D_Y, N * 8));
    TRY(ensure_dev(c, D_S, N * 8));
    HIPCHK(hipMemcpyAsync(D<void>(c, D_X), in->x, N * 8, hipMemcpyHostToDevice, s));
    HIPCHK(hipMemcpyAsync(D<void>(c, D_Y), in->y, N * 8, hipMemcpyHostToDevice, s));
    HIPCHK(hipMemcpyAsync(D<void>(c, D_S), in->score, N * 8, hipMemcpyHostToDevice, s));
    x = D<double>(c, D_X);
    y = D<double>(c, D_Y);
    sc = D<double>(c, D_S);
  }

  // ---- fused passes.  Pass 0: f32-coordinate layout at the best occupancy; pass 1: the
  // micrographs it deferred (coordinates not exact in f32, or more edges than its ecap) with
  // f64 coordinates; pass 2: the edge-capacity overflows of pass 1 with the whole LDS.  What
  // is still deferred (or too large for LDS) runs through the multi-kernel path.
  int64_t fused_total = 0;
  int64_t fused_edges = 0;   // RGC_F_EDGES: edges dumped by the fused passes
  int64_t E_total = 0;
  std::vector<int32_t> deferred;
  std::vector<int32_t> todo0;
  auto mg_class = [&](int m) {
    const int64_t nm = in->box_off[(int64_t)(m + 1) * k] - in->box_off[(int64_t)m * k];
    return nm <= FUSED_MAX_BOXES ? fused_class(nm) : 0;
  };
  // per-call plan lookup: few distinct classes, so a linear list beats the shared memo
  std::vector<std::pair<int, const FusedPlan*>> local_plans;
  auto plan_of = [&](int pass, int cl) -> const FusedPlan& {
    const int key = cl * 4 + pass;
    for (const auto& lp : local_plans)
      if (lp.first == key) return *lp.second;
    local_plans.push_back({key, &cached_plan(k, pass, cl)});
    return *local_plans.back().second;
  };
  // fast path: every micrograph fits pass 0 and the largest class runs at the occupancy of
  // the smallest (feasibility and occupancy are monotone in n) -> one launch over all of them
  int64_t nmin = INT64_MAX, nmaxb = 0;
  for (int m = 0; m < n_mg; ++m) {
    const int64_t nm = in->box_off[(int64_t)(m + 1) * k] - in->box_off[(int64_t)m * k];
    nmin = std::min(nmin, nm);
    nmaxb = std::max(nmaxb, nm);
  }
  const bool all0 = !no_fused && n_mg > 0 && nmaxb <= FUSED_MAX_BOXES &&
                    plan_of(0, fused_class(nmaxb)).nmax &&
                    plan_of(0, fused_class(nmin)).wg == plan_of(0, fused_class(nmaxb)).wg &&
                    plan_of(0, fused_class(nmin)).nt == plan_of(0, fused_class(nmaxb)).nt;
  if (!all0) {
    todo0.reserve(n_mg);
    for (int m = 0; m < n_mg; ++m) {
      const int cl = mg_class(m);
      if (!no_fused && cl && plan_of(0, cl).nmax) todo0.push_back(m);
      else deferred.push_back(m);
    }
  }
  if (all0 || !todo0.empty()) {
    if (c->cap_cliques < 4096) c->cap_cliques = std::max<int64_t>(4096, N);
    if (want_edges && c->cap_edges < 4 * N + 4096) c->cap_edges = 4 * N + 4096;
    for (int attempt = 0; attempt < 2; ++attempt) {
      TRY(ensure_outputs(c, c->cap_cliques, 0, k, want_members, multi != 0));
      if (want_edges) TRY(ensure_edges(c, c->cap_edges, 0));
      // this run's cursor slot was zeroed by the previous run's kernel (or at allocation);
      // a regrow attempt re-zeroes it
      FusedIo io;
      TRY(fused_io(c, n_mg, cur_off, &io));
      if (attempt > 0) HIPCHK(hipMemsetAsync(io.cur, 0, CUR_BYTES, s));
      h_cur = io.h_cur;
      FusedArgs A{};
      A.k = k; A.flags = get_cc | (multi << 1) | (want_members ? 32 : 0);
      A.B = B; A.two_b2 = two_b2;
      A.box_off = d_bo; A.id_base = d_id;
      A.x = x; A.y = y; A.score = sc; A.o = io.o;
      A.cursor = io.cur; A.cap = c->cap_cliques;
      A.cursor_clear = io.clear;
      A.rows = D<int32_t>(c, D_ROWS); A.w = D<float>(c, D_W); A.conf = D<float>(c, D_CONF);
      A.consensus = D<int32_t>(c, D_CONS);
      A.members = want_members ? D<int32_t>(c, D_MEMBERS) : nullptr;
      A.order = multi ? D<uint8_t>(c, D_ORDER) : nullptr;
      A.stamps = nullptr;
      A.eu = want_edges ? D<int32_t>(c, D_EU) : nullptr;
      A.ev = want_edges ? D<int32_t>(c, D_EV) : nullptr;
      A.eji = want_edges ? D<double>(c, D_EJIOUT) : nullptr;
      A.ecap_out = c->cap_edges;
      A.tie_list = D<int32_t>(c, D_TIES);
      A.tie_cap = c->cap_cliques;
      A.esum_n = 0;   // (the host sums the finished micrographs' edges from the stats copy)
      A.wide_list = nullptr;   // (host-driven passes here)
      A.mg_count = nullptr;
      int64_t ties_done = 0;   // entries of earlier passes already resolved
#ifdef RGC_STAMPS
      TRY(ensure_dev(c, D_STAMPS, 3 * (size_t)n_mg * rgc::STAMP_SLOTS * 8));
      HIPCHK(hipMemsetAsync(D<void>(c, D_STAMPS), 0, 3 * (size_t)n_mg * rgc::STAMP_SLOTS * 8, s));
#endif
      std::vector<int32_t> todo = todo0, left;
      int ml_off = 0;   // mg-list slots used (earlier passes' lists stay intact)
      bool overflow = false;
      for (int pass = 0; pass < 3 && (!todo.empty() || (pass == 0 && all0)); ++pass) {
        const bool wide = pass > 0;
        const bool single = pass == 0 && all0;   // identity list: block b = micrograph b
        // bucket by size class (few classes: linear search of the bucket keys)
        std::vector<int> keys;
        std::vector<std::vector<int32_t>> lists;
        left.clear();
        if (single) {
          keys.assign(1, fused_class(nmaxb));
          lists.assign(1, std::vector<int32_t>());
        }
        int last = -1;
        for (int32_t m : todo) {
          const int cl = mg_class(m);
          if (!cl || !plan_of(pass, cl).nmax) { left.push_back(m); continue; }
          if (last < 0 || keys[last] != cl) {
            last = -1;
            for (size_t q = 0; q < keys.size(); ++q)
              if (keys[q] == cl) last = (int)q;
            if (last < 0) { keys.push_back(cl); lists.emplace_back(); last = (int)keys.size() - 1; }
          }
          lists[last].push_back(m);
        }
        std::vector<int32_t> by;
        std::vector<size_t> starts;
        if (single) {
          starts.push_back(0);
        } else {
          for (size_t q = 0; q < keys.size(); ++q) {
            starts.push_back(by.size());
            by.insert(by.end(), lists[q].begin(), lists[q].end());
          }
          std::memcpy(f_ml + ml_off, by.data(), by.size() * 4);
          if (!by.empty())
            HIPCHK(hipMemcpyAsync(D<int32_t>(c, D_MGLIST) + ml_off, f_ml + ml_off, by.size() * 4,
                                  hipMemcpyHostToDevice, s));
        }
        for (size_t q = 0; q < keys.size(); ++q) {
          const FusedPlan& pl = plan_of(pass, keys[q]);
          A.nmax = pl.nmax;
          A.ecap = pl.ecap;
          A.mg_list = single ? nullptr : D<int32_t>(c, D_MGLIST) + ml_off + starts[q];
#ifdef RGC_STAMPS
          A.stamps = D<unsigned long long>(c, D_STAMPS) + (size_t)(ml_off + starts[q]) * rgc::STAMP_SLOTS;
#endif
          TRY(ensure_qg(c, A, k, pl.nt));
          TRY(mark(c, "k_fused"));
          const int le = launch_fused(s, single ? n_mg : (int)lists[q].size(), pl.lds, A, wide,
                                      pl.nt);
          if (le != 0)
            return fail(std::string("fused kernel launch failed (k=") + std::to_string(k) +
                        (wide ? ", f64" : ", f32") + " layout, nmax " + std::to_string(pl.nmax) +
                        ", lds " + std::to_string(pl.lds) + ", " +
                        std::to_string(pl.nt) + " threads): " +
                        (le > 0 ? hipGetErrorString((hipError_t)le) : "unsupported k"));
        }
        TRY(mark(c, "k_fused_ties"));
        if (launch_fused_ties(s, A, ties_done) != 0) return fail("tie kernel launch failed");
        TRY(mark(c, "d2h_stats"));
        HIPCHK(hipMemcpyAsync(H<void>(c, H_MGOUT), D<void>(c, D_MGOUT), cur_off + 2 * CUR_BYTES,
                              hipMemcpyDeviceToHost, s));
        if (c->timing) {
          if (!c->ev_tail) HIPCHK(hipEventCreate(&c->ev_tail));
          HIPCHK(hipEventRecord(c->ev_tail, s));
        }
        HIPCHK(hipGetLastError());
        HIPCHK(hipStreamSynchronize(s));
        const int32_t* fst = ho.status;
        ties_done = std::min<int64_t>((int64_t)h_cur[rgc::CUR_TIES], A.tie_cap);
        ml_off += (int)by.size();
        todo.clear();
        auto check = [&](int32_t m) {
          const int stt = fst[m];
          if (stt == RGC_ST_OVERFLOW) overflow = true;
          else if (stt == RGC_ST_DEFER_WIDE || stt == RGC_ST_DEFER) todo.push_back(m);
        };
        if (single) {
          for (int32_t m = 0; m < n_mg; ++m)
            if (fst[m] >= RGC_ST_DEFER) check(m);
        } else {
          for (const int32_t m : by) check(m);
        }
        for (int32_t m : left) todo.push_back(m);
      }
      fused_total = (int64_t)h_cur[0];
      // this attempt's launches zeroed the other cursor slot: the next run (or regrow) uses it
      c->cur_slot = 1 - c->cur_slot;
#ifdef RGC_STAMPS
      const size_t n0w = all0 ? (size_t)n_mg : todo0.size();   // pass 0's workgroups
      c->stamps.resize(n0w * rgc::STAMP_SLOTS);
      HIPCHK(hipMemcpy(c->stamps.data(), D<void>(c, D_STAMPS), n0w * rgc::STAMP_SLOTS * 8,
                       hipMemcpyDeviceToHost));
#endif
      fused_edges = (int64_t)h_cur[2];
      const bool edge_over = want_edges && fused_edges > c->cap_edges;
      if (!overflow && fused_total <= c->cap_cliques && !edge_over) {
        for (int32_t m : todo) deferred.push_back(m);
        break;
      }
      if (attempt == 1) return fail("internal: output overflow after regrow");
      if (edge_over) c->cap_edges = fused_edges + fused_edges / 8 + 1024;
      if (overflow || fused_total > c->cap_cliques)   // grow and re-run once
        c->cap_cliques = fused_total + fused_total / 8 + 1024;
      c->n_ev = 0;
    }
    // edges of the micrographs the fused passes finished (the stats were copied after each
    // pass; micrographs never launched hold a previous run's stats, so only launched ones)
    auto fin_edges = [&](int32_t m) {
      if (ho.status[m] < RGC_ST_DEFER) E_total += ho.n_edges[m];
    };
    if (all0) {
      for (int32_t m = 0; m < n_mg; ++m) fin_edges(m);
    } else {
      for (int32_t m : todo0) fin_edges(m);
    }
  }

  int64_t C_total = fused_total;
  if (!deferred.empty()) {
    std::sort(deferred.begin(), deferred.end());
    const int ns = (int)deferred.size();
    std::vector<int64_t> sbo((size_t)ns * k + 1), sid(ns);
    std::vector<int32_t> sbo32((size_t)ns * k + 1);
    int64_t acc = 0;
    for (int i = 0; i < ns; ++i) {
      const int m = deferred[i];
      for (int p = 0; p < k; ++p) {
        sbo[(size_t)i * k + p] = acc;
        acc += in->box_off[(int64_t)m * k + p + 1] - in->box_off[(int64_t)m * k + p];
      }
      sid[i] = in->id_base[m];
    }
    sbo[(size_t)ns * k] = acc;
    for (size_t i = 0; i < sbo.size(); ++i) sbo32[i] = (int32_t)sbo[i];
    // every micrograph deferred (a batch of large micrographs): the sub-batch IS the batch,
    // no gather and no index remap
    const bool ident = ns == n_mg;
    const double *sx = x, *sy = y, *ss = sc;
    const int32_t* orig = nullptr;
    if (!ident) {
      TRY(ensure_dev(c, D_SUBMG, ns * 4));
      TRY(ensure_dev(c, D_SUBX, acc * 8));
      TRY(ensure_dev(c, D_SUBY, acc * 8));
      TRY(ensure_dev(c, D_SUBS, acc * 8));
      TRY(ensure_dev(c, D_ORIG, acc * 4));
      TRY(ensure_dev(c, D_BOXOFF, sbo32.size() * 4));
      HIPCHK(hipMemcpy(D<void>(c, D_SUBMG), deferred.data(), ns * 4, hipMemcpyHostToDevice));
      HIPCHK(hipMemcpy(D<void>(c, D_BOXOFF), sbo32.data(), sbo32.size() * 4,
                       hipMemcpyHostToDevice));
      TRY(mark(c, "k_gather"));
      launch_gather(s, ns, k, D<int32_t>(c, D_SUBMG), d_bo, D<int32_t>(c, D_BOXOFF),
                    x, y, sc, D<double>(c, D_SUBX), D<double>(c, D_SUBY), D<double>(c, D_SUBS),
                    D<int32_t>(c, D_ORIG));
      HIPCHK(hipStreamSynchronize(s));
      sx = D<double>(c, D_SUBX);
      sy = D<double>(c, D_SUBY);
      ss = D<double>(c, D_SUBS);
      orig = D<int32_t>(c, D_ORIG);
    }
    std::vector<MgStat> sst;
    int64_t Cm = 0, Em = 0;
    TRY(run_multi(c, ns, k, B, two_b2, get_cc, multi, want_members, want_edges, sbo.data(),
                  sid.data(), sx, sy, ss, fused_total, sst, &Cm, &Em));
    if (!ident) {
      TRY(mark(c, "k_remap"));
      launch_remap(s, Cm, k, orig, D<int32_t>(c, D_CONS) + fused_total,
                   want_members ? D<int32_t>(c, D_MEMBERS) + fused_total * k : nullptr);
    }
    if (want_edges) {
      TRY(ensure_edges(c, fused_edges + Em, fused_edges));
      launch_dump_edges(s, (int)acc, D<int64_t>(c, D_FWDOFF), D<int32_t>(c, D_EDST),
                        D<double>(c, D_EJI), orig, D<int32_t>(c, D_EU) + fused_edges,
                        D<int32_t>(c, D_EV) + fused_edges, D<double>(c, D_EJIOUT) + fused_edges);
      fused_edges += Em;
    }
    for (int i = 0; i < ns; ++i) {
      const int m = deferred[i];
      const MgStat& t = sst[i];
      int stt = t.status;
      if (stt == RGC_OK && t.clique_cnt == 0) stt = RGC_NO_CLIQUES;
      ho.status[m] = stt;
      ho.cc_max[m] = t.cc_max;
      ho.cc_cnt[m] = t.cc_cnt;
      ho.n_nodes[m] = t.n_nodes;
      ho.n_vert[m] = t.n_vert;
      ho.n_edges[m] = t.n_edges;
      ho.clique_base[m] = t.clique_base;
      ho.clique_cnt[m] = stt == RGC_OK ? t.clique_cnt : 0;
    }
    C_total += Cm;
    E_total += Em;
  }
  out->n_cliques = C_total;
  out->n_edges = E_total;

  if (want_edges) {
    const int64_t ne = fused_edges;
    TRY(ensure_host(c, H_EU, ne * 4));
    TRY(ensure_host(c, H_EV, ne * 4));
    TRY(ensure_host(c, H_EJIOUT, ne * 8));
    if (ne) {
      HIPCHK(hipMemcpyAsync(H<void>(c, H_EU), D<void>(c, D_EU), ne * 4, hipMemcpyDeviceToHost, s));
      HIPCHK(hipMemcpyAsync(H<void>(c, H_EV), D<void>(c, D_EV), ne * 4, hipMemcpyDeviceToHost, s));
      HIPCHK(hipMemcpyAsync(H<void>(c, H_EJIOUT), D<void>(c, D_EJIOUT), ne * 8,
                            hipMemcpyDeviceToHost, s));
    }
    HIPCHK(hipStreamSynchronize(s));
    c->n_edge_dump = ne;
  }
  if (flags & RGC_F_HOST_OUTPUTS) {
    TRY(mark(c, "d2h"));
    const int64_t C = C_total;
    TRY(ensure_host(c, H_ROWS, C * k * 4));
    TRY(ensure_host(c, H_W, C * 4));
    TRY(ensure_host(c, H_CONF, C * 4));
    TRY(ensure_host(c, H_CONS, C * 4));
    if (want_members) TRY(ensure_host(c, H_MEMBERS, C * k * 4));
    if (multi) TRY(ensure_host(c, H_ORDER, C * k));
    if (C) {
      HIPCHK(hipMemcpyAsync(H<void>(c, H_ROWS), D<void>(c, D_ROWS), C * k * 4, hipMemcpyDeviceToHost, s));
      HIPCHK(hipMemcpyAsync(H<void>(c, H_W), D<void>(c, D_W), C * 4, hipMemcpyDeviceToHost, s));
      HIPCHK(hipMemcpyAsync(H<void>(c, H_CONF), D<void>(c, D_CONF), C * 4, hipMemcpyDeviceToHost, s));
      HIPCHK(hipMemcpyAsync(H<void>(c, H_CONS), D<void>(c, D_CONS), C * 4, hipMemcpyDeviceToHost, s));
      if (want_members)
        HIPCHK(hipMemcpyAsync(H<void>(c, H_MEMBERS), D<void>(c, D_MEMBERS), C * k * 4,
                              hipMemcpyDeviceToHost, s));
      if (multi)
        HIPCHK(hipMemcpyAsync(H<void>(c, H_ORDER), D<void>(c, D_ORDER), C * k, hipMemcpyDeviceToHost, s));
    }
    out->rows = H<int32_t>(c, H_ROWS);
    out->w = H<float>(c, H_W);
    out->conf = H<float>(c, H_CONF);
    out->consensus = H<int32_t>(c, H_CONS);
    out->members = want_members ? H<int32_t>(c, H_MEMBERS) : nullptr;
    out->order = multi ? H<uint8_t>(c, H_ORDER) : nullptr;
  } else {
    out->rows = D<int32_t>(c, D_ROWS);
    out->w = D<float>(c, D_W);
    out->conf = D<float>(c, D_CONF);
    out->consensus = D<int32_t>(c, D_CONS);
    out->members = want_members ? D<int32_t>(c, D_MEMBERS) : nullptr;
    out->order = multi ? D<uint8_t>(c, D_ORDER) : nullptr;
  }
  // nothing enqueued since the fused passes' last sync -> no second round trip; their tail
  // event closes the timeline
  const bool fused_ran = all0 || !todo0.empty();
  const bool tail_work = !fused_ran || !deferred.empty() || (flags & RGC_F_HOST_OUTPUTS);
  HIPCHK(hipGetLastError());
  if (tail_work) {
    TRY(mark(c, "end"));
    HIPCHK(hipStreamSynchronize(s));
  }


  if (c->timing) {
    c->times.clear();
    c->time_names.clear();
    for (int i = 0; i + 1 < c->n_ev || (!tail_work && i < c->n_ev); ++i) {
      float ms = 0.f;
      hipEvent_t e1 = i + 1 < c->n_ev ? c->events[i + 1] : c->ev_tail;
      HIPCHK(hipEventElapsedTime(&ms, c->events[i], e1));
      c->times.push_back(ms);
      c->time_names.push_back(c->ev_names[i]);
    }
  }
  return 0;
}

// rgc_submit's fast path: a batch whose micrographs all take the single fused launch (pass 0,
// one workgroup size and occupancy) with HBM-resident inputs and offsets and device outputs is
// enqueued (kernel + stats copy + event) without waiting.  Returns 1 when enqueued, 0 when the
// batch needs the general path (run synchronously by the caller), < 0 on error.
static int submit_fast(rgc_ctx* c, const rgc_batch_in* in) {
  const int n_mg = in->n_mg, k = in->k;
  const uint32_t flags = in->flags;
  const uint32_t need = RGC_F_DEVICE_INPUTS | RGC_F_DEVICE_META;
  const uint32_t deny = RGC_F_HOST_OUTPUTS | RGC_F_EDGES | RGC_F_NO_FUSED;
  if ((flags & need) != need || (flags & deny) || n_mg <= 0 || k < 2 || k > MAX_K) return 0;
  if (in->box_size > (1LL << 26) || !in->dev_box_off || !in->dev_id_base) return 0;
  const int64_t N = in->box_off[(int64_t)n_mg * k];
  if (N >= (1LL << 31) - 1) return 0;
  int64_t nmin = INT64_MAX, nmaxb = 0;
  for (int m = 0; m < n_mg; ++m) {
    const int64_t nm = in->box_off[(int64_t)(m + 1) * k] - in->box_off[(int64_t)m * k];
    nmin = std::min(nmin, nm);
    nmaxb = std::max(nmaxb, nm);
  }
  if (nmaxb > FUSED_MAX_BOXES) return 0;
  // launch groups: micrographs whose size classes share a plan's occupancy and workgroup
  // size run as one launch at the group's largest class; several groups (C3 / C4 classes
  // straddle an occupancy step) launch back to back over HBM micrograph lists, still without
  // a host sync (deferrals show up in rgc_wait, which falls back to the general path)
  struct Grp {
    int wg, nt, cl;
    std::vector<int32_t> mg;
  };
  std::vector<Grp> grp;
  {
    const FusedPlan& pl = cached_plan(k, 0, fused_class(nmaxb));
    const FusedPlan& p0 = cached_plan(k, 0, fused_class(nmin));
    if (!pl.nmax || !p0.nmax) return 0;
    if (p0.wg == pl.wg && p0.nt == pl.nt) {
      grp.push_back({pl.wg, pl.nt, fused_class(nmaxb), {}});
    } else {
      std::vector<std::pair<int, const FusedPlan*>> cp;   // few classes: linear cache
      for (int m = 0; m < n_mg; ++m) {
        const int cl = fused_class(in->box_off[(int64_t)(m + 1) * k] - in->box_off[(int64_t)m * k]);
        const FusedPlan* p = nullptr;
        for (const auto& e : cp)
          if (e.first == cl) p = e.second;
        if (!p) {
          p = &cached_plan(k, 0, cl);
          cp.push_back({cl, p});
        }
        if (!p->nmax) return 0;
        Grp* g = nullptr;
        for (auto& e : grp)
          if (e.wg == p->wg && e.nt == p->nt) g = &e;
        if (!g) {
          grp.push_back({p->wg, p->nt, cl, {}});
          g = &grp.back();
        }
        g->cl = std::max(g->cl, cl);
        g->mg.push_back(m);
      }
      for (const auto& g : grp)   // the group's largest class must keep its occupancy
        if (cached_plan(k, 0, g.cl).wg != g.wg || cached_plan(k, 0, g.cl).nt != g.nt) return 0;
    }
  }
  const bool multi = (flags & RGC_F_MULTI_OUT) != 0;
  const bool want_members = (flags & (RGC_F_MEMBERS | RGC_F_MULTI_OUT)) != 0;
  hipStream_t s = c->stream;
  c->timing = (flags & RGC_F_TIMING) != 0;
  c->n_ev = 0;
  c->n_edge_dump = 0;
  const size_t cur_off = (mgout_bytes(n_mg) + 15) & ~(size_t)15;
  if (c->cap_cliques < 4096) c->cap_cliques = std::max<int64_t>(4096, N);
  TRY(ensure_outputs(c, c->cap_cliques, 0, k, want_members, multi));
  FusedIo io;
  TRY(fused_io(c, n_mg, cur_off, &io));
  FusedArgs A{};
  A.k = k;
  A.flags = ((flags & RGC_F_GET_CC) ? 1 : 0) | (multi ? 2 : 0) | (want_members ? 32 : 0);
  A.B = (double)in->box_size;
  A.two_b2 = (double)(2 * in->box_size * in->box_size);
  A.box_off = in->dev_box_off; A.id_base = in->dev_id_base;
  A.x = in->x; A.y = in->y; A.score = in->score;
  A.o = io.o;
  A.cursor = io.cur; A.cap = c->cap_cliques;
  A.cursor_clear = io.clear;
  A.rows = D<int32_t>(c, D_ROWS); A.w = D<float>(c, D_W); A.conf = D<float>(c, D_CONF);
  A.consensus = D<int32_t>(c, D_CONS);
  A.members = want_members ? D<int32_t>(c, D_MEMBERS) : nullptr;
  A.order = multi ? D<uint8_t>(c, D_ORDER) : nullptr;
  A.stamps = nullptr;
  A.eu = nullptr; A.ev = nullptr; A.eji = nullptr; A.ecap_out = 0;
  A.mg_list = nullptr;
  A.tie_list = D<int32_t>(c, D_TIES);
  A.tie_cap = c->cap_cliques;
  A.esum_n = n_mg;   // k_fused_ties sums the edges of the finished micrographs (cursor[1])
  A.mg_count = nullptr;
  // the last run on this context deferred micrographs to the f64 layout: this one appends its
  // DEFER_WIDE micrographs to a device list and runs their f64 pass right after, on the
  // stream (no host round trip, no rerun of the batch through the general path)
  const FusedPlan* pw = c->wide_hint ? &cached_plan(k, 1, fused_class(nmaxb)) : nullptr;
  if (pw && !pw->nmax) pw = nullptr;
  A.wide_list = nullptr;
  if (pw) {
    TRY(ensure_dev(c, D_WIDELIST, (size_t)n_mg * 4));
    A.wide_list = D<int32_t>(c, D_WIDELIST);
  }
#ifdef RGC_STAMPS
  return 0;   // the diagnostic build times through rgc_run only
#endif
  int32_t* d_ml = nullptr;
  if (grp.size() > 1) {   // micrograph lists, group after group, through the pinned stage
    TRY(ensure_host(c, H_FSTAGE, (size_t)n_mg * 4));
    TRY(ensure_dev(c, D_MGLIST, (size_t)n_mg * 4));
    int32_t* h_ml = H<int32_t>(c, H_FSTAGE);
    size_t o = 0;
    for (const auto& g : grp) {
      std::memcpy(h_ml + o, g.mg.data(), g.mg.size() * 4);
      o += g.mg.size();
    }
    d_ml = D<int32_t>(c, D_MGLIST);
    HIPCHK(hipMemcpyAsync(d_ml, h_ml, (size_t)n_mg * 4, hipMemcpyHostToDevice, s));
  }
  size_t o = 0;
  for (const auto& g : grp) {
    const FusedPlan& pl = cached_plan(k, 0, g.cl);
    const int nb = grp.size() > 1 ? (int)g.mg.size() : n_mg;
    A.nmax = pl.nmax;
    A.ecap = pl.ecap;
    A.mg_list = grp.size() > 1 ? d_ml + o : nullptr;
    o += g.mg.size();
    TRY(ensure_qg(c, A, k, pl.nt));
    TRY(mark(c, "k_fused"));
    const int le = launch_fused(s, nb, pl.lds, A, false, pl.nt);
    if (le != 0) return fail("fused kernel launch failed (submit): " +
                             std::string(le > 0 ? hipGetErrorString((hipError_t)le) : "unsupported k"));
  }
  if (pw) {
    FusedArgs Aw = A;
    Aw.mg_list = A.wide_list;
    Aw.mg_count = io.cur + 5;
    Aw.wide_list = nullptr;
    Aw.nmax = pw->nmax;
    Aw.ecap = pw->ecap;
    TRY(ensure_qg(c, Aw, k, pw->nt));
    TRY(mark(c, "k_fused"));
    const int le = launch_fused(s, n_mg, pw->lds, Aw, true, pw->nt);
    if (le != 0) return fail("fused f64 kernel launch failed (submit): " +
                             std::string(le > 0 ? hipGetErrorString((hipError_t)le) : "unsupported k"));
  }
  // every micrograph's stats to the host from the ties kernel (the run's last kernel) when
  // the caller wants them with every run
  const bool stats_in_ties = !(flags & RGC_F_LAZY_STATS) && A.tie_list && A.tie_cap > 0;
  if (stats_in_ties) {
    A.stats_dev = D<char>(c, D_MGOUT);
    A.host_stats = H<char>(c, H_MGOUT);
    A.stats_bytes = (int64_t)cur_off;
  }
  TRY(mark(c, "k_fused_ties"));
  if (launch_fused_ties(s, A, 0) != 0) return fail("tie kernel launch failed (submit)");
  c->pend_slot = io.slot;
  c->cur_slot = 1 - c->cur_slot;   // the launch zeroes the other slot: the next run's
  if (c->timing) {
    if (!c->ev_tail) HIPCHK(hipEventCreate(&c->ev_tail));
    HIPCHK(hipEventRecord(c->ev_tail, s));
  }
  // The stats copy.  A lazy run's (its 128-B totals) on the launch stream: the next run on
  // THIS context is submitted after rgc_wait, and other contexts launch on streams of their
  // own (bench.py: one stream per context), whose hardware queues a side copy stream per
  // context would share (3-4 % with two or three contexts in flight,
  // profiles/r05w_ab_copy_on_stream.txt).  Every micrograph's stats (48 B each): written to
  // the pinned host block by the ties kernel itself (stats_in_ties).  As a copy they were a
  // blit kernel: on the launch stream it waited for CUs behind the other contexts'
  // workgroups (C2: 0.39 -> 0.56 ms per step), on a side stream after an event its wait
  // packet sat in a hardware queue that, depending on how a process's streams mapped onto
  // the 4 queues, a launch stream could share (14.3-14.8 M against 25 M micrographs/s on
  // half the processes measured, profiles/r06az_*).
  if (!c->ev_sub) HIPCHK(hipEventCreateWithFlags(&c->ev_sub, hipEventDisableTiming));
  if (stats_in_ties || (flags & RGC_F_LAZY_STATS)) {
    // the run's totals (a lazy run's other stats: rgc_fetch_stats; a non-lazy run's: the
    // ties kernel wrote them)
    const size_t so = cur_off + (size_t)io.slot * CUR_BYTES;
    HIPCHK(hipMemcpyAsync(H<char>(c, H_MGOUT) + so, D<char>(c, D_MGOUT) + so, CUR_BYTES,
                          hipMemcpyDeviceToHost, s));
    HIPCHK(hipEventRecord(c->ev_sub, s));
  } else {
    if (!c->copy_set) {
      TRY(shared_copy_stream(c->device, &c->copy_stream));
      c->copy_set = true;
    }
    if (!c->ev_k) HIPCHK(hipEventCreateWithFlags(&c->ev_k, hipEventDisableTiming));
    HIPCHK(hipEventRecord(c->ev_k, s));
    HIPCHK(hipStreamWaitEvent(c->copy_stream, c->ev_k, 0));
    HIPCHK(hipMemcpyAsync(H<void>(c, H_MGOUT), D<void>(c, D_MGOUT), cur_off + 2 * CUR_BYTES,
                          hipMemcpyDeviceToHost, c->copy_stream));
    HIPCHK(hipEventRecord(c->ev_sub, c->copy_stream));
  }
  HIPCHK(hipGetLastError());
  return 1;
}

// completes a submit_fast run: 1 = outputs in *out; 0 = some micrograph needs another pass or
// the outputs overflowed (the caller re-runs the batch with rgc_run's general path)
static int wait_fast(rgc_ctx* c, rgc_batch_out* out) {
  const rgc_batch_in* in = &c->pin;
  const int n_mg = in->n_mg, k = in->k;
  HIPCHK(hipEventSynchronize(c->ev_sub));
  const size_t cur_off = (mgout_bytes(n_mg) + 15) & ~(size_t)15;
  const MgOut ho = mgout_bind(H<void>(c, H_MGOUT), n_mg);
  const unsigned long long* h_cur = reinterpret_cast<const unsigned long long*>(
      H<char>(c, H_MGOUT) + cur_off + c->pend_slot * CUR_BYTES);
  bool again = (int64_t)h_cur[0] > c->cap_cliques || h_cur[4] != 0;
  // the next submit on this context runs the f64 pass on the device when this batch had
  // micrographs for it
  c->wide_hint = h_cur[5] != 0;
  const bool lazy = (in->flags & RGC_F_LAZY_STATS) != 0;
  for (int m = 0; m < n_mg && !again && !lazy; ++m) again = ho.status[m] >= RGC_ST_DEFER;
  if (again) return 0;
  c->lazy_n_mg = lazy ? n_mg : -1;   // rgc_fetch_stats copies them on demand
  const bool multi = (in->flags & RGC_F_MULTI_OUT) != 0;
  const bool want_members = (in->flags & (RGC_F_MEMBERS | RGC_F_MULTI_OUT)) != 0;
  std::memset(out, 0, sizeof(*out));
  out->status = ho.status;
  out->cc_max = ho.cc_max;
  out->cc_cnt = ho.cc_cnt;
  out->n_nodes = ho.n_nodes;
  out->n_vert = ho.n_vert;
  out->n_edges_mg = ho.n_edges;
  out->clique_base = ho.clique_base;
  out->clique_cnt = ho.clique_cnt;
  out->n_boxes = in->box_off[(int64_t)n_mg * k];
  out->n_cliques = (int64_t)h_cur[0];
  out->n_edges = (int64_t)h_cur[1];
  out->rows = D<int32_t>(c, D_ROWS);
  out->w = D<float>(c, D_W);
  out->conf = D<float>(c, D_CONF);
  out->consensus = D<int32_t>(c, D_CONS);
  out->members = want_members ? D<int32_t>(c, D_MEMBERS) : nullptr;
  out->order = multi ? D<uint8_t>(c, D_ORDER) : nullptr;
  if (c->timing) {
    c->times.clear();
    c->time_names.clear();
    for (int i = 0; i < c->n_ev; ++i) {
      float ms = 0.f;
      HIPCHK(hipEventElapsedTime(&ms, c->events[i], i + 1 < c->n_ev ? c->events[i + 1] : c->ev_tail));
      c->times.push_back(ms);
      c->time_names.push_back(c->ev_names[i]);
    }
  }
  return 1;
}

extern "C" {

int rgc_abi_version(void) { return RGC_ABI_VERSION; }

const char* rgc_last_error(void) { return g_err.c_str(); }

int rgc_device_count(int* n) {
  HIPCHK(hipGetDeviceCount(n));
  return 0;
}

int rgc_ctx_set_copy_stream(rgc_ctx* c, void* hip_stream) {
  if (!c) return fail("null context");
  if (c->pend) return fail("rgc_ctx_set_copy_stream: a submitted run awaits rgc_wait");
  if (c->copy_set) HIPCHK(hipStreamSynchronize(c->copy_stream));
  c->copy_stream = reinterpret_cast<hipStream_t>(hip_stream);
  c->copy_set = true;
  return 0;
}

int rgc_ctx_create(int device, void* hip_stream, rgc_ctx** out) {
  *out = nullptr;
  HIPCHK(hipSetDevice(device));
  rgc_ctx* c = new rgc_ctx();
  c->device = device;
  if (hip_stream) {
    c->stream = reinterpret_cast<hipStream_t>(hip_stream);
  } else {
    hipError_t e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
    if (e != hipSuccess) {
      delete c;
      return fail(std::string("hipStreamCreate: ") + hipGetErrorString(e));
    }
    c->own_stream = true;
  }
  *out = c;
  return 0;
}

void rgc_ctx_destroy(rgc_ctx* c) {
  if (!c) return;
  if (c->worker.joinable()) c->worker.join();
  (void)hipSetDevice(c->device);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  for (auto& b : c->d)
    if (b.p) (void)hipFree(b.p);
  for (auto& b : c->h)
    if (b.p) (void)hipHostFree(b.p);
  for (auto e : c->events) (void)hipEventDestroy(e);
  if (c->ev_tail) (void)hipEventDestroy(c->ev_tail);
  if (c->ev_sub) (void)hipEventDestroy(c->ev_sub);
  if (c->ev_k) (void)hipEventDestroy(c->ev_k);
  if (c->copy_set) (void)hipStreamSynchronize(c->copy_stream);   // (not owned: never destroyed)
  if (c->own_stream) (void)hipStreamDestroy(c->stream);
  delete c;
}

int rgc_run(rgc_ctx* c, const rgc_batch_in* in, rgc_batch_out* out) {
  if (!c || !in || !out) return fail("null argument");
  if (c->pend) return fail("rgc_run: a submitted run awaits rgc_wait on this context");
  HIPCHK(hipSetDevice(c->device));
  c->lazy_n_mg = -1;
  return run_impl(c, in, out);
}

int rgc_submit(rgc_ctx* c, const rgc_batch_in* in) {
  if (!c || !in) return fail("null argument");
  if (c->pend) return fail("rgc_submit: a submitted run awaits rgc_wait on this context");
  HIPCHK(hipSetDevice(c->device));
  c->lazy_n_mg = -1;
  c->pin = *in;
  const int r = submit_fast(c, in);
  if (r < 0) return r;
  c->pend = true;
  c->pend_fast = r == 1;
  if (!c->pend_fast) {
    // the general path syncs on the host once per clique level: on a worker thread, so the
    // caller's next submit (another context, another stream) overlaps this run's device work
    // and its host round trips; rgc_wait joins it.  (No thread: the run happens here.)
    try {
      c->worker = std::thread([c] {
        if (hipSetDevice(c->device) != hipSuccess) {
          c->pend_rc = fail("hipSetDevice failed on the submit worker");
        } else {
          c->pend_rc = run_impl(c, &c->pin, &c->pend_out);
        }
        if (c->pend_rc != 0) c->pend_err = g_err;
      });
    } catch (...) {
      c->pend_rc = run_impl(c, &c->pin, &c->pend_out);
      if (c->pend_rc != 0) c->pend_err = g_err;
    }
  }
  return 0;
}

int rgc_wait(rgc_ctx* c, rgc_batch_out* out) {
  if (!c || !out) return fail("null argument");
  if (!c->pend) return fail("rgc_wait: nothing submitted on this context");
  HIPCHK(hipSetDevice(c->device));
  c->pend = false;
  if (!c->pend_fast) {
    if (c->worker.joinable()) c->worker.join();
    *out = c->pend_out;
    if (c->pend_rc != 0) g_err = c->pend_err;
    return c->pend_rc;
  }
  const int r = wait_fast(c, out);
  if (r < 0) return r;
  if (r == 0) return run_impl(c, &c->pin, out);   // deferrals / overflow: the general path
  return 0;
}

int rgc_fetch_stats(rgc_ctx* c) {
  if (!c) return fail("null ctx");
  if (c->lazy_n_mg < 0) return 0;
  HIPCHK(hipSetDevice(c->device));
  HIPCHK(hipMemcpy(H<void>(c, H_MGOUT), D<void>(c, D_MGOUT), mgout_bytes(c->lazy_n_mg),
                   hipMemcpyDeviceToHost));
  c->lazy_n_mg = -1;
  return 0;
}

// ABI 7: the host buffers the last run's outputs point into, handed to the caller
struct rgc_host_block {
  std::vector<void*> bufs;
};

int rgc_detach_host(rgc_ctx* c, void** block) {
  if (!c || !block) return fail("null argument");
  *block = nullptr;
  if (c->pend) return fail("rgc_detach_host: a submitted run awaits rgc_wait on this context");
  HIPCHK(hipSetDevice(c->device));
  TRY(rgc_fetch_stats(c));   // a lazy run's per-micrograph block lands in the detached buffer
  HIPCHK(hipStreamSynchronize(c->stream));
  if (c->copy_set) HIPCHK(hipStreamSynchronize(c->copy_stream));
  rgc_host_block* b = new rgc_host_block();
  for (auto& h : c->h) {
    if (h.p) b->bufs.push_back(h.p);
    h.p = nullptr;   // the next run allocates fresh pinned buffers
    h.cap = 0;
  }
  c->n_edge_dump = 0;
  *block = b;
  return 0;
}

void rgc_host_block_free(void* block) {
  rgc_host_block* b = static_cast<rgc_host_block*>(block);
  if (!b) return;
  for (void* p : b->bufs) (void)hipHostFree(p);
  delete b;
}

int rgc_kernel_times(rgc_ctx* c, int max_n, float* ms, const char** names) {
  if (!c) return fail("null ctx");
  const int n = std::min<int>(max_n, (int)c->times.size());
  for (int i = 0; i < n; ++i) {
    if (ms) ms[i] = c->times[i];
    if (names) names[i] = c->time_names[i];
  }
  return (int)c->times.size();
}

int64_t rgc_last_edges(rgc_ctx* c, const int32_t** u, const int32_t** v, const double** ji) {
  if (!c) return fail("null ctx");
  if (u) *u = H<int32_t>(c, H_EU);
  if (v) *v = H<int32_t>(c, H_EV);
  if (ji) *ji = H<double>(c, H_EJIOUT);
  return c->n_edge_dump;
}

int rgc_score_pairs(rgc_ctx* c, const rgc_score_in* in, int64_t* counts) {
  if (!c || !in || !counts) return fail("null argument");
  if (c->pend) return fail("rgc_score_pairs: a submitted run awaits rgc_wait on this context");
  HIPCHK(hipSetDevice(c->device));
  const int64_t np = in->n_pairs;
  if (np < 0 || np > INT32_MAX) return fail("n_pairs out of range");
  c->times.clear();
  c->time_names.clear();
  if (np == 0) return 0;
  const int64_t nb = std::max(in->pk_off[np], in->gt_off[np]);   // boxes in the array
  if (in->gt_off[0] < 0 || in->pk_off[0] < 0) return fail("negative box offset");
  // tiles: R rows x TW words, R * TW = the kernel's LDS words per mask
  const int words_cap = rgc::score_tile_words();
  std::vector<int> tp, tr, tw;
  int R = 0, TW = 0;
  int64_t maxw = 1;
  for (int64_t p = 0; p < np; ++p) maxw = std::max<int64_t>(maxw, (in->width[p] + 63) / 64);
  TW = (int)std::min<int64_t>(maxw, 32);
  R = words_cap / TW;
  for (int64_t p = 0; p < np; ++p) {
    const int64_t H = in->height[p], W = in->width[p];
    if (H < 0 || W < 0 || H > (1 << 30) || W > (1 << 30)) return fail("mask size out of range");
    if (in->gt_off[p + 1] < in->gt_off[p] || in->pk_off[p + 1] < in->pk_off[p] ||
        in->pk_off[p + 1] > nb)
      return fail("box offsets must be non-decreasing and within the box array");
    for (int which = 0; which < 2; ++which) {
      const int64_t* off = which ? in->pk_off : in->gt_off;
      for (int64_t b = off[p]; b < off[p + 1]; ++b) {
        const int32_t* q = in->boxes + 4 * b;
        if (!(0 <= q[0] && q[0] < q[1] && q[1] <= H && 0 <= q[2] && q[2] < q[3] && q[3] <= W))
          return fail("box " + std::to_string(b) + " is not a normalised non-empty slice");
      }
    }
    const int64_t nw = (W + 63) / 64;
    for (int64_t r0 = 0; r0 < H; r0 += R)
      for (int64_t w0 = 0; w0 < nw; w0 += TW) {
        tp.push_back((int)p);
        tr.push_back((int)r0);
        tw.push_back((int)w0);
      }
  }
  const int64_t nt = (int64_t)tp.size();
  if (nt > INT32_MAX) return fail("too many tiles");
  TRY(ensure_dev(c, D_SC_BOX, (size_t)nb * 16));
  TRY(ensure_dev(c, D_SC_GOFF, (size_t)(np + 1) * 8));
  TRY(ensure_dev(c, D_SC_POFF, (size_t)(np + 1) * 8));
  TRY(ensure_dev(c, D_SC_TP, (size_t)nt * 4));
  TRY(ensure_dev(c, D_SC_TR, (size_t)nt * 4));
  TRY(ensure_dev(c, D_SC_TW, (size_t)nt * 4));
  TRY(ensure_dev(c, D_SC_CNT, (size_t)np * 24));
  hipStream_t s = c->stream;
  if (nb) HIPCHK(hipMemcpyAsync(c->d[D_SC_BOX].p, in->boxes, (size_t)nb * 16, hipMemcpyHostToDevice, s));
  HIPCHK(hipMemcpyAsync(c->d[D_SC_GOFF].p, in->gt_off, (size_t)(np + 1) * 8, hipMemcpyHostToDevice, s));
  HIPCHK(hipMemcpyAsync(c->d[D_SC_POFF].p, in->pk_off, (size_t)(np + 1) * 8, hipMemcpyHostToDevice, s));
  if (nt) {
    HIPCHK(hipMemcpyAsync(c->d[D_SC_TP].p, tp.data(), (size_t)nt * 4, hipMemcpyHostToDevice, s));
    HIPCHK(hipMemcpyAsync(c->d[D_SC_TR].p, tr.data(), (size_t)nt * 4, hipMemcpyHostToDevice, s));
    HIPCHK(hipMemcpyAsync(c->d[D_SC_TW].p, tw.data(), (size_t)nt * 4, hipMemcpyHostToDevice, s));
  }
  HIPCHK(hipMemsetAsync(c->d[D_SC_CNT].p, 0, (size_t)np * 24, s));
  rgc::ScoreArgs A;
  A.boxes = D<int4>(c, D_SC_BOX);
  A.gt_off = D<int64_t>(c, D_SC_GOFF);
  A.pk_off = D<int64_t>(c, D_SC_POFF);
  A.tile_pair = D<int>(c, D_SC_TP);
  A.tile_r0 = D<int>(c, D_SC_TR);
  A.tile_w0 = D<int>(c, D_SC_TW);
  A.R = R;
  A.TW = TW;
  A.counts = D<unsigned long long>(c, D_SC_CNT);
  const bool timing = (in->flags & RGC_F_TIMING) != 0;
  hipEvent_t e0 = nullptr, e1 = nullptr;
  if (timing) {
    HIPCHK(hipEventCreate(&e0));
    HIPCHK(hipEventCreate(&e1));
    HIPCHK(hipEventRecord(e0, s));
  }
  rgc::launch_score_raster(s, (int)nt, A);
  HIPCHK(hipGetLastError());
  if (timing) HIPCHK(hipEventRecord(e1, s));
  HIPCHK(hipMemcpyAsync(counts, c->d[D_SC_CNT].p, (size_t)np * 24, hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  if (timing) {
    float ms = 0.f;
    HIPCHK(hipEventElapsedTime(&ms, e0, e1));
    c->times.push_back(ms);
    c->time_names.push_back("k_score_raster");
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
  }
  return 0;
}

// One pass of the device solver over a CSC batch (rgc_ilp_solve runs it once, then once more
// on the reduced-cost-fixed columns of the components it left unproven): x, statuses and the
// per-component gaps (gap_out, at one column of each component) on the host.  With fix set,
// the kept columns of the certified components come back too (rgc_ilp.hip k_fs_*).
struct IlpFix {
  std::vector<uint8_t> keep;    // [n_cols] kept by reduced-cost fixing
  std::vector<int32_t> comp;    // [n_cols] component of each column
  std::vector<uint32_t> cnt;    // [n_comp] kept columns per component
  std::vector<uint8_t> cert;    // [n_comp] 0: proven by the search, else certified
};

static int ilp_core(rgc_ctx* c, const rgc_ilp_in* in, uint8_t* x, uint8_t* exact,
                    double* gap_out, IlpFix* fix) {
  const int64_t nc = in->n_cols, nr = in->n_rows;
  if (nc == 0) return 0;
  const int64_t nnz = in->col_ptr[nc];
  if (in->col_ptr[0] != 0 || nnz < 0) return fail("col_ptr must start at 0");
  int kmax = 1;
  for (int64_t j = 0; j < nc; ++j) {
    const int64_t d = in->col_ptr[j + 1] - in->col_ptr[j];
    if (d < 1) return fail("every column needs at least one row");
    kmax = (int)std::max<int64_t>(kmax, d);
  }
  if (kmax > 8) return fail("columns of more than 8 rows (cliques of more than 8 boxes)");
  for (int64_t e = 0; e < nnz; ++e)
    if (in->row_idx[e] < 0 || in->row_idx[e] >= nr) return fail("row index out of range");
  hipStream_t s = c->stream;
  TRY(ensure_dev(c, D_IL_CPTR, (nc + 1) * 8));
  TRY(ensure_dev(c, D_IL_ROW, nnz * 4));
  TRY(ensure_dev(c, D_IL_W, nc * 8));
  TRY(ensure_dev(c, D_IL_REP, nr * 4));
  TRY(ensure_dev(c, D_IL_PAR, nc * 4));
  TRY(ensure_dev(c, D_IL_ROOT, nc * 4));
  TRY(ensure_dev(c, D_IL_CSIZE, nc * 4));
  TRY(ensure_dev(c, D_IL_RCNT, nr * 4));
  TRY(ensure_dev(c, D_IL_RCUR, nr * 4));
  TRY(ensure_dev(c, D_IL_RPTR, (nr + 1) * 8));
  TRY(ensure_dev(c, D_IL_RCOLS, nnz * 4));
  TRY(ensure_dev(c, D_IL_CID, (nc + 1) * 8));
  TRY(ensure_dev(c, D_IL_MEM, nc * 4));
  TRY(ensure_dev(c, D_IL_LOC, nc * 4));
  TRY(ensure_dev(c, D_IL_SCR, (size_t)nc * (2 * kmax + 8) * 8));
  TRY(ensure_dev(c, D_IL_RLOC, nr * 4));
  TRY(ensure_dev(c, D_IL_NBIG, 16));
  TRY(ensure_dev(c, D_IL_X, nc));
  TRY(ensure_dev(c, D_IL_EX, nc));
  TRY(ensure_dev(c, D_TILES, scan_tiles_needed(std::max(nc, nr) + 1) * 8));
  TRY(tiles_refresh(c));
  TRY(ensure_dev(c, D_TOTAL, 32));
  TRY(ensure_host(c, H_TOTAL, 64));
  HIPCHK(hipMemcpyAsync(c->d[D_IL_CPTR].p, in->col_ptr, (nc + 1) * 8, hipMemcpyHostToDevice, s));
  HIPCHK(hipMemcpyAsync(c->d[D_IL_ROW].p, in->row_idx, nnz * 4, hipMemcpyHostToDevice, s));
  HIPCHK(hipMemcpyAsync(c->d[D_IL_W].p, in->w, nc * 8, hipMemcpyHostToDevice, s));
  HIPCHK(hipMemsetAsync(c->d[D_IL_NBIG].p, 0, 16, s));
  rgc::IlpArgs A{};
  A.n_cols = nc;
  A.n_rows = nr;
  A.kmax = kmax;
  A.node_limit = in->node_limit > 0 ? in->node_limit : (int64_t)RGC_ILP_DEFAULT_NODES;
  A.col_ptr = D<int64_t>(c, D_IL_CPTR);
  A.row_idx = D<int32_t>(c, D_IL_ROW);
  A.w = D<double>(c, D_IL_W);
  A.rep = D<int32_t>(c, D_IL_REP);
  A.rloc = D<int32_t>(c, D_IL_RLOC);
  A.parent = D<int32_t>(c, D_IL_PAR);
  A.is_root = D<int32_t>(c, D_IL_ROOT);
  A.csize = D<int32_t>(c, D_IL_CSIZE);
  A.rcnt = D<int32_t>(c, D_IL_RCNT);
  A.rcur = D<int32_t>(c, D_IL_RCUR);
  A.rptr = D<int64_t>(c, D_IL_RPTR);
  A.rcols = D<int32_t>(c, D_IL_RCOLS);
  A.comp_id = D<int64_t>(c, D_IL_CID);
  A.members = D<int32_t>(c, D_IL_MEM);
  A.loc = D<int32_t>(c, D_IL_LOC);
  A.scratch = D<uint64_t>(c, D_IL_SCR);
  A.n_big = D<unsigned int>(c, D_IL_NBIG);
  A.x = D<uint8_t>(c, D_IL_X);
  A.exact = D<uint8_t>(c, D_IL_EX);
  TRY(mark(c, "k_ilp_components"));
  rgc::launch_ilp(s, 0, A, 0, 0);
  launch_scan(s, nc, A.is_root, D<int64_t>(c, D_IL_CID), D<int64_t>(c, D_TILES),
              D<int64_t>(c, D_TOTAL));
  HIPCHK(hipMemcpyAsync(H<int64_t>(c, H_TOTAL), D<int64_t>(c, D_TOTAL), 8, hipMemcpyDeviceToHost, s));
  launch_scan(s, nr, A.rcnt, D<int64_t>(c, D_IL_RPTR), D<int64_t>(c, D_TILES),
              D<int64_t>(c, D_TOTAL) + 1);
  HIPCHK(hipStreamSynchronize(s));
  const int64_t ncomp = H<int64_t>(c, H_TOTAL)[0];
  if (ncomp < 0) return fail("component scan: look-back guard exhausted (stale tile buffer)");
  TRY(ensure_dev(c, D_IL_CN, (ncomp + 1) * 4));
  TRY(ensure_dev(c, D_IL_COFF, (ncomp + 1) * 8));
  TRY(ensure_dev(c, D_IL_CCUR, (ncomp + 1) * 4));
  TRY(ensure_dev(c, D_IL_BIG, (ncomp + 1) * 4));
  A.n_comp = ncomp;
  A.comp_n = D<int32_t>(c, D_IL_CN);
  A.comp_off = D<int64_t>(c, D_IL_COFF);
  A.comp_cur = D<int32_t>(c, D_IL_CCUR);
  A.big = D<int32_t>(c, D_IL_BIG);
  rgc::launch_ilp(s, 1, A, 0, 0);
  launch_scan(s, ncomp, A.comp_n, D<int64_t>(c, D_IL_COFF), D<int64_t>(c, D_TILES),
              D<int64_t>(c, D_TOTAL) + 2);
  HIPCHK(hipMemsetAsync(A.comp_cur, 0, (ncomp + 1) * 4, s));
  rgc::launch_ilp(s, 2, A, 0, 0);
  TRY(mark(c, "k_ilp_small"));
  rgc::launch_ilp(s, 3, A, 0, 0);
  HIPCHK(hipMemcpyAsync(H<int64_t>(c, H_TOTAL) + 1, A.n_big, 4, hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  const int n_big = (int)*reinterpret_cast<uint32_t*>(H<int64_t>(c, H_TOTAL) + 1);
  // certification arrays (rgc_ilp.hip): also the wave search's pre-search multipliers
  TRY(ensure_dev(c, D_IL_CERT, ncomp + 1));
  TRY(ensure_dev(c, D_IL_KEY, nc * 8));
  TRY(ensure_dev(c, D_IL_ST, nc));
  TRY(ensure_dev(c, D_IL_RMAX, nr * 8 + 8));
  TRY(ensure_dev(c, D_IL_OWN, nr * 4 + 4));
  TRY(ensure_dev(c, D_IL_LAM, nr * 8 + 8));
  TRY(ensure_dev(c, D_IL_GRAD, nr * 8 + 8));
  TRY(ensure_dev(c, D_IL_CS, (ncomp + 1) * 10 * 8));
  TRY(ensure_dev(c, D_IL_STSAVE, nc));
  TRY(ensure_dev(c, D_IL_CNT, 16));
  A.cert = D<uint8_t>(c, D_IL_CERT);
  A.key = D<uint64_t>(c, D_IL_KEY);
  A.st = D<uint8_t>(c, D_IL_ST);
  A.rmax = D<uint64_t>(c, D_IL_RMAX);
  A.owner = D<int32_t>(c, D_IL_OWN);
  A.lam = D<double>(c, D_IL_LAM);
  A.grad = D<double>(c, D_IL_GRAD);
  A.cs = D<double>(c, D_IL_CS);
  A.count = D<unsigned int>(c, D_IL_CNT);
  A.st_save = D<uint8_t>(c, D_IL_STSAVE);
  // per-component gaps: zero for proven components
  TRY(ensure_dev(c, D_IL_GAP, nc * 8));
  A.gap = D<double>(c, D_IL_GAP);
  HIPCHK(hipMemsetAsync(A.gap, 0, nc * 8, s));
  // rounds until a pass changes nothing (each round settles at least the heaviest undecided
  // clique / makes at least one improving swap, so both terminate); counters read every 4
  auto rounds = [&](int phase, int cap) -> int {
    for (int it = 0; it < cap; it += 4) {
      HIPCHK(hipMemsetAsync(A.count, 0, 4, s));
      for (int j = 0; j < 4; ++j) rgc::launch_ilp_cert(s, phase, A);
      HIPCHK(hipMemcpyAsync(H<int64_t>(c, H_TOTAL) + 3, A.count, 4, hipMemcpyDeviceToHost, s));
      HIPCHK(hipStreamSynchronize(s));
      if (*reinterpret_cast<uint32_t*>(H<int64_t>(c, H_TOTAL) + 3) == 0) break;
    }
    return 0;
  };
  // Lagrangian repack of the flagged components (rgc_ilp.hip k_rp_*): greedy by reduced cost
  // with the best multipliers, swaps, kept per component when better
  auto repack = [&]() -> int {
    rgc::launch_ilp_cert(s, 8, A);
    TRY(rounds(1, 1 << 20));
    TRY(rounds(2, 1 << 16));
    rgc::launch_ilp_cert(s, 9, A);
    return 0;
  };
  if (n_big > 0) {
    std::vector<int32_t> big(n_big), cn(ncomp);
    HIPCHK(hipMemcpyAsync(big.data(), A.big, n_big * 4, hipMemcpyDeviceToHost, s));
    HIPCHK(hipMemcpyAsync(cn.data(), A.comp_n, ncomp * 4, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    int nmax = 0;
    for (int b : big) nmax = std::max(nmax, std::min(cn[b], rgc::ilp_big_max()));
    const int64_t W = (nmax + 63) / 64;
    // adjacency n W, stack n (W + 2), weights n, tmpid K n / 2, row info (K + 1) n / 4; then
    // the Lagrangian bound's row multipliers K n and member weights n
    A.wlag_off = (int64_t)nmax * W + (int64_t)nmax * (W + 2) + nmax +
                 ((int64_t)kmax * nmax + 1) / 2 + ((int64_t)(kmax + 1) * nmax + 3) / 4 + 8;
    A.wstride = A.wlag_off + (int64_t)(kmax + 1) * nmax;
    const int n_waves = std::min(n_big, 2048);
    TRY(ensure_dev(c, D_IL_WSCR, (size_t)n_waves * A.wstride * 8));
    A.wscratch = D<uint64_t>(c, D_IL_WSCR);
    // multipliers for the search's Lagrangian bound: the certification's greedy primal,
    // swaps and projected subgradient (rgc_ilp.hip) on the wave components (cert 3)
    TRY(mark(c, "k_ilp_lagrange"));
    HIPCHK(hipMemsetAsync(A.count, 0, 16, s));
    rgc::launch_ilp_cert(s, 6, A);
    TRY(rounds(1, 1 << 20));
    TRY(rounds(2, 1 << 16));
    rgc::launch_ilp_cert(s, 3, A);
    for (int it = 0; it < 400; ++it) rgc::launch_ilp_cert(s, 4, A);
    rgc::launch_ilp_cert(s, 7, A);
    // the packing repacked by reduced cost when better: it seeds the search's incumbent
    TRY(repack());
    TRY(mark(c, "k_ilp_wave"));
    rgc::launch_ilp(s, 4, A, n_big, n_waves);
  }
  TRY(mark(c, "k_ilp_cert"));
  HIPCHK(hipMemsetAsync(A.count, 0, 16, s));
  rgc::launch_ilp_cert(s, 0, A);
  // no component left unproven by the branch and bound (the common case): nothing to certify
  HIPCHK(hipMemcpyAsync(H<int64_t>(c, H_TOTAL) + 3, A.count, 8, hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  const bool any_flagged = reinterpret_cast<uint32_t*>(H<int64_t>(c, H_TOTAL) + 3)[1] != 0;
  if (any_flagged) {
    TRY(rounds(1, 1 << 20));
    TRY(rounds(2, 1 << 16));
    rgc::launch_ilp_cert(s, 3, A);
    // projected subgradient iterations of the Lagrangian bound (per component Polyak steps
    // towards the primal; after 40 iterations without progress the step shrinks and lam
    // restarts from the best one), a repack by reduced cost from the multipliers, then more
    // iterations with the better primal's steps
    for (int it = 0; it < 1000; ++it) rgc::launch_ilp_cert(s, 4, A);
    TRY(repack());
    for (int it = 0; it < 4000; ++it) rgc::launch_ilp_cert(s, 4, A);
    TRY(repack());
    for (int it = 0; it < 2000; ++it) rgc::launch_ilp_cert(s, 4, A);
    rgc::launch_ilp_cert(s, 5, A);
    if (fix) {   // reduced-cost fixing of the certified components (the second pass's input)
      TRY(ensure_dev(c, D_IL_FS, (ncomp + 1) * 16));
      TRY(ensure_dev(c, D_IL_FSCNT, (ncomp + 1) * 4));
      TRY(ensure_dev(c, D_IL_FSKEEP, nc));
      A.fs = D<double>(c, D_IL_FS);
      A.fs_cnt = D<unsigned int>(c, D_IL_FSCNT);
      A.fs_keep = D<uint8_t>(c, D_IL_FSKEEP);
      rgc::launch_ilp_cert(s, 10, A);
      fix->keep.resize(nc);
      fix->comp.resize(nc);
      fix->cnt.resize(ncomp);
      fix->cert.resize(ncomp);
      HIPCHK(hipMemcpyAsync(fix->keep.data(), A.fs_keep, nc, hipMemcpyDeviceToHost, s));
      HIPCHK(hipMemcpyAsync(fix->comp.data(), A.loc, nc * 4, hipMemcpyDeviceToHost, s));
      HIPCHK(hipMemcpyAsync(fix->cnt.data(), A.fs_cnt, ncomp * 4, hipMemcpyDeviceToHost, s));
      HIPCHK(hipMemcpyAsync(fix->cert.data(), A.cert, ncomp, hipMemcpyDeviceToHost, s));
    }
  }
  TRY(mark(c, "d2h_x"));
  HIPCHK(hipGetLastError());
  HIPCHK(hipMemcpyAsync(x, A.x, nc, hipMemcpyDeviceToHost, s));
  HIPCHK(hipMemcpyAsync(exact, A.exact, nc, hipMemcpyDeviceToHost, s));
  HIPCHK(hipMemcpyAsync(gap_out, A.gap, nc * 8, hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  return 0;
}

// The device solver, then (depth < ILP_FIX_DEPTH) reduced-cost fixing of the components it
// left unproven, solved by the same function one level down.
constexpr int ILP_FIX_DEPTH = 4;

static int ilp_solve_rec(rgc_ctx* c, const rgc_ilp_in* in, uint8_t* x, uint8_t* exact,
                         double* gap, int depth) {
  const int64_t nc = in->n_cols, nr = in->n_rows;
  if (nc == 0) return 0;
  IlpFix fix;
  TRY(ilp_core(c, in, x, exact, gap, depth + 1 < ILP_FIX_DEPTH ? &fix : nullptr));
  // Next pass: the certified components whose reduced-cost-fixed column set is small enough
  // for the exact search (and smaller than the component), solved as one batch.  A packing of
  // component j that uses a fixed column is worth less than its packing P_j, so its optimum is
  // max(P_j, optimum over the kept columns): proven when the second pass proves its part.
  if (!fix.cnt.empty()) {
    const int64_t ncomp = (int64_t)fix.cnt.size();
    std::vector<int32_t> size(ncomp, 0);
    std::vector<double> pval(ncomp, 0.0), gap1(ncomp, 0.0);
    for (int64_t j = 0; j < nc; ++j) {
      const int32_t q = fix.comp[j];
      ++size[q];
      if (x[j]) pval[q] += in->w[j];
      gap1[q] += gap[j];
    }
    std::vector<uint8_t> elig(ncomp, 0);
    int64_t sub_nc = 0, sub_nnz = 0;
    for (int64_t q = 0; q < ncomp; ++q)
      elig[q] = fix.cert[q] != 0 && gap1[q] > 0.0 && fix.cnt[q] > 0 &&
                (int)fix.cnt[q] <= rgc::ilp_big_max() && (int32_t)fix.cnt[q] < size[q];
    std::vector<int64_t> sub_ptr(1, 0);
    std::vector<int32_t> sub_row;
    std::vector<double> sub_w;
    std::vector<int64_t> sub_col;   // original column of each sub column
    for (int64_t j = 0; j < nc; ++j) {
      if (!elig[fix.comp[j]] || !fix.keep[j]) continue;
      for (int64_t e = in->col_ptr[j]; e < in->col_ptr[j + 1]; ++e) sub_row.push_back(in->row_idx[e]);
      sub_nnz += in->col_ptr[j + 1] - in->col_ptr[j];
      sub_ptr.push_back(sub_nnz);
      sub_w.push_back(in->w[j]);
      sub_col.push_back(j);
      ++sub_nc;
    }
    if (sub_nc > 0) {
      TRY(mark(c, "k_ilp_fixsearch"));
      rgc_ilp_in sub{};
      sub.n_cols = sub_nc;
      sub.n_rows = nr;
      sub.col_ptr = sub_ptr.data();
      sub.row_idx = sub_row.data();
      sub.w = sub_w.data();
      // (4x the nodes one level down, up to 16x the first pass's: its components are the few
      // hard ones, restricted)
      const int64_t nl = in->node_limit > 0 ? in->node_limit : (int64_t)RGC_ILP_DEFAULT_NODES;
      sub.node_limit = depth < 2 ? 4 * nl : nl;
      std::vector<uint8_t> sx(sub_nc), sex(sub_nc);
      std::vector<double> sgap(sub_nc);
      // (with RGC_F_TIMING the second pass's sections follow "k_ilp_fixsearch" in the list)
      TRY(ilp_solve_rec(c, &sub, sx.data(), sex.data(), sgap.data(), depth + 1));
      std::vector<double> rval(ncomp, 0.0), rgap(ncomp, 0.0);
      std::vector<uint8_t> ropt(ncomp, 1);
      for (int64_t i = 0; i < sub_nc; ++i) {
        const int32_t q = fix.comp[sub_col[i]];
        if (sx[i]) rval[q] += sub_w[i];
        rgap[q] += sgap[i];
        if (sex[i] != RGC_ILP_OPTIMAL) ropt[q] = 0;
      }
      // per eligible component: bound min(L, max(P, R + sub gap)); the better packing
      std::vector<uint8_t> take(ncomp, 0), st(ncomp, 0);
      std::vector<double> g(ncomp, 0.0);
      for (int64_t q = 0; q < ncomp; ++q) {
        if (!elig[q]) continue;
        const double P = pval[q], L = P + gap1[q], R = rval[q];
        const double ub = std::min(L, std::max(P, R + (ropt[q] ? 0.0 : rgap[q])));
        take[q] = R > P;
        const double v = take[q] ? R : P;
        g[q] = std::max(0.0, ub - v);
        st[q] = g[q] <= 0.0 ? RGC_ILP_OPTIMAL : g[q] <= 1e-4 * std::fabs(v) ? RGC_ILP_GAP_OK : 0;
      }
      if (std::getenv("RGC_ILP_DEBUG")) {
        int64_t nel = 0, nopt = 0, nok = 0, ntake = 0, nflag = 0, nbig = 0, cmax = 0;
        for (int64_t q = 0; q < ncomp; ++q) {
          nflag += fix.cert[q] != 0;
          if (fix.cert[q] && gap1[q] > 0.0) {
            nbig += (int)fix.cnt[q] > rgc::ilp_big_max();
            cmax = std::max<int64_t>(cmax, fix.cnt[q]);
          }
          if (!elig[q]) continue;
          ++nel;
          nopt += st[q] == RGC_ILP_OPTIMAL;
          nok += st[q] == RGC_ILP_GAP_OK;
          ntake += take[q];
        }
        std::fprintf(stderr, "rgc_ilp fixsearch %d: %lld flagged, %lld eligible, %lld columns; "
                     "%lld optimal, %lld gap-ok, %lld improved; %lld kept > search limit "
                     "(largest kept set %lld)\n", depth, (long long)nflag, (long long)nel,
                     (long long)sub_nc, (long long)nopt, (long long)nok, (long long)ntake,
                     (long long)nbig, (long long)cmax);
      }
      std::vector<uint8_t> seen(ncomp, 0);
      for (int64_t j = 0; j < nc; ++j) {
        const int32_t q = fix.comp[j];
        if (!elig[q]) continue;
        if (take[q]) x[j] = 0;
        if (st[q]) exact[j] = st[q];
        gap[j] = 0.0;
        if (!seen[q]) {   // the component's gap at its first column
          seen[q] = 1;
          gap[j] = g[q];   // (<= the first pass's: the bound is min(L, ...))
        }
      }
      for (int64_t i = 0; i < sub_nc; ++i)
        if (take[fix.comp[sub_col[i]]] && sx[i]) x[sub_col[i]] = 1;
    }
  }
  return 0;
}

int rgc_ilp_solve(rgc_ctx* c, const rgc_ilp_in* in, uint8_t* x, uint8_t* exact) {
  if (!c || !in || !x || !exact) return fail("null argument");
  if (c->pend) return fail("rgc_ilp_solve: a submitted run awaits rgc_wait on this context");
  HIPCHK(hipSetDevice(c->device));
  const int64_t nc = in->n_cols, nr = in->n_rows;
  if (nc < 0 || nc >= INT32_MAX || nr < 0 || nr >= INT32_MAX) return fail("n_cols / n_rows out of range");
  c->times.clear();
  c->time_names.clear();
  c->n_ev = 0;
  c->timing = (in->flags & RGC_F_TIMING) != 0;
  if (nc == 0) return 0;
  std::vector<double> gap(nc);
  TRY(ilp_solve_rec(c, in, x, exact, gap.data(), 0));
  if (in->gap) std::memcpy(in->gap, gap.data(), nc * 8);
  TRY(mark(c, "end"));
  HIPCHK(hipStreamSynchronize(c->stream));
  if (c->timing) {
    for (int i = 0; i + 1 < c->n_ev; ++i) {
      float ms = 0.f;
      HIPCHK(hipEventElapsedTime(&ms, c->events[i], c->events[i + 1]));
      c->times.push_back(ms);
      c->time_names.push_back(c->ev_names[i]);
    }
  }
  return 0;
}

uint64_t rgc_py_hash_node(double x, double y, int64_t id) { return pyset::hash_node(x, y, id); }

#ifdef RGC_STAMPS
// Diagnostic build only: s_memtime stamps (8 per fused workgroup, launch order) of the
// last rgc_run.
int64_t rgc_diag_stamps(rgc_ctx* c, uint64_t* out, int64_t max_n) {
  const int64_t n = std::min<int64_t>(max_n, (int64_t)c->stamps.size());
  if (out) std::memcpy(out, c->stamps.data(), n * 8);
  return (int64_t)c->stamps.size();
}
#endif

int rgc_py_set_order(const uint64_t* hashes, int n, int8_t* out) {
  if (n < 0 || n > 18) return fail("set_order supports 0..18 keys");
  if (n >= 1 && n <= 8) {   // the register-packed variant the device epilogue uses
    uint32_t p = 0;
    switch (n) {
#define RGC_SO(NN)                                  \
  case NN: {                                        \
    uint64_t h[NN];                                 \
    for (int i = 0; i < NN; ++i) h[i] = hashes[i];  \
    p = pyset::set_order_packed<NN>(h);             \
    break;                                          \
  }
      RGC_SO(1) RGC_SO(2) RGC_SO(3) RGC_SO(4) RGC_SO(5) RGC_SO(6) RGC_SO(7) RGC_SO(8)
#undef RGC_SO
    }
    for (int i = 0; i < n; ++i) out[i] = (int8_t)((p >> (4 * i)) & 15);
    return n;
  }
  return pyset::set_order(hashes, n, out);
}

}  // extern "C"
