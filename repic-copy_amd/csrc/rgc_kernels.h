// rgc_kernels.h — device-side data structures and kernel launchers (see rgc_kernels.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <atomic>

namespace rgc {

// Raise a kernel's dynamic-LDS limit to `bytes` on the CURRENT device, once per (kernel,
// device): `done` is the kernel's own bitmask of devices already set (thread-safe; a racing
// second setter only repeats an idempotent call).  Returns the HIP error of the call.
inline hipError_t set_dyn_lds_once(std::atomic<uint64_t>& done, const void* fn, int bytes) {
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  const uint64_t bit = dev < 64 ? (1ULL << dev) : 0;
  if (bit && (done.load(std::memory_order_acquire) & bit)) return hipSuccess;
  e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
  if (e == hipSuccess && bit) done.fetch_or(bit, std::memory_order_acq_rel);
  return e;
}

constexpr int MAX_K = 8;            // largest picker count with a compiled clique kernel
constexpr int SCAN_TILE = 2048;     // elements per scan workgroup

// Per-picker grids of one micrograph (k1_bin): gx x gy cells per picker, columns `cell` =
// 1 / inv_cell wide (>= 1.08 B), rows >= 0.54 B tall, keys picker * ncell + cx * gy + cy;
// nkey = k * ncell (non-finite boxes); flags bit 0: integer layout (exact f32 JI test).
struct MgGrid {
  double minx, miny, cell, inv_cell, inv_celly;
  int gx, gy, ncell, nkey, flags, pad;
};
// cell-start entries of a micrograph of n boxes (k1_bin): its key budget + 2; wide = the u32
// counter variant (some micrograph of the batch has more than 65535 boxes)
__host__ __device__ inline int bin_budget(int64_t n, bool wide) {
  const int64_t cap = wide ? 32760 : 65528;
  return (int)(2 * n + 64 < cap ? 2 * n + 64 : cap);
}

// Per-micrograph results.
struct MgStat {
  int64_t n_edges;
  int64_t clique_base, clique_cnt;   // output range (fused path; host fills it for multi)
  int n_nodes, cc_cnt, cc_max, status, target, n_vert;
};

// cursor block word of the set-order tie count (a separate 64-B line from cursor[0])
constexpr int CUR_TIES = 8;

// internal per-micrograph status codes (0..2 are the public RGC_* codes)
constexpr int RGC_ST_NO_EDGES = 1;
constexpr int RGC_ST_NO_CLIQUES = 2;
constexpr int RGC_ST_DEFER = 3;      // does not fit the fused kernel's LDS capacities
constexpr int RGC_ST_OVERFLOW = 4;   // output capacity exceeded: host grows and re-runs
constexpr int RGC_ST_DEFER_WIDE = 5; // coordinates not exact in f32: rerun with the f64 layout

// LDS layout of the fused kernel for a size class (byte offsets into dynamic LDS)
struct FusedLayout {
  int off_sxy, off_cnt, off_fwd, off_pos, off_vrank, off_dst, off_union, off_cstart, off_parent,
      off_citems, off_scell, off_flags, off_smark, off_cbuf, total;
};

// Per-micrograph outputs of the fused kernel, SoA (the pinned host mirror has the same layout,
// so one copy hands them to the caller).  mgout_bytes / mgout_bind define the layout.
struct MgOut {
  int32_t* status;
  int32_t* cc_max;
  int32_t* cc_cnt;
  int32_t* n_nodes;
  int32_t* n_vert;
  int64_t* n_edges;
  int64_t* clique_base;
  int64_t* clique_cnt;
};
inline size_t mgout_bytes(int n_mg) { return (size_t)n_mg * 20 + 8 + (size_t)n_mg * 24; }
inline MgOut mgout_bind(void* base, int n_mg) {
  char* p = static_cast<char*>(base);
  MgOut o;
  o.status = reinterpret_cast<int32_t*>(p);
  o.cc_max = o.status + n_mg;
  o.cc_cnt = o.cc_max + n_mg;
  o.n_nodes = o.cc_cnt + n_mg;
  o.n_vert = o.n_nodes + n_mg;
  char* q = p + (((size_t)n_mg * 20 + 7) & ~(size_t)7);
  o.n_edges = reinterpret_cast<int64_t*>(q);
  o.clique_base = o.n_edges + n_mg;
  o.clique_cnt = o.clique_base + n_mg;
  return o;
}

// diagnostic build (RGC_STAMPS): per fused workgroup, 16 slots (phase releases by thread 0,
// the workgroup timeline, chunk and clique counts), then each wave's arrival at each of the
// 13 phase barriers (slot 16 + 16 * phase + wave)
constexpr int STAMP_SLOTS = 16 + 13 * 16;
struct FusedArgs {
  int k, flags;                 // flags: bit0 get_cc, bit1 multi_out, bit5 members
  double B, two_b2;
  int nmax, ecap;               // LDS capacities of this launch (boxes, forward edges)
  const int32_t* mg_list;       // micrographs of this launch (nullptr: block b = micrograph b)
  const int32_t* box_off;
  const int64_t* id_base;
  const double* x;
  const double* y;
  const double* score;
  MgOut o;                      // per-micrograph outputs (device)
  // [0] clique-range reservation, [1] edges of finished mgs (summed by k_fused_ties over the
  // first esum_n micrographs' stats; no per-workgroup atomic: 10k workgroups adding to one
  // word cost ~8 % of C2's kernel), [2] edge dump, [4] deferrals, [5] f32-pass micrographs
  // deferred to the f64 layout (DEFER_WIDE), [CUR_TIES] ties
  unsigned long long* cursor;
  // cursors of the context's other run slot: zeroed by block 0 for the next run (no memset
  // packet between runs)
  unsigned long long* cursor_clear;
  int64_t cap;                  // clique capacity of the output arrays
  int32_t* rows;
  float* w;
  float* conf;
  int32_t* consensus;
  int32_t* members;
  uint8_t* order;
  unsigned long long* stamps;   // diagnostic build (RGC_STAMPS) only: STAMP_SLOTS per WG
  // RGC_F_EDGES test hook (nullptr otherwise): every JI > 0.3 edge as (u, v, JI) with batch
  // box indices, reserved per micrograph on cursor[2]; nothing is written past ecap_out
  int32_t* eu;
  int32_t* ev;
  double* eji;
  int64_t ecap_out;
  // level trees of the 1024-thread launches (K = 4) in HBM: qg_nslots slots of qg_bytes,
  // claimed per workgroup through the qg_slots bitmap (nullptr: LDS queue only)
  char* qg_base;
  uint32_t* qg_slots;
  int qg_nslots, qg_bytes;
  // cliques whose consensus / --multi_out order needs CPython set order (degree ties with
  // 2k < |G|): entries of 4 + k int32 (j lo, j hi, micrograph, top | tie << 16 | multi << 17,
  // k batch box indices) for k_fused_ties, counted on cursor[CUR_TIES]; tie_cap entries
  int32_t* tie_list;
  int64_t tie_cap;
  int esum_n;   // k_fused_ties: micrographs whose finished edges it sums into cursor[1]
  // device-side f64 pass (rgc_submit): the f32 pass appends its DEFER_WIDE micrographs to
  // wide_list (count cursor[5]) instead of counting them as deferrals; the f64 launch that
  // follows on the stream takes mg_list = wide_list with mg_count = cursor + 5 (blocks past
  // the count exit at once), so no host round trip sits between the two passes
  int32_t* wide_list;
  const unsigned long long* mg_count;
  // rgc_submit without lazy stats: k_fused_ties, the run's last kernel, writes the
  // per-micrograph block [stats_dev, stats_dev + stats_bytes) to host_stats (pinned), so
  // only the run's 128-B cursor slot is copied, on the launch stream, as for a lazy run
  const char* stats_dev;
  char* host_stats;   // nullptr: none
  int64_t stats_bytes;
};

int fused_lds_bytes(int nmax, int ecap, bool wide);
int fused_vgprs(int k, bool wide, int nt);
bool fused_nt_ok(int k, int nt);
int launch_fused(hipStream_t stream, int n_blocks, int lds_bytes, const FusedArgs& A, bool wide,
                 int nt);
// the tie entries [from, cursor[CUR_TIES]) of the fused launches before it (CPython set order)
int launch_fused_ties(hipStream_t stream, const FusedArgs& A, int64_t from);
void launch_gather(hipStream_t stream, int n_sub, int k, const int32_t* sub_mg,
                   const int32_t* box_off, const int32_t* sub_box_off, const double* x,
                   const double* y, const double* s, double* ox, double* oy, double* os,
                   int32_t* orig);
void launch_remap(hipStream_t stream, int64_t C, int k, const int32_t* orig, int32_t* consensus,
                  int32_t* members);
void launch_dump_edges(hipStream_t stream, int N, const int64_t* fwd_off, const int32_t* e_dst,
                       const double* e_ji, const int32_t* orig, int32_t* eu, int32_t* ev,
                       double* eji);

// Clique stage of the large-micrograph route (rgc_cliques.hip + the DFS fallback in
// rgc_kernels.hip).  Boxes are sub-batch indices; outputs are offset by the caller.
constexpr int RB_W = 64;   // bitmap width: roots with <= RB_W forward neighbours (level kernels)

struct CliqueArgs {
  int k;
  int flags;                 // bit 0: --get_cc, bit 1: --multi_out
  int n_mg, n_roots;         // micrographs; picker-0 boxes (one wavefront each)
  int64_t C;                 // epilogue: cliques of the sub-batch
  double B, two_b2;          // box size, 2 B^2
  const int32_t* box_off;
  const int32_t* p0off;      // [n_mg + 1] exclusive prefix of picker-0 box counts
  const int64_t* id_base;
  const double* x;
  const double* y;
  const double* score;
  const int32_t* bmg;
  const uint8_t* bpick;
  const int64_t* fwd_off;
  const int32_t* e_dst;
  const int32_t* parent;
  const MgStat* st;
  const unsigned long long* ins_key;
  const int64_t* clique_off;
  const int32_t* vrow;
  double* pk;                // [N][4] epilogue gather record: x, y, score, vrow (k5_pack)
  int32_t* ccount;
  uint8_t* in_clique;
  uint64_t* adjg;            // [E] neighbourhood adjacency row of each root's i-th neighbour
  uint64_t* rbound;          // [N] picker run starts in each root's neighbourhood (bytes)
  uint8_t* rflag;            // [N] root enumerated by the level kernels
  uint8_t* dfs_mg;           // [n_mg] micrograph takes the DFS route (a root > RB_W nbrs)
  int32_t* root_box;         // [n_roots] box of each picker-0 root
  uint64_t* exmask;          // [ceil(C / 64)] epilogue: cliques deferred to the exact pass (one
                             // ballot word per epilogue wave) ...
  int64_t* exlist;           // [C] ... and as a list (k5_ex_compact)
  unsigned long long* excount;
  int32_t* exwtot;            // [ceil(C / 4096)] deferred cliques per compaction wave
  int64_t* exwoff;            // [ceil(C / 4096) + 1] their scanned offsets
  int64_t* tiles;             // scan tile buffer (launch_scan)
  int64_t dfs_base;          // first output clique of the DFS route
  int64_t epi_lo;            // first clique k5_epilogue handles (the level route's cliques
                             // [0, dfs_base) may come from k5_leaf_epi instead)
  int32_t* members;
  int32_t* rows;
  float* w;
  float* conf;
  int32_t* consensus;
  uint8_t* order;
};


void launch_bin(hipStream_t stream, int n_mg, int k, double B, const int32_t* box_off,
                const int32_t* cell_off, const double* x, const double* y, MgGrid* grid,
                int32_t* cell_start, double* sx, double* sy, int32_t* sbox, uint8_t* spick,
                int32_t* smg, int32_t* bmg, uint8_t* bpick, bool wide, int max_n);
void launch_pairs(hipStream_t stream, bool fill, int N, int k, double B, double two_b2,
                  const int32_t* box_off, const int32_t* cell_off, const MgGrid* grid,
                  const int32_t* cell_start, const double* sx, const double* sy,
                  const int32_t* sbox, const uint8_t* spick, const int32_t* smg,
                  int32_t* fwd_cnt, const int64_t* fwd_off, int32_t* e_dst, double* e_ji);
// up to 16 memsets in one launch (k_fill_multi): pointers 16-byte aligned
struct FillSegs {
  int n;
  void* p[16];
  size_t bytes[16];
  uint32_t val[16];
  void add(void* ptr, size_t b, uint32_t v) {
    if (n < 16 && b > 0) { p[n] = ptr; bytes[n] = b; val[n] = v & 0xFF; ++n; }
  }
};
void launch_fill_multi(hipStream_t stream, const FillSegs& F);
int64_t scan_tiles_needed(int64_t n);
// one-pass scan launches so far (process-wide); a tile buffer whose states are older than
// SCAN_EPOCH_REFRESH launches must be zeroed before its next scan (launch epochs repeat after
// 2^22 - 1 launches)
constexpr uint32_t SCAN_EPOCH_REFRESH = 1u << 20;
uint64_t scan_epoch_count();
// (bucket: also bucket[b] = the item whose output range holds position b * bq)
void launch_scan(hipStream_t stream, int64_t n, const int32_t* in, int64_t* out,
                 int64_t* tile_buf, int64_t* total, int32_t* bucket = nullptr, int bq = 1);
void launch_cc(hipStream_t stream, int phase, int N, int n_mg, int k, int get_cc,
               const int32_t* box_off, const int32_t* bmg, const uint8_t* bpick,
               const int64_t* fwd_off, const int32_t* e_dst, int32_t* parent, uint8_t* has_edge,
               int32_t* csize, MgStat* st, unsigned long long* ins_key,
               unsigned long long* comp_min, int max_n);   // max_n: largest micrograph
// One level of the prefix expansion (rgc_cliques.hip): level-D prefixes in, children out.
struct LevelArgs {
  int D;                     // members chosen so far (pickers 1..D)
  int64_t n_items;           // prefixes (FIRST level: N boxes)
  const int32_t* in_root;
  const uint64_t* in_M;
  const uint64_t* in_P;
  int32_t* cnt;              // count pass: children (or cliques) per prefix
  const int64_t* off;        // fill pass: scanned offsets
  int32_t* out_root;
  uint64_t* out_M;
  uint64_t* out_P;
  int32_t* next_cnt;         // fill whose children are the leaf prefixes: their leaf counts
                             // (and the clique-vertex marks), so no leaf count pass runs
};

void launch_clique_setup(hipStream_t stream, int N, const CliqueArgs& A);
int launch_clique_level(hipStream_t stream, bool first, bool leaf, bool fill, const CliqueArgs& A,
                        const LevelArgs& L);
int launch_clique_epilogue(hipStream_t stream, bool exact_pass, const CliqueArgs& A);
void launch_clique_pack(hipStream_t stream, int N, const CliqueArgs& A);
// cliques per wave of the fused leaf epilogue; bucket[w] = the leaf prefix holding clique
// LEAF_Q w (the leaf level's scan writes it: launch_scan's bucket output)
constexpr int LEAF_Q = 128;
int launch_clique_leaf_epi(hipStream_t stream, const CliqueArgs& A, const LevelArgs& L,
                           int32_t* bucket, int64_t C1);
void launch_clique_ranges(hipStream_t stream, const CliqueArgs& A, int64_t C1, int64_t* rlo,
                          int64_t* rhi, const int32_t* leaf_root, const int64_t* leaf_off,
                          int64_t n_leaf);
int launch_cliques_dfs(hipStream_t stream, bool fill, int N, const CliqueArgs& A);
void launch_rank(hipStream_t stream, int N, int n_mg, int k, const int32_t* box_off,
                 const int32_t* bmg, const MgGrid* grid, const double* x, const double* y,
                 const uint8_t* in_clique, int32_t* bcnt, int32_t* bslot, int32_t* bbk,
                 int64_t* boff, int64_t* tile_buf, int64_t* total, int32_t* vsort, int32_t* vrow,
                 MgStat* st);
// score_detections raster/reduce (rgc_score.hip): one workgroup per (pair, tile)
struct ScoreArgs {
  const int4* boxes;          // (row start, row end, col start, col end), numpy slice bounds
  const int64_t* gt_off;      // [n_pairs + 1]
  const int64_t* pk_off;      // [n_pairs + 1]
  const int* tile_pair;       // per tile: pair, first row, first 64-pixel word
  const int* tile_r0;
  const int* tile_w0;
  int R, TW;                  // tile = R rows x TW words (R * TW <= score_tile_words())
  unsigned long long* counts; // [n_pairs][3] = sum(gt), sum(pckr), sum(gt * pckr)
};
int score_tile_words();
void launch_score_raster(hipStream_t stream, int n_tiles, const ScoreArgs& A);

// run_ilp exact set packing (rgc_ilp.hip)
struct IlpArgs {
  int64_t n_cols, n_rows, n_comp;
  int kmax;                   // largest number of rows of a column
  int64_t node_limit;         // branch-and-bound nodes per component
  const int64_t* col_ptr;     // [n_cols + 1] CSC
  const int32_t* row_idx;     // global row ids
  const double* w;            // [n_cols]
  int32_t* rep;               // [n_rows] smallest column of each row
  int32_t* rloc;              // [n_rows] solvers: winning member slot of each row
  int32_t* parent;            // [n_cols]
  int32_t* is_root;           // [n_cols]
  int32_t* csize;             // [n_cols] component size by root
  int32_t* rcnt;              // [n_rows] columns per row
  int32_t* rcur;              // [n_rows]
  const int64_t* rptr;        // [n_rows + 1] scanned rcnt
  int32_t* rcols;             // [nnz] columns of each row
  const int64_t* comp_id;     // [n_cols] scanned is_root (valid on roots)
  int32_t* comp_n;            // [n_comp]
  const int64_t* comp_off;    // [n_comp + 1]
  int32_t* comp_cur;          // [n_comp]
  int32_t* members;           // [n_cols] by component
  int32_t* loc;               // [n_cols] local index in its component
  uint64_t* scratch;          // small solver: (2 kmax + 8) words per column
  int32_t* big;               // components for the wave solver
  unsigned int* n_big;
  uint64_t* wscratch;         // wave solver: wstride words per wave
  int64_t wstride;
  int64_t wlag_off;           // wave solver: offset (words) of the Lagrangian-bound arrays
  uint8_t* x;                 // [n_cols] solution
  uint8_t* exact;             // [n_cols] RGC_ILP_* status of the column's component
  // certification stage (components not proven optimal by the branch and bound)
  uint8_t* cert;              // [n_comp] 0 proven, 1 node limit, 2 too large to search
  uint64_t* key;              // [n_cols] greedy / swap priority
  uint8_t* st;                // [n_cols] 0 undecided, 1 chosen, 2 not chosen, 3 not certified
  uint64_t* rmax;             // [n_rows] claims
  int32_t* owner;             // [n_rows] chosen column covering the row, -1
  double* lam;                // [n_rows] Lagrange multipliers
  double* grad;               // [n_rows] subgradient (cover count in between)
  double* cs;                 // [n_comp * CS] per component: lsum g2 lbest mu primal step stall
                              // flag, repacked primal
  unsigned int* count;        // round counter
  double* gap;                // optional [n_cols]: component bound - packing at its first column
  uint8_t* st_save;           // [n_cols] certification: the packing before a Lagrangian repack
  // reduced-cost fixing (rgc_ilp.hip k_fs_*): per component the dual bound and packing value
  // of the certification (fixed point, fs[2 comp], fs[2 comp + 1]) and the number of columns
  // kept (fs_cnt); per column the kept flag
  double* fs;
  unsigned int* fs_cnt;
  uint8_t* fs_keep;
};
int ilp_small_max();
int ilp_big_max();
void launch_ilp(hipStream_t stream, int phase, const IlpArgs& A, int n_big, int n_waves);
// certification stage (rgc_ilp.hip): phase 0 setup, 1 greedy round, 2 swap round, 3 primal
// and multiplier init, 4 subgradient iteration, 5 final statuses; 6 pre-search setup of the
// wave components' multipliers (cert 3), 7 best multipliers -> lam
void launch_ilp_cert(hipStream_t stream, int phase, const IlpArgs& A);

}  // namespace rgc
