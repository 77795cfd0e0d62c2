/* repic_gc.h — C-ABI of librepic_gc.so, the MI355X-native `repic get_cliques` hot path.
 *
 * The reference has no FFI: its boundary is the Python subcommand plugin protocol
 * (`name`, `add_arguments(parser)`, `main(args)`; reference repic/commands/get_cliques.py
 * :13-27,72 registered in repic/main.py:17-29).  The Python host package
 * (repic-copy_amd/repic_amd/commands/get_cliques.py) keeps that protocol and calls the
 * entry points below through ctypes.  Each entry point replaces one stage of the
 * reference's per-micrograph loop (get_cliques.py:108-229):
 *
 *   rgc_parse_files  <- common.py:71-114 get_box_coords (BOX text -> x, y, score)
 *   rgc_write_outputs <- get_cliques.py:204-229 (the four pickles + runtime.tsv of each
 *                       micrograph; ABI 5)
 *   rgc_run          <- get_cliques.py:134-202: Jaccard pairs (:40-69,:134-138), graph
 *                       (:30-37,:142-143), connected components (:145-156), size-k
 *                       cliques (:49-56,:160-161), ILP weight / confidence / consensus
 *                       (:164-190) and constraint-matrix COO (:192-202), for a whole
 *                       batch of micrographs at once.
 *
 * Conventions: plain pointers and sizes, no torch types.  Returns 0 on success and a
 * negative code on error (message in rgc_last_error(), thread-local).  Outputs are owned
 * by the context and stay valid until the next rgc_run on it or rgc_ctx_destroy, unless the
 * caller takes over their host buffers with rgc_detach_host (ABI 7).
 */
#ifndef REPIC_GC_H
#define REPIC_GC_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RGC_ABI_VERSION 9

/* flags for rgc_batch_in.flags */
#define RGC_F_GET_CC         1u  /* --get_cc   (get_cliques.py:151-156) */
#define RGC_F_MULTI_OUT      2u  /* --multi_out (get_cliques.py:175-178,206-213) */
#define RGC_F_DEVICE_INPUTS  4u  /* x/y/score are device pointers (HBM-resident) */
#define RGC_F_HOST_OUTPUTS   8u  /* copy per-clique outputs to pinned host memory */
#define RGC_F_TIMING        16u  /* record per-kernel HIP events (rgc_kernel_times) */
#define RGC_F_MEMBERS       32u  /* also return the k member boxes of every clique */
#define RGC_F_NO_FUSED      64u  /* route every micrograph through the multi-kernel path
                                    (testing / comparison; outputs are identical) */
#define RGC_F_DEVICE_META  128u  /* dev_box_off / dev_id_base hold HBM-resident copies of
                                    box_off (as int32) and id_base: no offset upload per run
                                    (the host arrays are still read for launch planning) */
#define RGC_F_LAZY_STATS   512u  /* rgc_submit (ABI 6): the per-micrograph outputs of a run that
                                  * takes the single fused launch stay in HBM; rgc_wait copies
                                  * only the run's totals and rgc_fetch_stats copies the rest
                                  * (outputs kept in HBM, like RGC_F_HOST_OUTPUTS unset) */
#define RGC_F_EDGES        256u  /* test hook: also record every JI > 0.3 edge with its f64 JI
                                    (rgc_last_edges); outputs are unchanged */

/* per-micrograph status (rgc_batch_out.status) */
#define RGC_OK          0   /* outputs written as in get_cliques.py:215-229 */
#define RGC_NO_EDGES    1   /* reference raises ValueError (np.max([]), :148) */
#define RGC_NO_CLIQUES  2   /* reference raises UnboundLocalError (del clique, :203) */

typedef struct rgc_ctx rgc_ctx;

typedef struct rgc_batch_in {
  int32_t n_mg;            /* micrographs in the batch */
  int32_t k;               /* pickers (= clique size, get_cliques.py:160), 1..8 */
  int64_t box_size;        /* CLI box_size (int pixels, get_cliques.py:22-23) */
  uint32_t flags;
  const int64_t* box_off;  /* HOST [n_mg*k+1]: boxes of (mg m, picker p) are
                              [box_off[m*k+p], box_off[m*k+p+1]) in file order */
  const int64_t* id_base;  /* HOST [n_mg]: global box id of the first box of each
                              micrograph (common.py:23,108-112 counter) */
  const double* x;         /* [N] box x (common.py:87), host or device per flags */
  const double* y;         /* [N] box y */
  const double* score;     /* [N] score, sigmoid already applied on host (common.py:92-94) */
  const int32_t* dev_box_off;  /* DEVICE [n_mg*k+1], int32 copy of box_off (RGC_F_DEVICE_META) */
  const int64_t* dev_id_base;  /* DEVICE [n_mg], copy of id_base (RGC_F_DEVICE_META) */
} rgc_batch_in;

typedef struct rgc_batch_out {
  int64_t n_boxes, n_edges, n_cliques;
  /* per micrograph [n_mg], host memory */
  int32_t* status;
  int32_t* cc_max;         /* runtime.tsv column 2 (get_cliques.py:228) */
  int32_t* cc_cnt;         /* runtime.tsv column 3 */
  int32_t* n_nodes;        /* graph nodes (boxes with >= 1 edge) */
  int32_t* n_vert;         /* constraint-matrix rows V (get_cliques.py:164) */
  int64_t* n_edges_mg;     /* JI > 0.3 edges */
  int64_t* clique_base;    /* cliques of mg m are [clique_base[m], +clique_cnt[m]) in the */
  int64_t* clique_cnt;     /* per-clique arrays (ranges of different micrographs do not
                              overlap; their order is unspecified) */
  /* per clique; host (RGC_F_HOST_OUTPUTS) or device pointers */
  int32_t* rows;           /* [C*k] COO row indices of each clique column, ascending */
  float* w;                /* [C] weight vector (get_cliques.py:188-190) */
  float* conf;             /* [C] consensus confidences (:186-187) */
  int32_t* consensus;      /* [C] global box index of the consensus box (:182-183) */
  int32_t* members;        /* [C*k] global box index of each member, picker order
                              (with RGC_F_MEMBERS or RGC_F_MULTI_OUT, else NULL) */
  uint8_t* order;          /* [C*k] networkx node-iteration order as picker indices
                              (only with RGC_F_MULTI_OUT, else NULL) */
} rgc_batch_out;

typedef struct rgc_parsed {
  int64_t n_files;
  int32_t* status;         /* [n_files] RGC_PARSE_* */
  int64_t* off;            /* [n_files+1] boxes of file f are [off[f], off[f+1]) */
  double* x;
  double* y;
  double* score;           /* raw scores (sigmoid NOT applied) */
  uint8_t* sigmoid;        /* [n_files] 1 if min(score) < 0 (common.py:92) */
} rgc_parsed;

/* rgc_parsed.status — the exception get_box_coords would raise for that file */
#define RGC_PARSE_OK          0
#define RGC_PARSE_INDEX       1  /* IndexError: empty file / blank first line / no coords */
#define RGC_PARSE_VALUE       2  /* ValueError: shortest row != 5 tokens, bad weight */
#define RGC_PARSE_ASSERT      3  /* AssertionError: len(X) != len(Y) */
#define RGC_PARSE_FALLBACK    4  /* non-ASCII / unusual bytes: parse in Python instead */
#define RGC_PARSE_OSERROR     5  /* could not open / read */

int rgc_abi_version(void);
const char* rgc_last_error(void);
int rgc_device_count(int* n);

int rgc_ctx_create(int device, void* hip_stream, rgc_ctx** out);
void rgc_ctx_destroy(rgc_ctx* ctx);
/* ABI 9: the stream of a submitted non-lazy run's per-micrograph stats copy (hip_stream may be
 * 0: the device's null stream).  Without a call every context of the process shares one copy
 * stream per device, so N contexts on N launch streams take N + 1 hardware queues, not 2 N
 * (GPU_MAX_HW_QUEUES is 4 on the MI355X boxes). */
int rgc_ctx_set_copy_stream(rgc_ctx* ctx, void* hip_stream);
int rgc_run(rgc_ctx* ctx, const rgc_batch_in* in, rgc_batch_out* out);
/* Asynchronous rgc_run (ABI 3), one run in flight per context: rgc_submit enqueues the batch
 * on the context's stream and returns; rgc_wait blocks until it is done and fills *out exactly
 * as rgc_run would.  Host and device arrays of the batch must stay valid until rgc_wait.  A
 * batch that takes the single fused launch (HBM-resident inputs and offsets, RGC_F_DEVICE_INPUTS
 * | RGC_F_DEVICE_META, device outputs) runs while the caller continues, so with two contexts
 * on one stream the host prepares and launches batch i+1 while the device runs batch i (on
 * two streams the two launches also overlap on the device); any other batch runs through
 * rgc_run's general path on a worker thread of the context (since round 5: it syncs on the
 * host once per clique level, so a second context on its own stream keeps the device busy
 * meanwhile), and one whose micrographs need a second pass re-runs that path inside rgc_wait.
 * Outputs stay valid until the next submit/run on the same context.  While a submitted
 * run awaits rgc_wait, rgc_submit, rgc_run, rgc_score_pairs and rgc_ilp_solve on the same
 * context fail (negative return, rgc_last_error says why). */
int rgc_submit(rgc_ctx* ctx, const rgc_batch_in* in);
int rgc_wait(rgc_ctx* ctx, rgc_batch_out* out);
/* ABI 6: after rgc_wait of an RGC_F_LAZY_STATS run, copy its per-micrograph outputs into the
 * host arrays *out points to (a no-op for any other run).  Valid until the next run on ctx. */
int rgc_fetch_stats(rgc_ctx* ctx);
/* ABI 7: ownership hand-off of the last run's host outputs.  rgc_detach_host moves every
 * pinned host buffer of the context (the per-micrograph arrays, the RGC_F_HOST_OUTPUTS
 * per-clique arrays, a lazy run's stats, fetched first) into *block: the pointers the last
 * rgc_batch_out holds stay valid, and stay unchanged, until rgc_host_block_free(*block), even
 * after further runs or rgc_ctx_destroy; the context allocates new buffers for its next run.
 * Fails while a submitted run awaits rgc_wait.  (repic_amd/_lib.py calls it only when a
 * Result of the last run is still referenced when the next run starts or the context closes.) */
int rgc_detach_host(rgc_ctx* ctx, void** block);
void rgc_host_block_free(void* block);
/* Per-kernel device milliseconds of the last rgc_run with RGC_F_TIMING; returns the count. */
int rgc_kernel_times(rgc_ctx* ctx, int max_n, float* ms, const char** names);

/* Test hook (RGC_F_EDGES): the JI > 0.3 edges of the last rgc_run as host arrays (batch box
 * indices u < v by picker, JI in the reference's f64 op order, get_cliques.py:40-46,59-69),
 * valid until the next rgc_run; returns the edge count (order unspecified). */
int64_t rgc_last_edges(rgc_ctx* ctx, const int32_t** u, const int32_t** v, const double** ji);

/* score_detections (repic/utils/score_detections.py:16-48 get_segmentation_scores): for every
 * (ground truth, picker) pair, the pixel counts of the int16 masks the reference paints.
 * Boxes are given as numpy slice bounds already normalised on the host (row start < row end
 * <= height, col start < col end <= width; boxes with an empty slice are left out), picked
 * boxes already filtered by the confidence threshold.  counts[3p..3p+2] = sum(gt_arr),
 * sum(pckr_arr), sum(gt_arr * pckr_arr).  RGC_F_TIMING records "k_score_raster". */
typedef struct rgc_score_in {
  int64_t n_pairs;
  const int64_t* height;   /* [n_pairs] mask rows (mrc_h) */
  const int64_t* width;    /* [n_pairs] mask columns (mrc_w) */
  const int64_t* gt_off;   /* [n_pairs + 1] pair p's ground truth: boxes[gt_off[p], gt_off[p+1]) */
  const int64_t* pk_off;   /* [n_pairs + 1] pair p's picks: boxes[pk_off[p], pk_off[p+1]) */
  const int32_t* boxes;    /* [n_boxes][4] row start, row end, col start, col end */
  uint32_t flags;          /* RGC_F_TIMING */
} rgc_score_in;
int rgc_score_pairs(rgc_ctx* ctx, const rgc_score_in* in, int64_t* counts);

/* run_ilp (repic/commands/run_ilp.py:50-63): maximise w.x over binary x subject to A x <= 1,
 * exactly, for a batch of micrographs at once (rows are global box ids: micrographs never
 * share a row).  A is given in CSC form.  x[c] = 1 for the chosen columns (cliques);
 * exact[c] is the status of column c's conflict component:
 *   RGC_ILP_OPTIMAL  (1) proven optimal: by the branch and bound, or (ABI 9) for a component
 *                        the search could not finish, by the exact search of the columns its
 *                        Lagrangian reduced costs leave (reduced-cost fixing: every packing
 *                        that uses another column is worth less than the certified one);
 *   RGC_ILP_GAP_OK   (2) not searched to the end (more than 4096 cliques, or node_limit hit),
 *                        but a Lagrangian dual bound certifies x within a relative gap of 1e-4,
 *                        the default MIPGap at which Gurobi reports a model optimal;
 *   RGC_ILP_NODE_LIMIT (0) node_limit hit, x is the best packing found, gap above 1e-4;
 *   RGC_ILP_HEURISTIC (3) too large to search, x is a greedy + swap local-search packing,
 *                        gap above 1e-4.
 * RGC_F_TIMING records the stages in rgc_kernel_times. */
#define RGC_ILP_NODE_LIMIT 0
#define RGC_ILP_OPTIMAL 1
#define RGC_ILP_GAP_OK 2
#define RGC_ILP_HEURISTIC 3
#define RGC_ILP_DEFAULT_NODES (1 << 14)
typedef struct rgc_ilp_in {
  int64_t n_cols;          /* cliques */
  int64_t n_rows;          /* boxes */
  const int64_t* col_ptr;  /* [n_cols + 1] column c's rows: row_idx[col_ptr[c], col_ptr[c+1]) */
  const int32_t* row_idx;  /* [nnz] global row ids */
  const double* w;         /* [n_cols] objective */
  int64_t node_limit;      /* branch-and-bound nodes per component (0: RGC_ILP_DEFAULT_NODES);
                              components of more than 1024 cliques get node_limit * 16 / W,
                              W = 64-clique words (work-scaled); each reduced-cost-fixing pass
                              (up to 2 below the first) searches with 4x the nodes of the one
                              above.  The node budgets are the only limit of the search, so
                              the result is deterministic */
  uint32_t flags;          /* RGC_F_TIMING */
  double* gap;             /* optional (NULL: not returned), ABI 6: [n_cols] dual bound minus
                            * packing value of column c's component, at the component's first
                            * column (0 elsewhere and for proven-optimal components), so a
                            * caller can certify a whole micrograph the way Gurobi's MIPGap
                            * does (sum of gaps <= 1e-4 x its objective) */
  double time_limit_s;     /* ABI 8, ignored since ABI 9: the search ran under a wall-clock budget,
                            * which made x depend on the device's speed and load; it is bounded
                            * by node budgets only now (kept for the struct layout) */
} rgc_ilp_in;
int rgc_ilp_solve(rgc_ctx* ctx, const rgc_ilp_in* in, uint8_t* x, uint8_t* exact);

int rgc_parse_files(const char* const* paths, int64_t n_files, int n_threads, rgc_parsed** out);
void rgc_parsed_free(rgc_parsed* p);

/* Native output writer (ABI 5), reference get_cliques.py:204-229: the pickles are emitted in
 * the opcode layout of CPython's pickler for these objects (protocol 5, no FRAME opcodes);
 * the names below come from the installed numpy / scipy.  repic_amd/writers.py enables it
 * only after rgc_pickle_bytes matched pickle.dumps of the same objects. */
typedef struct rgc_pickle_fmt {
  const char* arr_mod;     /* numpy array reduction: module and function ("_frombuffer") */
  const char* arr_fn;
  const char* dtype_mod;   /* numpy.dtype class */
  const char* dtype_cls;
  const char* coo_mod;     /* scipy.sparse coo_matrix class */
  const char* coo_cls;
  int32_t maxprint;        /* coo_matrix().maxprint */
} rgc_pickle_fmt;

typedef struct rgc_write_in {
  const char* out_dir;
  int32_t n_mg;
  int32_t k;
  const char* const* bases;   /* [n_mg] output base names */
  const int64_t* clique_off;  /* [n_mg+1] ranges into the per-clique arrays */
  const int32_t* n_vert;      /* [n_mg] V (rows of the constraint matrix) */
  const int32_t* cc_max;      /* [n_mg] runtime.tsv columns 2-3 */
  const int32_t* cc_cnt;
  const double* seconds;      /* [n_mg] runtime.tsv column 1 */
  const float* w;             /* [C] */
  const float* conf;          /* [C] */
  const int32_t* rows;        /* [C*k] ascending per clique */
  const double* cx;           /* [C] consensus x, y, global id */
  const double* cy;
  const int64_t* cid;
} rgc_write_in;
/* Writes the 5 files of every micrograph (n_threads threads); on an I/O error returns -errno
 * and the failing micrograph in *failed_mg (the lowest of the failing ones). */
int rgc_write_outputs(const rgc_pickle_fmt* fmt, const rgc_write_in* in, int n_threads,
                      int64_t* failed_mg);
/* Bytes of pickle `which` (0 weight_vector, 1 consensus_coords, 2 consensus_confidences,
 * 3 constraint_matrix) of micrograph mg: *len always, copied when cap >= *len. */
int rgc_pickle_bytes(const rgc_pickle_fmt* fmt, const rgc_write_in* in, int mg, int which,
                     uint8_t* buf, int64_t cap, int64_t* len);
/* CPython str(float) (test hook of the runtime.tsv formatting); returns the length. */
int rgc_py_float_repr(double v, char* buf, int cap);

/* Host test hooks for the CPython set-order emulation (pyset.h). */
uint64_t rgc_py_hash_node(double x, double y, int64_t id);
int rgc_py_set_order(const uint64_t* hashes, int n, int8_t* out);
/* Host test hook: the device ILP epilogue of ONE clique (rgc_device.h epilogue<K>), run on
 * the CPU.  Members in picker order; ji[i*k+j] for i < j; ins only used when !set_order.
 * Outputs: consensus member index, node-iteration order (k entries), w, conf.
 * Reference: get_cliques.py:169-190 (median conf / w, weighted-degree consensus). */
int rgc_test_epilogue(int k, const double* x, const double* y, const double* score,
                      const int64_t* ids, const double* ji, int set_order, const uint64_t* ins,
                      int* arg, int8_t* ord, float* w, float* conf);

#ifdef __cplusplus
}
#endif
#endif
