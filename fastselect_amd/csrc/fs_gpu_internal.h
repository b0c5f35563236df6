// fs_gpu_internal.h -- what the GPU backend's translation units share: the
// Plan (one scoring job's device state), the device helpers the kernels use,
// the launch / allocation helpers and the entry points each unit offers the
// others.  One unit per stage of the pipeline:
//
//   fs_gpu_mem.hip   devices, the device block cache, pinned host staging
//   fs_pass1.hip     k_quantize, k_dist, row moments, mean correction glue,
//                    calibration / row guard, SURF's averages and scoring
//   fs_select.hip    MultiSURF thresholds, refinement of ambiguous pairs,
//                    exact thresholds of flagged rows, near / far counts
//   fs_pass2.hip     pair weights, dense and sparse pass 2, segment reduce,
//                    reference-order masks / chains glue
//   fs_relieff.hip   ReliefF selection and update
//   fs_plan.hip      plan create / layout / shard / score entry points
//   fs_devices.hip   single-process multi-GPU (the estimators' devices=)
//
// Kernel map and rooflines: DESIGN.md §3.  No float atomics touch scores:
// every reduction has a fixed order, so two runs of the same input are
// bit-identical.
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <thread>
#include <type_traits>
#include <unordered_map>
#include <vector>

#include "../../include/fastselect_amd.h"
#include "fs_internal.h"

namespace fs {
namespace gpu {

#define FS_HIP(expr)                                                                      \
  do {                                                                                    \
    hipError_t e_ = (expr);                                                               \
    if (e_ != hipSuccess) {                                                               \
      set_error(std::string("HIP error '") + hipGetErrorString(e_) + "' in " #expr);      \
      return FS_EHIP;                                                                     \
    }                                                                                     \
  } while (0)

// Launch shapes shared between units
constexpr int kRowcorrMaxSlices = 16;
constexpr int kExRows = 8, kExJ = 4, kExChunk = kExJ;
constexpr int kSWaves = 16;
constexpr int kStreamEntries = (kTile / kSWaves) * kTile;
constexpr int64_t kXsSlack = 512;
constexpr int kXcds = 8;

// ---------------------------------------------------------------------------
// Device helpers
// ---------------------------------------------------------------------------

__device__ __forceinline__ uint32_t sad_u32(uint32_t a, uint32_t b, uint32_t c) {
  uint32_t d;
  asm("v_sad_u32 %0, %1, %2, %3" : "=v"(d) : "v"(a), "v"(b), "v"(c));
  return d;
}

// c + |a.lo - b.lo| + |a.hi - b.hi| over unsigned 16-bit halves (two
// features per word; checked on gfx950 by tools/ubench/sad16_check.hip)
__device__ __forceinline__ uint32_t sad_u16(uint32_t a, uint32_t b, uint32_t c) {
  uint32_t d;
  asm("v_sad_u16 %0, %1, %2, %3" : "=v"(d) : "v"(a), "v"(b), "v"(c));
  return d;
}

// c + sc * [a != b] for small category codes, without lane masks (a
// compare would burn an SGPR pair per pair-accumulator).
__device__ __forceinline__ uint32_t mismatch_u32(uint32_t a, uint32_t b, uint32_t sc, uint32_t c) {
  uint32_t t, d;
  asm("v_xor_b32 %1, %2, %3\n\tv_min_u32 %1, %1, 1\n\tv_mad_u32_u24 %0, %1, %4, %5"
      : "=v"(d), "=&v"(t)
      : "v"(a), "v"(b), "v"(sc), "v"(c));
  return d;
}

// Fixed-shape block reduction of doubles (256 threads), deterministic.
__device__ __forceinline__ double block_sum_256(double v, double* red) {
  const int tid = threadIdx.x;
  red[tid] = v;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (tid < s) red[tid] += red[tid + s];
    __syncthreads();
  }
  const double r = red[0];
  __syncthreads();
  return r;
}

// Distance storage.  Full layout (ReliefF / SURF, whose neighbour selection
// reads whole rows): D[i][j] over n_pad x n_pad, both halves.  Tiled layout
// (MultiSURF, whose kernels only ever read inside an owned tile): one
// 128 x 128 block per owned tile t, T_t[b][a] = D(i0 + a, j0 + b) -- half the
// memory of the full matrix for the whole triangle, and a rank of an N-GPU
// job holds only its 1/N of the tiles.  d_at(..., a, b) addresses element
// (i0 + a, j0 + b) of owned tile t either way; consecutive a are consecutive
// doubles in both layouts (the full layout reads it as D[j][i]).
__device__ __forceinline__ int64_t d_at(int tiled, int64_t n_pad, int64_t t, int64_t i0,
                                        int64_t j0, int a, int b) {
  return tiled ? ((t * kTile + b) * kTile + a) : ((j0 + b) * n_pad + i0 + a);
}

// Row window of the full layout (ReliefF / SURF row plans): only the rows
// [win.x, win.y) -- the plan's focal 128-sample blocks -- are stored, and the
// plan's D points where row 0 would be, so row r of the full matrix is still
// D + r * n_pad.  A whole fit stores every row; a row-sharded plan (one rank
// of N, a row panel) 1/N of them.  Writes skip rows outside the window; a
// read of (i0 + a, j0 + b) takes row j0 + b when it is stored and row i0 + a
// otherwise (D is symmetric, and every tile of a row plan has one of its two
// blocks inside the window).
__device__ __forceinline__ bool d_row_in(int2 win, int64_t r) { return r >= win.x && r < win.y; }
__device__ __forceinline__ int64_t d_rd(int tiled, int2 win, int64_t n_pad, int64_t t, int64_t i0,
                                        int64_t j0, int a, int b) {
  if (tiled) return (t * kTile + b) * kTile + a;
  const int64_t j = j0 + b;
  return d_row_in(win, j) ? j * n_pad + i0 + a : (i0 + a) * n_pad + j;
}

// ---------------------------------------------------------------------------
// Host side
// ---------------------------------------------------------------------------
struct Plan {
  Prepared P;
  int device = 0, rank = 0, world = 1;
  int x_is_f64 = 0;
  hipStream_t stream = nullptr;
  bool own_stream = false;
  // MultiSURF's mean correction (k_colrank, k_rowcorr) runs on `side`,
  // forked after k_quantize and joined before k_rowstats_reduce, beside k_dist
  hipStream_t side = nullptr;
  hipEvent_t ev_fork = nullptr, ev_join = nullptr;
  // MultiSURF*: the star split's per-sample sums on a stream of their own
  // (beside k_dist and the correction), joined by run_weights
  hipStream_t side2 = nullptr;
  hipEvent_t ev_star = nullptr;
  int64_t nb = 0, n_tiles = 0, seg_len = 1, nseg = 1;
  int64_t nsegpart = 1;         // rows of spart (nseg, or 2 * nseg for the v2 sparse pass)
  int ksplit = 1;               // pass-1 K-split parts of the tail tiles (k_dist)
  int64_t kfull = 0;            // tiles k_dist computes whole (the rest are split)
  int use_q16 = 0;              // pass 1 on packed 16-bit continuous operands
  double calib[7] = {0, 0, 0, 0, 1, 0, 0};  // plan_calibration (calibrate_band, row_guard)
  double cal32[2] = {0, 0};     // sampled rms / max error of 32-bit operands (row_guard)
  int64_t c_lo = 0, c_hi = 0;   // this rank's continuous columns of the mean correction
  int64_t r_lo = 0, r_hi = 0;   // focal rows scored by this plan (row sharding)
  double2* rspart = nullptr;    // per owned tile row-moment partials [tiles][256]
  double* Dpart = nullptr;      // (ksplit - 1) partial distance planes
  int key_shift = 8;             // colsort_key shift of the current scale
  void* colsort_scratch = nullptr;  // large-n route of colsort_terms
  size_t colsort_scratch_bytes = 0;
  // device buffers
  void* x = nullptr;            // X on the device: the plan's own, or a staged copy
  const void* x_staged = nullptr;  // the staged copy x reads (staged_acquire), released by plan_destroy
  int64_t* src_col = nullptr;
  int64_t* out_pos = nullptr;
  double *off = nullptr, *qs = nullptr, *scl = nullptr;
  float* scl32 = nullptr;       // scl as float (k_exact_pairs_rows)
  bool rows_direct = false;     // kept features = X's columns, all continuous, f32, 16-B pitch
  int64_t* dtab_off = nullptr;
  double* dtab = nullptr;
  int32_t* lab = nullptr;
  uint8_t* lab8 = nullptr;  // ReliefF: class codes as bytes (zero padding)
  uint32_t* xqT = nullptr;
  float* xs = nullptr;
  float* epsT = nullptr;
  double* corr = nullptr;
  double* corr_part = nullptr;  // [rowcorr_slices][n_pad] k_rowcorr slice partials
  double* xT64 = nullptr;      // SURF: float64 feature-major operands (the float64 route)
  bool surf_int = false;        // SURF: integer distances resolved to float32 (fs_surfint.hip)
  double* D = nullptr;
  int tiled = 0;                // D in the tiled layout (MultiSURF; d_at)
  int64_t dplane = 0;           // doubles of one distance plane (D, each Dpart)
  int2 tw = make_int2(0, 0);    // k_exact_pairs' store_pair: (nb, world) when tiled
  int2 win = make_int2(0, 0);   // full layout: rows [win.x, win.y) stored (d_row_in)
  void* D_alloc = nullptr;      // allocation behind D (D itself points at row 0)
  float* Dk = nullptr;          // ReliefF: the float32 keys instead of D (same layout)
  int2* tiles = nullptr;
  double* thr = nullptr;
  float* Wt = nullptr;          // dense pair weights (sparse == 0)
  uint2* ent = nullptr;         // sparse pair-weight streams (sparse == 1)
  unsigned long long* nnz = nullptr;  // non-zero weights of the last pass 2
  bool nnz_valid = false;
  int sparse = 0;               // pass 2 over non-zero weights only
  // MultiSURF* / SURF* split (fs_starterm.hip): pass 2 weighs the near pairs
  // only and the far pairs' all-pairs part comes per column from its sorted
  // values: xsT (float32 pass-2 values, feature-major), the per-sample
  // coefficients `alpha` and the per-column terms `tcol` k_reduce adds
  bool star_split = false;
  float* xsT = nullptr;
  double* alpha = nullptr;
  double* tcol = nullptr;
  double* spart = nullptr;       // pass-2 segment partials (own block, shard_segments)
  size_t spart_cap = 0;           // doubles of spart
  // sparse pass-2 schedule (build_sparse_schedule): tile order, segment
  // offsets and the unit tables of the F = 8 / F = 4 launches (own blocks)
  std::vector<int2> h_tiles;      // the owned tiles (host copy of `tiles`)
  int32_t* sched = nullptr;
  int32_t* seg_off = nullptr;
  int2* units8 = nullptr;
  int2* units4 = nullptr;
  size_t sched_cap = 0;           // int32 slots of `sched` + `seg_off` (one block)
  size_t units_cap = 0;           // int2 slots of units8 + units4 (one block)
  int64_t nunits8 = 0, nunits4 = 0, nfb8 = 0, nfb4 = 0, f_tail = 0;
  // exact thresholds of uncertain rows (exact_thresholds)
  unsigned int* unc = nullptr;  // [n_pad] row flags
  int32_t* urows = nullptr;     // [n_pad + 1] flagged rows in index order, then their count
  double2* uparts = nullptr;    // [thr_rows][nchunk] exact row-moment partials
  size_t uparts_cap = 0;        // double2 slots of uparts
  int thr_rows = kExactThrRows; // rows fixed at most: exact_thr_rows(n) (thr_exact_all test hook: all)
  bool thr_all = false;
  int32_t n_exact_thr = 0;      // rows whose threshold the last select recomputed (-1: too many)
  // ambiguous-pair refinement
  int2* list = nullptr;
  int64_t list_cap = 0;
  double* pair_part = nullptr;  // k_exact_pairs_rows' per-pair sums between feature chunks
  int64_t pair_part_cap = 0;
  unsigned long long* list_count = nullptr;
  int64_t n_refined = 0;
  int64_t n_tie_rows = 0;      // ReliefF rows re-ordered by k_rf_ties
  void* sort_scratch = nullptr;  // pair-list sort (fs_sort.hip)
  size_t sort_scratch_bytes = 0;
  // ev[0..1] distance kernel, ev[2..3] score kernel(s) / ReliefF selection +
  // update, ev[4..5] ReliefF's first k_rf_select launch (plan_kernel_ms)
  hipEvent_t ev[6] = {nullptr, nullptr, nullptr, nullptr, nullptr, nullptr};
  std::vector<void*> owned;         // buffers sized by n (live as long as the plan)
  std::vector<void*> owned_layout;  // buffers sized by the feature layout (PW)
  std::vector<void*> scratch;       // buffers of one plan_score call
  std::vector<void*> owned_shard;   // buffers sized by the owned tiles (plan_set_shard)
  int alloc_target = 0;             // dalloc target: 0 owned, 1 owned_layout, 2 scratch, 3 shard
  bool row_mode = false;
  // the row guard's quantised operands and mean correction are the first
  // step's (one plan over every continuous column): pass 1 takes them
  bool corr_ready = false;
  bool guard_pending = false;       // the row guard waits for the first pass 1 (P.defer_guard)
  std::vector<char> colmin, colmax; // per input column, x's dtype (device-measured)
  // reference-order accumulation (P.ref_accum, fs_refacc.hip): the kept
  // columns of X (float32 [n_pad][Kp]), their recip / discreteness, the
  // discrete flag of each 256-feature block (layout buffers); MultiSURF's
  // decision masks [n_pad][n_pad / 64][4] (plan buffer) and the per-batch
  // flagged-row counts of exact_thresholds
  float* xk = nullptr;
  double* xk64 = nullptr;       // SURF: the kept columns of its float64 X [n_pad][Kp]
  int64_t Kp = 0;
  int64_t* kcol = nullptr;
  float* krecip = nullptr;
  uint8_t* kdisc = nullptr;
  uint8_t* kblk = nullptr;
  uint64_t* masks = nullptr;
  int32_t* bcnt = nullptr;
  float* temp = nullptr;        // the reference's temp rows [rows][Kp] (own block)
  size_t temp_cap = 0;
  int64_t ref_rows = -1;        // rows of temp the last plan_ref_pass2 / _temp wrote (-1: none)
  bool ref_defer = false;       // ReliefF reference order: stop at the temp rows (plan_ref_temp)
  float* rkeys = nullptr;       // ReliefF neighbour keys (own block)
  size_t rkeys_cap = 0;
  bool ref_seeded = false;      // ReliefF: the column sums continue from the sums buffer
  double* risk_dev = nullptr;   // plan_decision_guard's result (owned, allocated on first use)
};

template <typename T>
int dalloc(Plan* g, T** p, size_t count) {
  void* q = nullptr;
  if (count == 0) count = 1;
  if (int rc = dev_alloc(&q, count * sizeof(T), g->device)) return rc;
  (g->alloc_target == 1   ? g->owned_layout
   : g->alloc_target == 2 ? g->scratch
   : g->alloc_target == 3 ? g->owned_shard
                          : g->owned)
      .push_back(q);
  *p = (T*)q;
  return FS_OK;
}

#define FS_TRY(expr)              \
  do {                            \
    int rc_ = (expr);             \
    if (rc_ != FS_OK) return rc_; \
  } while (0)

template <typename T>
int h2d(Plan* g, T* dst, const T* src, size_t count) {
  if (count == 0) return FS_OK;
  FS_HIP(hipMemcpyAsync(dst, src, count * sizeof(T), hipMemcpyHostToDevice, g->stream));
  return FS_OK;
}

inline int launch_check(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error(std::string("kernel launch failed (") + what + "): " + hipGetErrorString(e));
    return FS_EHIP;
  }
  return FS_OK;
}

// ---------------------------------------------------------------------------
// Entry points between units
// ---------------------------------------------------------------------------
// fs_gpu_mem.hip: pooled streams (non-blocking) and events (timing or not)
hipStream_t stream_get(int device);
void stream_put(int device, hipStream_t s);
hipEvent_t event_get(int device, bool timing);
void event_put(int device, hipEvent_t e, bool timing);
// fs_pass1.hip
int choose_ksplit(int64_t tiles, int device, int nchunks, int64_t feats, bool beside);
int calibrate_band(Plan* g);
int row_guard(Plan* g);
// after a 32-bit switch: the operand scale and sort key on the device
int apply_operand_width(Plan* g);
int run_quantize_dist(Plan* g);
int plan_score_surf(Plan* g, double* sums_dev);
// fs_surfint.hip: after k_dist on a SURF plan's integer operands, the focal
// rows' means into thr and every stored distance as its float32 value
int surf_resolve(Plan* g);
// fs_starterm.hip: the star split's sizes (n <= 24576, up to 8 classes);
// SURF*'s per-column all-pairs terms of this plan's focal rows into g->tcol
// (star_terms, beside pass 1); MultiSURF*'s in two steps: star_sums (beside
// pass 1: every sample's sum over the other classes, into xsT in place; the
// continuous columns' come with the mean correction's sort, colsort_star_terms,
// unless `continuous`), then
// star_reduce once the neighbour counts are known (alpha-weighted column sums
// of this rank's column share into g->tcol).  All launched on st.
bool star_split_fits(int64_t n, int32_t n_classes);
int star_terms(Plan* g, hipStream_t st);
int star_sums(Plan* g, hipStream_t st, bool continuous);
int star_reduce(Plan* g, const double* counts, hipStream_t st);
// fs_pass2.hip
int shard_segments(Plan* g);
int run_weights(Plan* g, const double* counts, int algo, double inv_sc);
int run_pass2(Plan* g, double* scores_dev);
int ref_masks(Plan* g);
int ref_temp(Plan* g, int64_t rows, float** out);
int ref_chains(Plan* g, const double* counts, double* scores);
// SURF reference order (plan_score_surf): the focal rows' masks, chains and
// float32 column sums (seeded by sums when g->ref_seeded; stopping at the
// temp rows when g->ref_defer), after the distances and means.
int surf_ref(Plan* g, double* sums);
// dst[k] += src[k] over count doubles (k_accumulate)
int accumulate(double* dst, const double* src, int64_t count, hipStream_t st);
// sums[out_pos[c]] = the fixed-order sum of part[0..nrows)[c] (k_reduce),
// plus add[c] when add is given
int reduce_segments(const double* part, int64_t nrows, int64_t PW, const int64_t* out_pos,
                    double* sums, hipStream_t st, const double* add = nullptr);
// fs_relieff.hip
int plan_score_relieff(Plan* g, double* sums_dev);
int relieff_run_one(const Prepared& P, const void* x, int device, int64_t r_lo, int64_t r_hi,
                    double* sums_out, const double* seed = nullptr);
// fs_plan.hip
int plan_layout(Plan* g);
int copy_sums(Plan* g, const double* sums_dev, double* sums_out);
int surf_run_one(const Prepared& P, const void* x, int device, int64_t r_lo, int64_t r_hi,
                 double* sums_out, const double* seed = nullptr);
// the decision guard's last risk / re-run of this thread (plan_decision_guard)
extern thread_local double g_last_risk;
extern thread_local int g_last_rerun;

}  // namespace gpu
}  // namespace fs
