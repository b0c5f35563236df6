// fs_internal.h -- shared definitions of the Relief scoring pipeline.
//
// Pipeline (every algorithm):
//   quantize   X (row-major, kernel dtype) -> Xq (integer distance operands)
//                                          -> Xs (float32 per-feature diffs)
//   pass 1     D[i][j] = sum_f |q_if - q_jf| (+ SC * [c_if != c_jf] for discrete
//              features), exact integers, computed once per unordered pair
//              (upper-triangle 128x128 tiles), stored for both (i,j) and (j,i)
//   select     per-row neighbourhood: MultiSURF radius mu - sigma/2, SURF mean
//              radius, ReliefF k nearest hits / misses per class
//   pass 2     S_f = sum_{i<j} w_ij |xs_if - xs_jf| with w_ij = W_ij + W_ji the
//              symmetric pair weight (MultiSURF/SURF), or the ReliefF
//              neighbour gather
//   finalize   scores = S / n
//
// Integer distance unit: one unit of the reference's scaled diff
// |x_i - x_j| * recip corresponds to SC integer units, SC ~ 2^24 (chosen per
// problem so that the pass-1 accumulators cannot overflow; see choose_scale).
#pragma once

#include <cmath>
#include <condition_variable>
#include <cstdint>
#include <mutex>
#include <string>
#include <utility>
#include <vector>

#if defined(__HIPCC__)
#define FS_HD __host__ __device__
#else
#define FS_HD
#endif

namespace fs {

enum Algo : int { ALGO_MULTISURF = 0, ALGO_RELIEFF = 1, ALGO_SURF = 2 };

constexpr int kTile = 128;          // pair tile edge (pass 1 / pass 2 / weights)
constexpr int kBK64 = 16;           // features per LDS stage, float64 pass 1 (SURF)
constexpr int kBKQ = 16;            // features per LDS stage, integer pass 1
constexpr int kFlushChunks = 256 / kBKQ;  // pass-1 u32 window = 256 features
constexpr int kHiShift = 24;        // pass-1 high part = D >> 24 (16-bit packed)
constexpr int kFeatPad = 64;        // feature blocks (one wave of lanes in pass 2)
constexpr int kSubRows = 32;        // pass-2 rows held in registers per sweep

void set_error(const std::string& msg);
// Phase timing on stderr when the environment sets FS_TRACE (host wall clock;
// callers synchronise the stream first where device time matters).
bool trace_on();
void trace_mark(const char* phase);

// Host-side derived problem description, identical for both backends.
struct Prepared {
  int algo = ALGO_MULTISURF;
  int use_star = 0;
  int64_t k_neighbors = 0;
  int64_t n = 0, n_pad = 0;        // samples; n_pad = roundup(n, kTile)
  int64_t p_in = 0;                // columns of the input X
  int64_t n_kept = 0;              // scored features (feat_idx)
  int64_t pc = 0, pd = 0;          // continuous / discrete kept features
  int64_t PC = 0, PD = 0, PW = 0;  // padded block widths, PW = PC + PD
  // per permuted column c in [0, PW): source column in X (-1 = padding),
  // position in the output (kept-feature order, -1 = padding)
  std::vector<int64_t> src_col, out_pos;
  std::vector<double> offset;      // continuous: column minimum (kernel dtype)
  // per input column: recip and discreteness as given (the reference's
  // feature order, used where its arithmetic is replayed exactly)
  std::vector<float> recip_in;
  std::vector<uint8_t> disc_in;
  std::vector<int64_t> kept_col;   // input column of each kept feature, kept order
  std::vector<double> scale;       // continuous: (double)recip
  // discrete: per permuted column, [dtab_off[c], dtab_off[c+1]) slice of the
  // sorted distinct values (kernel dtype widened to double)
  std::vector<int64_t> dtab_off;
  std::vector<double> dtab;
  std::vector<int32_t> labels;     // class code per sample
  int32_t n_classes = 0;
  std::vector<double> class_prior; // ReliefF priors (float32 values widened)
  double SC = 0.0;                 // integer units per scaled-diff unit
  uint32_t SCu = 0;                // SC as an integer (discrete mismatch cost)
  // Half-width (real distance units) of the band around a row's threshold
  // inside which a quantised near/far decision is not trusted; rows with a
  // pair in the band are recomputed with reference-exact arithmetic.
  double amb_delta = 0.0;
  double amb_delta_model = 0.0;    // amb_delta of the independent-rounding model
  double Rmax = 0.0;               // largest scaled continuous range (finalize_scale)
  double qmax = 0.0;               // largest quantised continuous value
  // 0 while the continuous column ranges are still to be measured (the GPU
  // backend measures them on the device, then calls finalize_scale)
  int ranges_ready = 1;
  // discrete columns of a float32 X are coded by their value bits (equality
  // is all the kernels use), so no value tables are built on the host
  int disc_bits = 0;
  // GPU pass 1 on 16-bit continuous operands: q <= 65535 (SC ~ 2^16), two
  // features packed per u32 word and compared by one v_sad_u16 (twice the
  // pair-feature rate of v_sad_u32).  finalize_scale picks SC accordingly;
  // the wider quantisation error is absorbed by amb_delta (more pairs are
  // recomputed exactly) and the mean correction (k_colrank).
  int q16 = 0;
  // 1: never 16-bit pass-1 operands (the one-shot MultiSURF re-run after the
  // decision-risk check, fs_plan.hip q16_decision_risk)
  int no_q16 = 0;
  // 1: reference-order accumulation (fs_set_accumulation(FS_ACCUM_REFERENCE),
  // fs_refacc.hip): MultiSURF's per-(sample, feature) float32 hit / miss
  // chains in ascending j and ReliefF's float32 temp of its float64 update,
  // each followed by the reference's sequential float32 column sums.
  // MultiSURF then takes 32-bit pass-1 operands and exact thresholds for
  // every flagged row, however many.
  int ref_accum = 0;
  // 1: the row guard (fs_pass1.hip row_guard) of a plan over every continuous
  // column is decided after its first pass 1, from the correction that pass
  // computes beside k_dist, instead of before it (one-shot calls; a plan
  // switched to 32-bit operands then runs pass 1 again)
  int defer_guard = 0;
};

// Accumulation mode of the calling thread's next calls (fs_api.cpp,
// fs_set_accumulation): FS_ACCUM_FAST (0) or FS_ACCUM_REFERENCE (1).
int accumulation_mode();

// Overrides of internal choices for the tests (fs_test_hook, the one
// test-only entry point; every field at its default = the product's own
// choice).  No environment variable selects a kernel or a route (FS_TRACE
// only prints phase times, FS_DEVICE_CACHE_MB sizes the block cache).
struct TestHooks {
  int64_t q16 = -1;            // 0 / 1: 32- / 16-bit pass-1 operands (choose_q16); no decision check
  int64_t sparse = -1;         // 0 / 1: dense / sparse pass 2 (choose_sparse)
  int64_t shards = 0;          // >= 1: MultiSURF tile shards per device (multisurf_shards)
  int64_t ksplit = 0;          // pass-1 K-split parts of every tile (choose_ksplit)
  int64_t q16_guard_off = 0;   // 1: no coherence / row guard on 16-bit operands
  int64_t thr_exact_all = 0;   // 1: every MultiSURF row's threshold exact (exact_thresholds)
  int64_t exact_gather = 0;    // 1: k_exact_pairs (column gather) for every layout
  int64_t row_panel = 0;       // ReliefF / SURF one-shot row-panel height
  int64_t rf_xlds = -1;        // k_rf_select's LDS x cap in floats (-1: automatic)
  int64_t rf_fcap = -1;        // candidates listed per row in LDS (-1: 256)
  int64_t ties_1w = 0;         // 1: the one-wave quicksort replay
  int64_t ties_coop = 0;       // smallest range the tie workgroup partitions (0: 2048)
  int64_t rf_ref_replay = 0;   // 1: reference-order quicksort replay of every tied row
  int64_t ref_q16 = 0;         // 1: reference-order MultiSURF may take 16-bit operands
  int64_t surf_f64 = -1;       // 0 / 1: SURF on integer / float64 distances (surf_band)
  int64_t star_split = -1;     // 0 / 1: MultiSURF* / SURF* dense star weights / near-only + column terms
  int64_t colsort_star = -1;   // 0: MultiSURF* split plans sort twice (binned correction + star sort)
  int64_t colsort_bins12 = 0;  // 1: 4096 bins at every n
  int64_t colsort_global = 0;  // 1: the large-n (device sort) route at every n
};
TestHooks& test_hooks();

// Build the permutation, label codes, discrete tables and integer scale.
// x is row-major [n][p_in], float32 (x_is_f64 == 0) or float64.
// With device_ranges != 0 the continuous column minima/maxima (and, for a
// float32 X, the discrete value tables) are left to the GPU backend.
// With dtab_src (a Prepared of the same X) the discrete value tables are
// taken from it instead of being built from x (re-targeting a GPU plan whose
// X lives on the device).
int prepare(Prepared& P, int algo, const void* x, int x_is_f64, int64_t n, int64_t p_in,
            const int64_t* feat_idx, int64_t n_kept, const float* recip,
            const uint8_t* is_discrete, int n_jobs, int device_ranges = 0,
            const Prepared* dtab_src = nullptr);
// Offsets, integer scale and error band from the per-permuted-column minima
// and maxima of the continuous columns (c in [0, pc)).
int finalize_scale(Prepared& P, const double* cmin, const double* cmax);
// Integer scale, qmax and the model band for 16-bit (q16 = 1) or 32-bit
// operands, from the ranges finalize_scale measured (P.Rmax).
int set_integer_scale(Prepared& P, int q16);
// Refinement-band calibration (fs_pass1.hip calibrate_band, and the CPU
// backend's): `count` pairs i < j from a fixed generator over [0, n) (the
// same on every rank and backend), and the band from their measured errors:
// max(model, (3 max|err| + rms / 2) / SC) in real distance units.
constexpr int64_t kCalibPairs = 4096;
void calib_pairs(int64_t n, int64_t pc, int64_t count,
                 std::vector<std::pair<int64_t, int64_t>>& out);
double calibrated_delta(double model, double SC, double rms, double max_abs);
// Sort key of a quantised continuous value for the exact per-column order
// of MultiSURF's mean correction (fs_colsort.hip, fs_cpu.cpp
// mean_correction): with fx = rint(eps 2^24) (eps = q - t in (-1/2, 1/2]),
// key = (q << s) | min((2^23 - fx) >> (24 - s), 2^s - 1), monotone in
// t = q - eps; s = 32 - bits(qmax - 1), at most 24.  The device copy
// (fs_colsort.hip cs_key / cs_fx) computes the same integers.
inline int colsort_key_shift(double qmax) {
  int b = 0;
  while (b < 32 && std::ldexp(1.0, b) < qmax) b++;
  return 32 - b < 24 ? 32 - b : 24;
}
inline int32_t colsort_fx(float eps) { return (int32_t)std::llrint((double)eps * 16777216.0); }
inline uint32_t colsort_key(uint32_t q, int32_t fx, int s) {
  const uint32_t fr = (uint32_t)(((1 << 23) - fx) >> (24 - s));
  const uint32_t m = (1u << s) - 1u;
  return (q << s) | (fr < m ? fr : m);
}
// The per-column order of the mean correction (fs_colsort.hip k_colsort,
// fs_cpu.cpp mean_correction): samples binned on the key's top
// colsort_bin_bits(n) bits; a column whose fullest mixed bin holds more than
// kColsortMaxFill samples is sorted whole, else each sample is ordered within
// its bin against its neighbours' low 32 - bits key bits, with their eps at
// 2^-12 of a quantum: the eps code colsort_eq12(fx) = (fx + 2^23) >> 12
// clamped to [0, 4095], worth colsort_eq12_fx(q) = (2q + 1) 2^11 - 2^23 in
// 2^-24 units.
// The bin count is gpu::colsort_bin_bits(n).
constexpr int kColsortMaxFill = 64;
inline uint32_t colsort_eq12(int32_t fx) {
  const int32_t u = fx + (1 << 23);
  return (uint32_t)(u < 0 ? 0 : (u >= (1 << 24) ? 4095 : (u >> 12)));
}
inline int64_t colsort_eq12_fx(uint32_t q) { return (int64_t)(2 * q + 1) * 2048 - (int64_t(1) << 23); }
int encode_labels_f64(Prepared& P, const double* y);
int encode_labels_i32(Prepared& P, const int32_t* y);

// Upper-triangle tile enumeration: t -> (bi, bj), bi <= bj, row-major over
// the triangle.  Tile t is owned by rank t % world.
void owned_tiles(int64_t nb, int rank, int world, std::vector<int32_t>& bi,
                 std::vector<int32_t>& bj);
// Row sharding (ReliefF / SURF): every upper-triangle tile that touches a
// row block in [b_lo, b_hi), so that the distance rows of those blocks are
// complete (each pair's tile writes both halves of D).
void row_tiles(int64_t nb, int64_t b_lo, int64_t b_hi, std::vector<int32_t>& bi,
               std::vector<int32_t>& bj);
FS_HD inline int64_t tile_linear(int64_t nb, int64_t bi, int64_t bj) {
  // number of tiles in rows < bi is bi*nb - bi*(bi-1)/2
  return bi * nb - bi * (bi - 1) / 2 + (bj - bi);
}

int hardware_threads(int n_jobs);

// Rows whose MultiSURF threshold a select recomputes from exact distances
// at most (exact_thresholds in both backends): a refined pair that close to
// a quantised threshold could be decided differently from the reference.
// Each such row costs n p exact pair-features with float64 sums: up to
// max(64, min(n / 64, 3e10 / (n p))) rows -- at most ~3e10 pair-features
// (a few ms on an MI355X) beyond the first 64.  32-bit operands flag a
// handful of rows (the heavy-tailed family at n = 16384: 167); 16-bit ones
// ~1000 at n >= 16384, above the cap, where the decision check stays in
// charge.
constexpr int kExactThrRows = 64;
inline int64_t exact_thr_rows(int64_t n, int64_t p) {
  const double budget = 3e10 / ((double)(n > 1 ? n : 1) * (double)(p > 1 ? p : 1));
  int64_t r = n / 64 < (int64_t)budget ? n / 64 : (int64_t)budget;
  return r > kExactThrRows ? r : kExactThrRows;
}

// Thresholds shared by both backends (MultiSURF.py:193-196 in D units).
FS_HD inline double multisurf_threshold(double s1, double s2, int64_t n) {
  const double mu = s1 / (double)(n - 1);
  double var = s2 / (double)(n - 1) - mu * mu;
  if (var < 0.0) var = 0.0;
  return mu - 0.5 * __builtin_sqrt(var);
}

// Pair weight of focal sample i for neighbour j (MultiSURF.py:217-251):
// near hit -1/H_i, near miss +1/M_i, far miss (star) -1/max(M_i, 1).
FS_HD inline double multisurf_weight(bool near, bool hit, int use_star, double H, double M) {
  if (near) return hit ? -1.0 / H : 1.0 / M;
  if (use_star && !hit) return -1.0 / (M > 0.0 ? M : 1.0);
  return 0.0;
}

// SURF pair weight of focal sample i for neighbour j (SURF.py:180-193).
FS_HD inline double surf_weight(bool near, bool hit, int use_star) {
  if (near) return hit ? -1.0 : 1.0;
  if (use_star) return hit ? 1.0 : -1.0;
  return 0.0;
}

// ---- numba's quicksort argsort (ReliefF neighbour ties) ------------------
// The reference orders each ReliefF distance row with np.argsort inside
// @njit (ReliefF.py:157), i.e. numba's non-stable quicksort (numba 0.54.1
// numba/misc/quicksort.py: median-of-three pivot, Hoare partition with the
// pivot parked at `high`, larger side pushed, insertion sort below 15
// elements; floats compared with `<`, no NaNs here).  Which of several
// neighbours at exactly the k-th distance it takes depends on that order.
// This is the same algorithm over R (the index permutation), except that a
// sub-range holding no "interesting" element (interesting(j): a neighbour
// whose key equals a tied k-th distance) is dropped instead of sorted:
// ranges are disjoint once split, so the final relative order of the
// interesting elements is exactly numba's, at ~2n work instead of n log n.
// R holds one handle per element in the initial order (R[t] = element t,
// possibly tagged); key(h) takes a handle and has_interest(lo, hi) tells
// whether R[lo..hi] holds an interesting element.  Returns 0, or -1 if the
// explicit stack (numba's MAX_STACK = 100) would overflow.  On the GPU every
// lane of a wave may run it in lockstep (identical values, identical stores)
// so that has_interest can scan with the whole wave.
template <typename KeyFn, typename RangeFn>
FS_HD inline int numba_argsort_focus(int64_t len, int32_t* R, KeyFn key, RangeFn has_interest) {
  if (len < 2) return 0;
  constexpr int kSmall = 15, kMaxStack = 100;
  int64_t st_lo[kMaxStack], st_hi[kMaxStack];
  int ns = 1;
  st_lo[0] = 0;
  st_hi[0] = len - 1;
  while (ns > 0) {
    ns--;
    int64_t low = st_lo[ns], high = st_hi[ns];
    bool live = true;
    while (high - low >= kSmall) {
      const int64_t mid = (low + high) >> 1;
      int32_t tmp;
      if (key(R[mid]) < key(R[low])) { tmp = R[low]; R[low] = R[mid]; R[mid] = tmp; }
      if (key(R[high]) < key(R[mid])) { tmp = R[high]; R[high] = R[mid]; R[mid] = tmp; }
      if (key(R[mid]) < key(R[low])) { tmp = R[low]; R[low] = R[mid]; R[mid] = tmp; }
      const float pivot = key(R[mid]);
      tmp = R[high]; R[high] = R[mid]; R[mid] = tmp;
      int64_t i = low, j = high - 1;
      while (true) {
        while (i < high && key(R[i]) < pivot) i++;
        while (j >= low && pivot < key(R[j])) j--;
        if (i >= j) break;
        tmp = R[i]; R[i] = R[j]; R[j] = tmp;
        i++;
        j--;
      }
      tmp = R[i]; R[i] = R[high]; R[high] = tmp;
      // numba pushes the larger side and keeps partitioning the smaller one
      int64_t push_lo, push_hi, keep_lo, keep_hi;
      if (high - i > i - low) {
        push_lo = i + 1; push_hi = high; keep_lo = low; keep_hi = i - 1;
      } else {
        push_lo = low; push_hi = i - 1; keep_lo = i + 1; keep_hi = high;
      }
      if (push_hi >= push_lo && has_interest(push_lo, push_hi)) {
        if (ns >= kMaxStack) return -1;
        st_lo[ns] = push_lo;
        st_hi[ns] = push_hi;
        ns++;
      }
      low = keep_lo;
      high = keep_hi;
      if (high < low || !has_interest(low, high)) {
        live = false;
        break;
      }
    }
    if (!live) continue;
    for (int64_t i = low + 1; i <= high; i++) {  // insertion sort [low, high]
      const int32_t kk = R[i];
      const float v = key(kk);
      int64_t j = i;
      while (j > low && v < key(R[j - 1])) {
        R[j] = R[j - 1];
        j--;
      }
      R[j] = kk;
    }
  }
  return 0;
}

// ---- CPU backend ---------------------------------------------------------
namespace cpu {
// 1 if all `count` float32 / float64 elements of x are finite, else 0.
int all_finite(const void* x, int x_is_f64, int64_t count, int n_jobs);
// CPU state of a MultiSURF plan (the GPU keeps the same arrays in HBM).
struct CpuState {
  std::vector<double> D;      // n x n distances (integer units; exact for refined pairs)
  std::vector<float> xs;      // n x PW per-feature operands of pass 2
  std::vector<double> corr;   // per-row mean correction (see k_colrank)
  std::vector<double> thr;    // per-row thresholds (integer units)
  int64_t refined = 0;        // ambiguous pairs recomputed exactly in the last select
};
int multisurf_pass1(const Prepared& P, const void* x, int rank, int world, int n_jobs,
                    CpuState& S, double* rowstats);
int multisurf_select(const Prepared& P, const void* x, int rank, int world,
                     const double* rowstats, int n_jobs, CpuState& S, double* counts);
// Score sums of the focal samples [r_lo, r_hi) only (each pair side counts
// for its own focal sample; [0, n) = the whole fit).
// x: the problem's float32 X (read only by reference-order accumulation,
// whose chains use the reference's raw diffs; world must then be 1).
int multisurf_pass2(const Prepared& P, const void* x, const CpuState& S, const double* counts,
                    int rank, int world, int n_jobs, int64_t r_lo, int64_t r_hi, double* scores);
// Score sums (not divided by n) of the focal samples [r_lo, r_hi).
int surf_run(const Prepared& P, const void* x, int n_jobs, int64_t r_lo, int64_t r_hi,
             double* scores);
int relieff_run(const Prepared& P, const void* x, int n_jobs, int64_t r_lo, int64_t r_hi,
                double* scores);
int column_stats(const void* x, int x_is_f64, int64_t n, int64_t p, int64_t cap, int n_jobs,
                 void* colmin, void* colmax, int64_t* ndistinct);
}  // namespace cpu

// ---- GPU backend ---------------------------------------------------------
// Barrier of the device threads that also agrees on failure: every thread
// hands in its status; when one failed, all of them return after the barrier
// instead of waiting for a peer that will never arrive at the next one.
// Status 0 is success (FS_OK).  Host code; tests/native/stage_barrier_check.cpp.
class StageBarrier {
 public:
  explicit StageBarrier(int n) : n_(n) {}
  bool arrive(int rc, const std::string& err) {
    std::unique_lock<std::mutex> lk(mu_);
    if (rc != 0 && rc_ == 0) {
      rc_ = rc;
      err_ = err;
    }
    const uint64_t gen = gen_;
    if (++count_ == n_) {
      // the stage's verdict, fixed when the last thread arrives: a faster
      // thread may fail the NEXT stage (setting rc_) before a slow waiter
      // wakes, and that waiter must still see this stage as passed
      count_ = 0;
      last_ok_ = rc_ == 0;
      gen_++;
      cv_.notify_all();
    } else {
      cv_.wait(lk, [&] { return gen_ != gen; });
    }
    return last_ok_;
  }
  int rc() const { return rc_; }
  const std::string& err() const { return err_; }
  int waiting() {  // threads blocked in the current stage (tests)
    std::lock_guard<std::mutex> lk(mu_);
    return count_;
  }

 private:
  std::mutex mu_;
  std::condition_variable cv_;
  int n_, count_ = 0, rc_ = 0;
  bool last_ok_ = true;
  uint64_t gen_ = 0;
  std::string err_;
};


namespace gpu {
int device_count();
// Device block cache (fs_gpu_mem.hip): dev_alloc hands out a cached block of
// `device` that covers `bytes` (within 2x) or a fresh hipMalloc; dev_free
// keeps the block for the next request (up to the cache cap) or frees it.
// Blocks come back with stale contents.  Returns FS_OK / FS_EOOM.
int dev_alloc(void** p, size_t bytes, int device);
void dev_free(void* p);
void dev_cache_release();
// Pinned host blocks (hipHostMalloc), cached between fits (fs_host_alloc).
int host_alloc(void** p, size_t bytes);
void host_free(void* p);
// Staged X (fs_stage_x): one device copy of a host matrix that the column
// statistics and the plan of the same fit read instead of uploading it again.
// staged_lookup returns the device copy of (host, n, p, f64) on `device`, or
// nullptr.
int stage_x(int device, const void* x, int x_is_f64, int64_t n, int64_t p, uint64_t* handle);
int stage_x_cast(int device, const void* x, int x_is_f64, int64_t n, int64_t p, int n_jobs,
                 float* out, int* finite, uint64_t* handle);
int stage_x_device(int device, const void* x, const void* x_dev, int x_is_f64, int64_t n,
                   int64_t p, uint64_t* handle);
int unstage_x(uint64_t handle);
const void* staged_lookup(const void* host, int64_t n, int64_t p, int x_is_f64, int device);
// staged_lookup of a library-owned copy (fs_stage_x, fs_stage_x_cast) plus a
// reference that keeps it alive past fs_unstage_x until staged_release
// (plans read such copies in place); nullptr for caller-owned copies
const void* staged_acquire(const void* host, int64_t n, int64_t p, int x_is_f64, int device);
void staged_release(const void* dev);
// the column extrema of a staged copy (X's dtype, p values each), when known
bool staged_extrema(const void* dev, void* cmin, void* cmax);
int column_stats(const void* x, int x_is_f64, int64_t n, int64_t p, int64_t cap, int device,
                 void* colmin, void* colmax, int64_t* ndistinct);
// Column minima / maxima of a device-resident X, copied to host arrays in
// x's dtype; runs on `stream` (a hipStream_t) and synchronises it.
int column_minmax(const void* dx, int x_is_f64, int64_t n, int64_t p, void* hmin, void* hmax,
                  void* stream);
// Sort a pair list (int2 (i, j) entries) by (i, j) in place (fs_sort.hip);
// scratch of pair_sort_scratch_bytes(count) bytes of device memory, `stream`
// a hipStream_t.
size_t pair_sort_scratch_bytes(int64_t count);
int sort_pairs(void* list, int64_t count, void* scratch, size_t scratch_bytes, void* stream);
// MultiSURF mean-correction terms of the continuous columns [c_lo, c_hi)
// from exact per-column order (fs_colsort.hip; colsort_key): epsT[c][i]
// (quantisation errors, from k_quantize) is overwritten with
// eps_i (L_i - G_i) - (E_below - E_above).  Columns of n <= 24576 samples
// are ordered in LDS, larger n by a device segmented sort; either way the
// call needs colsort_scratch_bytes(n, c_hi - c_lo) bytes of device scratch.
// `stream` is a hipStream_t.
bool colsort_lds(int64_t n);
// Bits of the key the LDS route bins on: 13 (8192 bins) where the
// workgroup's LDS holds them next to the column's entries (12288 < n <=
// 20480: half the within-bin work of 4096 bins at cfg4's n = 20000), 12
// elsewhere; the colsort_bins12 test hook keeps 12 everywhere.  Both
// backends bin alike, so their terms stay identical -- except MultiSURF*
// plans with the star split on the GPU, which sort every column whole
// (colsort_star_terms: the exact eps of every neighbour, not 2^-12 quanta).
int colsort_bin_bits(int64_t n);
size_t colsort_scratch_bytes(int64_t n, int64_t ncols);
int colsort_terms(const uint32_t* xqT, float* epsT, int64_t n, int64_t n_pad, int64_t c_lo,
                  int64_t c_hi, int q16, int key_shift, void* scratch, size_t scratch_bytes,
                  void* stream);
// MultiSURF* star split (n <= 24576): the same terms from a full sort of
// every column (no bin rounding), and in that order each sample's sum over
// the other classes of |v_i - v_j| written over xsT (fs_starterm.hip
// star_reduce); padding columns (out_pos < 0) get the terms only.
int colsort_star_terms(const uint32_t* xqT, float* epsT, float* xsT, const int32_t* lab,
                       const int64_t* out_pos, int ncls, int64_t n, int64_t n_pad, int64_t c_lo,
                       int64_t c_hi, int q16, int key_shift, void* stream);
struct Plan;
// Tile sharding (MultiSURF): tile t belongs to rank t % world.  Row
// sharding (r_hi >= 0): the tiles touching the 128-row blocks of [r_lo, r_hi).
int plan_create(Plan** out, const Prepared& P, const void* x, int x_is_f64, int device,
                int rank, int world, uint64_t stream, int64_t r_lo = 0, int64_t r_hi = -1);
// Re-target a plan (resident X, distances storage) to another feature
// subset: P is the new layout (same samples, labels and algorithm).
int plan_set_features(Plan* g, const Prepared& P);
int plan_pass1(Plan* g, double* rowstats_dev);
int plan_select(Plan* g, const double* rowstats_dev, double* counts_dev);
int plan_pass2(Plan* g, const double* counts_dev, double* scores_dev);
int64_t ref_mask_words(const Plan* g);
int plan_ref_masks(Plan* g, uint64_t* masks_dev);
int plan_ref_pass2(Plan* g, const uint64_t* masks_dev, const double* counts_dev, int64_t row_lo,
                   int64_t row_hi);
int plan_ref_sums(Plan* g, const double* init_dev, double* sums_dev);
int plan_ref_temp(Plan* g);
// After a step on 16-bit operands: decision risk from the step's summed
// exchange vectors (device memory); above the bound the plan switches to
// 32-bit operands and *switched = 1 (run the step again).  risk = -1: no check.
int plan_decision_guard(Plan* g, const double* rowstats, const double* counts,
                        const double* sums, double* risk, int* switched);
// MultiSURF focal-sample slice: the next pass2 sums the pair sides of the
// focal samples [r_lo, r_hi) only (thresholds and counts stay global).
int plan_set_rows(Plan* g, int64_t r_lo, int64_t r_hi);
// Re-target a MultiSURF plan to the tiles of (rank, world) (tile t belongs to
// rank t % world): frees the previous shard's tile buffers and lays out the
// new ones.  X and its quantised operands stay resident.
int plan_set_shard(Plan* g, int rank, int world);
// Tile shards per device for a MultiSURF job of `world` ranks so that the
// tile buffers fit the device (1 = no sharding; the shards test hook forces it); with
// share > 1 that many plans split the device's memory (repeated ordinals).
int multisurf_shards(const Prepared& P, int device, int world, int share = 1);
// ReliefF / SURF plans: float64 score sums of the plan's focal rows
// (sums_dev[n_kept], device memory), for the plan's current feature subset.
int plan_score(Plan* g, double* sums_dev);
int plan_info(const Plan* g, int64_t* tiles, double* pfe, int64_t* refined);
// Band calibration of the plan's current layout: out[0] = 16-bit operands in
// use, out[1] / out[2] = rms / max |error| of the sampled pairs' quantised
// distances (integer units, final operand width), out[3] = the model's
// standard deviation sqrt(pc/6 + 1), out[4] = band / model band, out[5] = 1
// if the coherence guard turned 16-bit operands off.
int plan_calibration(const Plan* g, double* out);
double plan_kernel_ms(const Plan* g, int which);
int plan_weighted_pairs(Plan* g, int64_t* pairs);
void plan_destroy(Plan* g);
// Single-GPU one-shot runs (host in/out).  MultiSURF: scores already divided
// by n.  SURF / ReliefF: float64 score sums of the focal samples [r_lo, r_hi)
// (row sharding; the full range gives the single-GPU result times n).
int multisurf_run(const Prepared& P, const void* x, int device, float* scores_out);
// The 16-bit decision check of this thread's last multisurf_run (risk, re-run).
int multisurf_last_guard(double* risk, int* rerun);
// One process, several devices (devices[0..ndev), repeats allowed): MultiSURF
// tile partition / ReliefF and SURF row partition with host-side rank-order
// sums in place of the all-reduces.  Score sums of [r_lo, r_hi) (not / n).
int multisurf_run_devices(const Prepared& P, const void* x, const int* devices, int ndev,
                          int64_t r_lo, int64_t r_hi, double* sums_out);
int rows_run_devices(const Prepared& P, const void* x, const int* devices, int ndev,
                     int64_t r_lo, int64_t r_hi, double* sums_out);
// MultiSURF float64 score sums of the focal samples [r_lo, r_hi).
int multisurf_rows(const Prepared& P, const void* x, int device, int64_t r_lo, int64_t r_hi,
                   double* sums_out);
int surf_run(const Prepared& P, const void* x, int device, int64_t r_lo, int64_t r_hi,
             double* sums_out);
int relieff_run(const Prepared& P, const void* x, int device, int64_t r_lo, int64_t r_hi,
                double* sums_out);

// Reference-order accumulation kernels (fs_refacc.hip); `stream` is a
// hipStream_t, `tiles` the plan's int2 tile list.
namespace refacc {
// xk[j][k] = x[j][kcol[k]] (k < n_kept, j < n), zero padding to [n_pad][Kp];
// Kp a multiple of 256.
int gather_kept(const float* x, int64_t n, int64_t n_pad, int64_t p_in, const int64_t* kcol,
                int64_t n_kept, int64_t Kp, float* xk, void* stream);
// The same for SURF's float64 X (Kp a multiple of 128).
int gather_kept64(const double* x, int64_t n, int64_t n_pad, int64_t p_in, const int64_t* kcol,
                  int64_t n_kept, int64_t Kp, double* xk, void* stream);
// SURF: near-hit / near-miss / far-hit / far-miss bit masks of the focal
// rows [r_lo, r_hi) from their float32 distance rows and means (avg[n]):
// masks[((i - r_lo) * (n_pad / 64) + word) * 4 + type].
int surf_masks(const double* D, int64_t n, int64_t n_pad, const double* avg, const int32_t* lab,
               int use_star, int64_t r_lo, int64_t r_hi, uint64_t* masks, void* stream);
// temp[i - r_lo][k] = (near miss - near hit) [+ (far hit - far miss)], each
// a float32 chain over ascending j (SURF.py:165-193).
int surf_chains(const double* xk, int64_t Kp, const float* krecip, const uint8_t* kdisc,
                const uint8_t* blkdisc, const uint64_t* masks, int64_t n, int64_t n_pad,
                int use_star, int64_t r_lo, int64_t r_hi, float* temp, void* stream);
// Near-hit / miss-chain / far-miss bit masks of the owned tiles' pairs:
// masks[(row * (n_pad / 64) + word) * 4 + type].
int multisurf_masks(const double* D, int64_t n, int64_t n_pad, const void* tiles, int64_t n_tiles,
                    const double* thr, const int32_t* lab, int use_star, uint64_t* masks,
                    void* stream);
// temp[i - r_lo][k] = f32(miss chain / M_i) - f32(hit chain / H_i) for the
// focal rows [r_lo, r_hi) (MultiSURF.py:198-251).
int multisurf_chains(const float* xk, int64_t Kp, const float* krecip, const uint8_t* kdisc,
                     const uint8_t* blkdisc, const uint64_t* masks, int64_t n, int64_t n_pad,
                     const double* counts, int use_star, int64_t r_lo, int64_t r_hi, float* temp,
                     void* stream);
// out[k] = float32 sequential sum of temp[0..rows)[k] (starting from
// (float) init[k] when init is not null; init may alias out), as a double.
int column_sums(const float* temp, int64_t rows, int64_t Kp, int64_t n_kept, const double* init,
                double* out, void* stream);
// ReliefF: each (row, class) neighbour list in ascending exact key, equal
// keys by sample index (keys[rows * C * k]: the sorted keys), dup[rows * C] =
// 1 where a list holds equal keys (k_rf_ref_ties then orders those runs as
// numba's quicksort does).
int relieff_order(const float* xk, int64_t Kp, const float* krecip, const uint8_t* kdisc,
                  int64_t n_kept, int C, int64_t k, int32_t* nbr, const int32_t* nfound,
                  int64_t r_lo, int64_t r_hi, float* keys, int32_t* dup, void* stream);
// keys[r][j] = the reference's key of (rows[r], j), +inf at j = rows[r].
int relieff_row_keys(const float* xk, int64_t Kp, const float* krecip, const uint8_t* kdisc,
                     int64_t n_kept, const int32_t* rows, int64_t nr, int64_t n, float* keys,
                     void* stream);
// matters[r] = 1 when some list of row rows[r] flagged in dup could sum to
// different float64 values in another order (a continuous feature whose
// float32 diffs span 2^29 or more); 0 = any order gives the same sums.
int relieff_order_matters(const float* xk, int64_t Kp, const float* krecip,
                          const uint8_t* kdisc, int64_t n_kept, const int32_t* rows, int64_t nr,
                          const int32_t* dup, const int32_t* nbr, const int32_t* nfound,
                          int64_t r_lo, int C, int64_t k, int32_t* matters, void* stream);
// temp[i - r_lo][k] = f32(update) over the lists in their order
// (ReliefF.py:177-216).
int relieff_update(const float* xk, int64_t Kp, const float* krecip, const uint8_t* kdisc,
                   const int32_t* lab, const double* prior, int C, int64_t k, const int32_t* nbr,
                   const int32_t* nfound, int64_t r_lo, int64_t r_hi, float* temp, void* stream);
}  // namespace refacc
}  // namespace gpu

}  // namespace fs
