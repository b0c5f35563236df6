/*
 * relief_oracle.c -- TEST INFRASTRUCTURE ONLY (parity oracle + timed CPU
 * baseline).  Never linked into or called by the product (fastselect_amd/).
 *
 * A plain-C restatement of the reference's `backend='cpu'` Relief kernels
 * (GavinLynch04/FastSelect v0.2.0, Numba `@njit(parallel=True, fastmath=True)`):
 *
 *   oracle_multisurf  <- src/fast_select/MultiSURF.py:165-253 (+ host caller :256-270)
 *   oracle_relieff    <- src/fast_select/ReliefF.py:137-220  (+ host caller :222-236)
 *   oracle_surf       <- src/fast_select/SURF.py:131-195     (+ host caller :198-218)
 *   numba_argsort_f32 <- numba 0.54.1 numba/misc/quicksort.py:27-197 with
 *                        lt_floats (numba/np/arrayobj.py:5214-5215), the
 *                        algorithm behind `np.argsort` inside @njit
 *                        (ReliefF.py:157).
 *
 * Numerics follow Numba's typing of those kernels: `diff`
 * and `dist` are float64 (the 1.0/0.0 literals unify with the float32
 * product), the continuous diff itself is computed in the kernel's X dtype
 * with a float32 `recip`, per-sample arrays are float32 with a float64
 * right-hand side rounded on store, and `temp[:, k].sum()` is a sequential
 * float32 accumulation.  Numba's fastmath may reassociate the float64 sums;
 * that freedom is below every tolerance used by the tests.
 *
 * Parity pinning: the reference ships no golden score vectors and cannot be
 * executed in this image (numba absent).  The oracle is pinned by the
 * reference's own known-answer tests (tests/test_{multisurf,relieff,surf}.py
 * fixtures and assertions, re-run against this oracle in
 * tests/test_oracle.py) and cross-checked against an independent
 * vectorised numpy restatement (oracle/relief_np.py).
 *
 * Parallelism: OpenMP over focal samples, like numba.prange; per-sample rows
 * go to a temp matrix and are column-summed sequentially, so results do not
 * depend on the thread count.  SURF's per-thread private_scores are replaced
 * by that same deterministic per-sample layout (== the reference run with
 * n_jobs=1).
 *
 * Every entry point can score a contiguous range of focal samples
 * [i_begin, i_end) (the bounded CPU-baseline sample of bench.py); scores are
 * then the partial sum over that range divided by n, as the host caller does.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define ORACLE_API __attribute__((visibility("default")))

static void set_threads(int n_jobs) {
#ifdef _OPENMP
  if (n_jobs > 0) omp_set_num_threads(n_jobs);
#else
  (void)n_jobs;
#endif
}

ORACLE_API int oracle_max_threads(void) {
#ifdef _OPENMP
  return omp_get_max_threads();
#else
  return 1;
#endif
}

/* ------------------------------------------------------------------------ */
/* MultiSURF / MultiSURF*   (MultiSURF.py:165-253, host caller :256-270)      */
/* ------------------------------------------------------------------------ */

/* diff of one feature, MultiSURF.py:184-187: discrete -> 1.0/0.0, else the
 * float32 product |x_i - x_j| * recip, widened to float64. */
static inline double ms_diff(const float* xi, const float* xj, const float* recip,
                             const uint8_t* is_discrete, int64_t f) {
  if (is_discrete[f]) return xi[f] != xj[f] ? 1.0 : 0.0;
  float d = fabsf(xi[f] - xj[f]) * recip[f];
  return (double)d;
}

/* accum64 = 0: the reference's arithmetic (float32 per-sample sums, float32
 * rows, float32 sequential column sum).  accum64 = 1 (parity attribution,
 * not the reference): the same diffs, distances and near/far decisions, but
 * every sum after them -- per-sample hit/miss sums, the division, the row and
 * the column sum -- in float64, rounded to float32 once at the end.  The
 * difference between the two is the reference's own float32 accumulation
 * error (tests/test_parity_attribution.py). */
static inline double acc_round(int accum64, double v) { return accum64 ? v : (double)(float)v; }

/* Column sum of the per-sample rows (float32 sequential as the reference's
 * `.sum()`, or float64 with accum64), then `/ n` (host callers). */
static void colsum(const double* temp, int64_t m, int64_t p, int64_t n, int accum64, float* out) {
#pragma omp parallel for schedule(static)
  for (int64_t k = 0; k < p; k++) {
    if (accum64) {
      double s = 0.0;
      for (int64_t r = 0; r < m; r++) s += temp[r * p + k];
      out[k] = (float)(s / (double)n);
    } else {
      float s = 0.0f;
      for (int64_t r = 0; r < m; r++) s += (float)temp[r * p + k];
      out[k] = s / (float)n;
    }
  }
}

ORACLE_API int oracle_multisurf_acc(const float* x, int64_t n, int64_t p, const double* y,
                                    const float* recip, const int64_t* feat_idx, int64_t n_kept,
                                    int use_star, const uint8_t* is_discrete, int64_t i_begin,
                                    int64_t i_end, int n_jobs, int accum64, float* scores_out) {
  if (n < 2 || i_begin < 0 || i_end > n || i_begin > i_end) return -1;
  int64_t m = i_end - i_begin;
  double* temp = (double*)calloc((size_t)(m > 0 ? m : 1) * (size_t)n_kept, sizeof(double));
  if (!temp) return -2;
  set_threads(n_jobs);
#pragma omp parallel
  {
    double* hit_diffs = (double*)malloc(sizeof(double) * (size_t)n_kept);
    double* miss_diffs = (double*)malloc(sizeof(double) * (size_t)n_kept);
#pragma omp for schedule(dynamic, 1)
    for (int64_t i = i_begin; i < i_end; i++) {
      const float* xi = x + i * p;
      /* pass 1: mean and spread of the distance row (MultiSURF.py:175-196) */
      double sum_d = 0.0, sum_d2 = 0.0;
      for (int64_t j = 0; j < n; j++) {
        if (i == j) continue;
        const float* xj = x + j * p;
        double dist = 0.0;
        for (int64_t k = 0; k < n_kept; k++) dist += ms_diff(xi, xj, recip, is_discrete, feat_idx[k]);
        sum_d += dist;
        sum_d2 += dist * dist;
      }
      double mu = sum_d / (double)(n - 1);
      double var = sum_d2 / (double)(n - 1) - mu * mu;
      if (var < 0.0) var = 0.0;
      double thresh = mu - 0.5 * sqrt(var);
      /* pass 2: near hits / near misses (/ far misses) (MultiSURF.py:198-243) */
      memset(hit_diffs, 0, sizeof(double) * (size_t)n_kept);
      memset(miss_diffs, 0, sizeof(double) * (size_t)n_kept);
      int64_t n_hits = 0, n_miss = 0;
      for (int64_t j = 0; j < n; j++) {
        if (i == j) continue;
        const float* xj = x + j * p;
        double dist = 0.0;
        for (int64_t k = 0; k < n_kept; k++) dist += ms_diff(xi, xj, recip, is_discrete, feat_idx[k]);
        int is_hit = y[i] == y[j];
        if (dist < thresh) {
          if (is_hit) {
            n_hits++;
            for (int64_t k = 0; k < n_kept; k++)
              hit_diffs[k] = acc_round(accum64, hit_diffs[k] + ms_diff(xi, xj, recip, is_discrete, feat_idx[k]));
          } else {
            n_miss++;
            for (int64_t k = 0; k < n_kept; k++)
              miss_diffs[k] = acc_round(accum64, miss_diffs[k] + ms_diff(xi, xj, recip, is_discrete, feat_idx[k]));
          }
        } else if (use_star && !is_hit) {
          for (int64_t k = 0; k < n_kept; k++)
            miss_diffs[k] = acc_round(accum64, miss_diffs[k] - ms_diff(xi, xj, recip, is_discrete, feat_idx[k]));
        }
      }
      /* MultiSURF.py:245-251: in-place float32 /= int (computed in float64) */
      if (n_hits > 0)
        for (int64_t k = 0; k < n_kept; k++) hit_diffs[k] = acc_round(accum64, hit_diffs[k] / (double)n_hits);
      if (n_miss > 0)
        for (int64_t k = 0; k < n_kept; k++) miss_diffs[k] = acc_round(accum64, miss_diffs[k] / (double)n_miss);
      double* row = temp + (i - i_begin) * n_kept;
      for (int64_t k = 0; k < n_kept; k++)
        row[k] = accum64 ? miss_diffs[k] - hit_diffs[k]
                         : (double)((float)miss_diffs[k] - (float)hit_diffs[k]);
    }
    free(hit_diffs);
    free(miss_diffs);
  }
  /* MultiSURF.py:252-253 column sum (float32, sequential), host caller :270 `/ n` */
  colsum(temp, m, n_kept, n, accum64, scores_out);
  free(temp);
  return 0;
}

/* The near/far decisions of MultiSURF.py:175-217 alone (parity attribution:
 * a score difference is either flipped decisions or accumulation): per focal
 * sample i in [i_begin, i_end) the threshold mu - sigma/2 (thr_out) and the
 * near hit / near miss counts (counts_out[2 (i - i_begin)], [.. + 1]), in the
 * reference's arithmetic as oracle_multisurf_acc. */
ORACLE_API int oracle_multisurf_decisions(const float* x, int64_t n, int64_t p, const double* y,
                                          const float* recip, const int64_t* feat_idx,
                                          int64_t n_kept, const uint8_t* is_discrete,
                                          int64_t i_begin, int64_t i_end, int n_jobs,
                                          double* thr_out, int64_t* counts_out) {
  if (n < 2 || i_begin < 0 || i_end > n || i_begin > i_end) return -1;
  set_threads(n_jobs);
  int fail = 0;
#pragma omp parallel
  {
    double* drow = (double*)malloc(sizeof(double) * (size_t)n);
    if (!drow) fail = 1;
#pragma omp for schedule(dynamic, 1)
  for (int64_t i = i_begin; i < i_end; i++) {
    if (!drow) continue;
    const float* xi = x + i * p;
    double sum_d = 0.0, sum_d2 = 0.0;
    for (int64_t j = 0; j < n; j++) {
      if (i == j) continue;
      const float* xj = x + j * p;
      double d = 0.0;
      for (int64_t k = 0; k < n_kept; k++) d += ms_diff(xi, xj, recip, is_discrete, feat_idx[k]);
      drow[j] = d;
      sum_d += d;
      sum_d2 += d * d;
    }
    double mu = sum_d / (double)(n - 1);
    double var = sum_d2 / (double)(n - 1) - mu * mu;
    if (var < 0.0) var = 0.0;
    double thresh = mu - 0.5 * sqrt(var);
    int64_t h = 0, m = 0;
    for (int64_t j = 0; j < n; j++) {
      if (i == j || !(drow[j] < thresh)) continue;
      if (y[i] == y[j]) h++;
      else m++;
    }
    thr_out[i - i_begin] = thresh;
    counts_out[2 * (i - i_begin)] = h;
    counts_out[2 * (i - i_begin) + 1] = m;
  }
    free(drow);
  }
  return fail ? -2 : 0;
}

ORACLE_API int oracle_multisurf(const float* x, int64_t n, int64_t p, const double* y,
                                const float* recip, const int64_t* feat_idx, int64_t n_kept,
                                int use_star, const uint8_t* is_discrete, int64_t i_begin,
                                int64_t i_end, int n_jobs, float* scores_out) {
  return oracle_multisurf_acc(x, n, p, y, recip, feat_idx, n_kept, use_star, is_discrete, i_begin,
                              i_end, n_jobs, 0, scores_out);
}

/* ------------------------------------------------------------------------ */
/* numba quicksort argsort (numba/misc/quicksort.py:27-197, lt_floats)       */
/* ------------------------------------------------------------------------ */

static inline int lt_floats(float a, float b) { return isnan(b) || a < b; }

#define SMALL_QUICKSORT 15
#define MAX_STACK 100

static void nb_insertion_sort(const float* A, int64_t* R, int64_t low, int64_t high) {
  if (high <= low) return;
  for (int64_t i = low + 1; i <= high; i++) {
    int64_t k = R[i];
    float v = A[k];
    int64_t j = i;
    while (j > low && lt_floats(v, A[R[j - 1]])) {
      R[j] = R[j - 1];
      j--;
    }
    R[j] = k;
  }
}

static int64_t nb_partition(const float* A, int64_t* R, int64_t low, int64_t high) {
  int64_t mid = (low + high) >> 1, t;
  if (lt_floats(A[R[mid]], A[R[low]])) { t = R[low]; R[low] = R[mid]; R[mid] = t; }
  if (lt_floats(A[R[high]], A[R[mid]])) { t = R[high]; R[high] = R[mid]; R[mid] = t; }
  if (lt_floats(A[R[mid]], A[R[low]])) { t = R[low]; R[low] = R[mid]; R[mid] = t; }
  float pivot = A[R[mid]];
  t = R[high]; R[high] = R[mid]; R[mid] = t;
  int64_t i = low, j = high - 1;
  for (;;) {
    while (i < high && lt_floats(A[R[i]], pivot)) i++;
    while (j >= low && lt_floats(pivot, A[R[j]])) j--;
    if (i >= j) break;
    t = R[i]; R[i] = R[j]; R[j] = t;
    i++;
    j--;
  }
  t = R[i]; R[i] = R[high]; R[high] = t;
  return i;
}

ORACLE_API void numba_argsort_f32(const float* A, int64_t len, int64_t* R) {
  for (int64_t i = 0; i < len; i++) R[i] = i;
  if (len < 2) return;
  int64_t st_lo[MAX_STACK], st_hi[MAX_STACK];
  int n = 1;
  st_lo[0] = 0;
  st_hi[0] = len - 1;
  while (n > 0) {
    n--;
    int64_t low = st_lo[n], high = st_hi[n];
    while (high - low >= SMALL_QUICKSORT) {
      int64_t i = nb_partition(A, R, low, high);
      if (high - i > i - low) {
        if (high > i) { st_lo[n] = i + 1; st_hi[n] = high; n++; }
        high = i - 1;
      } else {
        if (i > low) { st_lo[n] = low; st_hi[n] = i - 1; n++; }
        low = i + 1;
      }
    }
    nb_insertion_sort(A, R, low, high);
  }
}

/* ------------------------------------------------------------------------ */
/* ReliefF   (ReliefF.py:137-220, host caller :222-236)                      */
/* ------------------------------------------------------------------------ */

static inline double rf_diff(const float* xi, const float* xj, const float* recip,
                             const uint8_t* is_discrete, int64_t f) {
  if (is_discrete[f]) return xi[f] != xj[f] ? 1.0 : 0.0;
  return (double)(fabsf(xi[f] - xj[f]) * recip[f]);
}

ORACLE_API int oracle_relieff_acc(const float* x, int64_t n, int64_t p, const int32_t* y_enc,
                                  const float* recip, const uint8_t* is_discrete, int64_t k,
                                  const float* class_probs, int64_t n_classes, int64_t i_begin,
                                  int64_t i_end, int n_jobs, int accum64, float* scores_out) {
  if (n < 2 || k < 0 || i_begin < 0 || i_end > n || i_begin > i_end) return -1;
  int64_t m = i_end - i_begin;
  double* temp = (double*)calloc((size_t)(m > 0 ? m : 1) * (size_t)p, sizeof(double));
  if (!temp) return -2;
  set_threads(n_jobs);
#pragma omp parallel
  {
    float* dists = (float*)malloc(sizeof(float) * (size_t)n);
    int64_t* order = (int64_t*)malloc(sizeof(int64_t) * (size_t)n);
    int64_t* hits = (int64_t*)malloc(sizeof(int64_t) * (size_t)(k > 0 ? k : 1));
    int64_t* misses = (int64_t*)malloc(sizeof(int64_t) * (size_t)(n_classes * (k > 0 ? k : 1)));
    int64_t* m_found = (int64_t*)malloc(sizeof(int64_t) * (size_t)n_classes);
#pragma omp for schedule(dynamic, 1)
    for (int64_t i = i_begin; i < i_end; i++) {
      const float* xi = x + i * p;
      /* ReliefF.py:144-155: float64 distance stored as float32, self = inf */
      for (int64_t j = 0; j < n; j++) {
        if (i == j) { dists[j] = INFINITY; continue; }
        const float* xj = x + j * p;
        double d = 0.0;
        for (int64_t f = 0; f < p; f++) d += rf_diff(xi, xj, recip, is_discrete, f);
        dists[j] = (float)d;
      }
      numba_argsort_f32(dists, n, order); /* ReliefF.py:157 */
      int32_t lbl_i = y_enc[i];
      int64_t h_found = 0;
      for (int64_t c = 0; c < n_classes; c++) m_found[c] = 0;
      /* ReliefF.py:164-175.  The early exit at :174 can never fire (the
       * own-class slot of m_found stays 0 < k), so scanning all is exact. */
      for (int64_t t = 0; t < n; t++) {
        int64_t idx = order[t];
        int32_t lbl = y_enc[idx];
        if (lbl == lbl_i) {
          if (h_found < k) hits[h_found++] = idx;
        } else {
          if (m_found[lbl] < k) misses[lbl * k + m_found[lbl]++] = idx;
        }
      }
      /* ReliefF.py:177-179 */
      double denom = 1.0 - (double)class_probs[lbl_i];
      if (denom == 0.0) denom = 1.0;
      double* row = temp + (i - i_begin) * p;
      /* ReliefF.py:181-216 */
      for (int64_t f = 0; f < p; f++) {
        double hit_sum = 0.0;
        for (int64_t ki = 0; ki < h_found; ki++) hit_sum += rf_diff(xi, x + hits[ki] * p, recip, is_discrete, f);
        double miss_sum = 0.0;
        for (int64_t c = 0; c < n_classes; c++) {
          if (c == lbl_i) continue;
          double weight = (double)class_probs[c] / denom;
          double cur = 0.0;
          for (int64_t ki = 0; ki < m_found[c]; ki++)
            cur += rf_diff(xi, x + misses[c * k + ki] * p, recip, is_discrete, f);
          miss_sum += weight * cur;
        }
        double update = 0.0;
        if (h_found > 0) update -= hit_sum / (double)h_found;
        if (k > 0) update += miss_sum / (double)k;
        row[f] = acc_round(accum64, update);
      }
    }
    free(dists);
    free(order);
    free(hits);
    free(misses);
    free(m_found);
  }
  /* ReliefF.py:219-220 column sum, host caller :236 `/ n` */
  colsum(temp, m, p, n, accum64, scores_out);
  free(temp);
  return 0;
}

ORACLE_API int oracle_relieff(const float* x, int64_t n, int64_t p, const int32_t* y_enc,
                              const float* recip, const uint8_t* is_discrete, int64_t k,
                              const float* class_probs, int64_t n_classes, int64_t i_begin,
                              int64_t i_end, int n_jobs, float* scores_out) {
  return oracle_relieff_acc(x, n, p, y_enc, recip, is_discrete, k, class_probs, n_classes, i_begin,
                            i_end, n_jobs, 0, scores_out);
}

/* ------------------------------------------------------------------------ */
/* SURF / SURF*   (SURF.py:131-195, host caller :198-218)                    */
/* ------------------------------------------------------------------------ */

/* SURF.py:153-156: X is float64 here; the float32 recip is widened. */
static inline double sf_diff(const double* xi, const double* xj, const float* recip,
                             const uint8_t* is_discrete, int64_t f) {
  if (is_discrete[f]) return xi[f] != xj[f] ? 1.0 : 0.0;
  return fabs(xi[f] - xj[f]) * (double)recip[f];
}

ORACLE_API int oracle_surf_acc(const double* x, int64_t n, int64_t p, const int32_t* y,
                               const float* recip, int use_star, const uint8_t* is_discrete,
                               int64_t i_begin, int64_t i_end, int n_jobs, int accum64,
                               float* scores_out) {
  if (n < 2 || i_begin < 0 || i_end > n || i_begin > i_end) return -1;
  int64_t m = i_end - i_begin;
  double* temp = (double*)calloc((size_t)(m > 0 ? m : 1) * (size_t)p, sizeof(double));
  if (!temp) return -2;
  set_threads(n_jobs);
#pragma omp parallel
  {
    float* dists = (float*)malloc(sizeof(float) * (size_t)n);
    double* nh = (double*)malloc(sizeof(double) * (size_t)p);
    double* nm = (double*)malloc(sizeof(double) * (size_t)p);
    double* fh = (double*)malloc(sizeof(double) * (size_t)p);
    double* fm = (double*)malloc(sizeof(double) * (size_t)p);
#pragma omp for schedule(dynamic, 1)
    for (int64_t i = i_begin; i < i_end; i++) {
      const double* xi = x + i * p;
      /* SURF.py:146-160: diffs stored float32, distance float64 -> float32.
       * The n x p diffs_from_i buffer is recomputed below instead of stored;
       * the recomputation is bit-identical. */
      for (int64_t j = 0; j < n; j++) {
        if (i == j) { dists[j] = 0.0f; continue; }
        const double* xj = x + j * p;
        double dist = 0.0;
        for (int64_t f = 0; f < p; f++) dist += sf_diff(xi, xj, recip, is_discrete, f);
        dists[j] = (float)dist;
      }
      /* SURF.py:162-163: np.sum of a float32 array (float32 accumulator,
       * sequential), divided by (n - 1) in float64 */
      float sum_d = 0.0f;
      for (int64_t j = 0; j < n; j++) sum_d += dists[j];
      double avg = (double)sum_d / (double)(n - 1);
      memset(nh, 0, sizeof(double) * (size_t)p);
      memset(nm, 0, sizeof(double) * (size_t)p);
      memset(fh, 0, sizeof(double) * (size_t)p);
      memset(fm, 0, sizeof(double) * (size_t)p);
      /* SURF.py:170-189 */
      for (int64_t j = 0; j < n; j++) {
        if (i == j) continue;
        int is_hit = y[i] == y[j];
        int is_near = (double)dists[j] < avg;
        double* acc;
        if (is_near) acc = is_hit ? nh : nm;
        else if (use_star) acc = is_hit ? fh : fm;
        else continue;
        const double* xj = x + j * p;
        /* float32 diffs (diffs_from_i), float32 sums (or float64 with accum64) */
        for (int64_t f = 0; f < p; f++)
          acc[f] = accum64 ? acc[f] + (double)(float)sf_diff(xi, xj, recip, is_discrete, f)
                           : (double)((float)acc[f] + (float)sf_diff(xi, xj, recip, is_discrete, f));
      }
      /* SURF.py:191-195 */
      double* row = temp + (i - i_begin) * p;
      for (int64_t f = 0; f < p; f++) {
        if (accum64) {
          double u = nm[f] - nh[f];
          if (use_star) u += fh[f] - fm[f];
          row[f] = u;
        } else {
          float u = (float)nm[f] - (float)nh[f];
          if (use_star) u += (float)fh[f] - (float)fm[f];
          row[f] = (double)u;
        }
      }
    }
    free(dists);
    free(nh);
    free(nm);
    free(fh);
    free(fm);
  }
  /* SURF.py:195/216-218: private_scores accumulation then `/ n` */
  colsum(temp, m, p, n, accum64, scores_out);
  free(temp);
  return 0;
}

ORACLE_API int oracle_surf(const double* x, int64_t n, int64_t p, const int32_t* y,
                           const float* recip, int use_star, const uint8_t* is_discrete,
                           int64_t i_begin, int64_t i_end, int n_jobs, float* scores_out) {
  return oracle_surf_acc(x, n, p, y, recip, use_star, is_discrete, i_begin, i_end, n_jobs, 0,
                         scores_out);
}
