// fs_cpu.cpp -- native multithreaded CPU backend (backend='cpu').
//
// Runs the same pipeline as the GPU backend (fs_internal.h): the same
// integer distances, mean correction, thresholds, ambiguous-pair refinement
// and pair weights, on std::threads; only the order of the floating-point
// score accumulation differs.  Built with -ffp-contract=off so the
// quantisation rounds exactly like k_quantize.  This is the product's CPU
// path -- it is NOT the parity oracle (oracle/ restates the reference kernels
// independently and is never linked here).
#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <thread>

#include "../../include/fastselect_amd.h"
#include "fs_internal.h"

namespace fs {
namespace cpu {

template <typename F>
static void parallel_for(int64_t count, int n_jobs, F&& body) {
  const int nt = (int)std::max<int64_t>(1, std::min<int64_t>(hardware_threads(n_jobs), count));
  if (nt <= 1) {
    for (int64_t t = 0; t < count; t++) body(t);
    return;
  }
  std::atomic<int64_t> next{0};
  std::vector<std::thread> th;
  th.reserve(nt);
  for (int w = 0; w < nt; w++)
    th.emplace_back([&]() {
      for (int64_t t = next++; t < count; t = next++) body(t);
    });
  for (auto& t : th) t.join();
}

// 1 if every element of x is finite (no NaN, no infinity), else 0: the
// exponent-all-ones test on the bit patterns, chunks of 1M elements over
// std::threads.
int all_finite(const void* x, int x_is_f64, int64_t count, int n_jobs) {
  constexpr int64_t kChunk = 1 << 20;
  std::atomic<int> bad{0};
  parallel_for((count + kChunk - 1) / kChunk, n_jobs, [&](int64_t c) {
    const int64_t lo = c * kChunk, hi = std::min<int64_t>(count, lo + kChunk);
    bool b = false;
    if (x_is_f64) {
      const uint64_t* u = (const uint64_t*)x;
      for (int64_t i = lo; i < hi; i++) b |= (u[i] & 0x7ff0000000000000ull) == 0x7ff0000000000000ull;
    } else {
      const uint32_t* u = (const uint32_t*)x;
      for (int64_t i = lo; i < hi; i++) b |= (u[i] & 0x7f800000u) == 0x7f800000u;
    }
    if (b) bad.store(1, std::memory_order_relaxed);
  });
  return bad.load() ? 0 : 1;
}

static inline double load_x(const void* x, int x_is_f64, int64_t idx) {
  return x_is_f64 ? ((const double*)x)[idx] : (double)((const float*)x)[idx];
}

// The refinement band from measured pairs, as the GPU backend's
// calibrate_band (32-bit operands only here): kCalibPairs sampled pairs get
// their quantised distance error against the reference's arithmetic (f32
// diffs summed in f64) and the band becomes max(model, 3 max|err| + rms/2).
static double calibrated_band(const Prepared& P, const void* x, int x_is_f64, int n_jobs) {
  if (P.pc == 0 || P.n < 2) return P.amb_delta;
  std::vector<std::pair<int64_t, int64_t>> pr;
  calib_pairs(P.n, P.pc, std::min<int64_t>(kCalibPairs, P.n * (P.n - 1) / 2), pr);
  std::vector<double> err(pr.size(), 0.0);
  std::vector<double> qs(P.pc);
  for (int64_t c = 0; c < P.pc; c++) qs[c] = P.scale[c] * P.SC;
  parallel_for((int64_t)pr.size(), n_jobs, [&](int64_t k) {
    const int64_t i = pr[k].first, j = pr[k].second;
    double e = 0.0;
    for (int64_t c = 0; c < P.pc; c++) {
      const int64_t col = P.src_col[c];
      const double a = load_x(x, x_is_f64, i * P.p_in + col);
      const double b = load_x(x, x_is_f64, j * P.p_in + col);
      const double ta = (a - P.offset[c]) * qs[c], tb = (b - P.offset[c]) * qs[c];
      const uint32_t qa = (uint32_t)(ta + 0.5), qb = (uint32_t)(tb + 0.5);
      const double ref = (double)(std::fabs((float)a - (float)b) * P.recip_in[col]);
      e += (qa > qb ? (double)(qa - qb) : (double)(qb - qa)) - P.SC * ref;
    }
    err[k] = e;
  });
  double ss = 0.0, mx = 0.0;
  for (double e : err) {
    ss += e * e;
    mx = std::max(mx, std::fabs(e));
  }
  return calibrated_delta(P.amb_delta_model > 0.0 ? P.amb_delta_model : P.amb_delta, P.SC,
                          std::sqrt(ss / (double)err.size()), mx);
}

// Same arithmetic as k_quantize (fs_pass1.hip): t = (x - off) * qs,
// q = trunc(t + 0.5), eps = q - t, every double operation rounded separately.
static void quantize(const Prepared& P, const void* x, int x_is_f64, int n_jobs,
                     std::vector<uint32_t>& xq, std::vector<float>& xs,
                     std::vector<float>* eps) {
  xq.assign((size_t)P.n * P.PW, 0);
  xs.assign((size_t)P.n * P.PW, 0.0f);
  if (eps) eps->assign((size_t)P.n * P.PW, 0.0f);
  std::vector<double> qs(P.PW);
  for (int64_t c = 0; c < P.PW; c++) qs[c] = P.scale[c] * P.SC;
  parallel_for(P.n, n_jobs, [&](int64_t i) {
    for (int64_t c = 0; c < P.PW; c++) {
      const int64_t col = P.src_col[c];
      if (col < 0) continue;
      const double xv = load_x(x, x_is_f64, i * P.p_in + col);
      uint32_t q;
      float v;
      if (c < P.pc) {
        const double u = xv - P.offset[c];
        const double t = u * qs[c];
        q = (uint32_t)(t + 0.5);
        v = (float)(u * P.scale[c]);
        if (eps) (*eps)[(size_t)i * P.PW + c] = (float)((double)q - t);
      } else {
        const double* b = P.dtab.data() + P.dtab_off[c];
        const double* e = P.dtab.data() + P.dtab_off[c + 1];
        q = (uint32_t)(std::lower_bound(b, e, xv) - b);
        v = (float)q;
      }
      xq[(size_t)i * P.PW + c] = q;
      xs[(size_t)i * P.PW + c] = v;
    }
  });
}

static inline bool owned(int64_t nb, int64_t i, int64_t j, int rank, int world) {
  if (world == 1) return true;
  int64_t a = i / kTile, b = j / kTile;
  if (a > b) std::swap(a, b);
  return tile_linear(nb, a, b) % world == rank;
}

static void distances(const Prepared& P, const std::vector<uint32_t>& xq, int rank, int world,
                      int n_jobs, std::vector<double>& D) {
  const int64_t n = P.n, nb = P.n_pad / kTile;
  D.assign((size_t)n * n, 0.0);
  std::vector<int32_t> bi, bj;
  owned_tiles(nb, rank, world, bi, bj);
  parallel_for((int64_t)bi.size(), n_jobs, [&](int64_t t) {
    const int64_t i0 = (int64_t)bi[t] * kTile, j0 = (int64_t)bj[t] * kTile;
    for (int64_t i = i0; i < std::min(i0 + kTile, n); i++) {
      const uint32_t* a = xq.data() + (size_t)i * P.PW;
      for (int64_t j = std::max(j0, bi[t] == bj[t] ? i : j0); j < std::min(j0 + kTile, n); j++) {
        const uint32_t* b = xq.data() + (size_t)j * P.PW;
        uint64_t d = 0;
        for (int64_t c = 0; c < P.PC; c++) d += a[c] > b[c] ? a[c] - b[c] : b[c] - a[c];
        uint64_t mism = 0;
        for (int64_t c = P.PC; c < P.PW; c++) mism += a[c] != b[c];
        d += mism * (uint64_t)P.SCu;
        D[(size_t)i * n + j] = (double)d;
        D[(size_t)j * n + i] = (double)d;
      }
    }
  });
}

// Mean correction of k_colsort / k_rowcorr (fs_colsort.hip), the same
// integer arithmetic: every continuous column is ordered by t (colsort_key).
// Binned on the key's top gpu::colsort_bin_bits(n) bits, a sample is ordered exactly against every
// other bin by the bin counts and fixed-point eps sums, and within its own
// bin against its neighbours' low key bits (their eps at 2^-12 of a quantum,
// equal keys tied; a bin whose samples share one key needs nothing); a
// column with a mixed bin fuller than kColsortMaxFill is sorted whole instead (std::sort on (key, index), as the GPU's stable sort),
// where position k, the eps prefix P before it and the column total T give
//   term_i = eps_i (2k - n) - 2 P + T.
// Either way term_i = eps_i (L - G) - (E_below - E_above), and
// corr[i] = sum_c term_ic: bit-identical terms to the GPU's.  The correction
// of the continuous columns [c_lo, c_hi) (a rank's share; the shares are
// summed across ranks with the row moments).
static void mean_correction(const Prepared& P, const std::vector<uint32_t>& xq,
                            const std::vector<float>& eps, int64_t c_lo, int64_t c_hi,
                            int n_jobs, std::vector<double>& corr) {
  const int64_t n = P.n;
  const int s = colsort_key_shift(P.qmax);
  // the GPU's route for this n: binned columns (k_colsort) up to 24576
  // samples, beyond that (or under the colsort_global test hook) every column sorted
  // whole by the device segmented sort -- position terms, ties by index
  const bool binned = gpu::colsort_lds(n);
  const int bins = 1 << gpu::colsort_bin_bits(n), shift = 32 - gpu::colsort_bin_bits(n);
  const uint32_t low_mask = (1u << shift) - 1u;
  std::vector<float> term((size_t)n * std::max<int64_t>(P.pc, 1), 0.0f);
  parallel_for(c_hi - c_lo, n_jobs, [&](int64_t cc) {
    const int64_t c = c_lo + cc;
    constexpr double kFx = 16777216.0;  // eps fixed point 2^24, as k_colsort
    std::vector<uint32_t> key((size_t)n);
    std::vector<int64_t> fx((size_t)n);
    std::vector<int64_t> cnt(bins + 1, 0), esum(bins + 1, 0);
    // per bin: first low key seen, and whether another one followed (mixed)
    std::vector<uint32_t> first(bins, 0xFFFFFFFFu);
    std::vector<char> mixed(bins, 0);
    int64_t T = 0;
    for (int64_t i = 0; i < n; i++) {
      fx[i] = colsort_fx(eps[(size_t)i * P.PW + c]);
      key[i] = colsort_key(xq[(size_t)i * P.PW + c], (int32_t)fx[i], s);
      const uint32_t b = key[i] >> shift, kl = key[i] & low_mask;
      cnt[b + 1]++;
      esum[b + 1] += fx[i];
      T += fx[i];
      if (first[b] == 0xFFFFFFFFu) first[b] = kl;
      else if (first[b] != kl) mixed[b] = 1;
    }
    int64_t fill = 0;
    for (int b = 0; b < bins; b++) {
      if (mixed[b]) fill = std::max(fill, cnt[b + 1]);
      cnt[b + 1] += cnt[b];     // exclusive prefix at b, inclusive at b + 1
      esum[b + 1] += esum[b];
    }
    if (fill > kColsortMaxFill || !binned) {
      std::vector<uint64_t> ord((size_t)n);
      for (int64_t i = 0; i < n; i++) ord[i] = ((uint64_t)key[i] << 32) | (uint64_t)i;
      std::sort(ord.begin(), ord.end());
      int64_t Pk = 0;
      for (int64_t k = 0; k < n; k++) {
        const int64_t i = (int64_t)(ord[k] & 0xFFFFFFFFull);
        term[(size_t)i * P.pc + c] = (float)((double)(fx[i] * (2 * k - n) - 2 * Pk + T) / kFx);
        Pk += fx[i];
      }
      return;
    }
    // the samples of bins holding >= 2, in bin order (low key bits, eps code)
    std::vector<uint32_t> seg((size_t)n), cur(cnt.begin(), cnt.end() - 1);
    for (int64_t i = 0; i < n; i++) {
      const uint32_t b = key[i] >> shift;
      if (cnt[b + 1] - cnt[b] < 2 || !mixed[b]) continue;
      seg[cur[b]++] = ((key[i] & low_mask) << 12) | colsort_eq12((int32_t)fx[i]);
    }
    for (int64_t i = 0; i < n; i++) {
      const uint32_t b = key[i] >> shift;
      int64_t L = cnt[b], G = n - cnt[b + 1], Eb = esum[b], Ea = T - esum[b + 1];
      if (cnt[b + 1] - cnt[b] >= 2 && mixed[b]) {  // a pure bin's samples all tie
        const uint32_t mine = key[i] & low_mask;
        for (int64_t j = cnt[b]; j < cnt[b + 1]; j++) {
          const uint32_t kl = seg[j] >> 12;
          const int64_t q = colsort_eq12_fx(seg[j] & 0xFFFu);
          if (kl < mine) {
            L++;
            Eb += q;
          } else if (kl > mine) {
            G++;
            Ea += q;
          }
        }
      }
      term[(size_t)i * P.pc + c] = (float)((double)(fx[i] * (L - G) - (Eb - Ea)) / kFx);
    }
  });
  corr.assign(n, 0.0);
  for (int64_t i = 0; i < n; i++) {
    double s = 0.0;
    for (int64_t c = c_lo; c < c_hi; c++) s += (double)term[(size_t)i * P.pc + c];
    corr[i] = s;
  }
}

// Reference-exact distance of one pair (same arithmetic as k_exact_pairs):
// float32 diffs for float32 X (MultiSURF.py:184-187, ReliefF.py:151-154),
// float64 diffs for float64 X (SURF.py:153-156), summed in float64.
static double exact_pair(const Prepared& P, const void* x, int x_is_f64, int64_t i, int64_t j) {
  double acc = 0.0;
  for (int64_t c = 0; c < P.pc; c++) {
    const int64_t col = P.src_col[c];
    if (x_is_f64) {
      const double* X = (const double*)x;
      acc += std::fabs(X[i * P.p_in + col] - X[j * P.p_in + col]) * P.scale[c];
    } else {
      const float* X = (const float*)x;
      const float dv = std::fabs(X[i * P.p_in + col] - X[j * P.p_in + col]) * (float)P.scale[c];
      acc += (double)dv;
    }
  }
  for (int64_t c = P.PC; c < P.PC + P.pd; c++) {
    const int64_t col = P.src_col[c];
    acc += load_x(x, x_is_f64, i * P.p_in + col) != load_x(x, x_is_f64, j * P.p_in + col) ? 1.0
                                                                                          : 0.0;
  }
  return acc;
}

// Flag and refine the ambiguous owned pairs (k_flag_pairs + k_exact_pairs).
template <typename Amb>
static int64_t refine_pairs(const Prepared& P, const void* x, int x_is_f64, int rank, int world,
                            int n_jobs, std::vector<double>& D, Amb&& ambiguous,
                            std::vector<std::pair<int32_t, int32_t>>* refined = nullptr) {
  const int64_t n = P.n, nb = P.n_pad / kTile;
  std::vector<std::pair<int32_t, int32_t>> pairs;
  std::mutex mu;
  parallel_for(n, n_jobs, [&](int64_t i) {
    std::vector<std::pair<int32_t, int32_t>> loc;
    for (int64_t j = i + 1; j < n; j++)
      if (owned(nb, i, j, rank, world) && ambiguous(i, j, D[(size_t)i * n + j]))
        loc.push_back({(int32_t)i, (int32_t)j});
    if (!loc.empty()) {
      std::lock_guard<std::mutex> g(mu);
      pairs.insert(pairs.end(), loc.begin(), loc.end());
    }
  });
  parallel_for((int64_t)pairs.size(), n_jobs, [&](int64_t k) {
    const int64_t i = pairs[k].first, j = pairs[k].second;
    const double v = exact_pair(P, x, x_is_f64, i, j) * P.SC;
    D[(size_t)i * n + j] = v;
    D[(size_t)j * n + i] = v;
  });
  if (refined) *refined = pairs;
  return (int64_t)pairs.size();
}

// exact_thresholds (fs_select.hip): thresholds from exact distances for the
// rows a refined pair lies within thr_tol of, when at most exact_thr_rows(n, p)
// (every row under the thr_exact_all test hook, fs_test_hook).
static void exact_thresholds(const Prepared& P, const void* x, int n_jobs, const CpuState& S,
                             const std::vector<std::pair<int32_t, int32_t>>& refined,
                             double thr_tol, std::vector<double>& thr) {
  const int64_t n = P.n;
  std::vector<int32_t> rows;
  if (test_hooks().thr_exact_all) {
    for (int64_t i = 0; i < n; i++) rows.push_back((int32_t)i);
  } else {
    std::vector<uint8_t> unc((size_t)n, 0);
    for (const auto& pr : refined) {
      const double v = S.D[(size_t)pr.first * n + pr.second];
      if (std::fabs(v - thr[pr.first]) < thr_tol) unc[pr.first] = 1;
      if (std::fabs(v - thr[pr.second]) < thr_tol) unc[pr.second] = 1;
    }
    for (int64_t i = 0; i < n; i++)
      if (unc[i]) rows.push_back((int32_t)i);
    if ((int64_t)rows.size() > exact_thr_rows(n, P.pc + P.pd)) return;
  }
  parallel_for((int64_t)rows.size(), n_jobs, [&](int64_t k) {
    const int64_t i = rows[k];
    double s1 = 0.0, s2 = 0.0;
    for (int64_t j = 0; j < n; j++) {
      if (j == i) continue;
      const double d = exact_pair(P, x, 0, i, j);
      s1 += d;
      s2 += d * d;
    }
    thr[i] = multisurf_threshold(s1, s2, n) * P.SC;
  });
}

int multisurf_pass1(const Prepared& P, const void* x, int rank, int world, int n_jobs,
                    CpuState& S, double* rowstats) {
  std::vector<uint32_t> xq;
  std::vector<float> eps;
  quantize(P, x, 0, n_jobs, xq, S.xs, &eps);
  mean_correction(P, xq, eps, P.pc * rank / world, P.pc * (rank + 1) / world, n_jobs, S.corr);
  distances(P, xq, rank, world, n_jobs, S.D);
  const int64_t n = P.n, nb = P.n_pad / kTile;
  parallel_for(n, n_jobs, [&](int64_t i) {
    double s1 = 0.0, s2 = 0.0;
    for (int64_t j = 0; j < n; j++) {
      if (j == i || !owned(nb, i, j, rank, world)) continue;
      const double d = S.D[(size_t)i * n + j];
      s1 += d;
      s2 += d * d;
    }
    rowstats[3 * i] = s1;
    rowstats[3 * i + 1] = s2;
    rowstats[3 * i + 2] = S.corr[i];
  });
  return FS_OK;
}

int multisurf_select(const Prepared& P, const void* x, int rank, int world,
                     const double* rowstats, int n_jobs, CpuState& S, double* counts) {
  const int64_t n = P.n, nb = P.n_pad / kTile;
  S.thr.assign(n, 0.0);
  const double nm1 = (double)(n - 1);
  for (int64_t i = 0; i < n; i++) {  // k_thr_ms
    const double mu = rowstats[3 * i] / nm1;
    double var = rowstats[3 * i + 1] / nm1 - mu * mu;
    if (var < 0.0) var = 0.0;
    S.thr[i] = (mu - rowstats[3 * i + 2] / nm1) - 0.5 * std::sqrt(var);
  }
  const double dq = calibrated_band(P, x, 0, n_jobs) * P.SC;
  std::vector<std::pair<int32_t, int32_t>> refined;
  S.refined = refine_pairs(
      P, x, 0, rank, world, n_jobs, S.D,
      [&](int64_t i, int64_t j, double d) {
        return std::fabs(d - S.thr[i]) < dq || std::fabs(d - S.thr[j]) < dq;
      },
      &refined);
  exact_thresholds(P, x, n_jobs, S, refined, dq / std::sqrt((double)std::max<int64_t>(n - 1, 1)) + 2.0,
                   S.thr);
  parallel_for(n, n_jobs, [&](int64_t i) {  // k_count_ms
    double h = 0.0, m = 0.0;
    for (int64_t j = 0; j < n; j++) {
      if (j == i || !owned(nb, i, j, rank, world)) continue;
      if (S.D[(size_t)i * n + j] < S.thr[i]) {
        if (P.labels[j] == P.labels[i]) h += 1.0;
        else m += 1.0;
      }
    }
    counts[2 * i] = h;
    counts[2 * i + 1] = m;
  });
  return FS_OK;
}

// S_c = sum over owned pairs i < j of w_ij * |xs_ic - xs_jc| (or the
// mismatch indicator for discrete columns), w_ij already combined.
struct PairW {
  int32_t i, j;
  float w;
};

static void weighted_sum(const Prepared& P, const std::vector<float>& xs,
                         const std::vector<PairW>& pairs, int n_jobs, double* S_perm) {
  const int64_t nblk = (P.PW + 63) / 64;
  parallel_for(nblk, n_jobs, [&](int64_t blk) {
    const int64_t c0 = blk * 64, c1 = std::min<int64_t>(c0 + 64, P.PW);
    double acc[64] = {0};
    for (const PairW& pw : pairs) {
      const float* a = xs.data() + (size_t)pw.i * P.PW;
      const float* b = xs.data() + (size_t)pw.j * P.PW;
      for (int64_t c = c0; c < c1; c++) {
        const float d = c < P.PC ? std::fabs(a[c] - b[c]) : (a[c] != b[c] ? 1.0f : 0.0f);
        acc[c - c0] += (double)pw.w * (double)d;
      }
    }
    for (int64_t c = c0; c < c1; c++) S_perm[c] = acc[c - c0];
  });
}

static void scatter_scores(const Prepared& P, const std::vector<double>& S_perm,
                           double* scores) {
  for (int64_t k = 0; k < P.n_kept; k++) scores[k] = 0.0;
  for (int64_t c = 0; c < P.PW; c++)
    if (P.out_pos[c] >= 0) scores[P.out_pos[c]] = S_perm[c];
}

// The reference's diff of kept feature k between samples i and j
// (MultiSURF.py:184-187, ReliefF.py:151-154): float32 |x_i - x_j| * recip,
// or 1 / 0 for a discrete feature.
static inline float ref_diff(const Prepared& P, const float* X, int64_t i, int64_t j, int64_t k) {
  const int64_t col = P.kept_col[k];
  const float a = X[i * P.p_in + col], b = X[j * P.p_in + col];
  if (P.disc_in[col]) return a != b ? 1.0f : 0.0f;
  return std::fabs(a - b) * P.recip_in[col];
}

// temp[:, k].sum() of the reference (numba's float32 .sum(): sequential,
// MultiSURF.py:252-253, ReliefF.py:219-220) over rows [0, rows).
static void ref_column_sums(const std::vector<float>& temp, int64_t rows, int64_t nk,
                            double* scores) {
  for (int64_t k = 0; k < nk; k++) {
    float s = 0.0f;
    for (int64_t r = 0; r < rows; r++) s += temp[(size_t)r * nk + k];
    scores[k] = (double)s;
  }
}

// Reference-order pass 2 (P.ref_accum; fs_refacc.hip k_ms_chains): per focal
// sample the float32 hit / miss chains over j in ascending order, the
// float64 division rounded to float32, temp = miss - hit in float32, then
// the float32 column sums over the focal rows (MultiSURF.py:198-253).
static int multisurf_pass2_ref(const Prepared& P, const float* X, const CpuState& S,
                               const double* counts, int n_jobs, int64_t r_lo, int64_t r_hi,
                               double* scores) {
  const int64_t n = P.n, nk = P.n_kept, rows = r_hi - r_lo;
  std::vector<float> temp((size_t)std::max<int64_t>(rows, 0) * nk);
  parallel_for(rows, n_jobs, [&](int64_t r) {
    const int64_t i = r_lo + r;
    std::vector<float> hit((size_t)nk, 0.0f), miss((size_t)nk, 0.0f);
    for (int64_t j = 0; j < n; j++) {
      if (j == i) continue;
      const bool near = S.D[(size_t)i * n + j] < S.thr[i];
      const bool is_hit = P.labels[j] == P.labels[i];
      if (near) {
        float* acc = is_hit ? hit.data() : miss.data();
        for (int64_t k = 0; k < nk; k++) acc[k] += ref_diff(P, X, i, j, k);
      } else if (P.use_star && !is_hit) {
        for (int64_t k = 0; k < nk; k++) miss[k] -= ref_diff(P, X, i, j, k);
      }
    }
    const double H = counts[2 * i], M = counts[2 * i + 1];
    float* row = temp.data() + (size_t)r * nk;
    for (int64_t k = 0; k < nk; k++) {
      const float h = H > 0.0 ? (float)((double)hit[k] / H) : hit[k];
      const float m = M > 0.0 ? (float)((double)miss[k] / M) : miss[k];
      row[k] = m - h;
    }
  });
  ref_column_sums(temp, rows, nk, scores);
  return FS_OK;
}

int multisurf_pass2(const Prepared& P, const void* x, const CpuState& S, const double* counts,
                    int rank, int world, int n_jobs, int64_t r_lo, int64_t r_hi, double* scores) {
  if (P.ref_accum) {
    if (world != 1 || !x) {
      set_error("reference-order accumulation: pass 2 needs every pair's decisions (world 1)");
      return FS_ENOTSUP;
    }
    return multisurf_pass2_ref(P, (const float*)x, S, counts, n_jobs, r_lo, r_hi, scores);
  }
  const int64_t n = P.n, nb = P.n_pad / kTile;
  std::vector<PairW> pairs;
  for (int64_t i = 0; i < n; i++)
    for (int64_t j = i + 1; j < n; j++) {
      if (!owned(nb, i, j, rank, world)) continue;
      const double d = S.D[(size_t)i * n + j];
      const bool hit = P.labels[i] == P.labels[j];
      const double wi =
          (i >= r_lo && i < r_hi)
              ? multisurf_weight(d < S.thr[i], hit, P.use_star, counts[2 * i], counts[2 * i + 1])
              : 0.0;
      const double wj =
          (j >= r_lo && j < r_hi)
              ? multisurf_weight(d < S.thr[j], hit, P.use_star, counts[2 * j], counts[2 * j + 1])
              : 0.0;
      const float w = (float)(wi + wj);
      if (w != 0.0f) pairs.push_back({(int32_t)i, (int32_t)j, w});
    }
  std::vector<double> Sp(P.PW, 0.0);
  weighted_sum(P, S.xs, pairs, n_jobs, Sp.data());
  scatter_scores(P, Sp, scores);
  return FS_OK;
}

int surf_run(const Prepared& P, const void* x, int n_jobs, int64_t r_lo, int64_t r_hi,
             double* scores) {
  // SURF compares float32-rounded distances with a float32 sequential mean,
  // so distances are accumulated in float64 from float64 diffs (as
  // k_dist_f64 does; exact to ~1e-16, SURF.py:146-160) rather than quantised.
  std::vector<uint32_t> xq;
  std::vector<float> xs;
  quantize(P, x, 1, n_jobs, xq, xs, nullptr);
  const int64_t n = P.n;
  std::vector<float> Df((size_t)n * n, 0.0f);
  parallel_for(n, n_jobs, [&](int64_t i) {
    for (int64_t j = i + 1; j < n; j++) {
      const float d = (float)exact_pair(P, x, 1, i, j);
      Df[(size_t)i * n + j] = d;
      Df[(size_t)j * n + i] = d;
    }
  });
  // float32 sequential mean (SURF.py:162-163)
  std::vector<double> avg(n);
  parallel_for(n, n_jobs, [&](int64_t i) {
    if (i < r_lo || i >= r_hi) return;  // not a focal sample of this call
    float s = 0.0f;
    for (int64_t j = 0; j < n; j++) s += Df[(size_t)i * n + j];
    avg[i] = (double)s / (double)(n - 1);
  });
  if (P.ref_accum) {
    // the reference's n_jobs = 1 order (fs_refacc.hip k_surf_chains): per
    // focal sample four float32 chains over ascending j of the float32-stored
    // float64 diffs, score_update in float32, then the float32 column sums
    // (SURF.py:165-195, 216)
    const double* X = (const double*)x;
    const int64_t nk = P.n_kept, rows = r_hi - r_lo;
    std::vector<float> temp((size_t)std::max<int64_t>(rows, 0) * nk);
    parallel_for(rows, n_jobs, [&](int64_t r) {
      const int64_t i = r_lo + r;
      std::vector<float> acc((size_t)4 * nk, 0.0f);  // near hit, near miss, far hit, far miss
      for (int64_t j = 0; j < n; j++) {
        if (j == i) continue;
        const bool near = (double)Df[(size_t)i * n + j] < avg[i];
        const bool hit = P.labels[j] == P.labels[i];
        if (!near && !P.use_star) continue;
        float* a = acc.data() + (size_t)((near ? 0 : 2) + (hit ? 0 : 1)) * nk;
        for (int64_t k = 0; k < nk; k++) {
          const int64_t col = P.kept_col[k];
          const double u = X[i * P.p_in + col], v = X[j * P.p_in + col];
          a[k] += P.disc_in[col] ? (u != v ? 1.0f : 0.0f)
                                 : (float)(std::fabs(u - v) * (double)P.recip_in[col]);
        }
      }
      float* row = temp.data() + (size_t)r * nk;
      for (int64_t k = 0; k < nk; k++) {
        float u = acc[nk + k] - acc[k];
        if (P.use_star) u += acc[2 * nk + k] - acc[3 * nk + k];
        row[k] = u;
      }
    });
    ref_column_sums(temp, rows, nk, scores);
    return FS_OK;
  }
  std::vector<PairW> pairs;
  for (int64_t i = 0; i < n; i++)
    for (int64_t j = i + 1; j < n; j++) {
      const double df = (double)Df[(size_t)i * n + j];
      const bool hit = P.labels[i] == P.labels[j];
      // each side counts only for the focal samples [r_lo, r_hi)
      const double wi = (i >= r_lo && i < r_hi) ? surf_weight(df < avg[i], hit, P.use_star) : 0.0;
      const double wj = (j >= r_lo && j < r_hi) ? surf_weight(df < avg[j], hit, P.use_star) : 0.0;
      const float w = (float)(wi + wj);
      if (w != 0.0f) pairs.push_back({(int32_t)i, (int32_t)j, w});
    }
  std::vector<double> S(P.PW, 0.0);
  weighted_sum(P, xs, pairs, n_jobs, S.data());
  scatter_scores(P, S, scores);
  return FS_OK;
}

// The reference's float32 distance key of (i, j) (ReliefF.py:145-155):
// float32 diffs accumulated in float64 in feature order, stored as float32.
static float relieff_exact_key(const Prepared& P, const float* x, int64_t i, int64_t j) {
  const float* xi = x + i * P.p_in;
  const float* xj = x + j * P.p_in;
  double d = 0.0;
  for (int64_t f : P.kept_col) {  // the scored features, in their order
    if (P.disc_in[f]) d += xi[f] != xj[f] ? 1.0 : 0.0;
    else d += (double)(std::fabs(xi[f] - xj[f]) * P.recip_in[f]);
  }
  return (float)d;
}

// ReliefF neighbour selection for focal row i (ReliefF.py:157-175), same
// pipeline as the GPU: quantised keys, exact keys for every candidate near
// a class's k-th distance, then -- only when several candidates share the
// k-th distance exactly -- numba's quicksort order over the exact row.
// nbr[c] receives the chosen neighbours of class c.
static void relieff_select_row(const Prepared& P, const float* x, const std::vector<double>& D,
                               int64_t i, double amb, std::vector<std::vector<int32_t>>& nbr) {
  const int64_t n = P.n, k = P.k_neighbors;
  const int C = P.n_classes;
  const double inv_sc = 1.0 / P.SC;
  std::vector<float> key((size_t)n);
  for (int64_t j = 0; j < n; j++) key[j] = (float)(D[(size_t)i * n + j] * inv_sc);
  key[i] = INFINITY;
  const int32_t li = P.labels[i];
  std::vector<std::vector<int32_t>> members(C);
  for (int64_t j = 0; j < n; j++)
    if (j != i) members[P.labels[j]].push_back((int32_t)j);
  std::vector<float> T(C, INFINITY);
  std::vector<int64_t> need(C, 0), eq(C, 0);
  std::vector<uint8_t> exact((size_t)n, 0);
  auto kth = [&](int c, int64_t kc) {
    std::vector<float> v;
    v.reserve(members[c].size());
    for (int32_t j : members[c]) v.push_back(key[j]);
    std::nth_element(v.begin(), v.begin() + (kc - 1), v.end());
    return v[kc - 1];
  };
  bool tie = false;
  for (int c = 0; c < C; c++) {
    const int64_t kc = std::min<int64_t>(k, (int64_t)members[c].size());
    if (kc == 0 || kc == (int64_t)members[c].size()) continue;  // take all
    // exact keys for every candidate within the quantisation band of T
    const float t0 = kth(c, kc);
    const double band = 2.0 * (amb + (double)t0 * 1.2e-7);
    for (int32_t j : members[c])
      if (std::fabs((double)key[j] - (double)t0) <= band) {
        key[j] = relieff_exact_key(P, x, i, j);
        exact[j] = 1;
      }
    T[c] = kth(c, kc);
    int64_t lt = 0;
    for (int32_t j : members[c]) {
      lt += key[j] < T[c];
      eq[c] += key[j] == T[c];
    }
    need[c] = kc - lt;
    tie = tie || eq[c] > need[c];
  }
  std::vector<std::vector<int32_t>> tied(C);
  if (tie) {
    // numba's order decides: replay its quicksort over the exact row
    if (P.pc > 0)
      for (int64_t j = 0; j < n; j++)
        if (j != i && !exact[j]) key[j] = relieff_exact_key(P, x, i, j);
    std::vector<int32_t> R((size_t)n);
    for (int64_t j = 0; j < n; j++) R[j] = (int32_t)j;
    auto is_tied = [&](int32_t j) {
      const int c = P.labels[j];
      return j != i && eq[c] > need[c] && key[j] == T[c];
    };
    numba_argsort_focus(n, R.data(), [&](int32_t j) { return key[j]; },
                        [&](int64_t lo, int64_t hi) {
                          for (int64_t t = lo; t <= hi; t++)
                            if (is_tied(R[t])) return true;
                          return false;
                        });
    for (int64_t t = 0; t < n; t++)
      if (is_tied(R[t])) tied[P.labels[R[t]]].push_back(R[t]);
  }
  for (int c = 0; c < C; c++) {
    nbr[c].clear();
    const int64_t kc = std::min<int64_t>(k, (int64_t)members[c].size());
    if (kc == (int64_t)members[c].size()) {
      nbr[c] = members[c];
      continue;
    }
    for (int32_t j : members[c])
      if (key[j] < T[c]) nbr[c].push_back(j);
    if (eq[c] > need[c]) {
      for (int64_t t = 0; t < need[c]; t++) nbr[c].push_back(tied[c][t]);
    } else {
      for (int32_t j : members[c])
        if (key[j] == T[c]) nbr[c].push_back(j);
    }
  }
  (void)li;
}

// Reference order of ReliefF's neighbour lists (nbr[c], ascending keys
// nkey[c]): every run of equal keys re-ordered as numba's quicksort argsort
// of row i's exact keys orders those samples (numba_argsort_focus, focused on
// them: the relative order of the focus samples is numba's exactly).
static void ref_tie_order(const Prepared& P, const float* X, int64_t i,
                          const std::vector<std::vector<float>>& nkey,
                          std::vector<std::vector<int32_t>>& nbr) {
  const int64_t n = P.n;
  std::vector<float> key((size_t)n);
  for (int64_t j = 0; j < n; j++) key[j] = j == i ? INFINITY : relieff_exact_key(P, X, i, j);
  std::vector<uint8_t> focus((size_t)n, 0);
  for (size_t c = 0; c < nbr.size(); c++)
    for (size_t t = 1; t < nbr[c].size(); t++)
      if (nkey[c][t] == nkey[c][t - 1]) focus[nbr[c][t]] = focus[nbr[c][t - 1]] = 1;
  std::vector<int32_t> R((size_t)n);
  for (int64_t j = 0; j < n; j++) R[j] = (int32_t)j;
  numba_argsort_focus(n, R.data(), [&](int32_t j) { return key[j]; },
                      [&](int64_t lo, int64_t hi) {
                        for (int64_t t = lo; t <= hi; t++)
                          if (focus[R[t]]) return true;
                        return false;
                      });
  std::vector<int64_t> pos((size_t)n, 0);
  for (int64_t t = 0; t < n; t++) pos[R[t]] = t;
  for (size_t c = 0; c < nbr.size(); c++) {
    std::vector<int32_t>& L = nbr[c];
    for (size_t s = 0; s < L.size();) {
      size_t e = s + 1;
      while (e < L.size() && nkey[c][e] == nkey[c][s]) e++;
      std::sort(L.begin() + s, L.begin() + e,
                [&](int32_t a, int32_t b) { return pos[a] < pos[b]; });
      s = e;
    }
  }
}

// Whether another order of row i's tied lists could change their float64
// sums (as k_rf_ref_order_matters): a list whose float32 diffs at some
// feature are multiples of u = ulp(smallest non-zero diff) summing below
// 2^53 u has every partial sum exact, in any order.
static bool ref_order_matters(const Prepared& P, const float* X, int64_t i,
                              const std::vector<std::vector<float>>& nkey,
                              const std::vector<std::vector<int32_t>>& nbr) {
  for (size_t c = 0; c < nbr.size(); c++) {
    bool run = false;
    for (size_t t = 1; t < nbr[c].size(); t++) run = run || nkey[c][t] == nkey[c][t - 1];
    if (!run) continue;
    for (int64_t f = 0; f < P.n_kept; f++) {
      float vmin = INFINITY;
      double s = 0.0;
      for (int32_t j : nbr[c]) {
        const float v = ref_diff(P, X, i, j, f);
        if (v > 0.0f && v < vmin) vmin = v;
        s += (double)v;
      }
      if (vmin == INFINITY) continue;
      int e;
      (void)std::frexp(vmin, &e);
      if (s >= std::ldexp(1.0, e - 24 + 53)) return true;
    }
  }
  return false;
}

int relieff_run(const Prepared& P, const void* x, int n_jobs, int64_t r_lo, int64_t r_hi,
                double* scores) {
  std::vector<uint32_t> xq;
  std::vector<float> xs;
  std::vector<double> D;
  quantize(P, x, 0, n_jobs, xq, xs, nullptr);
  distances(P, xq, 0, 1, n_jobs, D);
  const int64_t n = P.n, k = P.k_neighbors;
  const int C = P.n_classes;
  const double amb = calibrated_band(P, x, 0, n_jobs);
  if (P.ref_accum) {
    // the reference's order (ReliefF.py:157-220): each class's neighbours in
    // argsort order (exact float32 keys ascending; equal keys by index, see
    // fs_refacc.hip k_rf_ref_sort), float64 sums in that order, temp =
    // f32(update), float32 column sums
    const float* X = (const float*)x;
    const int64_t nk = P.n_kept, rows = r_hi - r_lo;
    std::vector<float> temp((size_t)std::max<int64_t>(rows, 0) * nk);
    parallel_for(rows, n_jobs, [&](int64_t r) {
      const int64_t i = r_lo + r;
      std::vector<std::vector<int32_t>> nbr(C);
      relieff_select_row(P, X, D, i, amb, nbr);
      std::vector<std::vector<float>> nkey(C);
      bool dup = false;
      for (int c = 0; c < C; c++) {
        std::vector<std::pair<float, int32_t>> kv;
        for (int32_t j : nbr[c]) kv.push_back({relieff_exact_key(P, X, i, j), j});
        std::sort(kv.begin(), kv.end());
        for (size_t t = 0; t < kv.size(); t++) {
          nbr[c][t] = kv[t].second;
          nkey[c].push_back(kv[t].first);
          dup = dup || (t > 0 && kv[t].first == kv[t - 1].first);
        }
      }
      // Neighbours of one list at the same key: the reference takes them in
      // numba's quicksort order of the whole row (ReliefF.py:157-175), which
      // decides the order of its float64 sums below (ReliefF.py:181-207).
      // With continuous features that order can change a sum's rounding, so
      // replay the quicksort over the row's exact keys (as k_rf_ref_ties
      // does) when it can (ref_order_matters); 0 / 1 diffs of an
      // all-discrete layout add exactly in any order.
      if (dup && P.pc > 0 &&
          (test_hooks().rf_ref_replay || ref_order_matters(P, X, i, nkey, nbr)))
        ref_tie_order(P, X, i, nkey, nbr);
      const int32_t li = P.labels[i];
      double denom = 1.0 - P.class_prior[li];
      if (denom == 0.0) denom = 1.0;
      const int64_t kc_own = (int64_t)nbr[li].size();
      const int64_t h_found = kc_own < k ? kc_own + 1 : k;
      float* row = temp.data() + (size_t)r * nk;
      for (int64_t f = 0; f < nk; f++) {
        double hit_sum = 0.0, miss_sum = 0.0;
        for (int c = 0; c < C; c++) {
          double s = 0.0;
          for (int32_t j : nbr[c]) s += (double)ref_diff(P, X, i, j, f);
          if (c == li) hit_sum = s;
          else miss_sum += (P.class_prior[c] / denom) * s;
        }
        double update = 0.0;
        if (h_found > 0) update -= hit_sum / (double)h_found;
        if (k > 0) update += miss_sum / (double)k;
        row[f] = (float)update;
      }
    });
    ref_column_sums(temp, rows, nk, scores);
    return FS_OK;
  }
  // per-row partial sums, folded in row order for determinism
  std::vector<double> part((size_t)n * P.PW, 0.0);
  parallel_for(n, n_jobs, [&](int64_t i) {
    if (i < r_lo || i >= r_hi) return;  // not a focal sample of this call
    std::vector<std::vector<int32_t>> nbr(C);
    relieff_select_row(P, (const float*)x, D, i, amb, nbr);
    const int32_t li = P.labels[i];
    double denom = 1.0 - P.class_prior[li];
    if (denom == 0.0) denom = 1.0;
    double* out = part.data() + (size_t)i * P.PW;
    const float* a = xs.data() + (size_t)i * P.PW;
    for (int c = 0; c < C; c++) {
      const std::vector<int32_t>& v = nbr[c];
      const int64_t kc = (int64_t)v.size();
      if (kc == 0) continue;
      // self is a zero-diff hit when its class has < k other members
      // (ReliefF.py:144-168: dists[i] = inf sorts last but is still scanned)
      const int64_t h_found = kc < k ? kc + 1 : k;
      const double wgt =
          (c == li) ? -1.0 / (double)h_found : (P.class_prior[c] / denom) / (double)k;
      for (int64_t col = 0; col < P.PW; col++) {
        double s = 0.0;
        for (int64_t t = 0; t < kc; t++) {
          const float* b = xs.data() + (size_t)v[t] * P.PW;
          s += col < P.PC ? (double)std::fabs(a[col] - b[col]) : (a[col] != b[col] ? 1.0 : 0.0);
        }
        out[col] += wgt * s;
      }
    }
  });
  std::vector<double> S(P.PW, 0.0);
  for (int64_t i = 0; i < n; i++)
    for (int64_t c = 0; c < P.PW; c++) S[c] += part[(size_t)i * P.PW + c];
  scatter_scores(P, S, scores);
  return FS_OK;
}

}  // namespace cpu
}  // namespace fs
