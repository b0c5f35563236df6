// fs_cpu.cpp -- native multithreaded CPU backend (backend='cpu').
//
// Runs the same pipeline as the GPU backend (fs_internal.h) with the same
// integer distances, thresholds and pair weights, on std::threads; only the
// order of the floating-point score accumulation differs.  Built with
// -ffp-contract=off so the quantisation rounds exactly like k_quantize.  This is the
// product's CPU path -- it is NOT the parity oracle (oracle/ restates the
// reference kernels independently and is never linked here).
#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdlib>
#include <cstring>
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

static inline double load_x(const void* x, int x_is_f64, int64_t idx) {
  return x_is_f64 ? ((const double*)x)[idx] : (double)((const float*)x)[idx];
}

// Same arithmetic as k_quantize (fs_gpu.hip): q = trunc((x - off) * qs + 0.5)
// with every double operation rounded separately.
static void quantize(const Prepared& P, const void* x, int x_is_f64, int n_jobs,
                     std::vector<uint32_t>& xq, std::vector<float>& xs) {
  xq.assign((size_t)P.n * P.PW, 0);
  xs.assign((size_t)P.n * P.PW, 0.0f);
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
        double t = u * qs[c];
        t = t + 0.5;
        q = (uint32_t)t;
        v = (float)(u * P.scale[c]);
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

static void distances(const Prepared& P, const std::vector<uint32_t>& xq, int rank, int world,
                      int n_jobs, std::vector<uint64_t>& D) {
  const int64_t n = P.n, nb = P.n_pad / kTile;
  D.assign((size_t)n * n, 0);
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
        D[(size_t)i * n + j] = d;
        D[(size_t)j * n + i] = d;
      }
    }
  });
}

static inline bool owned(int64_t nb, int64_t i, int64_t j, int rank, int world) {
  if (world == 1) return true;
  int64_t a = i / kTile, b = j / kTile;
  if (a > b) std::swap(a, b);
  return tile_linear(nb, a, b) % world == rank;
}

// Reference-exact distance row of sample i (same arithmetic as
// k_exact_rows): float32 diffs for float32 X (MultiSURF.py:184-187,
// ReliefF.py:151-154), float64 diffs for float64 X (SURF.py:153-156), summed
// in float64.
static void exact_row(const Prepared& P, const void* x, int x_is_f64, int64_t i,
                      double* out) {
  for (int64_t j = 0; j < P.n; j++) {
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
      acc += load_x(x, x_is_f64, i * P.p_in + col) != load_x(x, x_is_f64, j * P.p_in + col) ? 1.0 : 0.0;
    }
    out[j] = j == i ? 0.0 : acc;
  }
}

int multisurf_pass1(const Prepared& P, const void* x, int x_is_f64, int rank, int world,
                    int n_jobs, std::vector<uint64_t>& D, std::vector<float>& xs,
                    double* rowstats) {
  std::vector<uint32_t> xq;
  quantize(P, x, x_is_f64, n_jobs, xq, xs);
  distances(P, xq, rank, world, n_jobs, D);
  const int64_t n = P.n, nb = P.n_pad / kTile;
  parallel_for(n, n_jobs, [&](int64_t i) {
    double s1 = 0.0, s2 = 0.0;
    for (int64_t j = 0; j < n; j++) {
      if (j == i || !owned(nb, i, j, rank, world)) continue;
      const double d = (double)D[(size_t)i * n + j];
      s1 += d;
      s2 += d * d;
    }
    rowstats[2 * i] = s1;
    rowstats[2 * i + 1] = s2;
  });
  return FS_OK;
}

int multisurf_select(const Prepared& P, const std::vector<uint64_t>& D, int rank, int world,
                     const double* rowstats, std::vector<double>& thr, double* counts,
                     int n_jobs) {
  const int64_t n = P.n, nb = P.n_pad / kTile;
  thr.assign(n, 0.0);
  parallel_for(n, n_jobs, [&](int64_t i) {
    const double t = multisurf_threshold(rowstats[2 * i], rowstats[2 * i + 1], n);
    const double delta_q = P.amb_delta * P.SC;
    double h = 0.0, m = 0.0, a = 0.0;
    for (int64_t j = 0; j < n; j++) {
      if (j == i || !owned(nb, i, j, rank, world)) continue;
      const double d = (double)D[(size_t)i * n + j];
      if (d < t) {
        if (P.labels[j] == P.labels[i]) h += 1.0;
        else m += 1.0;
      }
      if (std::fabs(d - t) < delta_q) a += 1.0;
    }
    thr[i] = t;
    counts[3 * i] = h;
    counts[3 * i + 1] = m;
    counts[3 * i + 2] = a;
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

int multisurf_pass2(const Prepared& P, const void* x, const std::vector<uint64_t>& D,
                    const std::vector<float>& xs, const std::vector<double>& thr,
                    const double* counts, int rank, int world, int n_jobs, double* scores,
                    int64_t* refined_rows) {
  const int64_t n = P.n, nb = P.n_pad / kTile;
  // Ambiguous rows (all-reduced counts) -> exact rows, thresholds and counts.
  std::vector<double> H(n), M(n);
  std::vector<int64_t> rows;
  for (int64_t i = 0; i < n; i++) {
    H[i] = counts[3 * i];
    M[i] = counts[3 * i + 1];
    if (counts[3 * i + 2] > 0.0) rows.push_back(i);
  }
  if (refined_rows) *refined_rows = (int64_t)rows.size();
  std::vector<int64_t> rmap(n, -1);
  std::vector<double> Dx(rows.size() * (size_t)n), thrx(rows.size());
  parallel_for((int64_t)rows.size(), n_jobs, [&](int64_t r) {
    const int64_t i = rows[r];
    double* row = Dx.data() + (size_t)r * n;
    exact_row(P, x, 0, i, row);
    double s1 = 0.0, s2 = 0.0;
    for (int64_t j = 0; j < n; j++)
      if (j != i) {
        s1 += row[j];
        s2 += row[j] * row[j];
      }
    thrx[r] = multisurf_threshold(s1, s2, n);
    double h = 0.0, m = 0.0;
    for (int64_t j = 0; j < n; j++)
      if (j != i && row[j] < thrx[r]) (P.labels[j] == P.labels[i] ? h : m) += 1.0;
    H[i] = h;
    M[i] = m;
  });
  for (size_t r = 0; r < rows.size(); r++) rmap[rows[r]] = (int64_t)r;
  auto near = [&](int64_t i, int64_t j, double dq) {
    const int64_t r = rmap[i];
    return r >= 0 ? Dx[(size_t)r * n + j] < thrx[r] : dq < thr[i];
  };
  std::vector<PairW> pairs;
  for (int64_t i = 0; i < n; i++)
    for (int64_t j = i + 1; j < n; j++) {
      if (!owned(nb, i, j, rank, world)) continue;
      const double d = (double)D[(size_t)i * n + j];
      const bool hit = P.labels[i] == P.labels[j];
      const double wi = multisurf_weight(near(i, j, d), hit, P.use_star, H[i], M[i]);
      const double wj = multisurf_weight(near(j, i, d), hit, P.use_star, H[j], M[j]);
      const float w = (float)(wi + wj);
      if (w != 0.0f) pairs.push_back({(int32_t)i, (int32_t)j, w});
    }
  std::vector<double> S(P.PW, 0.0);
  weighted_sum(P, xs, pairs, n_jobs, S.data());
  scatter_scores(P, S, scores);
  return FS_OK;
}

int surf_run(const Prepared& P, const void* x, int n_jobs, double* scores) {
  std::vector<uint32_t> xq;
  std::vector<float> xs;
  std::vector<uint64_t> D;
  quantize(P, x, 1, n_jobs, xq, xs);
  distances(P, xq, 0, 1, n_jobs, D);
  const int64_t n = P.n;
  const double inv_sc = 1.0 / P.SC;
  // float32 distance row, float32 sequential mean (SURF.py:146-163)
  std::vector<float> Df((size_t)n * n);
  for (size_t e = 0; e < Df.size(); e++) Df[e] = (float)((double)D[e] * inv_sc);
  std::vector<double> avg(n);
  std::vector<char> amb(n, 0);
  parallel_for(n, n_jobs, [&](int64_t i) {
    float s = 0.0f;
    for (int64_t j = 0; j < n; j++) s += Df[(size_t)i * n + j];
    avg[i] = (double)s / (double)(n - 1);
    const float af = (float)avg[i];
    const double band = P.amb_delta + 4.0 * ((double)std::nextafter(af, 3.0e38f) - (double)af);
    for (int64_t j = 0; j < n && !amb[i]; j++)
      if (j != i && std::fabs((double)D[(size_t)i * n + j] * inv_sc - avg[i]) < band) amb[i] = 1;
  });
  // ambiguous rows: exact float32 distance row and exact sequential mean
  std::vector<int64_t> rows;
  for (int64_t i = 0; i < n; i++)
    if (amb[i]) rows.push_back(i);
  parallel_for((int64_t)rows.size(), n_jobs, [&](int64_t r) {
    const int64_t i = rows[r];
    std::vector<double> row(n);
    exact_row(P, x, 1, i, row.data());
    float s = 0.0f;
    for (int64_t j = 0; j < n; j++) {
      Df[(size_t)i * n + j] = (float)row[j];
      s += (float)row[j];
    }
    avg[i] = (double)s / (double)(n - 1);
  });
  std::vector<PairW> pairs;
  for (int64_t i = 0; i < n; i++)
    for (int64_t j = i + 1; j < n; j++) {
      const bool hit = P.labels[i] == P.labels[j];
      const float w = (float)(surf_weight((double)Df[(size_t)i * n + j] < avg[i], hit, P.use_star) +
                              surf_weight((double)Df[(size_t)j * n + i] < avg[j], hit, P.use_star));
      if (w != 0.0f) pairs.push_back({(int32_t)i, (int32_t)j, w});
    }
  std::vector<double> S(P.PW, 0.0);
  weighted_sum(P, xs, pairs, n_jobs, S.data());
  scatter_scores(P, S, scores);
  return FS_OK;
}

int relieff_run(const Prepared& P, const void* x, int n_jobs, double* scores) {
  std::vector<uint32_t> xq;
  std::vector<float> xs;
  std::vector<uint64_t> D;
  quantize(P, x, 0, n_jobs, xq, xs);
  distances(P, xq, 0, 1, n_jobs, D);
  const int64_t n = P.n, k = P.k_neighbors;
  const int C = P.n_classes;
  const double inv_sc = 1.0 / P.SC;
  // per-row partial sums, folded in row order for determinism
  std::vector<double> part((size_t)n * P.PW, 0.0);
  parallel_for(n, n_jobs, [&](int64_t i) {
    std::vector<std::vector<std::pair<uint32_t, int32_t>>> cand(C);
    for (int64_t j = 0; j < n; j++) {
      if (j == i) continue;
      const float df = (float)((double)D[(size_t)i * n + j] * inv_sc);
      uint32_t key;
      std::memcpy(&key, &df, 4);
      cand[P.labels[j]].push_back({key, (int32_t)j});
    }
    const int32_t li = P.labels[i];
    double denom = 1.0 - P.class_prior[li];
    if (denom == 0.0) denom = 1.0;
    double* out = part.data() + (size_t)i * P.PW;
    const float* a = xs.data() + (size_t)i * P.PW;
    for (int c = 0; c < C; c++) {
      auto& v = cand[c];
      const int64_t kc = std::min<int64_t>(k, (int64_t)v.size());
      if (kc == 0) continue;
      std::partial_sort(v.begin(), v.begin() + kc, v.end());
      // self is a zero-diff hit when its class has < k other members
      // (ReliefF.py:144-168: dists[i] = inf sorts last but is still scanned)
      const int64_t h_found = kc < k ? kc + 1 : k;
      const double wgt = (c == li) ? -1.0 / (double)h_found : (P.class_prior[c] / denom) / (double)k;
      for (int64_t col = 0; col < P.PW; col++) {
        double s = 0.0;
        for (int64_t t = 0; t < kc; t++) {
          const float* b = xs.data() + (size_t)v[t].second * P.PW;
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
