// fs_prep.cpp -- host-side problem preparation shared by both backends:
// feature permutation (continuous block, then discrete block, each padded to
// whole 64-feature blocks), discrete value tables, label codes and the
// integer distance scale.  Mirrors the per-feature preprocessing each
// reference fit() hands to its host caller (MultiSURF.py:409-420,
// ReliefF.py:366-380, SURF.py:347-355); the caller still computes recip and
// is_discrete exactly as the reference does.
#include <algorithm>
#include <cmath>
#include <thread>

#include "fs_internal.h"

namespace fs {

int hardware_threads(int n_jobs) {
  int hw = (int)std::thread::hardware_concurrency();
  if (hw <= 0) hw = 1;
  if (n_jobs > 0) return n_jobs;
  return hw;
}

static inline double load_x(const void* x, int x_is_f64, int64_t idx) {
  return x_is_f64 ? ((const double*)x)[idx] : (double)((const float*)x)[idx];
}

void owned_tiles(int64_t nb, int rank, int world, std::vector<int32_t>& bi,
                 std::vector<int32_t>& bj) {
  bi.clear();
  bj.clear();
  int64_t t = 0;
  for (int64_t a = 0; a < nb; a++)
    for (int64_t b = a; b < nb; b++, t++)
      if (t % world == rank) {
        bi.push_back((int32_t)a);
        bj.push_back((int32_t)b);
      }
}

int prepare(Prepared& P, int algo, const void* x, int x_is_f64, int64_t n, int64_t p_in,
            const int64_t* feat_idx, int64_t n_kept, const float* recip,
            const uint8_t* is_discrete, int n_jobs) {
  if (!x || !recip || !is_discrete || n < 2 || p_in < 1) {
    set_error("invalid problem: need x, recip, is_discrete, n >= 2 and p >= 1");
    return -1;
  }
  if (!feat_idx) n_kept = p_in;
  if (n_kept < 1) {
    set_error("n_kept must be >= 1");
    return -1;
  }
  P.algo = algo;
  P.n = n;
  P.n_pad = (n + kTile - 1) / kTile * kTile;
  P.p_in = p_in;
  P.n_kept = n_kept;
  std::vector<int64_t> cont, disc;  // (kept position)
  for (int64_t k = 0; k < n_kept; k++) {
    const int64_t f = feat_idx ? feat_idx[k] : k;
    if (f < 0 || f >= p_in) {
      set_error("feat_idx entry out of range");
      return -1;
    }
    (is_discrete[f] ? disc : cont).push_back(k);
  }
  P.pc = (int64_t)cont.size();
  P.pd = (int64_t)disc.size();
  P.PC = (P.pc + kFeatPad - 1) / kFeatPad * kFeatPad;
  P.PD = (P.pd + kFeatPad - 1) / kFeatPad * kFeatPad;
  P.PW = P.PC + P.PD;
  P.src_col.assign(P.PW, -1);
  P.out_pos.assign(P.PW, -1);
  P.offset.assign(P.PW, 0.0);
  P.scale.assign(P.PW, 0.0);
  P.dtab_off.assign(P.PW + 1, 0);
  P.dtab.clear();
  for (int64_t c = 0; c < P.pc; c++) {
    P.out_pos[c] = cont[c];
    P.src_col[c] = feat_idx ? feat_idx[cont[c]] : cont[c];
  }
  for (int64_t c = 0; c < P.pd; c++) {
    P.out_pos[P.PC + c] = disc[c];
    P.src_col[P.PC + c] = feat_idx ? feat_idx[disc[c]] : disc[c];
  }

  // Column minima / maxima of continuous columns (threads over columns).
  std::vector<double> cmax(P.PW, 0.0);
  const int nt = std::max(1, std::min<int>(hardware_threads(n_jobs), (int)std::max<int64_t>(1, P.pc)));
  {
    std::vector<std::thread> th;
    for (int t = 0; t < nt; t++)
      th.emplace_back([&, t]() {
        for (int64_t c = t; c < P.pc; c += nt) {
          const int64_t col = P.src_col[c];
          double lo = load_x(x, x_is_f64, col), hi = lo;
          for (int64_t i = 1; i < n; i++) {
            const double v = load_x(x, x_is_f64, i * p_in + col);
            lo = v < lo ? v : lo;
            hi = v > hi ? v : hi;
          }
          P.offset[c] = lo;
          cmax[c] = hi;
          P.scale[c] = (double)recip[col];
        }
      });
    for (auto& t : th) t.join();
  }
  double R = 0.0;
  for (int64_t c = 0; c < P.pc; c++) {
    const double r = (cmax[c] - P.offset[c]) * P.scale[c];
    if (!(r >= 0.0) || std::isinf(r)) {
      set_error("non-finite or negative scaled feature range (check recip)");
      return -1;
    }
    R = r > R ? r : R;
  }
  // Discrete value tables (sorted distinct values, float equality semantics).
  for (int64_t c = P.PC; c < P.PC + P.pd; c++) {
    const int64_t col = P.src_col[c];
    std::vector<double> v((size_t)n);
    for (int64_t i = 0; i < n; i++) v[i] = load_x(x, x_is_f64, i * p_in + col);
    std::sort(v.begin(), v.end());
    std::vector<double> u;
    for (double a : v)
      if (u.empty() || a != u.back()) u.push_back(a);
    P.dtab_off[c] = (int64_t)P.dtab.size();
    P.dtab.insert(P.dtab.end(), u.begin(), u.end());
  }
  // Slices are contiguous in column order: slice c ends where c+1 starts.
  for (int64_t c = P.PC + P.pd; c <= P.PW; c++) P.dtab_off[c] = (int64_t)P.dtab.size();

  // Integer distance scale.  Per-feature |q_a - q_b| <= Rm*SC + 1 must keep
  // (a) a 256-feature window on top of a 24-bit remainder inside u32 and
  // (b) the whole distance below 2^40 (16-bit high part above bit 24).
  const double Rm = R > 1.0 ? R : 1.0;
  const double feats = (double)(P.pc + P.pd);
  const double lim_a = ((4294967295.0 - 16777216.0) / 256.0 - 1.0) / Rm;
  const double lim_b = (1099511627775.0 / feats - 1.0) / Rm;
  const double sc = std::floor(std::min(lim_a, lim_b));
  if (!(sc >= 1.0)) {
    set_error("too many features for the 40-bit integer distance");
    return -1;
  }
  P.SC = sc;
  P.SCu = (uint32_t)sc;
  P.qmax = std::floor(R * sc + 0.5) + 1.0;
  // Error model of a quantised distance vs the reference's (float64 sum of
  // float32-rounded diffs): per continuous feature a rounding error of at
  // most 1/SC (std ~ 1/sqrt(6)/SC) plus the reference's own float32
  // rounding (< 1.2e-7 relative).  16 standard deviations of the sum bound
  // both the distance and the threshold error with a wide margin.
  const double pcd = (double)P.pc;
  P.amb_delta = 16.0 * std::sqrt(pcd / 6.0 + 1.0) / sc + 4.0e-7 * std::sqrt(pcd);
  return 0;
}

int encode_labels_f64(Prepared& P, const double* y) {
  if (!y) {
    set_error("y is NULL");
    return -1;
  }
  std::vector<double> u(y, y + P.n);
  std::sort(u.begin(), u.end());
  std::vector<double> cls;
  for (double a : u)
    if (cls.empty() || a != cls.back()) cls.push_back(a);
  P.labels.resize(P.n);
  for (int64_t i = 0; i < P.n; i++) {
    auto it = std::lower_bound(cls.begin(), cls.end(), y[i]);
    P.labels[i] = (int32_t)(it - cls.begin());
  }
  P.n_classes = (int32_t)cls.size();
  return 0;
}

int encode_labels_i32(Prepared& P, const int32_t* y) {
  if (!y) {
    set_error("y is NULL");
    return -1;
  }
  std::vector<int32_t> u(y, y + P.n);
  std::sort(u.begin(), u.end());
  u.erase(std::unique(u.begin(), u.end()), u.end());
  P.labels.resize(P.n);
  for (int64_t i = 0; i < P.n; i++)
    P.labels[i] = (int32_t)(std::lower_bound(u.begin(), u.end(), y[i]) - u.begin());
  P.n_classes = (int32_t)u.size();
  return 0;
}

}  // namespace fs
