// fs_prep.cpp -- host-side problem preparation shared by both backends:
// feature permutation (continuous block, then discrete block, each padded to
// whole 64-feature blocks), discrete value tables, label codes and the
// integer distance scale.  Mirrors the per-feature preprocessing each
// reference fit() hands to its host caller (MultiSURF.py:409-420,
// ReliefF.py:366-380, SURF.py:347-355); the caller still computes recip and
// is_discrete exactly as the reference does.
#include <sched.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <unordered_set>

#include "../../include/fastselect_amd.h"
#include "fs_internal.h"

namespace fs {

// n_jobs > 0: that many threads.  Otherwise the CPUs this process may run on
// (its affinity mask, not the machine's count: a container or a GPU box's
// share), capped by OMP_NUM_THREADS when it is set -- the pool a
// numba / OpenMP program of the reference would get.
int hardware_threads(int n_jobs) {
  if (n_jobs > 0) return n_jobs;
  int hw = 0;
  cpu_set_t set;
  if (sched_getaffinity(0, sizeof(set), &set) == 0) hw = CPU_COUNT(&set);
  if (hw <= 0) hw = (int)std::thread::hardware_concurrency();
  if (hw <= 0) hw = 1;
  if (const char* e = std::getenv("OMP_NUM_THREADS")) {
    const int cap = std::atoi(e);
    if (cap > 0 && cap < hw) hw = cap;
  }
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

void row_tiles(int64_t nb, int64_t b_lo, int64_t b_hi, std::vector<int32_t>& bi,
               std::vector<int32_t>& bj) {
  bi.clear();
  bj.clear();
  for (int64_t a = 0; a < nb; a++)
    for (int64_t b = a; b < nb; b++)
      if ((a >= b_lo && a < b_hi) || (b >= b_lo && b < b_hi)) {
        bi.push_back((int32_t)a);
        bj.push_back((int32_t)b);
      }
}

int prepare(Prepared& P, int algo, const void* x, int x_is_f64, int64_t n, int64_t p_in,
            const int64_t* feat_idx, int64_t n_kept, const float* recip,
            const uint8_t* is_discrete, int n_jobs, int device_ranges,
            const Prepared* dtab_src) {
  // x may be NULL only when nothing here reads it: ranges left to the
  // device and discrete columns coded by their bits (float32 X) or tables
  // taken from dtab_src
  const bool x_needed = !(device_ranges && (!x_is_f64 || dtab_src));
  if ((!x && x_needed) || !recip || !is_discrete || n < 2 || p_in < 1) {
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

  for (int64_t c = 0; c < P.pc; c++) P.scale[c] = (double)recip[P.src_col[c]];
  P.recip_in.assign(recip, recip + p_in);
  P.disc_in.assign(is_discrete, is_discrete + p_in);
  P.kept_col.resize((size_t)n_kept);
  for (int64_t k = 0; k < n_kept; k++) P.kept_col[k] = feat_idx ? feat_idx[k] : k;
  P.disc_bits = (device_ranges && !x_is_f64) ? 1 : 0;
  const int nthreads = hardware_threads(n_jobs);

  // Discrete value tables (sorted distinct values, float equality
  // semantics), one column per task.
  if (!P.disc_bits && P.pd > 0 && dtab_src) {
    // slices of the source's tables, looked up by input column
    std::vector<int64_t> perm_of((size_t)p_in, -1);
    const Prepared& S = *dtab_src;
    for (int64_t c = S.PC; c < S.PC + S.pd; c++) perm_of[(size_t)S.src_col[c]] = c;
    for (int64_t k = 0; k < P.pd; k++) {
      const int64_t c = perm_of[(size_t)P.src_col[P.PC + k]];
      if (c < 0) {
        set_error("discrete column without a value table in the source plan");
        return -1;
      }
      P.dtab_off[P.PC + k] = (int64_t)P.dtab.size();
      P.dtab.insert(P.dtab.end(), S.dtab.begin() + S.dtab_off[c], S.dtab.begin() + S.dtab_off[c + 1]);
    }
  } else if (!P.disc_bits && P.pd > 0) {
    std::vector<std::vector<double>> tabs((size_t)P.pd);
    const int nt = (int)std::max<int64_t>(1, std::min<int64_t>(nthreads, P.pd));
    std::vector<std::thread> th;
    for (int t = 0; t < nt; t++)
      th.emplace_back([&, t]() {
        std::vector<double> v((size_t)n);
        for (int64_t k = t; k < P.pd; k += nt) {
          const int64_t col = P.src_col[P.PC + k];
          for (int64_t i = 0; i < n; i++) v[i] = load_x(x, x_is_f64, i * p_in + col);
          std::sort(v.begin(), v.end());
          std::vector<double>& u = tabs[k];
          for (double a : v)
            if (u.empty() || a != u.back()) u.push_back(a);
        }
      });
    for (auto& t : th) t.join();
    for (int64_t k = 0; k < P.pd; k++) {
      P.dtab_off[P.PC + k] = (int64_t)P.dtab.size();
      P.dtab.insert(P.dtab.end(), tabs[k].begin(), tabs[k].end());
    }
  }
  // Slices are contiguous in column order: slice c ends where c+1 starts.
  for (int64_t c = P.PC + P.pd; c <= P.PW; c++) P.dtab_off[c] = (int64_t)P.dtab.size();

  if (device_ranges) {
    P.ranges_ready = 0;
    return 0;
  }
  // Column minima / maxima on the host: all columns, streamed by row blocks.
  const size_t esz = x_is_f64 ? 8 : 4;
  std::vector<char> mn((size_t)p_in * esz), mx((size_t)p_in * esz);
  std::vector<int64_t> nd((size_t)p_in);
  cpu::column_stats(x, x_is_f64, n, p_in, 0, n_jobs, mn.data(), mx.data(), nd.data());
  std::vector<double> cmin((size_t)P.pc), cmax((size_t)P.pc);
  for (int64_t c = 0; c < P.pc; c++) {
    const int64_t col = P.src_col[c];
    cmin[c] = x_is_f64 ? ((const double*)mn.data())[col] : (double)((const float*)mn.data())[col];
    cmax[c] = x_is_f64 ? ((const double*)mx.data())[col] : (double)((const float*)mx.data())[col];
  }
  return finalize_scale(P, cmin.data(), cmax.data());
}

int finalize_scale(Prepared& P, const double* cmin, const double* cmax) {
  double R = 0.0;
  for (int64_t c = 0; c < P.pc; c++) {
    P.offset[c] = cmin[c];
    const double r = (cmax[c] - cmin[c]) * P.scale[c];
    if (!(r >= 0.0) || std::isinf(r)) {
      set_error("non-finite or negative scaled feature range (check recip)");
      return -1;
    }
    R = r > R ? r : R;
  }
  P.Rmax = R;
  return set_integer_scale(P, P.q16);
}

int set_integer_scale(Prepared& P, int q16) {
  P.q16 = q16;
  const double R = P.Rmax;
  // Integer distance scale.  Per-feature |q_a - q_b| <= Rm*SC + 1 must keep
  // (a) a 256-feature window on top of a 24-bit remainder inside u32 and
  // (b) the whole distance below 2^40 (16-bit high part above bit 24).
  const double Rm = R > 1.0 ? R : 1.0;
  const double feats = (double)(P.pc + P.pd);
  const double lim_a = ((4294967295.0 - 16777216.0) / 256.0 - 1.0) / Rm;
  const double lim_b = (1099511627775.0 / feats - 1.0) / Rm;
  // 16-bit operands: q = round(t) <= Rm * SC + 0.5 must stay <= 65535
  const double lim_16 = P.q16 ? 65534.0 / Rm : lim_a;
  const double sc = std::floor(std::min(std::min(lim_a, lim_16), lim_b));
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
  // rounding (< 1.2e-7 relative).  12 standard deviations of the sum (a
  // tail of 4e-33 per pair; the sum of bounded terms has lighter tails than
  // a Gaussian, and for pc <= 23 the band exceeds the worst case pc / SC)
  // bound the distance error; the threshold error is far smaller.  The GPU
  // backend checks this model against measured pairs (calibrate_band in
  // fs_pass1.hip) and widens the band where the errors of different columns
  // add up coherently (duplicated, collinear or same-grid columns).
  const double pcd = (double)P.pc;
  P.amb_delta = 12.0 * std::sqrt(pcd / 6.0 + 1.0) / sc + 4.0e-7 * std::sqrt(pcd);
  // SURF's terms are float64 (SURF.py:156): the quantisation error alone
  if (P.algo == ALGO_SURF) P.amb_delta = 12.0 * std::sqrt(pcd / 6.0 + 1.0) / sc;
  P.amb_delta_model = P.amb_delta;
  P.ranges_ready = 1;
  return 0;
}

void calib_pairs(int64_t n, int64_t pc, int64_t count, std::vector<std::pair<int64_t, int64_t>>& out) {
  out.clear();
  if (n < 2) return;
  uint64_t st = 0x9E3779B97F4A7C15ull ^ ((uint64_t)n << 20) ^ (uint64_t)pc;
  auto next = [&]() {  // splitmix64
    uint64_t z = (st += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
  };
  for (int64_t k = 0; k < count; k++) {
    const int64_t i = (int64_t)(next() % (uint64_t)n);
    int64_t j = (int64_t)(next() % (uint64_t)(n - 1));
    if (j >= i) j++;
    out.emplace_back(std::min(i, j), std::max(i, j));
  }
}

double calibrated_delta(double model, double SC, double rms, double max_abs) {
  return std::max(model, (3.0 * max_abs + 0.5 * rms) / SC);
}

namespace cpu {

// Host column statistics (the CPU backend of fs_column_stats).  Threads own
// blocks of 64 adjacent columns and stream the rows, so every row segment is
// read once and contiguously; a column stops collecting values once it has
// more than `cap` distinct ones.
template <typename T>
static void colstats_block(const T* x, int64_t n, int64_t p, int64_t cap, int64_t c0, int64_t c1,
                           T* mn, T* mx, int64_t* nd) {
  const int64_t w = c1 - c0;
  std::vector<std::vector<uint64_t>> small(w);
  std::vector<std::unordered_set<uint64_t>> big(cap > 32 ? w : 0);
  std::vector<int64_t> cnt(w, 0);
  for (int64_t c = c0; c < c1; c++) mn[c] = mx[c] = x[c];
  for (int64_t i = 0; i < n; i++) {
    const T* row = x + i * p;
    for (int64_t c = c0; c < c1; c++) {
      const T v = row[c];
      mn[c] = v < mn[c] ? v : mn[c];
      mx[c] = v > mx[c] ? v : mx[c];
      const int64_t k = c - c0;
      if (cnt[k] > cap) continue;
      double d = (double)v;
      if (d == 0.0) d = 0.0;  // np.unique: -0.0 == +0.0
      uint64_t key;
      std::memcpy(&key, &d, 8);
      if (cap > 32) {
        if (big[k].insert(key).second) cnt[k]++;
      } else if (std::find(small[k].begin(), small[k].end(), key) == small[k].end()) {
        small[k].push_back(key);
        cnt[k]++;
      }
    }
  }
  for (int64_t c = c0; c < c1; c++) nd[c] = std::min(cnt[c - c0], cap + 1);
}

int column_stats(const void* x, int x_is_f64, int64_t n, int64_t p, int64_t cap, int n_jobs,
                 void* colmin, void* colmax, int64_t* ndistinct) {
  const int64_t nblk = (p + 63) / 64;
  const int nt = (int)std::max<int64_t>(1, std::min<int64_t>(hardware_threads(n_jobs), nblk));
  std::vector<std::thread> th;
  for (int t = 0; t < nt; t++)
    th.emplace_back([&, t]() {
      for (int64_t b = t; b < nblk; b += nt) {
        const int64_t c0 = b * 64, c1 = std::min(p, c0 + 64);
        if (x_is_f64)
          colstats_block((const double*)x, n, p, cap, c0, c1, (double*)colmin, (double*)colmax,
                         ndistinct);
        else
          colstats_block((const float*)x, n, p, cap, c0, c1, (float*)colmin, (float*)colmax,
                         ndistinct);
      }
    });
  for (auto& t : th) t.join();
  return FS_OK;
}

}  // namespace cpu

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
