// fs_starterm.hip -- the star variants' far pairs without a dense pass 2.
//
// MultiSURF* (MultiSURF.py:217-251) weighs EVERY miss of focal sample i:
// +1/M_i when near, -1/M'_i when far (M' = max(M, 1); a near miss implies
// M >= 1, so M' = M there).  SURF* (SURF.py:180-193) weighs every pair: near
// hit -1, near miss +1, far hit +1, far miss -1.  Both split into a near-only
// part and an all-pairs part that does not depend on the decisions:
//
//   MultiSURF*  w_ij = [near] (hit ? -1/H_i : +2/M'_i)  -  [miss] / M'_i
//   SURF*       w_ij = [near] (hit ? -2 : +2)           +  (hit ? +1 : -1)
//
// The near part is the sparse pass 2 (k_weights_sparse2 with use_star = 2:
// cfg5 holds 41.7% near pairs for MultiSURF, 62.4% for SURF, against 62%
// and 100% non-zero star weights; profiles/r06/near_density.txt).  The
// all-pairs part of feature f is
//
//   U_f = sum_i alpha_i (gamma S_same(i) - S_all(i)),
//   S_all(i) = sum_{j != i} d_f(i, j),   S_same(i) = the same over j of i's class
//
// (MultiSURF*: alpha = 1/M'_i, gamma = 1; SURF*: alpha = 1, gamma = 2;
// alpha = 0 outside the plan's focal rows), which one sort of the column
// gives: with v_k the k-th smallest value, P_k the sum of the values before
// it and T the column total,  S_all = v_k (2k - n) - 2 P_k + T,  and the
// same within a class from the class's own prefix sums (equal values add 0
// on either side, so ties need no order).  A discrete column's d is
// [v_i != v_j]: S_all = n - eq(v_i), S_same = n_c - eq_c(v_i), with the
// equal-value counts from the sorted run bounds.
//
// One 1024-thread workgroup per column, n <= 24576 (kStMaxIpt items per
// thread): the column's (key, 16-bit index) pairs sorted in LDS by rocPRIM's
// block radix sort, one block scan of the values, one (count, sum) scan per
// class, a fixed-order reduction -- deterministic, sums in float64 of the
// float32 pass-2 values (the pair terms of the dense pass are float32 |a - b|
// summed in float32; the split is the more precise of the two).
#include <hip/hip_runtime.h>

#include <rocprim/block/block_radix_sort.hpp>

#include "fs_gpu_internal.h"

namespace fs {
namespace gpu {

namespace {

constexpr int kStThreads = 1024;
// minimum waves per SIMD the compiler plans registers for (A/B builds only:
// make variant DEFS=-DFS_ST_MIN_WAVES=8 -> two workgroups per CU)
#ifndef FS_ST_MIN_WAVES
#define FS_ST_MIN_WAVES 1
#endif
constexpr int kStMaxIpt = 24;
constexpr int kStMaxClasses = 8;
constexpr int kStWaves = kStThreads / 64;

// order-preserving float -> u32 (continuous values are >= 0, but any sign
// sorts right); 0xFFFFFFFF is never produced (it would be a negative NaN)
__device__ __forceinline__ uint32_t st_key(float v) {
  const uint32_t u = __float_as_uint(v);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float st_val(uint32_t k) {
  return __uint_as_float((k & 0x80000000u) ? (k & 0x7FFFFFFFu) : ~k);
}

// Exclusive block scan of two doubles (counts are exact integers in a
// double); fixed order, so the same column gives the same bits every run.
__device__ __forceinline__ void st_scan2(double& a, double& b, double (*ws)[kStWaves],
                                         double& ta, double& tb) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  double x = a, y = b;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const double tx = __shfl_up(x, o), ty = __shfl_up(y, o);
    if (lane >= o) {
      x += tx;
      y += ty;
    }
  }
  if (lane == 63) {
    ws[0][wave] = x;
    ws[1][wave] = y;
  }
  __syncthreads();
  double pa = 0.0, pb = 0.0, sa = 0.0, sb = 0.0;
#pragma unroll
  for (int w = 0; w < kStWaves; w++) {
    const double u = ws[0][w], v = ws[1][w];
    if (w < wave) {
      pa += u;
      pb += v;
    }
    sa += u;
    sb += v;
  }
  __syncthreads();  // ws is reused by the next scan
  ta = sa;
  tb = sb;
  a = pa + x - a;
  b = pb + y - b;
}

// rocPRIM's block radix sort (8-bit digits, match ranking: 4 passes).  Its
// scatters leave ~74% of the kernel's LDS-active cycles in bank conflicts at
// cfg5 (profiles/r06/starsplit/pmc_cfg5m_table.txt); neither the padding
// hint nor odd items per thread moved the step (starsplit/ipt_ab.txt)
template <int IPT>
using StSort = rocprim::block_radix_sort<uint32_t, kStThreads, IPT, uint16_t>;

template <int IPT, bool DISC>
struct StLds {
  union {
    typename StSort<IPT>::storage_type sort;
    struct {
      uint32_t key[DISC ? kStThreads * IPT : 1];      // sorted keys (run bounds)
      uint16_t cnt[DISC ? kStThreads * IPT + 2 : 1];  // class-c items before each position
    } d;
  } u;
  double ws[2][kStWaves];
};

// first position in [lo, hi) whose key is >= k (upper: > k)
template <bool UPPER>
__device__ __forceinline__ int st_bound(const uint32_t* __restrict__ key, int lo, int hi,
                                        uint32_t k) {
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (UPPER ? key[mid] <= k : key[mid] < k) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

// SUMS = false (SURF*): the column's term U_f into tcol.  SUMS = true
// (MultiSURF*, before the counts are known): each sample's S_other(i) =
// S_all(i) - S_same(i), summed class by class over the other classes
// (G_k(i) = sum over class k of |v_i - v_j|, from class k's prefix at i's
// position -- valid for a sample of any class), written over the column's
// xsT values (the workgroup holds them in registers by then); star_reduce
// weighs them with alpha.
template <int IPT, bool DISC, bool SUMS>
__global__ __launch_bounds__(kStThreads, FS_ST_MIN_WAVES) void k_star_terms(
    float* __restrict__ xsT, int64_t n, int64_t n_pad, const int32_t* __restrict__ lab,
    const double* __restrict__ alpha, int ncls, double gamma, int64_t c_first, int64_t s_lo,
    int64_t s_hi, const int64_t* __restrict__ out_pos, double* __restrict__ tcol) {
  using Sort = StSort<IPT>;
  __shared__ StLds<IPT, DISC> sm;
  const int64_t c = c_first + blockIdx.x;
  const int tid = threadIdx.x;
  if (c < s_lo || c >= s_hi || out_pos[c] < 0) {
    if (!SUMS && tid == 0) tcol[c] = 0.0;
    return;
  }
  const int nn = (int)n;
  float* __restrict__ col = xsT + c * n_pad;
  uint32_t key[IPT];
  uint16_t idx[IPT];
#pragma unroll
  for (int j = 0; j < IPT; j++) {  // striped loads (coalesced); the sort ignores the arrangement
    const int i = j * kStThreads + tid;
    key[j] = i < nn ? (DISC ? __float_as_uint(col[i]) : st_key(col[i])) : 0xFFFFFFFFu;
    idx[j] = (uint16_t)i;
  }
  Sort().sort(key, idx, sm.u.sort);  // blocked: positions tid * IPT + j; padding last
  __syncthreads();                   // the sort's storage is reused below
  const int base = tid * IPT;
  // per item only its class, (discrete) run bounds and (SUMS) its sum stay
  // in registers: the value decodes from the key, alpha reloads from L1 / L2
  int cl[IPT];
  float so[SUMS ? IPT : 1];
  double loc = 0.0;
#pragma unroll
  for (int j = 0; j < IPT; j++) {
    const bool ok = base + j < nn;
    cl[j] = ok ? lab[idx[j]] : -1;
    if (SUMS) so[j] = 0.0f;
    if (!DISC && !SUMS) loc += ok ? (double)st_val(key[j]) : 0.0;
  }
  double acc = 0.0;
  uint32_t run[DISC ? IPT : 1];  // lo | hi << 16
  if (!DISC && !SUMS) {
    double P = loc, zero = 0.0, T, z;
    st_scan2(P, zero, sm.ws, T, z);
#pragma unroll
    for (int j = 0; j < IPT; j++) {
      if (base + j < nn) {
        const double v = (double)st_val(key[j]);
        acc -= alpha[idx[j]] * (v * (double)(2 * (base + j) - nn) - 2.0 * P + T);
        P += v;
      }
    }
  } else if (DISC) {
#pragma unroll
    for (int j = 0; j < IPT; j++)
      if (base + j < nn) sm.u.d.key[base + j] = key[j];
    __syncthreads();
#pragma unroll
    for (int j = 0; j < IPT; j++) {
      const int p = base + j;
      run[j] = 0u;
      if (p < nn) {
        const int lo = st_bound<false>(sm.u.d.key, 0, p, key[j]);
        const int hi = st_bound<true>(sm.u.d.key, p + 1, nn, key[j]);
        run[j] = (uint32_t)lo | ((uint32_t)hi << 16);
        if (!SUMS) acc -= alpha[idx[j]] * (double)(nn - (hi - lo));
      }
    }
  }
  for (int k = 0; k < ncls; k++) {
    double lc = 0.0, ls = 0.0;
#pragma unroll
    for (int j = 0; j < IPT; j++)
      if (cl[j] == k) {
        lc += 1.0;
        if (!DISC) ls += (double)st_val(key[j]);
      }
    double tc, ts;
    st_scan2(lc, ls, sm.ws, tc, ts);
    if (!DISC) {
#pragma unroll
      for (int j = 0; j < IPT; j++) {
        const double v = (double)st_val(key[j]);
        const double G = v * (2.0 * lc - tc) - 2.0 * ls + ts;  // sum over class k of |v - v_j|
        if (SUMS) {
          if (cl[j] >= 0 && cl[j] != k) so[j] += (float)G;
        } else if (cl[j] == k) {
          acc += gamma * alpha[idx[j]] * G;
        }
        if (cl[j] == k) {
          lc += 1.0;
          ls += v;
        }
      }
    } else {
      // class-k items before each position, then eq_k = cnt[hi] - cnt[lo]
#pragma unroll
      for (int j = 0; j < IPT; j++) {
        if (base + j < nn) sm.u.d.cnt[base + j] = (uint16_t)lc;
        if (cl[j] == k) lc += 1.0;
      }
      if (tid == 0) sm.u.d.cnt[nn] = (uint16_t)tc;
      __syncthreads();
#pragma unroll
      for (int j = 0; j < IPT; j++) {
        if (cl[j] < 0 || (SUMS ? cl[j] == k : cl[j] != k)) continue;
        const int eq = (int)sm.u.d.cnt[run[j] >> 16] - (int)sm.u.d.cnt[run[j] & 0xFFFFu];
        if (SUMS) so[j] += (float)(tc - (double)eq);
        else acc += gamma * alpha[idx[j]] * (tc - (double)eq);
      }
      __syncthreads();  // cnt is rewritten for the next class
    }
  }
  if (SUMS) {
#pragma unroll
    for (int j = 0; j < IPT; j++)
      if (base + j < nn) col[idx[j]] = so[j];
    return;
  }
  // fixed-order reduction of acc
  const int lane = tid & 63, wave = tid >> 6;
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) acc += __shfl_xor(acc, o);
  if (lane == 0) sm.ws[0][wave] = acc;
  __syncthreads();
  if (tid == 0) {
    double s = 0.0;
    for (int w = 0; w < kStWaves; w++) s += sm.ws[0][w];
    tcol[c] = s;
  }
}

// MultiSURF*'s column terms from the per-sample sums: tcol[c] = -sum_i
// alpha_i S_other(i) over this share's columns, 4 columns per 256-thread
// workgroup (alpha read once for the four), fixed-order reduction.
constexpr int kGvCols = 4;
__global__ __launch_bounds__(256) void k_star_gemv(const float* __restrict__ So, int64_t n,
                                                   int64_t n_pad, int64_t PW,
                                                   const double* __restrict__ alpha, int64_t s0,
                                                   int64_t s1, int64_t d0, int64_t d1,
                                                   const int64_t* __restrict__ out_pos,
                                                   double* __restrict__ tcol) {
  __shared__ double red[kGvCols][256];
  const int tid = threadIdx.x;
  const int64_t c0 = (int64_t)blockIdx.x * kGvCols;
  bool live[kGvCols];
  double acc[kGvCols];
#pragma unroll
  for (int q = 0; q < kGvCols; q++) {
    const int64_t c = c0 + q;
    live[q] = c < PW && ((c >= s0 && c < s1) || (c >= d0 && c < d1)) && out_pos[c] >= 0;
    acc[q] = 0.0;
  }
  for (int64_t i = tid; i < n; i += 256) {
    const double a = alpha[i];
#pragma unroll
    for (int q = 0; q < kGvCols; q++)
      if (live[q]) acc[q] += a * (double)So[(c0 + q) * n_pad + i];
  }
#pragma unroll
  for (int q = 0; q < kGvCols; q++) red[q][tid] = acc[q];
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if (tid < w)
#pragma unroll
      for (int q = 0; q < kGvCols; q++) red[q][tid] += red[q][tid + w];
    __syncthreads();
  }
  if (tid < kGvCols && c0 + tid < PW) tcol[c0 + tid] = live[tid] ? -red[tid][0] : 0.0;
}

// alpha_i: 1 / max(M_i, 1) (MultiSURF*, counts[2i + 1] = M_i) or 1 (SURF*)
// on the focal rows [r_lo, r_hi), 0 elsewhere
__global__ void k_star_alpha(int64_t n_pad, const double* __restrict__ counts, int64_t r_lo,
                             int64_t r_hi, double* __restrict__ alpha) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n_pad) return;
  double a = 0.0;
  if (i >= r_lo && i < r_hi) {
    if (counts) {
      const double m = counts[2 * i + 1];
      a = 1.0 / (m > 0.0 ? m : 1.0);
    } else {
      a = 1.0;
    }
  }
  alpha[i] = a;
}

template <bool DISC, bool SUMS>
int launch_terms(Plan* g, int64_t c_first, int64_t ncols, int64_t s_lo, int64_t s_hi,
                 double gamma, hipStream_t st) {
  const Prepared& Q = g->P;
  if (ncols <= 0) return FS_OK;
  const unsigned grid = (unsigned)ncols;
#define FS_ST(IPT)                                                                              \
  k_star_terms<IPT, DISC, SUMS><<<grid, kStThreads, 0, st>>>(                                \
      g->xsT, Q.n, Q.n_pad, g->lab, g->alpha, Q.n_classes, gamma, c_first, s_lo, s_hi,           \
      g->out_pos, g->tcol)
  const int64_t ipt = (Q.n + kStThreads - 1) / kStThreads;
  if (ipt <= 4) FS_ST(4);
  else if (ipt <= 8) FS_ST(8);
  else if (ipt <= 10) FS_ST(10);
  else if (ipt <= 12) FS_ST(12);
  else if (ipt <= 16) FS_ST(16);
  else if (ipt <= 20) FS_ST(20);
  else FS_ST(24);
#undef FS_ST
  return launch_check(DISC ? "k_star_terms<disc>" : "k_star_terms");
}

int check_split(const Plan* g) {
  const Prepared& Q = g->P;
  if (!g->xsT || !g->alpha || !g->tcol || !star_split_fits(Q.n, Q.n_classes)) {
    set_error("star split: plan without its buffers or outside the split's sizes");
    return FS_EINVAL;
  }
  return FS_OK;
}

// this rank's columns of the split: the continuous ones of its mean
// correction ([c_lo, c_hi): pc r / N ... pc (r + 1) / N, so that one sort
// can serve both, fs_colsort.hip k_colsort_star) and PD r / N ... of the
// discrete ones.  Tile-sharded MultiSURF* ranks add their columns' terms
// before the sum all-reduce; a row plan (world 1) covers every column.
void shares(const Plan* g, int64_t& c0, int64_t& c1, int64_t& d0, int64_t& d1) {
  const Prepared& Q = g->P;
  c0 = g->c_lo;
  c1 = g->c_hi;
  d0 = Q.PC + (Q.PW - Q.PC) * g->rank / g->world;
  d1 = Q.PC + (Q.PW - Q.PC) * (g->rank + 1) / g->world;
}

int run_alpha(Plan* g, const double* counts, hipStream_t st) {
  const Prepared& Q = g->P;
  k_star_alpha<<<(unsigned)((Q.n_pad + 255) / 256), 256, 0, st>>>(Q.n_pad, counts, g->r_lo,
                                                                 g->r_hi, g->alpha);
  return launch_check("k_star_alpha");
}

}  // namespace

bool star_split_fits(int64_t n, int32_t n_classes) {
  return n >= 2 && n <= (int64_t)kStThreads * kStMaxIpt && n_classes >= 1 &&
         n_classes <= kStMaxClasses;
}

int star_terms(Plan* g, hipStream_t st) {
  const Prepared& Q = g->P;
  FS_TRY(check_split(g));
  FS_TRY(run_alpha(g, nullptr, st));  // SURF*: alpha = 1 on the focal rows
  int64_t c0, c1, d0, d1;
  shares(g, c0, c1, d0, d1);
  FS_TRY((launch_terms<false, false>(g, 0, Q.PC, c0, c1, 2.0, st)));
  return launch_terms<true, false>(g, Q.PC, Q.PW - Q.PC, d0, d1, 2.0, st);
}

int star_sums(Plan* g, hipStream_t st, bool continuous) {
  const Prepared& Q = g->P;
  FS_TRY(check_split(g));
  int64_t c0, c1, d0, d1;
  shares(g, c0, c1, d0, d1);
  if (continuous) FS_TRY((launch_terms<false, true>(g, 0, Q.PC, c0, c1, 1.0, st)));
  return launch_terms<true, true>(g, Q.PC, Q.PW - Q.PC, d0, d1, 1.0, st);
}

int star_reduce(Plan* g, const double* counts, hipStream_t st) {
  const Prepared& Q = g->P;
  FS_TRY(check_split(g));
  FS_TRY(run_alpha(g, counts, st));
  int64_t c0, c1, d0, d1;
  shares(g, c0, c1, d0, d1);
  k_star_gemv<<<(unsigned)((Q.PW + kGvCols - 1) / kGvCols), 256, 0, st>>>(
      g->xsT, Q.n, Q.n_pad, Q.PW, g->alpha, c0, c1, d0, d1, g->out_pos, g->tcol);
  return launch_check("k_star_gemv");
}

}  // namespace gpu
}  // namespace fs
