// fs_surfint.hip -- SURF / SURF* on integer pass-1 distances: the float32
// distances of the reference recovered exactly from 32-bit quantised ones.
// Shared state and helpers: fs_gpu_internal.h.
//
// The reference stores every distance as float32 (SURF.py:146-160: float64
// terms |x_i - x_j| * recip summed in float64, then rounded), sums each row
// of them sequentially in float32 for the mean (:162-163) and compares the
// float32 distance with that mean (:176).  Those float32 values are all the
// neighbourhood ever reads, so pass 1 does not need float64 distances --
// only their float32 roundings.  k_dist (32-bit SAD, ~2x the float64 kernel's
// pair-feature rate) gives y = D_q / SC within the calibrated band b of the
// reference's distance D (calibrate_band: 12 sigma of the quantisation error
// or 3x the largest sampled one), so f32(D) lies in [f32(y - b), f32(y + b)]:
// one value for most pairs, two for the ~2 b / ulp of them whose y sits
// near a float32 rounding midpoint.  Such a pair matters only where the
// choice changes something the reference computes from it:
//   * a row's float32 running sum: k_surf_avg_int adds both candidates and
//     lists the pairs where the two sums differ (about sum_k 2 b / ulp(s_k),
//     ~2.4 per row at cfg5), following both sums past each; the listed
//     distances are recomputed in the reference's arithmetic
//     (k_surf_exact_pairs) and those rows summed again, until every row
//     finishes without one -- 2 to 4 rounds;
//   * a near / far decision: k_surf_decisions lists the pairs whose two
//     candidates fall on both sides of a focal endpoint's mean;
// then k_surf_normalize writes every distance as its float32 value (the
// refined ones exactly, the others f32(y)), which is what the float64 path
// wrote, so selection, pass 2 and the reference-order chains read D as
// before.  A distance recomputed exactly is stored as -f32(D) until the
// normalisation (the sign marks it: the band test would otherwise call a
// float32 value near zero ambiguous again).
#include "fs_gpu_internal.h"

namespace fs {
namespace gpu {

// The float32 candidates of one stored distance d of pair (i, j): d <= -0
// holds an exact float32 value, otherwise y = d / SC (integer units) lies
// within band of the reference's distance.
__device__ __forceinline__ void surf_candidates(double d, bool self, double inv_sc, double band,
                                                float& lo, float& hi) {
  if (self) {
    lo = hi = 0.0f;  // dists_from_i[i] = 0 (SURF.py:147-149)
  } else if (__builtin_signbit(d)) {
    lo = hi = (float)(-d);
  } else {
    const double y = d * inv_sc;
    lo = (float)(y - band);
    hi = (float)(y + band);
  }
}

// Row means of the focal rows rows[0..nr): avg[i] = the float32 sequential
// sum of row i's float32 distances over j (self included, 0), / (n - 1) in
// float64 (SURF.py:162-163), as k_surf_avg.  A workgroup takes 64 rows and
// walks them in blocks of kAvgCols columns: wave 0 adds the current block
// from LDS in j order (lane r along row r) while waves 1-4 turn the next
// block into candidate pairs in the other LDS buffer from registers loaded
// a block earlier -- the dependent float32 adds of wave 0 are the round's
// critical path, so nothing else runs on that wave.  Where
// the two candidates give different running sums the row stops: (i, j) goes
// to the pair list (counts[1]) for refinement and i to next_rows (counts[0])
// for the next round.  (Following both sums past such a pair, up to 3 pairs
// a round, took 5 rounds instead of 10 at cfg5 but tripled the cost of a
// round: the add chain is issue-bound, one wave per SIMD.)
constexpr int kAvgCols = 128;
constexpr int kAvgPairsPerRound = 1;
constexpr int kAvgPer = 64 * kAvgCols / 256;  // distances a staging thread stages per block
__global__ __launch_bounds__(320) void k_surf_avg_int(const double* __restrict__ D, int64_t n,
                                                      int64_t n_pad, double inv_sc, double band,
                                                      const int32_t* __restrict__ rows, int64_t nr,
                                                      double* __restrict__ avg,
                                                      int32_t* __restrict__ next_rows,
                                                      int32_t* __restrict__ counts,
                                                      int2* __restrict__ pairs) {
  __shared__ float lo_s[2][64][kAvgCols + 1], hi_s[2][64][kAvgCols + 1];
  __shared__ int32_t rid[64];
  __shared__ int any_live[2];  // by block parity: a slot is rewritten only after the next barrier
  // wave 0 sums; waves 1-4 stage (sw = 0..3)
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, sw = wave - 1;
  const int64_t base = (int64_t)blockIdx.x * 64;
  const int nrows = nr - base < 64 ? (int)(nr - base) : 64;
  if (tid < 64) rid[tid] = rows[base + (tid < nrows ? tid : 0)];  // padding: a stored row
  __syncthreads();
  // thread (wave w, lane l) stages rows w, w + 4, ..., w + 60 at columns l
  // and l + 64 of the block: the 16 row pointers and indices live in
  // registers (padding rows repeat the list's first row; never summed)
  constexpr int kRowsPer = kAvgPer / 2;
  const double* rowp[kRowsPer];
  int32_t rowi[kRowsPer];
#pragma unroll
  for (int q = 0; q < kRowsPer; q++) {
    rowi[q] = rid[(sw < 0 ? 0 : sw) + 4 * q];
    rowp[q] = D + (int64_t)rowi[q] * n_pad + lane;
  }
  // two register sets: block b + 2 is loaded while block b is summed and
  // block b + 1 (loaded one block earlier) goes to LDS
  double dA[kAvgPer], dB[kAvgPer];
  auto load = [&](double (&d)[kAvgPer], int64_t j0) {
    const bool in0 = j0 + lane < n, in1 = j0 + lane + 64 < n;
#pragma unroll
    for (int k = 0; k < kAvgPer; k++) d[k] = ((k & 1) ? in1 : in0) ? rowp[k >> 1][j0 + 64 * (k & 1)] : 0.0;
  };
  auto put = [&](int buf, const double (&d)[kAvgPer], int64_t j0) {
#pragma unroll
    for (int k = 0; k < kAvgPer; k++) {
      const int r = sw + 4 * (k >> 1);
      const int c = lane + 64 * (k & 1);
      const int64_t j = j0 + c;
      float lo = 0.0f, hi = 0.0f;
      if (j < n) surf_candidates(d[k], j == rowi[k >> 1], inv_sc, band, lo, hi);
      lo_s[buf][r][c] = lo;
      hi_s[buf][r][c] = hi;
    }
  };
  const int64_t i = rid[lane];
  bool live = wave == 0 && lane < nrows;
  float s = 0.0f;
  // wave 0: row lane's sum over block j0 (in LDS buffer buf)
  auto sum = [&](int buf, int64_t j0) {
    const int cnt = n - j0 < kAvgCols ? (int)(n - j0) : kAvgCols;
    // 8 columns' candidates in registers, the next 8 read while these are
    // added (the LDS latency off the dependent float32 adds)
    float nlo[8], nhi[8];
#pragma unroll
    for (int u = 0; u < 8; u++) {
      nlo[u] = lo_s[buf][lane][u];
      nhi[u] = hi_s[buf][lane][u];
    }
    for (int c0 = 0; c0 < cnt && __any(live); c0 += 8) {
      float lo[8], hi[8];
#pragma unroll
      for (int u = 0; u < 8; u++) {
        lo[u] = nlo[u];
        hi[u] = nhi[u];
      }
      if (c0 + 8 < kAvgCols) {
#pragma unroll
        for (int u = 0; u < 8; u++) {
          nlo[u] = lo_s[buf][lane][c0 + 8 + u];  // inside the padded row
          nhi[u] = hi_s[buf][lane][c0 + 8 + u];
        }
      }
      // branch-free per column: the first column of the 8 whose two sums
      // differ (columns past n hold 0 / 0, never such a column); a row that
      // met one stops there (its later sums are not used)
      int stop = 8;
#pragma unroll
      for (int u = 0; u < 8; u++) {
        const float a = s + lo[u];
        const bool crit = a != s + hi[u];
        stop = (crit && stop == 8) ? u : stop;
        s = a;
      }
      const bool rec = live && stop < 8;
      if (__any(rec)) {
        if (rec) {  // the sum depends on which one it is
          pairs[atomicAdd(&counts[1], 1)] = make_int2((int)i, (int)(j0 + c0 + stop));
          next_rows[atomicAdd(&counts[0], 1)] = (int32_t)i;
          live = false;
        }
      }
    }
  };
  // one block: load j0 + 2 blocks into `ld`, sum j0 from `buf`, stage j0 + 1
  // block from `st` into the other buffer; false when every row stopped
  auto block = [&](int buf, int64_t j0, int64_t it, double (&ld)[kAvgPer],
                   const double (&st)[kAvgPer]) {
    if (sw >= 0 && j0 + 2 * kAvgCols < n) load(ld, j0 + 2 * kAvgCols);
    if (wave == 0) {
      sum(buf, j0);
      const bool more = __any(live);
      if (lane == 0) any_live[it & 1] = more ? 1 : 0;
    }
    if (sw >= 0 && j0 + kAvgCols < n) put(buf ^ 1, st, j0 + kAvgCols);
    __syncthreads();
    return any_live[it & 1] != 0;  // a slot is rewritten only after the next barrier
  };
  if (sw >= 0) {
    load(dA, 0);
    put(0, dA, 0);
    if (kAvgCols < n) load(dA, kAvgCols);
  }
  __syncthreads();
  for (int64_t j0 = 0, it = 0; j0 < n; j0 += 2 * kAvgCols, it += 2) {
    if (!block(0, j0, it, dB, dA)) break;  // every row stopped: the workgroup leaves together
    if (j0 + kAvgCols >= n) break;
    if (!block(1, j0 + kAvgCols, it + 1, dA, dB)) break;
  }
  if (live) avg[i] = (double)s / (double)(n - 1);
}

// Pairs whose two candidates sit on both sides of a focal endpoint's mean
// (the decision f32(D) < avg of SURF.py:176, as pair_weight tests it), over
// the stored rows [win.x, win.y) x [0, n): appended to pairs (*count may
// exceed cap: the caller grows the list and runs again).  Grid (ceil(n /
// 256), stored rows).
__global__ __launch_bounds__(256) void k_surf_decisions(
    const double* __restrict__ D, int64_t n, int64_t n_pad, int2 win, double inv_sc, double band,
    const double* __restrict__ avg, int64_t r_lo, int64_t r_hi, int2* __restrict__ pairs,
    int64_t cap, unsigned long long* __restrict__ count) {
  const int64_t i = win.x + (int64_t)blockIdx.y;
  const int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n || j >= n) return;
  float lo, hi;
  surf_candidates(D[i * n_pad + j], i == j, inv_sc, band, lo, hi);
  if (lo == hi) return;
  bool flag = false;
  if (i >= r_lo && i < r_hi) flag = ((double)lo < avg[i]) != ((double)hi < avg[i]);
  if (j >= r_lo && j < r_hi) flag = flag || (((double)lo < avg[j]) != ((double)hi < avg[j]));
  if (!flag) return;
  const unsigned long long k = atomicAdd(count, 1ull);
  if ((int64_t)k < cap) pairs[k] = make_int2((int)i, (int)j);
}

// Every stored distance as its float32 value in float64 (what k_dist_f64's
// consumers read with inv_sc = 1): the exact ones (-f) as f, the others
// f32(y) -- either candidate where two remain, since no sum or decision
// depends on which.  Grid (ceil(n / 256), stored rows).
__global__ __launch_bounds__(256) void k_surf_normalize(double* __restrict__ D, int64_t n,
                                                        int64_t n_pad, int2 win, double inv_sc) {
  const int64_t i = win.x + (int64_t)blockIdx.y;
  const int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n || j >= n) return;
  double* p = D + i * n_pad + j;
  const double d = *p;
  *p = i == j ? 0.0 : __builtin_signbit(d) ? -d : (double)(float)(d * inv_sc);
}

// The reference's float32 distance of each listed pair (SURF.py:151-160:
// float64 |x_i - x_j| * recip over the continuous kept columns, 1 per
// differing discrete one), one 256-thread workgroup per pair -- a round's
// last pairs are few, so the per-pair chain of loads sets the time: thread
// t takes features t, t + 256, ..., four loads of each row in flight, and
// the partial sums are added in a fixed order (float64: the order changes
// the float32 rounding only within ~1e-16 of a midpoint, as k_dist_f64's).
// Stored as -f in both halves of the full layout where their rows are in
// the window.
__global__ __launch_bounds__(256) void k_surf_exact_pairs(
    const double* __restrict__ x, int64_t p_in, int64_t pc, int64_t PC, int64_t pd,
    const int64_t* __restrict__ src_col, const double* __restrict__ scl,
    const int2* __restrict__ pairs, double* __restrict__ D, int64_t n_pad, int2 win) {
  __shared__ double red[256];
  const int tid = threadIdx.x;
  const int2 pr = pairs[blockIdx.x];
  const double* xi = x + (int64_t)pr.x * p_in;
  const double* xj = x + (int64_t)pr.y * p_in;
  double a4[4] = {0.0, 0.0, 0.0, 0.0};
  int64_t c = tid;
  for (; c + 768 < pc; c += 1024) {
    double u[4], v[4], w[4];
#pragma unroll
    for (int q = 0; q < 4; q++) {
      const int64_t col = src_col[c + 256 * q];
      u[q] = xi[col];
      v[q] = xj[col];
      w[q] = scl[c + 256 * q];
    }
#pragma unroll
    for (int q = 0; q < 4; q++) a4[q] += __builtin_fabs(u[q] - v[q]) * w[q];
  }
  for (; c < pc; c += 256) {
    const int64_t col = src_col[c];
    a4[0] += __builtin_fabs(xi[col] - xj[col]) * scl[c];
  }
  for (int64_t c2 = PC + tid; c2 < PC + pd; c2 += 256) {
    const int64_t col = src_col[c2];
    a4[1] += xi[col] != xj[col] ? 1.0 : 0.0;
  }
  const double acc = block_sum_256((a4[0] + a4[1]) + (a4[2] + a4[3]), red);
  if (tid != 0) return;
  const double v = -(double)(float)acc;  // -0.0 for a zero distance: still marked
  if (d_row_in(win, pr.x)) D[(int64_t)pr.x * n_pad + pr.y] = v;
  if (d_row_in(win, pr.y)) D[(int64_t)pr.y * n_pad + pr.x] = v;
}

static int exact_pairs(Plan* g, int64_t count) {
  const Prepared& Q = g->P;
  if (count <= 0) return FS_OK;
  k_surf_exact_pairs<<<(unsigned)count, 256, 0, g->stream>>>(
      (const double*)g->x, Q.p_in, Q.pc, Q.PC, Q.pd, g->src_col, g->scl, g->list, g->D, Q.n_pad,
      g->win);
  return launch_check("k_surf_exact_pairs");
}

int surf_resolve(Plan* g) {
  const Prepared& Q = g->P;
  const int64_t rows = g->r_hi - g->r_lo, n = Q.n;
  if (rows <= 0 || n < 2) return FS_OK;
  const double inv_sc = 1.0 / Q.SC, band = Q.amb_delta;
  int32_t *ra = nullptr, *rb = nullptr, *cnt = nullptr;
  g->alloc_target = 2;
  int rc;
  if ((rc = dalloc(g, &ra, (size_t)rows)) || (rc = dalloc(g, &rb, (size_t)rows)) ||
      (rc = dalloc(g, &cnt, 2))) {
    g->alloc_target = 0;
    return rc;
  }
  g->alloc_target = 0;
  if (g->list_cap < kAvgPairsPerRound * rows) {  // the list lives with the plan
    g->list_cap = kAvgPairsPerRound * rows;
    FS_TRY(dalloc(g, &g->list, (size_t)g->list_cap));
  }
  {
    std::vector<int32_t> all((size_t)rows);
    for (int64_t r = 0; r < rows; r++) all[(size_t)r] = (int32_t)(g->r_lo + r);
    FS_TRY(h2d(g, ra, all.data(), all.size()));
    FS_HIP(hipStreamSynchronize(g->stream));  // `all` leaves scope
  }
  // the row means, refining the pairs that decide a running sum
  int64_t cur = rows, rounds = 0, refined_sum = 0;
  while (cur > 0) {
    FS_HIP(hipMemsetAsync(cnt, 0, 2 * sizeof(int32_t), g->stream));
    k_surf_avg_int<<<(unsigned)((cur + 63) / 64), 320, 0, g->stream>>>(
        g->D, n, Q.n_pad, inv_sc, band, ra, cur, g->thr, rb, cnt, g->list);
    FS_TRY(launch_check("k_surf_avg_int"));
    int32_t next[2] = {0, 0};
    FS_HIP(hipMemcpyAsync(next, cnt, sizeof(next), hipMemcpyDeviceToHost, g->stream));
    FS_HIP(hipStreamSynchronize(g->stream));
    FS_TRY(exact_pairs(g, next[1]));
    std::swap(ra, rb);
    cur = next[0];
    refined_sum += next[1];
    if (++rounds > n) {  // every round settles a pair of each row it sends on
      set_error("SURF distances: row means did not settle");
      return FS_EHIP;
    }
  }
  // the decisions that depend on the candidate
  int64_t ndec = 0;
  for (int attempt = 0; attempt < 2; attempt++) {
    FS_HIP(hipMemsetAsync(g->list_count, 0, sizeof(unsigned long long), g->stream));
    const dim3 grid((unsigned)((n + 255) / 256), (unsigned)(g->win.y - g->win.x));
    k_surf_decisions<<<grid, 256, 0, g->stream>>>(g->D, n, Q.n_pad, g->win, inv_sc, band, g->thr,
                                                  g->r_lo, g->r_hi, g->list, g->list_cap,
                                                  g->list_count);
    FS_TRY(launch_check("k_surf_decisions"));
    unsigned long long c = 0;
    FS_HIP(hipMemcpyAsync(&c, g->list_count, sizeof(c), hipMemcpyDeviceToHost, g->stream));
    FS_HIP(hipStreamSynchronize(g->stream));
    ndec = (int64_t)c;
    if (ndec <= g->list_cap) break;
    g->list_cap = ndec + ndec / 4;
    FS_TRY(dalloc(g, &g->list, (size_t)g->list_cap));
  }
  FS_TRY(exact_pairs(g, ndec));
  const dim3 grid((unsigned)((n + 255) / 256), (unsigned)(g->win.y - g->win.x));
  k_surf_normalize<<<grid, 256, 0, g->stream>>>(g->D, n, Q.n_pad, g->win, inv_sc);
  FS_TRY(launch_check("k_surf_normalize"));
  g->n_refined = refined_sum + ndec;
  if (trace_on()) {
    char msg[192];
    snprintf(msg, sizeof msg,
             "surf: integer distances, %lld rounds, %lld pairs for the row sums, %lld for the "
             "decisions",
             (long long)rounds, (long long)refined_sum, (long long)ndec);
    trace_mark(msg);
  }
  return FS_OK;
}

}  // namespace gpu
}  // namespace fs
