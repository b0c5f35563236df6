// fs_pass2.hip -- pass 2: pair weights, dense and sparse scoring, the segment reduce; reference-order masks and chains glue.
// Shared state and helpers: fs_gpu_internal.h.
#include "fs_gpu_internal.h"
#include "fs_sparse_asm.inc"

namespace fs {
namespace gpu {

// ---------------------------------------------------------------------------
// Pair weights per owned tile: Wt[t][jj][ii] = W_ij + W_ji for i < j
// ---------------------------------------------------------------------------
// Symmetric pair weight W_ij + W_ji of one pair (i, j) of an owned tile.
__device__ __forceinline__ float pair_weight(const double* __restrict__ D, int64_t n, int64_t n_pad,
                                             int tiled, int2 win, int64_t t, int64_t i0, int64_t j0, int ii,
                                             int jj, bool upper,
                                             const double* __restrict__ thr,
                                             const int32_t* __restrict__ lab,
                                             const double* __restrict__ counts, int algo,
                                             int use_star, double inv_sc, int64_t r_lo,
                                             int64_t r_hi) {
  const int64_t i = i0 + ii, j = j0 + jj;
  if (!(i < n && j < n && upper)) return 0.0f;
  const double d = D[d_rd(tiled, win, n_pad, t, i0, j0, ii, jj)];  // == D[i][j]
  const bool hit = lab[i] == lab[j];
  // use_star == 2: the star split (fs_starterm.hip) -- near pairs only, the
  // star weight minus its all-pairs part: MultiSURF* near misses 2 / M_i,
  // SURF* near pairs +-2; the far pairs' weight is in the per-column terms
  const int ws = use_star == 2 ? 0 : use_star;
  double wi, wj;
  if (algo == ALGO_MULTISURF) {
    wi = multisurf_weight(d < thr[i], hit, ws, counts[2 * i], counts[2 * i + 1]);
    wj = multisurf_weight(d < thr[j], hit, ws, counts[2 * j], counts[2 * j + 1]);
    if (use_star == 2 && !hit) {
      wi *= 2.0;
      wj *= 2.0;
    }
  } else {  // SURF: float32 distance against the float64 mean
    const double df = (double)(float)(d * inv_sc);
    wi = surf_weight(df < thr[i], hit, ws);
    wj = surf_weight(df < thr[j], hit, ws);
    if (use_star == 2) {
      wi *= 2.0;
      wj *= 2.0;
    }
  }
  // Only focal samples in [r_lo, r_hi) contribute their side of a pair (row
  // sharding: another rank scores the other side); MultiSURF passes [0, n).
  if (i < r_lo || i >= r_hi) wi = 0.0;
  if (j < r_lo || j >= r_hi) wj = 0.0;
  return (float)(wi + wj);
}

__global__ __launch_bounds__(256) void k_weights(const double* __restrict__ D, int64_t n,
                                                 int64_t n_pad, int tiled, int2 win,
                                                 const int2* __restrict__ tiles,
                                                 const double* __restrict__ thr,
                                                 const int32_t* __restrict__ lab,
                                                 const double* __restrict__ counts, int algo,
                                                 int use_star, double inv_sc, int64_t r_lo,
                                                 int64_t r_hi, float* __restrict__ Wt) {
  const int2 tl = tiles[blockIdx.x];
  const int64_t i0 = (int64_t)tl.x * kTile, j0 = (int64_t)tl.y * kTile;
  float* out = Wt + (int64_t)blockIdx.x * kTile * kTile;
  for (int e = threadIdx.x; e < kTile * kTile; e += 256) {
    const int jj = e / kTile, ii = e % kTile;
    out[jj * kTile + ii] = pair_weight(D, n, n_pad, tiled, win, blockIdx.x, i0, j0, ii, jj,
                                       tl.x < tl.y || ii < jj, thr, lab, counts, algo, use_star,
                                       inv_sc, r_lo, r_hi);
  }
}

// Sparse pair weights (pass 2 skips zero weights; MultiSURF: ~42% of the
// pairs are near one of their two samples): k_weights_sparse2 / k_score_sparse2
// below.  A workgroup of the sparse kernels has kSWaves waves.
// entries a tile's streams may hold: 16 streams x 8 columns x 128 rows (both halves)
// floats past xs's last spare row that a pass-2 B-row read may touch (the
// widest feature block of k_score_sparse2)

__device__ __forceinline__ uint32_t weight_bits(float w, bool last) {
  return (__float_as_uint(w) & ~1u) | (last ? 1u : 0u);
}

// ---------------------------------------------------------------------------
// Pass 2: weighted per-feature accumulation over owned tiles
// ---------------------------------------------------------------------------
// Grid (ceil(PW/128) feature blocks, segments of seg_len tiles); 4 waves per
// workgroup, wave w handles rows w*32 .. w*32+31 of every tile; lane l scores
// the two features c0 = blk*128 + l and c1 = c0 + 64 (each half is wholly
// continuous or wholly discrete because PC is a multiple of 64).  For each
// column jj the 32 pair weights of the wave's sub-tile are wave-uniform and
// live in SGPRs; they feed 2 x 32 (sub, fma|.|) pairs.  Software pipeline:
// the next column's weights are requested (s_load) right after the current
// column's have been consumed once, and the B values run two columns ahead
// (in-order vector loads), so neither latency is exposed.  A rows stay in
// VGPRs across consecutive tiles of the same row block.  Per feature, 4 f32
// partial sums are folded into a double every 32 columns.
template <bool DISC>
__device__ __forceinline__ float pair_term(float a, float b, float w, float acc) {
  if (DISC) return acc + ((a != b) ? w : 0.0f);
  return __builtin_fmaf(__builtin_fabsf(a - b), w, acc);
}

// Order point: everything computing `v` happens before, and no memory access
// moves across (so a scalar load placed after it is issued after the wait
// for the weights `v` depends on).
#define FS_ORDER_AFTER(v) asm volatile("" : "+v"(v)::"memory")

template <bool D0, bool D1, bool TWO>
__device__ __forceinline__ void score_column(const float (&a0)[kSubRows],
                                             const float (&a1)[kSubRows],
                                             const float* __restrict__ w, float b0, float b1,
                                             float (&acc)[8], const float* __restrict__ wnext,
                                             float (&wn)[kSubRows]) {
  acc[0] = pair_term<D0>(a0[0], b0, w[0], acc[0]);
  FS_ORDER_AFTER(acc[0]);
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int r = 0; r < kSubRows; r++) wn[r] = wnext[r];
  __builtin_amdgcn_sched_barrier(0);  // issue the s_loads here, not later
#pragma unroll
  for (int r = 0; r < kSubRows; r++) {
    if (r != 0) acc[r & 3] = pair_term<D0>(a0[r], b0, w[r], acc[r & 3]);
    if (TWO) acc[4 + (r & 3)] = pair_term<D1>(a1[r], b1, w[r], acc[4 + (r & 3)]);
  }
  // keep the next column's arithmetic (which waits for wn) below this point
  __builtin_amdgcn_sched_barrier(0);
}

template <bool D0, bool D1, bool TWO>
__device__ __forceinline__ void score_tiles(const float* __restrict__ xs, int64_t PW,
                                            int64_t c0, int wave,
                                            const int2* __restrict__ tiles,
                                            const float* __restrict__ Wt, int64_t t_begin,
                                            int64_t t_end, double& out0, double& out1) {
  double s0 = 0.0, s1 = 0.0;
  float a0[kSubRows], a1[kSubRows];
  int cur_bi = -1;
  // wA always holds column 0 of the current tile: the last prefetch of a
  // tile is column 0 of the next one (tiles of a segment are consecutive).
  float wA[kSubRows], wB[kSubRows];
  {
    const float* __restrict__ w0 = Wt + t_begin * (kTile * kTile) + wave * kSubRows;
#pragma unroll
    for (int r = 0; r < kSubRows; r++) wA[r] = w0[r];
  }
  for (int64_t t = t_begin; t < t_end; t++) {
    const int2 tl = tiles[t];
    if (tl.x != cur_bi) {
      cur_bi = tl.x;
      const float* __restrict__ xa = xs + ((int64_t)tl.x * kTile + wave * kSubRows) * PW + c0;
#pragma unroll
      for (int r = 0; r < kSubRows; r++) {
        a0[r] = xa[(int64_t)r * PW];
        a1[r] = TWO ? xa[(int64_t)r * PW + 64] : 0.0f;
      }
    }
    const float* __restrict__ wt = Wt + t * (kTile * kTile) + wave * kSubRows;
    const float* __restrict__ xb = xs + (int64_t)tl.y * kTile * PW + c0;
    float bA0 = xb[0], bA1 = TWO ? xb[64] : 0.0f;
    float bB0 = xb[PW], bB1 = TWO ? xb[PW + 64] : 0.0f;
    // The prefetches of the last column pair reach 2 rows past the tile (xs
    // has 2 spare rows) and column 0 of tile t+1 (Wt has a spare tile).
    const float* __restrict__ xn = xb + 2 * PW;
    const float* __restrict__ wn = wt + kTile;
    for (int jb = 0; jb < kTile; jb += 32) {
      float acc[8] = {0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f};
      for (int jj = 0; jj < 32; jj += 2) {
        const float cA0 = xn[0], cA1 = TWO ? xn[64] : 0.0f;
        const float cB0 = xn[PW], cB1 = TWO ? xn[PW + 64] : 0.0f;
        score_column<D0, D1, TWO>(a0, a1, wA, bA0, bA1, acc, wn, wB);
        score_column<D0, D1, TWO>(a0, a1, wB, bB0, bB1, acc, wn + kTile, wA);
        bA0 = cA0; bA1 = cA1; bB0 = cB0; bB1 = cB1;
        xn += 2 * PW;
        wn += 2 * kTile;
      }
      s0 += ((double)acc[0] + (double)acc[1]) + ((double)acc[2] + (double)acc[3]);
      if (TWO) s1 += ((double)acc[4] + (double)acc[5]) + ((double)acc[6] + (double)acc[7]);
    }
  }
  out0 = s0;
  out1 = s1;
}

// XCD-aware grid: workgroup w normally runs on XCD w % 8, so XCD x is given
// the segments s = x, x + 8, ... with all nfb feature blocks of a segment in
// consecutive slots.  The ~160 workgroups an XCD holds at a time then share
// one segment's pair weights (30 tiles x 64 KB) in that XCD's L2 instead of
// ~8 segments thrashing it; the 1-D grid has 8 * max_x(segments of x) * nfb
// slots, the few beyond nseg exit at once.
// row blocks per group of the sparse pass-2 schedule (build_sparse_schedule;
// 16 / kSchedRows feature blocks per block of units)

__global__ __launch_bounds__(256) void k_score(const float* __restrict__ xs, int64_t PW,
                                               int64_t PC, const int2* __restrict__ tiles,
                                               const float* __restrict__ Wt, int64_t n_tiles,
                                               int64_t seg_len, int64_t nseg, int64_t nfb,
                                               double* __restrict__ spart) {
  __shared__ double red[2][4][64];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t w = blockIdx.x;
  const int64_t xcd = w % kXcds, k = w / kXcds;
  const int64_t seg = xcd + kXcds * (k / nfb), fb = k % nfb;
  if (seg >= nseg) return;
  const int64_t f0 = fb * 128;
  const int64_t c0 = f0 + lane;
  const int64_t t_begin = seg * seg_len;
  const int64_t t_end = t_begin + seg_len < n_tiles ? t_begin + seg_len : n_tiles;
  const bool two = f0 + 64 < PW;
  const bool d0 = f0 >= PC, d1 = f0 + 64 >= PC;
  double s0 = 0.0, s1 = 0.0;
  if (two) {
    if (!d1) score_tiles<false, false, true>(xs, PW, c0, wave, tiles, Wt, t_begin, t_end, s0, s1);
    else if (d0) score_tiles<true, true, true>(xs, PW, c0, wave, tiles, Wt, t_begin, t_end, s0, s1);
    else score_tiles<false, true, true>(xs, PW, c0, wave, tiles, Wt, t_begin, t_end, s0, s1);
  } else {
    if (d0) score_tiles<true, true, false>(xs, PW, c0, wave, tiles, Wt, t_begin, t_end, s0, s1);
    else score_tiles<false, false, false>(xs, PW, c0, wave, tiles, Wt, t_begin, t_end, s0, s1);
  }
  red[0][wave][lane] = s0;
  red[1][wave][lane] = s1;
  __syncthreads();
  if (wave < 2 && (wave == 0 || two)) {
    const double v = (red[wave][0][lane] + red[wave][1][lane]) + (red[wave][2][lane] + red[wave][3][lane]);
    spart[seg * PW + c0 + wave * 64] = v;
  }
}

// ---------------------------------------------------------------------------
// Pass 2, sparse v2: 64-row half tiles, 8 features per lane
// ---------------------------------------------------------------------------
// Grid as k_score (XCD-aware, segments of consecutive tiles), 16 waves per
// workgroup (one workgroup per CU).  The round-1/2 form (v1, retired in
// round 4) held a whole 128-row tile per wave, so a workgroup
// kept 128 rows x 256 features (128 KB) in LDS and every entry fed 4
// features per lane: the entry streams were re-read once per 256-feature
// block (79 times at cfg4) and each scalar load of 8 entries covered 8 x 9
// VALU.  v2 splits each tile into its two 64-row halves: a workgroup keeps 64 rows x
// 512 features (the same 128 KB) and every entry feeds 8 features per lane --
// one v_add_u32 address, two ds_read_b128, 8 x (v_sub_f32, v_fma_f32 |.|): 17
// VALU per 8 pair-features instead of 18, half the scalar loads and half the
// entry-stream reads per pair-feature (40 feature blocks at cfg4), and twice
// the arithmetic behind every scalar load.  The B rows (the tile's columns)
// are read once per half instead of once per tile; the two halves of a
// (segment, feature block) sit in adjacent grid slots of one XCD, so the
// second read is mostly an L2 hit.
//
// Stream (t, h, w) (k_weights_sparse2): the columns jj = w, w + 16, ... (8)
// of owned tile t, each column's non-zero weights of the rows ii in
// [64h, 64h + 64) as entries ((ii - 64h) * 2048, weight) in ascending ii --
// 2048 = the byte stride of a row in the LDS block -- with NO padding: the
// lowest mantissa bit of a weight is set on the last entry of its column and
// clear elsewhere (a <= 1-ulp change, far below the 1e-5 bar), and an empty
// column holds one (0, 0x1) entry (a denormal weight, zero for every
// purpose).  Stream (t, h, w) starts at ent + ((t * 2 + h) * 16 + w) *
// kStreamEntries2; 8 columns x 64 rows fill it at most.
constexpr int kHalf = 64;
constexpr int kRowBytes2 = 2048;                           // 64 lanes x 8 floats
constexpr int kStreamEntries2 = (kTile / kSWaves) * kHalf;  // 512
static_assert(kStreamEntries2 * 2 == kStreamEntries, "v2 streams reuse the v1 buffer size");

__global__ __launch_bounds__(1024) void k_weights_sparse2(
    const double* __restrict__ D, int64_t n, int64_t n_pad, int tiled, int2 win,
    const int2* __restrict__ tiles, const double* __restrict__ thr,
    const int32_t* __restrict__ lab,
    const double* __restrict__ counts, int algo, int use_star, double inv_sc, int64_t r_lo,
    int64_t r_hi, uint2* __restrict__ ent, unsigned long long* __restrict__ nnz) {
  __shared__ int wave_nnz[kSWaves];
  const int2 tl = tiles[blockIdx.x];
  const int64_t i0 = (int64_t)tl.x * kTile, j0 = (int64_t)tl.y * kTile;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint2* out0 = ent + (((int64_t)blockIdx.x * 2 + 0) * kSWaves + wave) * kStreamEntries2;
  uint2* out1 = ent + (((int64_t)blockIdx.x * 2 + 1) * kSWaves + wave) * kStreamEntries2;
  const uint64_t below = lane ? (~0ull >> (64 - lane)) : 0ull;
  const uint32_t roff = (uint32_t)lane * (uint32_t)kRowBytes2;
  int off0 = 0, off1 = 0, nz = 0;
  for (int jj = wave; jj < kTile; jj += kSWaves) {
    const float w0 = pair_weight(D, n, n_pad, tiled, win, blockIdx.x, i0, j0, lane, jj,
                                 tl.x < tl.y || lane < jj, thr, lab, counts, algo, use_star,
                                 inv_sc, r_lo, r_hi);
    const float w1 = pair_weight(D, n, n_pad, tiled, win, blockIdx.x, i0, j0, lane + 64, jj,
                                 tl.x < tl.y || lane + 64 < jj, thr, lab, counts, algo, use_star,
                                 inv_sc, r_lo, r_hi);
    const uint64_t m0 = __ballot(w0 != 0.0f), m1 = __ballot(w1 != 0.0f);
    const int n0 = __popcll(m0), n1 = __popcll(m1);
    // stream lengths (at least one entry: an empty column still ends)
    const int p0 = n0 == 0 ? 1 : n0;
    const int p1 = n1 == 0 ? 1 : n1;
    const int e0 = __popcll(m0 & below), e1 = __popcll(m1 & below);
    if (w0 != 0.0f) out0[off0 + e0] = make_uint2(roff, weight_bits(w0, e0 == p0 - 1));
    if (w1 != 0.0f) out1[off1 + e1] = make_uint2(roff, weight_bits(w1, e1 == p1 - 1));
    if (n0 + lane < p0) out0[off0 + n0 + lane] = make_uint2(0u, n0 + lane == p0 - 1 ? 1u : 0u);
    if (n1 + lane < p1) out1[off1 + n1 + lane] = make_uint2(0u, n1 + lane == p1 - 1 ? 1u : 0u);
    off0 += p0;
    off1 += p1;
    nz += n0 + n1;
  }
  if (lane == 0) wave_nnz[wave] = nz;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long t = 0;
    for (int w = 0; w < kSWaves; w++) t += (unsigned long long)wave_nnz[w];
    atomicAdd(nnz, t);
  }
}

// Generic (plain HIP) walk of one v2 stream: F features per lane (8: chunks
// c = 0, 1 of the row, 4 each; 4: chunk 0 only), per-lane discrete flags.
// Used for feature blocks holding discrete features; continuous blocks take
// the generated loop of fs_sparse_asm.inc.
template <int F>
__device__ __forceinline__ void sparse2_stream_generic(const float4* __restrict__ As,
                                                       const uint2* __restrict__ e,
                                                       const float* __restrict__ xb, int64_t bstride,
                                                       int lane, const bool (&disc)[F],
                                                       float (&acc)[F]) {
  constexpr int C = F / 4;
  float b[F];
  int col = 0;
#pragma unroll
  for (int c = 0; c < C; c++) {
    const float4 v = *(const float4*)(xb + 256 * c);
    b[4 * c] = v.x; b[4 * c + 1] = v.y; b[4 * c + 2] = v.z; b[4 * c + 3] = v.w;
  }
  for (int q = 0; q < kStreamEntries2; q++) {
    const uint2 E = e[q];
    const float w = __uint_as_float(E.y);
#pragma unroll
    for (int c = 0; c < C; c++) {
      const float4 a = As[(E.x >> 4) + 64 * c + lane];
      const float av[4] = {a.x, a.y, a.z, a.w};
#pragma unroll
      for (int k = 0; k < 4; k++) {
        const int f = 4 * c + k;
        acc[f] = disc[f] ? pair_term<true>(av[k], b[f], w, acc[f])
                         : pair_term<false>(av[k], b[f], w, acc[f]);
      }
    }
    if (E.y & 1u) {  // last entry of the column
      if (++col == kTile / kSWaves) break;
      xb += bstride;
#pragma unroll
      for (int c = 0; c < C; c++) {
        const float4 v = *(const float4*)(xb + 256 * c);
        b[4 * c] = v.x; b[4 * c + 1] = v.y; b[4 * c + 2] = v.z; b[4 * c + 3] = v.w;
      }
    }
  }
}

// Grid: one workgroup per unit (segment, feature block, half) of the pass-2
// schedule (build_sparse_schedule, host side): units[w] = (seg, 2 fb + h),
// or seg = -1 for the padding slots of a short XCD list.  A segment is a run
// of tiles of one row block (its rows are staged into LDS once) in descending
// column-block order, tile indices sched[seg_off[seg] .. seg_off[seg + 1]).
// F = 8: 512-feature blocks f_base + 512 fb; F = 4: 256-feature blocks (the
// tail of a layout whose width is not a multiple of 512).  Lane l scores
// features f0 + 4l + k and (F = 8) f0 + 256 + 4l + k, k = 0..3; partials go
// to spart[(seg * 2 + h) * PW + f].
template <int F>
__global__ __launch_bounds__(1024) void k_score_sparse2(
    const float* __restrict__ xs, int64_t PW, int64_t PC, const int2* __restrict__ tiles,
    const uint2* __restrict__ ent, const int32_t* __restrict__ sched,
    const int32_t* __restrict__ seg_off, const int2* __restrict__ units, int64_t f_base,
    double* __restrict__ spart) {
  constexpr int C = F / 4;
  __shared__ float4 As[kHalf * 2 * 64];  // 64 rows x 2 chunks x 64 lanes (128 KB)
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int2 unit = units[blockIdx.x];
  if (unit.x < 0) return;
  const int64_t seg = unit.x, fb = unit.y >> 1, h = unit.y & 1;
  const int64_t f0 = f_base + fb * (64 * F);
  const int64_t t_begin = seg_off[seg];
  const int64_t t_end = seg_off[seg + 1];
  bool disc[F];
#pragma unroll
  for (int c = 0; c < C; c++)
#pragma unroll
    for (int q = 0; q < 4; q++) disc[4 * c + q] = f0 + 256 * c + 4 * lane + q >= PC;
  // the generated loop when every real feature of the block is continuous;
  // features past PW stage zeros and their accumulators are discarded (their
  // B values are read past the row's end: xs has kXsSlack floats of slack)
  const int64_t f_end = f0 + 64 * F < PW ? f0 + 64 * F : PW;
  const bool fast = f_end <= PC;
  const uint32_t lds_lane = (uint32_t)(uintptr_t)As + (uint32_t)lane * 16u;
  const uint32_t glb_lane = (uint32_t)lane * 16u;
  const uint32_t pf_lane = (uint32_t)lane * 32u;
  const int64_t bstride = kSWaves * PW;
  const uint32_t bstride_b = (uint32_t)(bstride * sizeof(float));
  const uint32_t ncols = kTile / kSWaves;
  double s[F];
#pragma unroll
  for (int q = 0; q < F; q++) s[q] = 0.0;
  // VALU issue goes to the oldest ready wave of a SIMD (MI355X_MICROARCH.md,
  // "Two waves per SIMD" item 2), so with equal static shares the 16 waves
  // of a unit finished staggered -- the oldest first, the youngest last with
  // few partners to hide its latency: 26% of the waves' lives waited at the
  // final barrier (round 4's clock-stamp build, profiles/r04/pass2_prio.txt).  A wave behind
  // the workgroup's mean progress (tiles done, an LDS counter) raises its
  // priority until it has caught up: 4.9% left waiting, pass 2 88.0 -> 81.2
  // ms at cfg4.  The scores do not change (same streams per wave, same order).
  __shared__ unsigned int wg_done;
  if (threadIdx.x == 0) wg_done = 0u;  // before the first staging barrier
  unsigned int my_done = 0;
  // The segment's tile list, 64 tiles per lane-indexed load: tile k - t_begin
  // is lane (k - t_begin) % 64 of my_t / my_x / my_y (v_readlane per tile,
  // instead of two dependent scalar loads -- sched, then tiles -- per tile).
  int my_t = 0, my_x = -1, my_y = 0;
  int cur_bi = -1;
  for (int64_t k = t_begin; k < t_end; k++) {
    const int idx = (int)((k - t_begin) & 63);
    if (idx == 0) {
      const int64_t kk = k + lane;
      my_t = kk < t_end ? sched[kk] : sched[k];
      const int2 tt = tiles[my_t];
      my_x = tt.x;
      my_y = tt.y;
    }
    const int64_t t = __builtin_amdgcn_readlane(my_t, idx);
    const int2 tl = make_int2(__builtin_amdgcn_readlane(my_x, idx), __builtin_amdgcn_readlane(my_y, idx));
    if (tl.x != cur_bi) {  // once per segment: its tiles share one row block
      __syncthreads();
      // 64 rows x 2 chunks = 128 float4 per lane: 8 per wave, all requested
      // before the first store (one HBM latency per segment, not eight)
      const float* __restrict__ xa = xs + ((int64_t)tl.x * kTile + h * kHalf) * PW + f0 + 4 * lane;
      constexpr int kPer = kHalf * 2 / kSWaves;
      float4 v[kPer];
#pragma unroll
      for (int m = 0; m < kPer; m++) {
        const int rc = wave + kSWaves * m, r = rc >> 1, c = rc & 1;
        v[m] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        if (c < C && f0 + 256 * c + 4 * lane < PW) v[m] = *(const float4*)(xa + (int64_t)r * PW + 256 * c);
      }
#pragma unroll
      for (int m = 0; m < kPer; m++) As[(wave + kSWaves * m) * 64 + lane] = v[m];
      __syncthreads();
      cur_bi = tl.x;
    }
    float acc[F];
#pragma unroll
    for (int q = 0; q < F; q++) acc[q] = 0.0f;
    const uint2* __restrict__ e = ent + ((t * 2 + h) * kSWaves + wave) * kStreamEntries2;
    const float* __restrict__ xb = xs + ((int64_t)tl.y * kTile + wave) * PW + f0;
    if (fast) {
      const uint64_t eb = (uint64_t)(uintptr_t)e;
      const uint64_t bp = (uint64_t)(uintptr_t)xb;
      // next-tile prefetch operands of the loop (the shipped loops are
      // generated without the prefetch: tools/gen_sparse_asm.py pfn)
      const uint64_t bpn = bp, enb = eb;
      if constexpr (F == 8) {
        FS_SPARSE2_ASM_F8(acc, lds_lane, glb_lane, eb, bp, bstride_b, ncols, bpn, pf_lane, enb);
      } else
        FS_SPARSE2_ASM_F4(acc, lds_lane, glb_lane, eb, bp, bstride_b, ncols, bpn, pf_lane, enb);
    } else {
      sparse2_stream_generic<F>(As, e, xb + 4 * lane, bstride, lane, disc, acc);
    }
#pragma unroll
    for (int q = 0; q < F; q++) s[q] += (double)acc[q];
    unsigned int tot = 0;
    if (lane == 0) tot = atomicAdd(&wg_done, 1u) + 1u;
    tot = __builtin_amdgcn_readfirstlane(tot);
    ++my_done;
    if (my_done * kSWaves < tot)
      __builtin_amdgcn_s_setprio(2);
    else
      __builtin_amdgcn_s_setprio(0);
  }
  // fixed-order reduction of the 16 waves' partials through the LDS block
  __syncthreads();
  double* red = (double*)As;  // [F][kSWaves][64] (64 KB at F = 8)
#pragma unroll
  for (int q = 0; q < F; q++) red[(q * kSWaves + wave) * 64 + lane] = s[q];
  __syncthreads();
  if (wave < F) {
    const int q = wave;                                  // feature f0 + 256 (q/4) + 4 lane + q%4
    const int64_t f = f0 + 256 * (q >> 2) + 4 * lane + (q & 3);
    const double* rr = red + q * kSWaves * 64 + lane;
    double v = 0.0;
#pragma unroll
    for (int w = 0; w < kSWaves; w += 4)
      v += (rr[w * 64] + rr[(w + 1) * 64]) + (rr[(w + 2) * 64] + rr[(w + 3) * 64]);
    if (f < PW) spart[(seg * 2 + h) * PW + f] = v;
  }
}

// dst[k] += src[k] (the tile shards' partial vectors, summed in shard order).
__global__ void k_accumulate(double* __restrict__ dst, const double* __restrict__ src,
                             int64_t count) {
  const int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (k < count) dst[k] += src[k];
}

// out[out_pos[c]] = sum over segments of part[seg][c] (fixed order).  One
// 1024-thread workgroup per 64 columns: wave w sums the segments w, w + 16,
// ... (one coalesced 512-byte read per segment), then the 16 partials are
// added in a fixed tree (deterministic run to run).  A thread per column
// walking every segment (the round-2 form) left ~80 workgroups on the chip:
// 0.3 ms for one rank of N = 8 at cfg4.
constexpr int kReduceWaves = 16;
__global__ __launch_bounds__(1024) void k_reduce(const double* __restrict__ part, int64_t nseg,
                                                 int64_t PW, const int64_t* __restrict__ out_pos,
                                                 const double* __restrict__ add,
                                                 double* __restrict__ out) {
  __shared__ double red[kReduceWaves][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t c = (int64_t)blockIdx.x * 64 + lane;
  double s = 0.0;
  if (c < PW)
    for (int64_t g = wave; g < nseg; g += kReduceWaves) s += part[g * PW + c];
  red[wave][lane] = s;
  __syncthreads();
  if (wave != 0 || c >= PW) return;
  const int64_t o = out_pos[c];
  if (o < 0) return;
  double q[4];
#pragma unroll
  for (int k = 0; k < 4; k++)
    q[k] = (red[4 * k][lane] + red[4 * k + 1][lane]) + (red[4 * k + 2][lane] + red[4 * k + 3][lane]);
  out[o] = ((q[0] + q[1]) + (q[2] + q[3])) + (add ? add[c] : 0.0);
}

int accumulate(double* dst, const double* src, int64_t count, hipStream_t st) {
  if (count <= 0) return FS_OK;
  k_accumulate<<<(unsigned)((count + 255) / 256), 256, 0, st>>>(dst, src, count);
  return launch_check("k_accumulate");
}

int reduce_segments(const double* part, int64_t nrows, int64_t PW, const int64_t* out_pos,
                    double* sums, hipStream_t st, const double* add) {
  k_reduce<<<(unsigned)((PW + 63) / 64), 1024, 0, st>>>(part, nrows, PW, out_pos, add, sums);
  return launch_check("k_reduce");
}

// Shard part of a plan's layout: this rank's continuous columns of the mean
// correction and the pass-2 segments (sized by the owned tiles and the
// feature blocks), with the segment partials' buffer grown when needed.
// plan_layout calls it, and plan_set_shard alone: re-targeting a plan to
// Pass-2 schedule of the sparse kernels (k_score_sparse2).  The B operand of
// a tile (its 128 column samples' values, 2 KB each per 512-feature block)
// is read once per (tile, feature block, half): ~250 GB per launch at cfg4,
// far more than L2 holds when the workgroups on an XCD all walk different
// column blocks.  Here the units an XCD runs at the same time walk the SAME
// column blocks in the same order:
//  * segment = the owned tiles of one row block I whose column block J falls
//    in one chunk of seg_len * world blocks (~seg_len tiles), in descending
//    J (so the segments of a group start aligned at the chunk's end);
//  * group = the segments of one chunk from kSchedRows consecutive row
//    blocks (they share every J they hold);
//  * block = one group x kSchedFb feature blocks x both halves (<= 64
//    units, two rounds of an XCD's 32 CUs), dealt to the XCD with the least
//    work so far (workgroup w runs on XCD w % 8; each XCD's list is padded
//    with empty units to the longest).
// Concurrent units then share their B rows through the XCD's L2 (kSchedRows
// row blocks x 2 halves read each) and their entry streams (kSchedFb
// feature blocks read each).  16 row blocks x 2 feature blocks against
// round 4's 8 x 2: pass 2 0.2-0.6 ms shorter at cfg4 on two boxes
// (profiles/r05/sched_ab.txt; 4 x 4 0.4-0.7 ms longer).
#ifndef FS_SCHED_ROWS
#define FS_SCHED_ROWS 16
#endif
#ifndef FS_SCHED_UNITS
#define FS_SCHED_UNITS 32
#endif
constexpr int kSchedRows = FS_SCHED_ROWS;
constexpr int kSchedFb = FS_SCHED_UNITS / kSchedRows;

static int ensure_dev(Plan* g, void** buf, size_t* cap, size_t bytes) {
  if (bytes <= *cap) return FS_OK;
  if (*buf) {
    FS_HIP(hipStreamSynchronize(g->stream));
    dev_free(*buf);
    *buf = nullptr;
    *cap = 0;
  }
  FS_TRY(dev_alloc(buf, bytes, g->device));
  *cap = bytes;
  return FS_OK;
}

static int build_sparse_schedule(Plan* g) {
  const Prepared& Q = g->P;
  const int64_t T = g->n_tiles;
  const int64_t CJ = std::max<int64_t>(1, g->seg_len * std::max(1, g->world));
  std::vector<int32_t> sched, seg_off{0};
  std::vector<int64_t> seg_tiles;
  std::map<std::pair<int64_t, int64_t>, std::vector<int32_t>> groups;  // (chunk, I group) -> segs
  sched.reserve((size_t)T);
  for (int64_t t = 0; t < T;) {  // h_tiles are ordered by (I, J)
    const int I = g->h_tiles[t].x;
    const int64_t c = g->h_tiles[t].y / CJ;
    int64_t e = t;
    // at most 64 tiles (a lane-indexed tile list per segment)
    while (e < T && e - t < 64 && g->h_tiles[e].x == I && g->h_tiles[e].y / CJ == c) e++;
    for (int64_t k = e - 1; k >= t; k--) sched.push_back((int32_t)k);
    groups[{c, I / kSchedRows}].push_back((int32_t)seg_tiles.size());
    seg_tiles.push_back(e - t);
    seg_off.push_back((int32_t)sched.size());
    t = e;
  }
  g->nseg = std::max<int64_t>(1, (int64_t)seg_tiles.size());
  // feature blocks of the two launches (run_pass2): 512-wide, then a tail
  // of <= 256 features in one 256-wide block (a longer tail takes one more,
  // partial, 512-wide block: its cost is mostly its entry walk)
  g->nfb8 = Q.PW / 512;
  if (Q.PW - g->nfb8 * 512 > 256) g->nfb8++;
  g->f_tail = std::min<int64_t>(g->nfb8 * 512, Q.PW);
  g->nfb4 = (Q.PW - g->f_tail + 255) / 256;
  auto units_of = [&](int64_t nfb, std::vector<int2>& table) {
    std::vector<std::vector<int2>> per(kXcds);
    std::vector<int64_t> load(kXcds, 0);
    for (const auto& gr : groups)
      for (int64_t f0 = 0; f0 < nfb; f0 += kSchedFb) {
        int x = 0;
        for (int q = 1; q < kXcds; q++)
          if (load[q] < load[x]) x = q;
        for (int64_t fb = f0; fb < std::min<int64_t>(nfb, f0 + kSchedFb); fb++)
          for (int32_t sg : gr.second)
            for (int h = 0; h < 2; h++) {
              per[x].push_back(make_int2(sg, (int)(2 * fb + h)));
              load[x] += seg_tiles[sg];
            }
      }
    size_t kmax = 0;
    for (const auto& v : per) kmax = std::max(kmax, v.size());
    table.assign(kXcds * kmax, make_int2(-1, 0));
    for (int x = 0; x < kXcds; x++)
      for (size_t k = 0; k < per[x].size(); k++) table[x + kXcds * k] = per[x][k];
  };
  std::vector<int2> u8, u4;
  units_of(g->nfb8, u8);
  units_of(g->nfb4, u4);
  g->nunits8 = (int64_t)u8.size();
  g->nunits4 = (int64_t)u4.size();
  if (sched.empty()) sched.push_back(0);
  const size_t ns = sched.size() + seg_off.size();
  const size_t nu = std::max<size_t>(1, u8.size() + u4.size());
  FS_TRY(ensure_dev(g, (void**)&g->sched, &g->sched_cap, ns * sizeof(int32_t)));
  FS_TRY(ensure_dev(g, (void**)&g->units8, &g->units_cap, nu * sizeof(int2)));
  g->seg_off = g->sched + sched.size();
  g->units4 = g->units8 + u8.size();
  FS_TRY(h2d(g, g->sched, sched.data(), sched.size()));
  FS_TRY(h2d(g, g->seg_off, seg_off.data(), seg_off.size()));
  if (!u8.empty()) FS_TRY(h2d(g, g->units8, u8.data(), u8.size()));
  if (!u4.empty()) FS_TRY(h2d(g, g->units4, u4.data(), u4.size()));
  return FS_OK;
}

// another tile shard keeps the feature layout, its tables and its band
// calibration (none of them depends on the shard).
int shard_segments(Plan* g) {
  const Prepared& Q = g->P;
  g->corr_ready = false;  // a new column share: the row guard's correction is not this shard's
  g->c_lo = Q.pc * g->rank / g->world;
  g->c_hi = Q.pc * (g->rank + 1) / g->world;
  // Pass-2 workgroups: ~64k for the dense pass (256 threads, 128-feature
  // blocks), ~32k for the sparse one (1024 threads, 256-feature blocks):
  // enough to fill 256 CUs and bound tail imbalance.  Measured for the sparse
  // pass at cfg4 (tools/pass2_wgs.sh, k_score_sparse ms at world 1 / one rank
  // of 8; profiles/r01k/pass2_wgs.txt): 8k 111.8 / 14.7, 16k 105.9 / 14.6,
  // then on one box, alternating, 32k 107.6 / 14.9 and 107.7 / 14.6 against
  // 64k 108.1 / 15.0 and 108.0 / 14.6 -- the tail costs more than the
  // per-workgroup row-block stage below 32k.
  // Small problems (cfg2: 820 tiles x 20 blocks) take a quarter of their
  // (tile, block) units as the target, at least 4096: segments of ~4 tiles
  // amortise each workgroup's row-block stage (tools/cfg2_sweep.sh,
  // profiles/r02/cfg2_sweep.txt: cfg2 step 6.11 -> 5.83 ms at 4096-8192).
  // sparse: (512-feature block, half) units, two per 512 features
  const int64_t nfb = !g->sparse ? (Q.PW + 127) / 128 : 2 * ((Q.PW + 511) / 512);
  // Round 4 (progress priority, build_sparse_schedule): small problems take
  // a sixteenth of their units as the target, at least 1024 -- longer
  // segments amortise each unit's staging and final barrier (cfg2: 16 tiles
  // per segment, pass 2 1.50-1.54 -> 1.39-1.42 ms, profiles/r04/seg_len_ab.txt;
  // cfg4 keeps ~31)
  const int64_t wgs =
      g->sparse ? std::min<int64_t>(32768, std::max<int64_t>(1024, g->n_tiles * nfb / 16)) : 65536;
  g->seg_len = std::max<int64_t>(1, (g->n_tiles * nfb + wgs - 1) / wgs);
  g->nseg = std::max<int64_t>(1, (g->n_tiles + g->seg_len - 1) / g->seg_len);
  if (Q.algo == ALGO_RELIEFF) return FS_OK;
  if (g->sparse) FS_TRY(build_sparse_schedule(g));  // its own segments (g->nseg)
  // partial rows per segment: one per half with the sparse streams
  g->nsegpart = g->sparse ? 2 * g->nseg : g->nseg;
  const size_t need = (size_t)g->nsegpart * Q.PW;
  if (need > g->spart_cap) {
    if (g->spart) {
      FS_HIP(hipStreamSynchronize(g->stream));
      dev_free(g->spart);
      g->spart = nullptr;
      g->spart_cap = 0;
    }
    void* q = nullptr;
    FS_TRY(dev_alloc(&q, need * sizeof(double), g->device));
    g->spart = (double*)q;
    g->spart_cap = need;
  }
  return FS_OK;
}

// Pair weights of the owned tiles in the form pass 2 reads (dense or sparse).
int run_weights(Plan* g, const double* counts, int algo, double inv_sc) {
  const Prepared& Q = g->P;
  // the star split's per-column terms (this rank's column share, whatever
  // tiles it owns); k_reduce adds them
  // (SURF*: forked beside pass 1, run_quantize_dist; MultiSURF*: the
  // per-sample sums too, weighed by the counts here)
  if (g->star_split && algo == ALGO_MULTISURF) {
    FS_HIP(hipStreamWaitEvent(g->stream, g->ev_star, 0));
    FS_TRY(star_reduce(g, counts, g->stream));
  }
  if (g->n_tiles == 0) return FS_OK;
  const int star = g->star_split ? 2 : Q.use_star;
  if (g->sparse) {
    FS_HIP(hipMemsetAsync(g->nnz, 0, sizeof(unsigned long long), g->stream));
    g->nnz_valid = true;
    k_weights_sparse2<<<(unsigned)g->n_tiles, 64 * kSWaves, 0, g->stream>>>(
        g->D, Q.n, Q.n_pad, g->tiled, g->win, g->tiles, g->thr, g->lab, counts, algo,
        star, inv_sc, g->r_lo, g->r_hi, g->ent, g->nnz);
    return launch_check("k_weights_sparse2");
  }
  k_weights<<<(unsigned)g->n_tiles, 256, 0, g->stream>>>(g->D, Q.n, Q.n_pad, g->tiled, g->win,
                                                         g->tiles,
                                                         g->thr,
                                                         g->lab, counts, algo, star, inv_sc,
                                                         g->r_lo, g->r_hi, g->Wt);
  return launch_check("k_weights");
}

int run_pass2(Plan* g, double* scores_dev) {
  const Prepared& Q = g->P;
  const int64_t nfb = (Q.PW + 127) / 128;
  const double* add = g->star_split ? g->tcol : nullptr;
  FS_HIP(hipMemsetAsync(scores_dev, 0, sizeof(double) * Q.n_kept, g->stream));
  if (add && Q.algo == ALGO_SURF) FS_HIP(hipStreamWaitEvent(g->stream, g->ev_join, 0));
  if (g->n_tiles == 0) {
    if (add) return reduce_segments(g->spart, 0, Q.PW, g->out_pos, scores_dev, g->stream, add);
    return FS_OK;
  }
  FS_HIP(hipEventRecord(g->ev[2], g->stream));
  const int64_t seg_per_xcd = (g->nseg + kXcds - 1) / kXcds;
  if (g->sparse) {
    // 512-feature blocks, then the tail block (build_sparse_schedule; one
    // F = 8 block is cheaper than two F = 4 ones -- cfg2, 448 features:
    // 0.24 -> 0.17 ms)
    if (g->nunits8 > 0) {
      k_score_sparse2<8><<<(unsigned)g->nunits8, 64 * kSWaves, 0, g->stream>>>(
          g->xs, Q.PW, Q.PC, g->tiles, g->ent, g->sched, g->seg_off, g->units8, 0, g->spart);
      FS_TRY(launch_check("k_score_sparse2<8>"));
    }
    if (g->nunits4 > 0) {
      k_score_sparse2<4><<<(unsigned)g->nunits4, 64 * kSWaves, 0, g->stream>>>(
          g->xs, Q.PW, Q.PC, g->tiles, g->ent, g->sched, g->seg_off, g->units4, g->f_tail,
          g->spart);
      FS_TRY(launch_check("k_score_sparse2<4>"));
    }
  } else {
    k_score<<<(unsigned)(kXcds * seg_per_xcd * nfb), 256, 0, g->stream>>>(
        g->xs, Q.PW, Q.PC, g->tiles, g->Wt, g->n_tiles, g->seg_len, g->nseg, nfb, g->spart);
    FS_TRY(launch_check("k_score"));
  }
  FS_HIP(hipEventRecord(g->ev[3], g->stream));
  k_reduce<<<(unsigned)((Q.PW + 63) / 64), 1024, 0, g->stream>>>(g->spart, g->nsegpart, Q.PW,
                                                                   g->out_pos, add, scores_dev);
  return launch_check("k_reduce");
}

// Reference-order pass 2 (P.ref_accum), split at the point where every
// owned tile's decisions are known: ref_masks writes the masks of the
// current shard's tiles; ref_chains, once every tile of the triangle has
// written its masks, runs the chains of the focal rows [r_lo, r_hi) and the
// float32 column sums into scores[n_kept] (as doubles; the reference's
// float32 sums, not yet divided by n).
int ref_masks(Plan* g) {
  const Prepared& Q = g->P;
  if (!g->masks) {  // the plan's own masks, on first use
    const int at = g->alloc_target;
    g->alloc_target = 0;
    const int rc = dalloc(g, &g->masks, (size_t)ref_mask_words(g));
    g->alloc_target = at;
    FS_TRY(rc);
  }
  return refacc::multisurf_masks(g->D, Q.n, Q.n_pad, g->tiles, g->n_tiles, g->thr, g->lab,
                                 Q.use_star, g->masks, g->stream);
}

// temp[rows][Kp] (float32 rows of the reference's temp matrix), kept between
// steps and grown on demand.
int ref_temp(Plan* g, int64_t rows, float** out) {
  const size_t need = (size_t)std::max<int64_t>(rows, 1) * (size_t)g->Kp;
  if (need > g->temp_cap) {
    if (g->temp) dev_free(g->temp);
    g->temp = nullptr;
    g->temp_cap = 0;
    void* p = nullptr;
    FS_TRY(dev_alloc(&p, need * sizeof(float), g->device));
    g->temp = (float*)p;
    g->temp_cap = need;
  }
  *out = g->temp;
  return FS_OK;
}

// SURF / SURF* in the reference's order (fs_refacc.hip): the masks of the
// focal rows (a per-call buffer, rows x n_pad / 2 bytes: row-local
// decisions), the four chains into the temp rows, then the float32 column
// sums -- continuing from `sums` for a later row panel (ref_seeded), or left
// for plan_ref_sums (ref_defer: row-sharded SURF over ranks).
int surf_ref(Plan* g, double* sums) {
  const Prepared& Q = g->P;
  const int64_t rows = g->r_hi - g->r_lo;
  if (!g->ref_defer && !g->ref_seeded)
    FS_HIP(hipMemsetAsync(sums, 0, sizeof(double) * Q.n_kept, g->stream));
  if (rows <= 0) {
    g->ref_rows = 0;
    return FS_OK;
  }
  uint64_t* m = nullptr;
  g->alloc_target = 2;  // scratch of this plan_score
  const int rc = dalloc(g, &m, (size_t)rows * (Q.n_pad / 64) * 4);
  g->alloc_target = 0;
  FS_TRY(rc);
  float* temp = nullptr;
  FS_TRY(ref_temp(g, rows, &temp));
  FS_HIP(hipEventRecord(g->ev[2], g->stream));
  FS_TRY(refacc::surf_masks(g->D, Q.n, Q.n_pad, g->thr, g->lab, Q.use_star, g->r_lo, g->r_hi, m,
                            g->stream));
  FS_TRY(refacc::surf_chains(g->xk64, g->Kp, g->krecip, g->kdisc, g->kblk, m, Q.n, Q.n_pad,
                             Q.use_star, g->r_lo, g->r_hi, temp, g->stream));
  FS_HIP(hipEventRecord(g->ev[3], g->stream));
  if (g->ref_defer) {
    g->ref_rows = rows;
    return FS_OK;
  }
  return refacc::column_sums(temp, rows, g->Kp, Q.n_kept, g->ref_seeded ? sums : nullptr, sums,
                             g->stream);
}

int ref_chains(Plan* g, const double* counts, double* scores) {
  const Prepared& Q = g->P;
  const int64_t rows = g->r_hi - g->r_lo;
  FS_HIP(hipMemsetAsync(scores, 0, sizeof(double) * Q.n_kept, g->stream));
  if (rows <= 0) return FS_OK;
  float* temp = nullptr;
  FS_TRY(ref_temp(g, rows, &temp));
  FS_HIP(hipEventRecord(g->ev[2], g->stream));
  FS_TRY(refacc::multisurf_chains(g->xk, g->Kp, g->krecip, g->kdisc, g->kblk, g->masks, Q.n,
                                  Q.n_pad, counts, Q.use_star, g->r_lo, g->r_hi, temp, g->stream));
  FS_HIP(hipEventRecord(g->ev[3], g->stream));
  return refacc::column_sums(temp, rows, g->Kp, Q.n_kept, nullptr, scores, g->stream);
}

// Reference order across ranks (fs_plan_ref_masks / fs_plan_ref_pass2):
// this plan's tile decisions into a caller-owned mask buffer, zeroed first
// (every (row, word) belongs to one tile, so the ranks' buffers add up to
// the whole matrix's -- a SUM all-reduce of the words), then the chains of
// the focal rows [lo, hi) over the combined masks into the plan's temp rows
// (every rank at once), and their float32 sequential column sums continuing
// from `init` (the previous rank's sums: the only serial link).
int64_t ref_mask_words(const Plan* g) {
  return g->P.n_pad * (g->P.n_pad / 64) * 4;
}

int plan_ref_masks(Plan* g, uint64_t* masks) {
  const Prepared& Q = g->P;
  FS_HIP(hipSetDevice(g->device));
  FS_HIP(hipMemsetAsync(masks, 0, sizeof(uint64_t) * (size_t)ref_mask_words(g), g->stream));
  FS_TRY(refacc::multisurf_masks(g->D, Q.n, Q.n_pad, g->tiles, g->n_tiles, g->thr, g->lab,
                                 Q.use_star, masks, g->stream));
  if (g->own_stream) FS_HIP(hipStreamSynchronize(g->stream));
  return FS_OK;
}

int plan_ref_pass2(Plan* g, const uint64_t* masks, const double* counts, int64_t lo,
                   int64_t hi) {
  const Prepared& Q = g->P;
  FS_HIP(hipSetDevice(g->device));
  g->ref_rows = std::max<int64_t>(hi - lo, 0);
  if (g->ref_rows > 0) {
    float* temp = nullptr;
    FS_TRY(ref_temp(g, g->ref_rows, &temp));
    FS_HIP(hipEventRecord(g->ev[2], g->stream));
    FS_TRY(refacc::multisurf_chains(g->xk, g->Kp, g->krecip, g->kdisc, g->kblk, masks, Q.n,
                                    Q.n_pad, counts, Q.use_star, lo, hi, temp, g->stream));
    FS_HIP(hipEventRecord(g->ev[3], g->stream));
  }
  if (g->own_stream) FS_HIP(hipStreamSynchronize(g->stream));
  return FS_OK;
}

int plan_ref_sums(Plan* g, const double* init, double* sums) {
  const Prepared& Q = g->P;
  FS_HIP(hipSetDevice(g->device));
  if (g->ref_rows < 0) {
    set_error("fs_plan_ref_sums: no fs_plan_ref_pass2 since the plan was created or re-targeted");
    return FS_EINVAL;
  }
  if (g->ref_rows == 0) {  // no rows: the running sums pass through
    if (init)
      FS_HIP(hipMemcpyAsync(sums, init, sizeof(double) * Q.n_kept, hipMemcpyDeviceToDevice,
                            g->stream));
    else
      FS_HIP(hipMemsetAsync(sums, 0, sizeof(double) * Q.n_kept, g->stream));
  } else {
    FS_TRY(refacc::column_sums(g->temp, g->ref_rows, g->Kp, Q.n_kept, init, sums, g->stream));
  }
  if (g->own_stream) FS_HIP(hipStreamSynchronize(g->stream));
  return FS_OK;
}

int plan_pass2(Plan* g, const double* counts, double* scores) {
  const Prepared& Q = g->P;
  FS_HIP(hipSetDevice(g->device));
  if (Q.ref_accum) {
    if (g->world > 1) {
      set_error("reference-order accumulation with world > 1: pass 2 is fs_plan_ref_masks, a "
                "SUM all-reduce of the masks, then fs_plan_ref_pass2 chained over the ranks");
      return FS_ENOTSUP;
    }
    FS_TRY(ref_masks(g));
    FS_TRY(ref_chains(g, counts, scores));
    if (g->own_stream) FS_HIP(hipStreamSynchronize(g->stream));
    return FS_OK;
  }
  FS_TRY(run_weights(g, counts, ALGO_MULTISURF, 1.0 / Q.SC));
  FS_TRY(run_pass2(g, scores));
  if (g->own_stream) FS_HIP(hipStreamSynchronize(g->stream));
  return FS_OK;
}

}  // namespace gpu
}  // namespace fs
