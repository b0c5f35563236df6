// fs_refacc.hip -- reference-order accumulation (FS_ACCUM_REFERENCE,
// fs_set_accumulation): the per-sample float32 sums and the float32
// sequential column sums of the reference's CPU kernels, replayed on the GPU
// so that the scores are the reference's arithmetic bit for bit wherever the
// near / far decisions are the reference's.
//
// The default pass 2 (fs_pass2.hip k_score_sparse2) folds both directed
// weights of a pair into one symmetric weight and sums in float32 streams
// and float64 partials: 10-60x closer to the exact (float64) sums than the
// reference, but not the reference's own rounding.  On inputs where the
// reference's float32 error is itself above 1e-5 of max |s| (signal-free or
// heavy-tailed data, VERDICT r4 missing #1) only replaying that rounding
// gives "within 1e-5 and identical top-k".  This mode replays it:
//
//   MultiSURF / MultiSURF* (MultiSURF.py:198-253): for every focal sample i
//   and kept feature k, hit_diffs[k] and miss_diffs[k] are float32 chains
//   over the near hits / near misses (and, for MultiSURF*, the far misses
//   subtracted) in ascending j; each diff is the reference's float32
//   |x_i - x_j| * recip (or 1 / 0 for a discrete feature); then
//   f32(chain / count) in float64 (numba's in-place /= int), temp[i][k] =
//   miss - hit in float32, and scores[k] = temp[:, k].sum() sequentially in
//   float32.  The decisions come from the plan's distances (32-bit operands,
//   every refined pair exact, every flagged row's threshold exact) as bit
//   masks: k_ref_masks.
//   ReliefF (ReliefF.py:181-220): the neighbours of each class in argsort
//   order (the exact float32 keys, ascending; k_rf_ref_keys / k_rf_ref_sort),
//   float64 hit / miss sums in that order, the float64 update, temp[i][k] =
//   f32(update), and the same sequential float32 column sum.
//
//   SURF / SURF* (SURF.py:139-218): the reference's order at n_jobs = 1 (its
//   only fixed one: with more threads the per-thread private score rows are
//   summed in schedule order) -- per focal sample four float32 chains in
//   ascending j (near hit / near miss / far hit / far miss) of the float32-
//   stored float64 diffs, score_update in float32, and one sequential float32
//   sum over the samples: k_surf_masks, k_surf_chains, k_ref_colsum.
//
// Kernels (cfg4 figures in DESIGN.md §Reference-order accumulation):
//   k_ref_gather   kept columns of X into a 256-padded row-major copy.  HBM
//   k_ref_masks    near-hit / miss-chain / far-miss bit masks per row and
//                  64-sample word, one owned distance tile per workgroup. HBM
//   k_ms_chains    the chains: 96 focal rows x 256 features per workgroup,
//                  6 rows per wave, 4 features per lane, the 64-sample j
//                  chunks staged HBM -> LDS by global_load_lds (double-
//                  buffered); each wave walks its rows' mask bits in
//                  ascending j: per entry one ds_read_b128 and 4 x
//                  (v_sub, v_mul |.|, v_add).                     VALU / LDS
//   k_ref_colsum   sequential float32 column sums, 64 rows of loads in
//                  flight per lane.                                 latency
//   k_surf_masks   SURF's four decision masks per focal row from its float32
//                  D row and mean.                                     HBM
//   k_surf_chains  k_ms_chains on float64 X: 128 features per workgroup,
//                  2 per lane; per entry one ds_read_b128 and 2 x (v_add_f64,
//                  v_mul_f64 |.|, v_cvt_f32_f64, v_add_f32).     VALU (f64)
#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>

#include "../../include/fastselect_amd.h"
#include "fs_internal.h"

namespace fs {
namespace gpu {
namespace refacc {

namespace {

int check(const char* what) {
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error(std::string("HIP error '") + hipGetErrorString(e) + "' launching " + what);
    return FS_EHIP;
  }
  return FS_OK;
}

#ifndef FS_CHAINS_CHUNK
#define FS_CHAINS_CHUNK 64
#endif
constexpr int kChunk = FS_CHAINS_CHUNK;  // samples j per staged chunk (a mask word, or half of one)
constexpr int kFeat = 256;   // features per workgroup (64 lanes x 4)
#ifndef FS_CHAINS_WAVES
#define FS_CHAINS_WAVES 16
#endif
#ifndef FS_CHAINS_ROWS
#define FS_CHAINS_ROWS 6
#endif
constexpr int kWaves = FS_CHAINS_WAVES;  // waves per k_ms_chains workgroup
constexpr int kRowsW = FS_CHAINS_ROWS;   // focal rows per wave
static_assert(kChunk % kWaves == 0 && 4 * kRowsW <= 64 && (kChunk == 64 || kChunk == 32),
              "k_ms_chains shape");

// chunk c's bits of a row's mask words (kChunk = 32: half a 64-sample word)
__device__ __forceinline__ uint64_t chunk_word(const uint64_t* mrow, int64_t c) {
  if (kChunk == 64) return mrow[c * 4];
  return (mrow[(c >> 1) * 4] >> ((c & 1) * 32)) & 0xFFFFFFFFull;
}
constexpr int kRowsWG = kWaves * kRowsW;

__device__ __forceinline__ uint64_t readlane64(uint64_t v, int l) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, l);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), l);
  return ((uint64_t)hi << 32) | lo;
}

// ---- kept columns ------------------------------------------------------------
// xk[j][k] = x[j][kcol[k]] for j < n, k < n_kept; 0 in the padding (rows up to
// n_pad, columns up to Kp), so staged padding rows / lanes contribute nothing.
// float32 X (MultiSURF, ReliefF) or float64 X (SURF, SURF.py:330-332).
template <typename T>
__global__ __launch_bounds__(256) void k_ref_gather(const T* __restrict__ x, int64_t n,
                                                    int64_t n_pad, int64_t p_in,
                                                    const int64_t* __restrict__ kcol,
                                                    int64_t n_kept, int64_t Kp,
                                                    T* __restrict__ xk) {
  const int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (k >= Kp) return;
  const int64_t col = k < n_kept ? kcol[k] : -1;
  for (int64_t j = blockIdx.y; j < n_pad; j += gridDim.y)
    xk[j * Kp + k] = (j < n && col >= 0) ? x[j * p_in + col] : (T)0;
}

// ---- MultiSURF decisions as bit masks ------------------------------------------
// masks[(row * nw + w) * 4 + t], nw = n_pad / 64, bit b of word w = sample
// 64 w + b: t = 0 near hits, 1 the miss chain (near misses, and for
// MultiSURF* the far misses too), 2 far misses (the chain's subtracted
// entries), 3 zero.  The rule is k_tile_counts' (D_ij < thr_i, j != i,
// MultiSURF.py:216-217; far := not near and not a hit, :236), on the tiled
// distances T_t[b][a] = D(i0 + a, j0 + b) of the owned tiles.  Every (row,
// word) pair of the triangle's blocks is written by exactly one tile.
__global__ __launch_bounds__(256) void k_ref_masks(const double* __restrict__ D, int64_t n,
                                                   int64_t nw, const int2* __restrict__ tiles,
                                                   const double* __restrict__ thr,
                                                   const int32_t* __restrict__ lab, int use_star,
                                                   uint64_t* __restrict__ masks) {
  const int2 tl = tiles[blockIdx.x];
  const int64_t i0 = (int64_t)tl.x * kTile, j0 = (int64_t)tl.y * kTile;
  const double* T = D + (int64_t)blockIdx.x * kTile * kTile;
  const int tid = threadIdx.x;
  if (tid < kTile) {
    // rows i0 + a over the tile's columns j0 + b (both 64-sample words)
    const int a = tid;
    const int64_t i = i0 + a;
    const bool row_ok = i < n;
    const double t = row_ok ? thr[i] : 0.0;
    const int32_t li = row_ok ? lab[i] : 0;
    uint64_t w[2][3] = {{0, 0, 0}, {0, 0, 0}};
#pragma unroll
    for (int h = 0; h < 2; h++) {
      for (int b0 = 0; b0 < 64; b0 += 8) {
#pragma unroll
        for (int u = 0; u < 8; u++) {
          const int b = 64 * h + b0 + u;
          const int64_t j = j0 + b;
          const bool ok = row_ok && j < n && j != i;
          const double d = T[b * kTile + a];
          const bool near = ok && d < t;
          const bool hit = ok && lab[j < n ? j : 0] == li;
          const bool far_miss = use_star && ok && !near && !hit;
          const uint64_t bit = 1ull << (b0 + u);
          if (near && hit) w[h][0] |= bit;
          if ((near && !hit) || far_miss) w[h][1] |= bit;
          if (far_miss) w[h][2] |= bit;
        }
      }
    }
    if (i < (int64_t)nw * 64) {
#pragma unroll
      for (int h = 0; h < 2; h++) {
        uint64_t* o = masks + ((size_t)i * nw + (size_t)(j0 / 64 + h)) * 4;
        o[0] = w[h][0];
        o[1] = w[h][1];
        o[2] = w[h][2];
        o[3] = 0;
      }
    }
    return;
  }
  if (tl.x == tl.y) return;
  // rows j0 + b over the tile's rows i0 + a: wave-wide ballots, lane k of
  // wave w2 keeps the words of row j0 + 64 w2 + k
  const int lane = tid & 63, w2 = (tid >> 6) - 2;
  const bool in0 = i0 + lane < n, in1 = i0 + 64 + lane < n;
  const int32_t l0 = in0 ? lab[i0 + lane] : -1, l1 = in1 ? lab[i0 + 64 + lane] : -1;
  uint64_t keep[2][3] = {{0, 0, 0}, {0, 0, 0}};
  for (int k = 0; k < 64; k++) {
    const int b = 64 * w2 + k;
    const int64_t self = j0 + b;
    if (self >= n) break;  // uniform across the wave
    const double t = thr[self];
    const int32_t ls = lab[self];
    const double v0 = T[b * kTile + lane], v1 = T[b * kTile + 64 + lane];
    const bool n0 = in0 && v0 < t, n1 = in1 && v1 < t;
    const bool h0 = l0 == ls, h1 = l1 == ls;
    const bool f0 = use_star && in0 && !n0 && !h0, f1 = use_star && in1 && !n1 && !h1;
    const uint64_t wh0 = __ballot(n0 && h0), wh1 = __ballot(n1 && h1);
    const uint64_t wm0 = __ballot((n0 && !h0) || f0), wm1 = __ballot((n1 && !h1) || f1);
    const uint64_t wf0 = __ballot(f0), wf1 = __ballot(f1);
    if (lane == k) {
      keep[0][0] = wh0;
      keep[0][1] = wm0;
      keep[0][2] = wf0;
      keep[1][0] = wh1;
      keep[1][1] = wm1;
      keep[1][2] = wf1;
    }
  }
  const int64_t row = j0 + 64 * w2 + lane;
  if (row < n) {
#pragma unroll
    for (int h = 0; h < 2; h++) {
      uint64_t* o = masks + ((size_t)row * nw + (size_t)(i0 / 64 + h)) * 4;
      o[0] = keep[h][0];
      o[1] = keep[h][1];
      o[2] = keep[h][2];
      o[3] = 0;
    }
  }
}

// ---- MultiSURF chains -------------------------------------------------------------
// One entry of a chain: acc[k] (+|-)= diff_k(a, v) for the lane's 4 features,
// the reference's diff (MultiSURF.py:184-187, 222-243).  `neg` (a far miss of
// MultiSURF*) is wave-uniform; fma(-1, d, acc) rounds acc - d exactly as the
// reference's `miss_diffs[k] -= diff` does.
template <bool DISC>
__device__ __forceinline__ void chain_step(const float4 v, const float (&a)[4],
                                           const float (&rc)[4], const uint32_t dk, float sgn,
                                           float (&acc)[4]) {
  const float vb[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int k = 0; k < 4; k++) {
    float d = __builtin_fabsf(a[k] - vb[k]) * rc[k];
    if (DISC && ((dk >> k) & 1u)) d = a[k] != vb[k] ? 1.0f : 0.0f;
    acc[k] = __builtin_fmaf(sgn, d, acc[k]);
  }
}

// the lowest set bit of m, cleared: s_ff1 + s_bitset0 (2 SALU; the builtin
// form, ctz and m &= m - 1, compiles to 5, and the chains are issue-bound
// enough that this alone took k_ms_chains 195.5 -> 186.7 ms at cfg4,
// profiles/r05/chains_ab.txt)
__device__ __forceinline__ int pop_bit(uint64_t& m) {
  int b;
  asm("s_ff1_i32_b64 %0, %1\n\ts_bitset0_b64 %1, %0" : "=&s"(b), "+s"(m));
  return b;
}

// Walk the set bits of one 64-sample mask word in ascending j (the
// reference's j loop) in groups of 8, then 4 entries: the group's LDS row
// reads are issued together ahead of its arithmetic (each step then waits
// only for its own read, counted lgkmcnt), the last 1-3 entries likewise.
template <bool SIGNED, bool DISC>
__device__ __forceinline__ void chain_walk(uint64_t m, uint64_t neg, const float4* __restrict__ buf,
                                           int lane, const float (&a)[4], const float (&rc)[4],
                                           uint32_t dk, float (&acc)[4]) {
  auto sg = [&](int b) { return SIGNED && ((neg >> b) & 1ull) ? -1.0f : 1.0f; };
  while (__builtin_popcountll(m) >= 8) {
    int b[8];
    float4 v[8];
#pragma unroll
    for (int q = 0; q < 8; q++) b[q] = pop_bit(m);
#pragma unroll
    for (int q = 0; q < 8; q++) v[q] = buf[b[q] * 64 + lane];
#pragma unroll
    for (int q = 0; q < 8; q++) chain_step<DISC>(v[q], a, rc, dk, sg(b[q]), acc);
  }
  while (__builtin_popcountll(m) >= 4) {
    const int b0 = pop_bit(m), b1 = pop_bit(m), b2 = pop_bit(m), b3 = pop_bit(m);
    const float4 v0 = buf[b0 * 64 + lane], v1 = buf[b1 * 64 + lane];
    const float4 v2 = buf[b2 * 64 + lane], v3 = buf[b3 * 64 + lane];
    chain_step<DISC>(v0, a, rc, dk, sg(b0), acc);
    chain_step<DISC>(v1, a, rc, dk, sg(b1), acc);
    chain_step<DISC>(v2, a, rc, dk, sg(b2), acc);
    chain_step<DISC>(v3, a, rc, dk, sg(b3), acc);
  }
  if (m == 0) return;
  const int b0 = pop_bit(m);
  const float4 v0 = buf[b0 * 64 + lane];
  if (m == 0) {
    chain_step<DISC>(v0, a, rc, dk, sg(b0), acc);
    return;
  }
  const int b1 = pop_bit(m);
  const float4 v1 = buf[b1 * 64 + lane];
  if (m == 0) {
    chain_step<DISC>(v0, a, rc, dk, sg(b0), acc);
    chain_step<DISC>(v1, a, rc, dk, sg(b1), acc);
    return;
  }
  const int b2 = pop_bit(m);
  const float4 v2 = buf[b2 * 64 + lane];
  chain_step<DISC>(v0, a, rc, dk, sg(b0), acc);
  chain_step<DISC>(v1, a, rc, dk, sg(b1), acc);
  chain_step<DISC>(v2, a, rc, dk, sg(b2), acc);
}

// The rows of a wave over one staged chunk: each row's hit chain, then
// its miss chain.
template <bool STAR, bool DISC>
__device__ __forceinline__ void chunk_rows(const float4* __restrict__ buf, uint64_t mw, int lane,
                                           const float (&a)[kRowsW][4], const float (&rc)[4],
                                           uint32_t dk, float (&ah)[kRowsW][4],
                                           float (&am)[kRowsW][4]) {
#pragma unroll
  for (int r = 0; r < kRowsW; r++) {
    const uint64_t mh = readlane64(mw, 4 * r), mm = readlane64(mw, 4 * r + 1);
    const uint64_t mf = STAR ? readlane64(mw, 4 * r + 2) : 0ull;
    chain_walk<false, DISC>(mh, 0ull, buf, lane, a[r], rc, dk, ah[r]);
    chain_walk<STAR, DISC>(mm, mf, buf, lane, a[r], rc, dk, am[r]);
  }
}

// Chunk c's samples (64 rows x 1 KB of the block's features) into LDS, one
// global_load_lds_dwordx4 per row (4 rows per wave).
__device__ __forceinline__ void stage_chunk(const float* __restrict__ xk, int64_t Kp, int64_t f0,
                                            int wave, int lane, float4* buf, int64_t c) {
#pragma unroll
  for (int s = 0; s < kChunk / kWaves; s++) {
    const int t = wave * (kChunk / kWaves) + s;
    const float* src = xk + (c * kChunk + t) * Kp + f0 + 4 * lane;
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                     (__attribute__((address_space(3))) void*)(buf + t * 64), 16,
                                     0, 0);
  }
}

// Grid (row blocks of 128 focal rows of [r_lo, r_hi), Kp / 256 feature
// blocks).  Wave w holds rows r_lo + 128 bx + 8 w + r (r < 8): x_i, and the
// hit and miss chains of its lane's features 4 lane + k of the block, in
// VGPRs.  The samples j come in chunks of 64 (one mask word): chunk c + 1 is
// copied into the other LDS buffer (64 rows x 1 KB, one global_load_lds per
// row) while chunk c is walked; the chunk's mask words of the wave's 8 rows
// come by one vector load (lane 4 r + t) taken apart with v_readlane.
template <bool STAR, bool DISC>
__device__ __forceinline__ void chains_body(
    const float* __restrict__ xk, int64_t Kp, const float* __restrict__ krecip,
    const uint8_t* __restrict__ kdisc, const uint64_t* __restrict__ masks, int64_t nw,
    int64_t nch, const double* __restrict__ counts, int64_t r_lo, int64_t r_hi,
    float* __restrict__ temp, float4* bufA, float4* bufB) {
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t f0 = (int64_t)blockIdx.y * kFeat;
  const int64_t row0 = r_lo + (int64_t)blockIdx.x * kRowsWG + wave * kRowsW;

  float rc[4];
  uint32_t dk = 0;
#pragma unroll
  for (int k = 0; k < 4; k++) {
    rc[k] = krecip[f0 + 4 * lane + k];
    if (DISC) dk |= (kdisc[f0 + 4 * lane + k] ? 1u : 0u) << k;
  }
  float a[kRowsW][4], ah[kRowsW][4], am[kRowsW][4];
#pragma unroll
  for (int r = 0; r < kRowsW; r++) {
    const int64_t i = row0 + r;
    const float4 v = i < r_hi ? *(const float4*)(xk + i * Kp + f0 + 4 * lane)
                              : make_float4(0.f, 0.f, 0.f, 0.f);
    a[r][0] = v.x;
    a[r][1] = v.y;
    a[r][2] = v.z;
    a[r][3] = v.w;
#pragma unroll
    for (int k = 0; k < 4; k++) ah[r][k] = am[r][k] = 0.0f;
  }
  // mask words of chunk c: lane 4 r + t <- masks[row0 + r][c][t] (rows past
  // r_hi read as empty)
  const int mr = lane >> 2, mt = lane & 3;
  const bool mload = lane < 4 * kRowsW && row0 + mr < r_hi;
  const uint64_t* mrow = masks + ((size_t)(row0 + (mload ? mr : 0)) * nw) * 4 + mt;

  uint64_t mw = mload ? chunk_word(mrow, 0) : 0ull;
  stage_chunk(xk, Kp, f0, wave, lane, bufA, 0);
  __syncthreads();
  for (int64_t c = 0; c < nch; c += 2) {
    uint64_t mn = 0;
    if (c + 1 < nch) {
      mn = mload ? chunk_word(mrow, c + 1) : 0ull;
      stage_chunk(xk, Kp, f0, wave, lane, bufB, c + 1);
    }
    chunk_rows<STAR, DISC>(bufA, mw, lane, a, rc, dk, ah, am);
    __syncthreads();
    if (c + 1 >= nch) break;
    mw = mn;
    if (c + 2 < nch) {
      mn = mload ? chunk_word(mrow, c + 2) : 0ull;
      stage_chunk(xk, Kp, f0, wave, lane, bufA, c + 2);
    }
    chunk_rows<STAR, DISC>(bufB, mw, lane, a, rc, dk, ah, am);
    __syncthreads();
    mw = mn;
  }

  // MultiSURF.py:245-251: f32(chain / count) when the count is non-zero
  // (numba's float32 /= int goes through float64), then temp = miss - hit
#pragma unroll
  for (int r = 0; r < kRowsW; r++) {
    const int64_t i = row0 + r;
    if (i >= r_hi) continue;
    const double H = counts[2 * i], M = counts[2 * i + 1];
    float o[4];
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const float h = H > 0.0 ? (float)((double)ah[r][k] / H) : ah[r][k];
      const float m = M > 0.0 ? (float)((double)am[r][k] / M) : am[r][k];
      o[k] = m - h;
    }
    *(float4*)(temp + (i - r_lo) * Kp + f0 + 4 * lane) = make_float4(o[0], o[1], o[2], o[3]);
  }
}

template <bool STAR>
__global__ __launch_bounds__(64 * kWaves) void k_ms_chains(
    const float* __restrict__ xk, int64_t Kp, const float* __restrict__ krecip,
    const uint8_t* __restrict__ kdisc, const uint8_t* __restrict__ blkdisc,
    const uint64_t* __restrict__ masks, int64_t nw, int64_t nch, const double* __restrict__ counts,
    int64_t r_lo, int64_t r_hi, float* __restrict__ temp) {
  __shared__ float4 bufA[kChunk * 64];
  __shared__ float4 bufB[kChunk * 64];
  if (blkdisc[blockIdx.y])
    chains_body<STAR, true>(xk, Kp, krecip, kdisc, masks, nw, nch, counts, r_lo, r_hi, temp, bufA,
                            bufB);
  else
    chains_body<STAR, false>(xk, Kp, krecip, kdisc, masks, nw, nch, counts, r_lo, r_hi, temp, bufA,
                             bufB);
}

// ---- sequential float32 column sums ---------------------------------------------
// out[k] = (double) (s0 + temp[0][k] + temp[1][k] + ... ) in float32, row by
// row, s0 = (float) init[k] or 0 (a row panel continuing the previous one's sum)
// (numba's float32 .sum(), MultiSURF.py:252-253, ReliefF.py:219-220).  One
// lane per column; 64 rows of loads are issued before their adds.
constexpr int kSumAhead = 64;
__global__ __launch_bounds__(64) void k_ref_colsum(const float* __restrict__ temp, int64_t rows,
                                                   int64_t Kp, int64_t n_kept,
                                                   const double* __restrict__ init,
                                                   double* __restrict__ out) {
  const int64_t k = (int64_t)blockIdx.x * 64 + threadIdx.x;
  if (k >= n_kept) return;
  float s = init ? (float)init[k] : 0.0f;
  int64_t i = 0;
  for (; i + kSumAhead <= rows; i += kSumAhead) {
    float v[kSumAhead];
#pragma unroll
    for (int u = 0; u < kSumAhead; u++) v[u] = temp[(i + u) * Kp + k];
#pragma unroll
    for (int u = 0; u < kSumAhead; u++) s += v[u];
  }
  for (; i < rows; i++) s += temp[i * Kp + k];
  out[k] = (double)s;
}

// ---- ReliefF ---------------------------------------------------------------------
// The reference's float32 key of (i, j): float32 diffs summed in float64 in
// kept-feature order, rounded to float32 (ReliefF.py:149-155).
__device__ __forceinline__ float rf_ref_key(const float* __restrict__ xi,
                                            const float* __restrict__ xj,
                                            const float* __restrict__ krecip,
                                            const uint8_t* __restrict__ kdisc, int64_t n_kept) {
  double d = 0.0;
  for (int64_t f = 0; f < n_kept; f++) {
    if (kdisc[f])
      d += xi[f] != xj[f] ? 1.0 : 0.0;
    else
      d += (double)(__builtin_fabsf(xi[f] - xj[f]) * krecip[f]);
  }
  return (float)d;
}

// The key of neighbour entry e = ((i - r_lo) C + c) k + t (t < nfound[i][c]).
// One lane per entry, each summing its own two rows sequentially.
__global__ __launch_bounds__(256) void k_rf_ref_keys(
    const float* __restrict__ xk, int64_t Kp, const float* __restrict__ krecip,
    const uint8_t* __restrict__ kdisc, int64_t n_kept, const int32_t* __restrict__ nbr,
    const int32_t* __restrict__ nfound, int64_t r_lo, int64_t r_hi, int C, int64_t k,
    float* __restrict__ keys) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t total = (r_hi - r_lo) * C * k;
  if (e >= total) return;
  const int64_t t = e % k, ic = e / k;
  const int64_t i = r_lo + ic / C, c = ic % C;
  if (t >= nfound[i * C + c]) return;
  const int64_t j = nbr[(i * C + c) * k + t];
  keys[e] = rf_ref_key(xk + i * Kp, xk + j * Kp, krecip, kdisc, n_kept);
}

// Every key of the rows rows[r] (j = i: +inf, the reference's dists[i]),
// for the tie rows' quicksort replay (k_rf_ref_ties).  Grid (rows,
// ceil(n / 256)), one lane per sample j.
__global__ __launch_bounds__(256) void k_rf_ref_rowkeys(
    const float* __restrict__ xk, int64_t Kp, const float* __restrict__ krecip,
    const uint8_t* __restrict__ kdisc, int64_t n_kept, const int32_t* __restrict__ rows,
    int64_t n, float* __restrict__ keys) {
  const int64_t r = blockIdx.x, i = rows[r];
  const int64_t j = (int64_t)blockIdx.y * 256 + threadIdx.x;
  if (j >= n) return;
  keys[r * n + j] =
      j == i ? __builtin_inff() : rf_ref_key(xk + i * Kp, xk + j * Kp, krecip, kdisc, n_kept);
}

// Each (i, c) list in ascending key order, equal keys by sample index (the
// reference's argsort order up to ties: k_rf_ref_ties then re-orders each
// run of equal keys as numba's quicksort does, ReliefF.py:157).  Insertion
// sort, one thread per list; dup[list] = 1 when the list holds a run.
__global__ __launch_bounds__(256) void k_rf_ref_sort(int32_t* __restrict__ nbr,
                                                     const int32_t* __restrict__ nfound,
                                                     float* __restrict__ keys, int64_t r_lo,
                                                     int64_t r_hi, int C, int64_t k,
                                                     int32_t* __restrict__ dup) {
  const int64_t ic = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (ic >= (r_hi - r_lo) * C) return;
  const int64_t i = r_lo + ic / C, c = ic % C;
  const int64_t m = nfound[i * C + c];
  int32_t* L = nbr + (i * C + c) * k;
  float* K = keys + ic * k;
  for (int64_t s = 1; s < m; s++) {
    const float kv = K[s];
    const int32_t jv = L[s];
    int64_t q = s;
    while (q > 0 && (K[q - 1] > kv || (K[q - 1] == kv && L[q - 1] > jv))) {
      K[q] = K[q - 1];
      L[q] = L[q - 1];
      q--;
    }
    K[q] = kv;
    L[q] = jv;
  }
  int32_t d = 0;
  for (int64_t s = 1; s < m; s++) d |= K[s] == K[s - 1] ? 1 : 0;
  dup[ic] = d;
}

// Whether the order of a row's tied neighbours can change its float64 sums
// (ReliefF.py:181-207): for every list holding a run of equal keys (dup) and
// every continuous feature, the list's float32 diffs are all multiples of
// u = ulp(smallest non-zero diff) (a float32 value is a multiple of its own
// ulp, and larger ones of u), so when their sum is below 2^53 u every partial
// sum, in ANY order, is exactly representable in float64 -- the order cannot
// matter.  Only a row where some sum reaches 2^53 u (diffs 2^29 or more
// apart) needs numba's quicksort order (k_rf_ref_ties); 0 / 1 diffs of
// discrete features are exact in any order.  Grid: one 256-thread workgroup
// per candidate row, the threads over the features.
__global__ __launch_bounds__(256) void k_rf_ref_order_matters(
    const float* __restrict__ xk, int64_t Kp, const float* __restrict__ krecip,
    const uint8_t* __restrict__ kdisc, int64_t n_kept, const int32_t* __restrict__ rows,
    const int32_t* __restrict__ dup, const int32_t* __restrict__ nbr,
    const int32_t* __restrict__ nfound, int64_t r_lo, int C, int64_t k,
    int32_t* __restrict__ matters) {
  __shared__ int any;
  if (threadIdx.x == 0) any = 0;
  __syncthreads();
  const int64_t r = blockIdx.x, i = rows[r];
  const float* xi = xk + i * Kp;
  int m = 0;
  for (int c = 0; c < C && !m; c++) {
    if (!dup[(i - r_lo) * C + c]) continue;
    const int64_t cnt = nfound[i * C + c];
    const int32_t* L = nbr + (i * C + c) * k;
    for (int64_t f = threadIdx.x; f < n_kept && !m; f += 256) {
      if (kdisc[f]) continue;
      float vmin = __builtin_inff();
      double s = 0.0;
      for (int64_t t = 0; t < cnt; t++) {
        const float v = __builtin_fabsf(xi[f] - xk[(int64_t)L[t] * Kp + f]) * krecip[f];
        if (v > 0.0f && v < vmin) vmin = v;
        s += (double)v;
      }
      if (vmin == __builtin_inff()) continue;
      int e;
      (void)__builtin_frexpf(vmin, &e);  // vmin in [2^(e-1), 2^e): ulp 2^(e-24)
      if (s >= __builtin_ldexp(1.0, e - 24 + 53)) m = 1;
    }
  }
  if (m) any = 1;  // benign race: every writer stores 1
  __syncthreads();
  if (threadIdx.x == 0) matters[r] = any;
}

// temp[i - r_lo][f] = f32(update) (ReliefF.py:177-216): hit_sum and each miss
// class's sum in float64 in argsort order, miss_sum += P_c / (1 - P_yi) * sum
// in class order, update = -hit_sum / h_found + miss_sum / k.  Grid (Kp / 64
// feature blocks, 64-row blocks); lane = feature, wave w the rows w, w+4, ...
__global__ __launch_bounds__(256) void k_rf_ref_update(
    const float* __restrict__ xk, int64_t Kp, const float* __restrict__ krecip,
    const uint8_t* __restrict__ kdisc, const int32_t* __restrict__ lab,
    const double* __restrict__ prior, int C, int64_t k, const int32_t* __restrict__ nbr,
    const int32_t* __restrict__ nfound, int64_t r_lo, int64_t r_hi, float* __restrict__ temp) {
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t f = (int64_t)blockIdx.x * 64 + lane;
  const float r = krecip[f];
  const bool disc = kdisc[f] != 0;
  const int64_t b0 = r_lo + (int64_t)blockIdx.y * 64;
  for (int64_t i = b0 + wave; i < r_hi && i < b0 + 64; i += 4) {
    const int32_t li = lab[i];
    const float a = xk[i * Kp + f];
    double denom = 1.0 - prior[li];
    if (denom == 0.0) denom = 1.0;
    double hit_sum = 0.0, miss_sum = 0.0;
    int64_t h_found = 0;
    for (int c = 0; c < C; c++) {
      const int64_t found = nfound[i * C + c];
      const int32_t* lst = nbr + (i * C + c) * k;
      double s = 0.0;
      for (int64_t t = 0; t < found; t++) {
        const float b = xk[(int64_t)lst[t] * Kp + f];
        s += disc ? (a != b ? 1.0 : 0.0) : (double)(__builtin_fabsf(a - b) * r);
      }
      if (c == li) {
        hit_sum = s;
        // the focal sample itself (distance inf, last in the order) is a
        // zero-diff hit when its class has fewer than k other members
        h_found = found < k ? found + 1 : k;
      } else {
        miss_sum += (prior[c] / denom) * s;
      }
    }
    double update = 0.0;
    if (h_found > 0) update -= hit_sum / (double)h_found;
    if (k > 0) update += miss_sum / (double)k;
    temp[(i - r_lo) * Kp + f] = (float)update;
  }
}

// ---- SURF / SURF* ----------------------------------------------------------------
// The reference's n_jobs = 1 order (SURF.py:139-218): for each focal sample i
// in turn, four float32 vector sums over j in ascending order -- near hits,
// near misses, far hits, far misses (the far ones for SURF* only) -- of the
// float32-stored diffs f32(|x_i - x_j| * recip) (x float64, SURF.py:153-158),
// then score_update = (near_miss - near_hit) [+ (far_hit - far_miss)] in
// float32 and private_scores[0] += score_update: one sequential float32 sum
// per feature over the focal samples (k_ref_colsum).  With several numba
// threads the reference adds its per-thread rows in schedule order; n_jobs =
// 1 is its one fixed order, and the one this mode replays.

// Decisions of the focal rows [r_lo, r_hi) as bit masks:
// masks[((i - r_lo) * nw + w) * 4 + t], t = 0 near hits, 1 near misses, 2 far
// hits, 3 far misses (SURF*; 0 for SURF), bit b of word w = sample 64 w + b.
// near: float32 D_ij < avg_i, j != i (SURF.py:170-189; the float32 D is the
// float64 distance rounded, as k_surf_avg and pair_weight take it).  Grid
// (ceil(rows / 4), ceil(nw / 64)): one wave per row and 64 words, lane l
// reads sample 64 w + l of every word (coalesced) and keeps word w0 + l's
// four ballots.  D: the plan's rows (full layout, row i = D + i n_pad).
__global__ __launch_bounds__(256) void k_surf_masks(const double* __restrict__ D, int64_t n,
                                                    int64_t n_pad, int64_t nw,
                                                    const double* __restrict__ avg,
                                                    const int32_t* __restrict__ lab, int use_star,
                                                    int64_t r_lo, int64_t r_hi,
                                                    uint64_t* __restrict__ masks) {
  const int lane = threadIdx.x & 63;
  const int64_t i = r_lo + (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (i >= r_hi) return;  // uniform across the wave
  const int64_t w0 = (int64_t)blockIdx.y * 64;
  const int wn = nw - w0 < 64 ? (int)(nw - w0) : 64;
  const double t = avg[i];
  const int32_t li = lab[i];
  const double* row = D + i * n_pad;
  uint64_t keep[4] = {0, 0, 0, 0};
  for (int u = 0; u < wn; u++) {
    const int64_t j = (w0 + u) * 64 + lane;  // < n_pad: row j and lab[j] exist
    const bool ok = j < n && j != i;
    const bool near = ok && (double)(float)row[j] < t;
    const bool hit = ok && lab[j] == li;
    const bool far = use_star && ok && !near;
    const uint64_t m0 = __ballot(near && hit), m1 = __ballot(near && !hit);
    const uint64_t m2 = __ballot(far && hit), m3 = __ballot(far && !hit);
    if (lane == u) {
      keep[0] = m0;
      keep[1] = m1;
      keep[2] = m2;
      keep[3] = m3;
    }
  }
  if (lane < wn) {
    uint64_t* o = masks + ((size_t)(i - r_lo) * nw + (size_t)(w0 + lane)) * 4;
    *(ulonglong2*)(o + 0) = make_ulonglong2(keep[0], keep[1]);
    *(ulonglong2*)(o + 2) = make_ulonglong2(keep[2], keep[3]);
  }
}

// One entry of a SURF chain for the lane's 2 features: the reference's
// float64 |x_i - x_j| * recip stored as float32 (1 / 0 for a discrete
// feature), added in float32.
template <bool DISC>
__device__ __forceinline__ void surf_step(const double2 v, const double (&a)[2],
                                          const double (&rc)[2], uint32_t dk, float (&acc)[2]) {
  const double vb[2] = {v.x, v.y};
#pragma unroll
  for (int k = 0; k < 2; k++) {
    float d = (float)(__builtin_fabs(a[k] - vb[k]) * rc[k]);
    if (DISC && ((dk >> k) & 1u)) d = a[k] != vb[k] ? 1.0f : 0.0f;
    acc[k] += d;
  }
}

// chain_walk's schedule (groups of 8, then 4, then the last 1-3 entries, each
// group's LDS reads issued ahead of its arithmetic) for a SURF chain.
template <bool DISC>
__device__ __forceinline__ void surf_walk(uint64_t m, const double2* __restrict__ buf, int lane,
                                          const double (&a)[2], const double (&rc)[2],
                                          uint32_t dk, float (&acc)[2]) {
  while (__builtin_popcountll(m) >= 8) {
    int b[8];
    double2 v[8];
#pragma unroll
    for (int q = 0; q < 8; q++) b[q] = pop_bit(m);
#pragma unroll
    for (int q = 0; q < 8; q++) v[q] = buf[b[q] * 64 + lane];
#pragma unroll
    for (int q = 0; q < 8; q++) surf_step<DISC>(v[q], a, rc, dk, acc);
  }
  while (__builtin_popcountll(m) >= 4) {
    const int b0 = pop_bit(m), b1 = pop_bit(m), b2 = pop_bit(m), b3 = pop_bit(m);
    const double2 v0 = buf[b0 * 64 + lane], v1 = buf[b1 * 64 + lane];
    const double2 v2 = buf[b2 * 64 + lane], v3 = buf[b3 * 64 + lane];
    surf_step<DISC>(v0, a, rc, dk, acc);
    surf_step<DISC>(v1, a, rc, dk, acc);
    surf_step<DISC>(v2, a, rc, dk, acc);
    surf_step<DISC>(v3, a, rc, dk, acc);
  }
  while (m != 0) {
    const int b0 = pop_bit(m);
    surf_step<DISC>(buf[b0 * 64 + lane], a, rc, dk, acc);
  }
}

// Chunk c's samples (64 rows x 128 float64 features = 1 KB each) into LDS,
// one global_load_lds_dwordx4 per row, as stage_chunk.
__device__ __forceinline__ void stage_chunk64(const double* __restrict__ xk, int64_t Kp,
                                              int64_t f0, int wave, int lane, double2* buf,
                                              int64_t c) {
#pragma unroll
  for (int s = 0; s < kChunk / kWaves; s++) {
    const int t = wave * (kChunk / kWaves) + s;
    const double* src = xk + (c * kChunk + t) * Kp + f0 + 2 * lane;
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                     (__attribute__((address_space(3))) void*)(buf + t * 64), 16,
                                     0, 0);
  }
}

// k_ms_chains' structure for SURF: grid (row blocks of kRowsWG focal rows of
// [r_lo, r_hi), Kp / 128 feature blocks); wave w holds kRowsW rows -- x_i
// (float64) and their 2 (SURF) or 4 (SURF*) float32 chains for the lane's
// features 2 lane + k -- in VGPRs; the j chunks (one mask word each) staged
// by global_load_lds, double-buffered; each row's chains walked in order
// near hit, near miss, far hit, far miss (independent sums, so the order of
// the walks does not matter, only the ascending j within each).
constexpr int kFeat64 = 128;  // features per k_surf_chains workgroup (64 lanes x 2)
template <bool STAR, bool DISC>
__device__ __forceinline__ void surf_chains_body(
    const double* __restrict__ xk, int64_t Kp, const float* __restrict__ krecip,
    const uint8_t* __restrict__ kdisc, const uint64_t* __restrict__ masks, int64_t nw,
    int64_t nch, int64_t r_lo, int64_t r_hi, float* __restrict__ temp, double2* bufA,
    double2* bufB) {
  constexpr int NC = STAR ? 4 : 2;  // chains per row
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t f0 = (int64_t)blockIdx.y * kFeat64;
  const int64_t row0 = r_lo + (int64_t)blockIdx.x * kRowsWG + wave * kRowsW;

  double rc[2];
  uint32_t dk = 0;
#pragma unroll
  for (int k = 0; k < 2; k++) {
    rc[k] = (double)krecip[f0 + 2 * lane + k];
    if (DISC) dk |= (kdisc[f0 + 2 * lane + k] ? 1u : 0u) << k;
  }
  double a[kRowsW][2];
  float acc[kRowsW][NC][2];
#pragma unroll
  for (int r = 0; r < kRowsW; r++) {
    const int64_t i = row0 + r;
    const double2 v = i < r_hi ? *(const double2*)(xk + i * Kp + f0 + 2 * lane)
                               : make_double2(0.0, 0.0);
    a[r][0] = v.x;
    a[r][1] = v.y;
#pragma unroll
    for (int t = 0; t < NC; t++) acc[r][t][0] = acc[r][t][1] = 0.0f;
  }
  // mask words of chunk c: lane 4 r + t <- masks[row0 + r - r_lo][c][t]
  const int mr = lane >> 2, mt = lane & 3;
  const bool mload = lane < 4 * kRowsW && row0 + mr < r_hi;
  const uint64_t* mrow = masks + ((size_t)(row0 + (mload ? mr : 0) - r_lo) * nw) * 4 + mt;
  auto rows_of = [&](const double2* buf, uint64_t mw) {
#pragma unroll
    for (int r = 0; r < kRowsW; r++)
#pragma unroll
      for (int t = 0; t < NC; t++)
        surf_walk<DISC>(readlane64(mw, 4 * r + t), buf, lane, a[r], rc, dk, acc[r][t]);
  };
  uint64_t mw = mload ? chunk_word(mrow, 0) : 0ull;
  stage_chunk64(xk, Kp, f0, wave, lane, bufA, 0);
  __syncthreads();
  for (int64_t c = 0; c < nch; c += 2) {
    uint64_t mn = 0;
    if (c + 1 < nch) {
      mn = mload ? chunk_word(mrow, c + 1) : 0ull;
      stage_chunk64(xk, Kp, f0, wave, lane, bufB, c + 1);
    }
    rows_of(bufA, mw);
    __syncthreads();
    if (c + 1 >= nch) break;
    mw = mn;
    if (c + 2 < nch) {
      mn = mload ? chunk_word(mrow, c + 2) : 0ull;
      stage_chunk64(xk, Kp, f0, wave, lane, bufA, c + 2);
    }
    rows_of(bufB, mw);
    __syncthreads();
    mw = mn;
  }
  // SURF.py:191-193: score_update = (near_miss - near_hit) [+ (far_hit - far_miss)]
#pragma unroll
  for (int r = 0; r < kRowsW; r++) {
    const int64_t i = row0 + r;
    if (i >= r_hi) continue;
    float o[2];
#pragma unroll
    for (int k = 0; k < 2; k++) {
      float u = acc[r][1][k] - acc[r][0][k];
      if (STAR) u += acc[r][2 % NC][k] - acc[r][3 % NC][k];
      o[k] = u;
    }
    *(float2*)(temp + (i - r_lo) * Kp + f0 + 2 * lane) = make_float2(o[0], o[1]);
  }
}

template <bool STAR>
__global__ __launch_bounds__(64 * kWaves) void k_surf_chains(
    const double* __restrict__ xk, int64_t Kp, const float* __restrict__ krecip,
    const uint8_t* __restrict__ kdisc, const uint8_t* __restrict__ blkdisc,
    const uint64_t* __restrict__ masks, int64_t nw, int64_t nch, int64_t r_lo, int64_t r_hi,
    float* __restrict__ temp) {
  __shared__ double2 bufA[kChunk * 64];
  __shared__ double2 bufB[kChunk * 64];
  if (blkdisc[blockIdx.y])
    surf_chains_body<STAR, true>(xk, Kp, krecip, kdisc, masks, nw, nch, r_lo, r_hi, temp, bufA,
                                 bufB);
  else
    surf_chains_body<STAR, false>(xk, Kp, krecip, kdisc, masks, nw, nch, r_lo, r_hi, temp, bufA,
                                  bufB);
}

}  // namespace

int gather_kept(const float* x, int64_t n, int64_t n_pad, int64_t p_in, const int64_t* kcol,
                int64_t n_kept, int64_t Kp, float* xk, void* stream) {
  const hipStream_t s = (hipStream_t)stream;
  const unsigned gy = (unsigned)(n_pad < 4096 ? n_pad : 4096);
  k_ref_gather<float><<<dim3((unsigned)(Kp / 256), gy), 256, 0, s>>>(x, n, n_pad, p_in, kcol,
                                                                       n_kept, Kp, xk);
  return check("k_ref_gather");
}

int gather_kept64(const double* x, int64_t n, int64_t n_pad, int64_t p_in, const int64_t* kcol,
                  int64_t n_kept, int64_t Kp, double* xk, void* stream) {
  const hipStream_t s = (hipStream_t)stream;
  const unsigned gy = (unsigned)(n_pad < 4096 ? n_pad : 4096);
  k_ref_gather<double><<<dim3((unsigned)((Kp + 255) / 256), gy), 256, 0, s>>>(
      x, n, n_pad, p_in, kcol, n_kept, Kp, xk);
  return check("k_ref_gather<double>");
}

int surf_masks(const double* D, int64_t n, int64_t n_pad, const double* avg, const int32_t* lab,
               int use_star, int64_t r_lo, int64_t r_hi, uint64_t* masks, void* stream) {
  if (r_hi <= r_lo) return FS_OK;
  const int64_t nw = n_pad / 64;
  k_surf_masks<<<dim3((unsigned)((r_hi - r_lo + 3) / 4), (unsigned)((nw + 63) / 64)), 256, 0,
                 (hipStream_t)stream>>>(D, n, n_pad, nw, avg, lab, use_star, r_lo, r_hi, masks);
  return check("k_surf_masks");
}

int surf_chains(const double* xk, int64_t Kp, const float* krecip, const uint8_t* kdisc,
                const uint8_t* blkdisc, const uint64_t* masks, int64_t n, int64_t n_pad,
                int use_star, int64_t r_lo, int64_t r_hi, float* temp, void* stream) {
  if (r_hi <= r_lo) return FS_OK;
  const dim3 grid((unsigned)((r_hi - r_lo + kRowsWG - 1) / kRowsWG), (unsigned)(Kp / kFeat64));
  const int64_t nch = (n + kChunk - 1) / kChunk;
  const hipStream_t s = (hipStream_t)stream;
  if (use_star)
    k_surf_chains<true><<<grid, 64 * kWaves, 0, s>>>(xk, Kp, krecip, kdisc, blkdisc, masks,
                                                      n_pad / 64, nch, r_lo, r_hi, temp);
  else
    k_surf_chains<false><<<grid, 64 * kWaves, 0, s>>>(xk, Kp, krecip, kdisc, blkdisc, masks,
                                                       n_pad / 64, nch, r_lo, r_hi, temp);
  return check("k_surf_chains");
}

int multisurf_masks(const double* D, int64_t n, int64_t n_pad, const void* tiles, int64_t n_tiles,
                    const double* thr, const int32_t* lab, int use_star, uint64_t* masks,
                    void* stream) {
  if (n_tiles == 0) return FS_OK;
  k_ref_masks<<<(unsigned)n_tiles, 256, 0, (hipStream_t)stream>>>(
      D, n, n_pad / 64, (const int2*)tiles, thr, lab, use_star, masks);
  return check("k_ref_masks");
}

int multisurf_chains(const float* xk, int64_t Kp, const float* krecip, const uint8_t* kdisc,
                     const uint8_t* blkdisc, const uint64_t* masks, int64_t n, int64_t n_pad,
                     const double* counts, int use_star, int64_t r_lo, int64_t r_hi, float* temp,
                     void* stream) {
  if (r_hi <= r_lo) return FS_OK;
  const dim3 grid((unsigned)((r_hi - r_lo + kRowsWG - 1) / kRowsWG), (unsigned)(Kp / kFeat));
  const int64_t nch = (n + kChunk - 1) / kChunk;
  const hipStream_t s = (hipStream_t)stream;
  if (use_star)
    k_ms_chains<true><<<grid, 64 * kWaves, 0, s>>>(xk, Kp, krecip, kdisc, blkdisc, masks,
                                                    n_pad / 64, nch, counts, r_lo, r_hi, temp);
  else
    k_ms_chains<false><<<grid, 64 * kWaves, 0, s>>>(xk, Kp, krecip, kdisc, blkdisc, masks,
                                                     n_pad / 64, nch, counts, r_lo, r_hi, temp);
  return check("k_ms_chains");
}

int column_sums(const float* temp, int64_t rows, int64_t Kp, int64_t n_kept, const double* init,
                double* out, void* stream) {
  k_ref_colsum<<<(unsigned)((n_kept + 63) / 64), 64, 0, (hipStream_t)stream>>>(temp, rows, Kp,
                                                                               n_kept, init, out);
  return check("k_ref_colsum");
}

int relieff_order(const float* xk, int64_t Kp, const float* krecip, const uint8_t* kdisc,
                  int64_t n_kept, int C, int64_t k, int32_t* nbr, const int32_t* nfound,
                  int64_t r_lo, int64_t r_hi, float* keys, int32_t* dup, void* stream) {
  if (r_hi <= r_lo || k <= 0) return FS_OK;
  const hipStream_t s = (hipStream_t)stream;
  const int64_t lists = (r_hi - r_lo) * C;
  k_rf_ref_keys<<<(unsigned)((lists * k + 255) / 256), 256, 0, s>>>(
      xk, Kp, krecip, kdisc, n_kept, nbr, nfound, r_lo, r_hi, C, k, keys);
  const int rc = check("k_rf_ref_keys");
  if (rc != FS_OK) return rc;
  k_rf_ref_sort<<<(unsigned)((lists + 255) / 256), 256, 0, s>>>(nbr, nfound, keys, r_lo, r_hi, C,
                                                                k, dup);
  return check("k_rf_ref_sort");
}

int relieff_row_keys(const float* xk, int64_t Kp, const float* krecip, const uint8_t* kdisc,
                     int64_t n_kept, const int32_t* rows, int64_t nr, int64_t n, float* keys,
                     void* stream) {
  if (nr <= 0) return FS_OK;
  k_rf_ref_rowkeys<<<dim3((unsigned)nr, (unsigned)((n + 255) / 256)), 256, 0,
                     (hipStream_t)stream>>>(xk, Kp, krecip, kdisc, n_kept, rows, n, keys);
  return check("k_rf_ref_rowkeys");
}

int relieff_order_matters(const float* xk, int64_t Kp, const float* krecip,
                          const uint8_t* kdisc, int64_t n_kept, const int32_t* rows, int64_t nr,
                          const int32_t* dup, const int32_t* nbr, const int32_t* nfound,
                          int64_t r_lo, int C, int64_t k, int32_t* matters, void* stream) {
  if (nr <= 0) return FS_OK;
  k_rf_ref_order_matters<<<(unsigned)nr, 256, 0, (hipStream_t)stream>>>(
      xk, Kp, krecip, kdisc, n_kept, rows, dup, nbr, nfound, r_lo, C, k, matters);
  return check("k_rf_ref_order_matters");
}

int relieff_update(const float* xk, int64_t Kp, const float* krecip, const uint8_t* kdisc,
                   const int32_t* lab, const double* prior, int C, int64_t k, const int32_t* nbr,
                   const int32_t* nfound, int64_t r_lo, int64_t r_hi, float* temp,
                   void* stream) {
  if (r_hi <= r_lo) return FS_OK;
  k_rf_ref_update<<<dim3((unsigned)(Kp / 64), (unsigned)((r_hi - r_lo + 63) / 64)), 256, 0,
                    (hipStream_t)stream>>>(xk, Kp, krecip, kdisc, lab, prior, C, k, nbr, nfound,
                                           r_lo, r_hi, temp);
  return check("k_rf_ref_update");
}

}  // namespace refacc
}  // namespace gpu
}  // namespace fs
