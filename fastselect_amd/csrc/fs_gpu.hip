// fs_gpu.hip -- hand-written HIP kernels for gfx950 (MI355X / CDNA4) and the
// GPU backend of the Relief scoring pipeline (see fs_internal.h).
//
// Kernel map (DESIGN.md §3 for rooflines and bytes per unit):
//   k_quantize      X (row-major) -> xqT (u32, feature-major) + xs (f32,
//                   row-major), 64x64 LDS transpose.                 HBM-bound
//   k_dist          pass 1: one 128x128 upper-triangle pair tile per
//                   workgroup, 8x8 pairs per lane, v_sad_u32 over LDS
//                   panels staged with global_load_lds (double-buffered),
//                   exact integer distances.                         VALU-bound
//   k_tile_rowstats per-row sum D, sum D^2 over owned tiles (+ reduce). HBM-bound
//   k_select_ms     MultiSURF thresholds + near hit / miss counts.   HBM-bound
//   k_surf_avg      SURF float32 sequential row mean (SURF.py:162).  HBM-bound
//   k_weights       symmetric pair weights w_ij = W_ij + W_ji per tile.
//   k_score         pass 2: lanes = features, a 32-row sub-tile of x in
//                   VGPRs, pair weights in SGPRs (scalar loads),
//                   acc += w * |a - b| (v_sub_f32 + v_fma_f32 |.|). VALU-bound
//   k_reduce        deterministic segment sum of pass-2 partials.
//   k_rf_select     ReliefF: per-row radix select of the k nearest per class,
//                   exact keys of the candidates at the k-th key, in one launch.
//   k_rf_update     ReliefF: neighbour-gather update.
//
// No float atomics touch scores: every reduction has a fixed order, so two
// runs of the same input are bit-identical.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <map>
#include <mutex>
#include <thread>
#include <type_traits>
#include <unordered_map>
#include <vector>

#include "../../include/fastselect_amd.h"
#include "fs_internal.h"
#include "fs_sparse_asm.inc"

namespace fs {
namespace gpu {

#define FS_HIP(expr)                                                                      \
  do {                                                                                    \
    hipError_t e_ = (expr);                                                               \
    if (e_ != hipSuccess) {                                                               \
      set_error(std::string("HIP error '") + hipGetErrorString(e_) + "' in " #expr);      \
      return FS_EHIP;                                                                     \
    }                                                                                     \
  } while (0)

int device_count() {
  int c = 0;
  if (hipGetDeviceCount(&c) != hipSuccess) {
    (void)hipGetLastError();
    return 0;
  }
  return c < 0 ? 0 : c;
}

// ---------------------------------------------------------------------------
// Device helpers
// ---------------------------------------------------------------------------

__device__ __forceinline__ uint32_t sad_u32(uint32_t a, uint32_t b, uint32_t c) {
  uint32_t d;
  asm("v_sad_u32 %0, %1, %2, %3" : "=v"(d) : "v"(a), "v"(b), "v"(c));
  return d;
}

// c + |a.lo - b.lo| + |a.hi - b.hi| over unsigned 16-bit halves (two
// features per word; checked on gfx950 by tools/ubench/sad16_check.hip)
__device__ __forceinline__ uint32_t sad_u16(uint32_t a, uint32_t b, uint32_t c) {
  uint32_t d;
  asm("v_sad_u16 %0, %1, %2, %3" : "=v"(d) : "v"(a), "v"(b), "v"(c));
  return d;
}

// c + sc * [a != b] for small category codes, without lane masks (a
// compare would burn an SGPR pair per pair-accumulator).
__device__ __forceinline__ uint32_t mismatch_u32(uint32_t a, uint32_t b, uint32_t sc, uint32_t c) {
  uint32_t t, d;
  asm("v_xor_b32 %1, %2, %3\n\tv_min_u32 %1, %1, 1\n\tv_mad_u32_u24 %0, %1, %4, %5"
      : "=v"(d), "=&v"(t)
      : "v"(a), "v"(b), "v"(sc), "v"(c));
  return d;
}

// Fixed-shape block reduction of doubles (256 threads), deterministic.
__device__ __forceinline__ double block_sum_256(double v, double* red) {
  const int tid = threadIdx.x;
  red[tid] = v;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (tid < s) red[tid] += red[tid + s];
    __syncthreads();
  }
  const double r = red[0];
  __syncthreads();
  return r;
}

// Distance storage.  Full layout (ReliefF / SURF, whose neighbour selection
// reads whole rows): D[i][j] over n_pad x n_pad, both halves.  Tiled layout
// (MultiSURF, whose kernels only ever read inside an owned tile): one
// 128 x 128 block per owned tile t, T_t[b][a] = D(i0 + a, j0 + b) -- half the
// memory of the full matrix for the whole triangle, and a rank of an N-GPU
// job holds only its 1/N of the tiles.  d_at(..., a, b) addresses element
// (i0 + a, j0 + b) of owned tile t either way; consecutive a are consecutive
// doubles in both layouts (the full layout reads it as D[j][i]).
__device__ __forceinline__ int64_t d_at(int tiled, int64_t n_pad, int64_t t, int64_t i0,
                                        int64_t j0, int a, int b) {
  return tiled ? ((t * kTile + b) * kTile + a) : ((j0 + b) * n_pad + i0 + a);
}

// Row window of the full layout (ReliefF / SURF row plans): only the rows
// [win.x, win.y) -- the plan's focal 128-sample blocks -- are stored, and the
// plan's D points where row 0 would be, so row r of the full matrix is still
// D + r * n_pad.  A whole fit stores every row; a row-sharded plan (one rank
// of N, a row panel) 1/N of them.  Writes skip rows outside the window; a
// read of (i0 + a, j0 + b) takes row j0 + b when it is stored and row i0 + a
// otherwise (D is symmetric, and every tile of a row plan has one of its two
// blocks inside the window).
__device__ __forceinline__ bool d_row_in(int2 win, int64_t r) { return r >= win.x && r < win.y; }
__device__ __forceinline__ int64_t d_rd(int tiled, int2 win, int64_t n_pad, int64_t t, int64_t i0,
                                        int64_t j0, int a, int b) {
  if (tiled) return (t * kTile + b) * kTile + a;
  const int64_t j = j0 + b;
  return d_row_in(win, j) ? j * n_pad + i0 + a : (i0 + a) * n_pad + j;
}

// ---------------------------------------------------------------------------
// Quantize: X -> xqT (u32, [PW][n_pad]) and xs (f32, [n_pad][PW])
// ---------------------------------------------------------------------------
// With q16 the continuous rows of xqT are packed: word row c/2 holds features
// c (low half) and c + 1 (high half), and the discrete rows follow at PC/2:
// [PC/2 + PD][n_pad] words in all (pass 1 then walks one contiguous range).
template <typename T>
__global__ __launch_bounds__(256) void k_quantize(
    const T* __restrict__ x, int64_t n, int64_t n_pad, int64_t p_in, int64_t PW, int64_t PC,
    int q16, int64_t pc,
    const int64_t* __restrict__ src_col, const double* __restrict__ off,
    const double* __restrict__ qs, const double* __restrict__ scl,
    const int64_t* __restrict__ dtab_off, const double* __restrict__ dtab, int disc_bits,
    int64_t eps_lo, int64_t eps_hi, uint32_t* __restrict__ xqT, float* __restrict__ xs,
    float* __restrict__ epsT) {
  __shared__ uint32_t tile[64][65];
  __shared__ float etile[64][65];
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const int64_t c0 = (int64_t)blockIdx.x * 64, i0 = (int64_t)blockIdx.y * 64;
  const int64_t c = c0 + tx;
  const int64_t col = src_col[c];
  const bool is_cont = c < pc;
  // all 16 of this thread's loads are issued before any value is used
  constexpr int kR = 16;
  T xr[kR];
#pragma unroll
  for (int k = 0; k < kR; k++) {
    const int64_t i = i0 + ty + 4 * k;
    xr[k] = (i < n && col >= 0) ? x[i * p_in + col] : (T)0;
  }
#pragma unroll
  for (int k = 0; k < kR; k++) {
    const int r = ty + 4 * k;
    const int64_t i = i0 + r;
    uint32_t q = 0;
    float v = 0.0f, e = 0.0f;
    if (i < n && col >= 0) {
      const double xv = (double)xr[k];
      if (is_cont) {
        const double u = __dadd_rn(xv, -off[c]);
        const double t = __dmul_rn(u, qs[c]);
        q = (uint32_t)__dadd_rn(t, 0.5);
        e = (float)((double)q - t);  // rounding error in integer units
        v = (float)__dmul_rn(u, scl[c]);
      } else if (disc_bits) {
        // float32 X: the value's bits are its code (-0.0 folded into +0.0);
        // discrete features only ever compare codes for equality
        float xf = (float)xv;
        if (xf == 0.0f) xf = 0.0f;
        q = __float_as_uint(xf);
        v = xf;
      } else {
        int64_t lo = dtab_off[c], hi = dtab_off[c + 1] - 1;
        while (lo < hi) {
          const int64_t mid = (lo + hi) >> 1;
          if (dtab[mid] < xv) lo = mid + 1;
          else hi = mid;
        }
        q = (uint32_t)(lo - dtab_off[c]);
        v = (float)q;
      }
    }
    xs[i * PW + c] = v;
    tile[r][tx] = q;
    etile[r][tx] = e;
  }
  __syncthreads();
  if (q16 && c0 < PC) {
    for (int r = ty; r < 32; r += 4)
      xqT[(c0 / 2 + r) * n_pad + i0 + tx] = tile[tx][2 * r] | (tile[tx][2 * r + 1] << 16);
  } else {
    const int64_t row0 = q16 ? c0 - PC / 2 : c0;  // discrete rows follow the packed ones
    for (int r = ty; r < 64; r += 4) xqT[(row0 + r) * n_pad + i0 + tx] = tile[tx][r];
  }
  // quantisation errors only for this rank's share of the correction
  for (int r = ty; r < 64; r += 4)
    if (c0 + r >= eps_lo && c0 + r < eps_hi) epsT[(c0 + r) * n_pad + i0 + tx] = etile[tx][r];
}

// Mean-distance correction terms: exact per-column order, fs_colsort.hip
// (colsort_terms): epsT[c][i] <- the bias of sample i's quantised row sum
// in column c, in integer units.

// corr[i] = sum over continuous columns [c_lo, c_hi) (this rank's share) of
// the per-feature bias terms, in two launches.  k_rowcorr: grid (row blocks
// of 64, column slices); workgroup = 64 rows x 16 waves, wave w sums the
// slice's columns w, w + 16, ... (one coalesced 256-byte read per column, two
// independent chains), the 16 partials are added in a fixed order into
// part[slice][i].  The slices fill the chip when there are few row blocks
// (cfg2: 79 row blocks alone left two thirds of the CUs idle, 0.14 ms;
// rowcorr_slices).  k_rowcorr_sum adds the slices in order (deterministic).
constexpr int kRowcorrMaxSlices = 16;
__global__ __launch_bounds__(1024) void k_rowcorr(const float* __restrict__ epsT, int64_t n_pad,
                                                  int64_t c_lo, int64_t c_hi,
                                                  double* __restrict__ part) {
  __shared__ double wp[16][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t i = (int64_t)blockIdx.x * 64 + lane;  // < n_pad
  const int64_t nc = c_hi - c_lo, ns = gridDim.y;
  const int64_t a = c_lo + nc * blockIdx.y / ns, b = c_lo + nc * (blockIdx.y + 1) / ns;
  double s0 = 0.0, s1 = 0.0;
  int64_t c = a + wave;
  for (; c + 16 < b; c += 32) {
    s0 += (double)epsT[c * n_pad + i];
    s1 += (double)epsT[(c + 16) * n_pad + i];
  }
  if (c < b) s0 += (double)epsT[c * n_pad + i];
  wp[wave][lane] = s0 + s1;
  __syncthreads();
  if (wave == 0) {
    double t = 0.0;
#pragma unroll
    for (int w = 0; w < 16; w++) t += wp[w][lane];
    part[(int64_t)blockIdx.y * n_pad + i] = t;
  }
}

__global__ __launch_bounds__(256) void k_rowcorr_sum(const double* __restrict__ part, int slices,
                                                     int64_t n, int64_t n_pad,
                                                     double* __restrict__ corr) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  double t = 0.0;
  for (int sl = 0; sl < slices; sl++) t += part[(int64_t)sl * n_pad + i];
  corr[i] = t;
}

// column slices of k_rowcorr: about 1024 workgroups, at least 64 columns each
static int rowcorr_slices(int64_t n_pad, int64_t ncols) {
  const int64_t rb = std::max<int64_t>(1, n_pad / 64);
  int64_t sl = (1024 + rb - 1) / rb;
  sl = std::min<int64_t>(sl, std::max<int64_t>(1, ncols / 64));
  return (int)std::max<int64_t>(1, std::min<int64_t>(sl, kRowcorrMaxSlices));
}

// ---------------------------------------------------------------------------
// Pass 1: exact integer distance tiles
// ---------------------------------------------------------------------------
// Workgroup = 256 lanes = one 128x128 tile (bi <= bj).  Lane (tx, ty) owns
// rows {ty*4 + r, 64 + ty*4 + r} x cols {tx*4 + c, 64 + tx*4 + c} (8x8).
// Per 16-feature chunk the A panel (rows) and B panel (cols) of xqT, each
// 16 x 128 u32 = 8 KB, are copied global -> LDS by global_load_lds_dwordx4
// (each wave moves 2 x 1 KB of A and of B), double-buffered: chunk c+1 is in
// flight while chunk c is consumed.  u32 accumulators absorb 256 features,
// then their bits >= 24 move into 16-bit halves of a packed high word, so the
// final distance D = hi * 2^24 + lo is exact below 2^40.
// One 16-row chunk from an LDS panel pair: SADs of 32-bit operands
// (kModeU32), of packed 16-bit pairs (kModeU16: 32 features) or mismatch
// counts (kModeDisc).
constexpr int kModeU32 = 0, kModeU16 = 1, kModeDisc = 2;
template <int MODE>
__device__ __forceinline__ void dist_chunk(const uint32_t* __restrict__ A,
                                           const uint32_t* __restrict__ B, int tx, int ty,
                                           uint32_t sc_disc, uint32_t (&acc)[8][8]) {
#pragma unroll 2
  for (int k = 0; k < kBKQ; k++) {
    const uint4 a0 = *(const uint4*)&A[k * kTile + ty * 4];
    const uint4 a1 = *(const uint4*)&A[k * kTile + 64 + ty * 4];
    const uint4 b0 = *(const uint4*)&B[k * kTile + tx * 4];
    const uint4 b1 = *(const uint4*)&B[k * kTile + 64 + tx * 4];
    const uint32_t av[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
    const uint32_t bv[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
#pragma unroll
    for (int r = 0; r < 8; r++)
#pragma unroll
      for (int c = 0; c < 8; c++)
        acc[r][c] = MODE == kModeDisc  ? mismatch_u32(av[r], bv[c], sc_disc, acc[r][c])
                    : MODE == kModeU16 ? sad_u16(av[r], bv[c], acc[r][c])
                                       : sad_u32(av[r], bv[c], acc[r][c]);
  }
}

// K-split: workgroups b < n_full compute whole tiles; the tiles from n_full
// on are split into `splits` parts of their chunk range, workgroup
// n_full + q taking part q % splits of tile n_full + q / splits.  Part 0
// writes D, part s > 0 the compact partial block
// Dpart[(q / splits) * (splits - 1) + s - 1] (tile-local layout T[b][a]);
// k_dist_merge adds them.  The plan splits all tiles or none (choose_ksplit).
__global__ __launch_bounds__(256, 3) void k_dist(const uint32_t* __restrict__ xqT, int64_t n_pad,
                                                 int nck_cont, int nck_disc, uint32_t sc_disc,
                                                 int q16,
                                                 const int2* __restrict__ tiles, int64_t n_full,
                                                 int splits, int tiled, int2 win,
                                                 double* __restrict__ D,
                                                 double* __restrict__ Dpart, float* __restrict__ Dk,
                                                 double inv_sc) {
  // Two distinct LDS objects (not one indexed array) so the compiler can
  // prove a pending global_load_lds into one buffer does not alias the
  // ds_reads of the other and keeps the copy in flight across the compute.
  __shared__ __attribute__((aligned(16))) uint32_t ldsA0[kBKQ * kTile], ldsB0[kBKQ * kTile];
  __shared__ __attribute__((aligned(16))) uint32_t ldsA1[kBKQ * kTile], ldsB1[kBKQ * kTile];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int tx = tid & 15, ty = tid >> 4;
  const int nck_all = nck_cont + nck_disc;
  // glds lane mapping: instruction s of wave w moves k-rows 2*(4w+s) and
  // 2*(4w+s)+1; lane l -> k-row offset l/32, 4 u32 at column (l%32)*4.
  constexpr int kIns = kBKQ / 8;  // glds instructions per wave and panel
  const int krow_l = lane >> 5, col_l = (lane & 31) * 4;

  // One tile's chunks [c_begin, c_end): accumulate, then write the block to
  // D (out_part < 0) or to the compact partial block Dpart[out_part]
  // (tile-local layout T[b][a]).
  auto segment = [&](int64_t t, int c_begin, int c_end, int64_t out_part) {
    const int2 tl = tiles[t];
    const int64_t i0 = (int64_t)tl.x * kTile, j0 = (int64_t)tl.y * kTile;
    double* Dout = D;
    int64_t t_out = t;
    int tiled_out = tiled;
    if (out_part >= 0) {
      Dout = Dpart;
      t_out = out_part;
      tiled_out = 1;
    }
    uint32_t acc[8][8];
    uint32_t hi[8][4];
#pragma unroll
    for (int r = 0; r < 8; r++) {
#pragma unroll
      for (int c = 0; c < 8; c++) acc[r][c] = 0;
#pragma unroll
      for (int c = 0; c < 4; c++) hi[r][c] = 0;
    }
    auto stage = [&](uint32_t* la_base, uint32_t* lb_base, int ck) {
      const int64_t k0 = (int64_t)ck * kBKQ;
#pragma unroll
      for (int s = 0; s < kIns; s++) {
        const int ins = wave * kIns + s;
        const int64_t krow = k0 + ins * 2 + krow_l;
        const uint32_t* ga = xqT + krow * n_pad + i0 + col_l;
        const uint32_t* gb = xqT + krow * n_pad + j0 + col_l;
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)ga,
                                         (__attribute__((address_space(3))) void*)(la_base + ins * 2 * kTile),
                                         16, 0, 0);
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)gb,
                                         (__attribute__((address_space(3))) void*)(lb_base + ins * 2 * kTile),
                                         16, 0, 0);
      }
    };
    auto flush = [&]() {
#pragma unroll
      for (int r = 0; r < 8; r++)
#pragma unroll
        for (int c = 0; c < 8; c++) {
          const uint32_t top = acc[r][c] >> kHiShift;
          acc[r][c] &= (1u << kHiShift) - 1u;
          hi[r][c >> 1] += (c & 1) ? (top << 16) : top;
        }
    };
    // Chunks [c0, c1) of one kind: chunk ck lives in buffer (ck - c0) & 1 and
    // chunk ck+1 is copied while ck is consumed.  Continuous and discrete
    // chunks run in separate loops (one dist_chunk instantiation each), which
    // keeps the register allocation of either loop to itself.
    auto run = [&](auto mode_tag, int c0, int c1) {
      constexpr int MODE = decltype(mode_tag)::value;
      if (c0 >= c1) return;
      stage(ldsA0, ldsB0, c0);
      __syncthreads();
      for (int ck = c0; ck < c1; ck += 2) {
        if (ck + 1 < c1) stage(ldsA1, ldsB1, ck + 1);
        dist_chunk<MODE>(ldsA0, ldsB0, tx, ty, sc_disc, acc);
        if ((ck % kFlushChunks) == kFlushChunks - 1) flush();
        __syncthreads();
        if (ck + 1 < c1) {
          if (ck + 2 < c1) stage(ldsA0, ldsB0, ck + 2);
          dist_chunk<MODE>(ldsA1, ldsB1, tx, ty, sc_disc, acc);
          if (((ck + 1) % kFlushChunks) == kFlushChunks - 1) flush();
          __syncthreads();
        }
      }
    };
    // continuous chunks (16-bit pairs or 32-bit values), then discrete ones
    if (q16)
      run(std::integral_constant<int, kModeU16>{}, c_begin, c_end < nck_cont ? c_end : nck_cont);
    else
      run(std::integral_constant<int, kModeU32>{}, c_begin, c_end < nck_cont ? c_end : nck_cont);
    run(std::integral_constant<int, kModeDisc>{}, c_begin > nck_cont ? c_begin : nck_cont, c_end);
    flush();

    // Epilogue.  Full layout: D[i][j] for the tile and, off the diagonal, the
    // mirror D[j][i], each only where its row is in the window.  Tiled: T_t[b][a]
    // only (the mirror pattern below), which for a diagonal tile is the whole
    // symmetric block.  ReliefF (Dk): the float32 keys f32(D / SC) instead, the
    // value k_rf_select sorts (full layout, whole tiles only).
    if (Dk != nullptr) {
      auto keyv = [&](int r, int c) {
        const uint64_t h = (hi[r][c >> 1] >> ((c & 1) * 16)) & 0xFFFFu;
        return (float)((double)((h << kHiShift) + acc[r][c]) * inv_sc);
      };
#pragma unroll
      for (int r = 0; r < 8; r++) {
        const int64_t i = i0 + ty * 4 + (r & 3) + (r >> 2) * 64;
        if (!d_row_in(win, i)) continue;
        float* row = Dk + i * n_pad + j0 + tx * 4;
        *(float4*)(row + 0) = make_float4(keyv(r, 0), keyv(r, 1), keyv(r, 2), keyv(r, 3));
        *(float4*)(row + 64) = make_float4(keyv(r, 4), keyv(r, 5), keyv(r, 6), keyv(r, 7));
      }
      if (tl.x != tl.y) {
#pragma unroll
        for (int c = 0; c < 8; c++) {
          const int b = tx * 4 + (c & 3) + (c >> 2) * 64;
          if (!d_row_in(win, j0 + b)) continue;
          float* row = Dk + (j0 + b) * n_pad + i0 + ty * 4;
          *(float4*)(row + 0) = make_float4(keyv(0, c), keyv(1, c), keyv(2, c), keyv(3, c));
          *(float4*)(row + 64) = make_float4(keyv(4, c), keyv(5, c), keyv(6, c), keyv(7, c));
        }
      }
      return;
    }
#pragma unroll
    for (int r = 0; r < 8 && !tiled_out; r++) {
      const int64_t i = i0 + ty * 4 + (r & 3) + (r >> 2) * 64;
      if (!d_row_in(win, i)) continue;
      double v[8];
#pragma unroll
      for (int c = 0; c < 8; c++) {
        const uint64_t h = (hi[r][c >> 1] >> ((c & 1) * 16)) & 0xFFFFu;
        v[c] = (double)((h << kHiShift) + acc[r][c]);
      }
      double* row = Dout + i * n_pad + j0 + tx * 4;
      *(double2*)(row + 0) = make_double2(v[0], v[1]);
      *(double2*)(row + 2) = make_double2(v[2], v[3]);
      *(double2*)(row + 64) = make_double2(v[4], v[5]);
      *(double2*)(row + 66) = make_double2(v[6], v[7]);
    }
    if (tl.x != tl.y || tiled_out) {
#pragma unroll
      for (int c = 0; c < 8; c++) {
        const int b = tx * 4 + (c & 3) + (c >> 2) * 64;
        if (!tiled_out && !d_row_in(win, j0 + b)) continue;
        double v[8];
#pragma unroll
        for (int r = 0; r < 8; r++) {
          const uint64_t h = (hi[r][c >> 1] >> ((c & 1) * 16)) & 0xFFFFu;
          v[r] = (double)((h << kHiShift) + acc[r][c]);
        }
        double* row = Dout + d_at(tiled_out, n_pad, t_out, i0, j0, ty * 4, b);
        *(double2*)(row + 0) = make_double2(v[0], v[1]);
        *(double2*)(row + 2) = make_double2(v[2], v[3]);
        *(double2*)(row + 64) = make_double2(v[4], v[5]);
        *(double2*)(row + 66) = make_double2(v[6], v[7]);
      }
    }
  };

  const int64_t b_id = blockIdx.x;
  const int64_t q = b_id - n_full;  // >= 0: a split tile's part
  const int part = q < 0 ? 0 : (int)(q % splits);
  const int nparts = q < 0 ? 1 : splits;
  const int64_t t = q < 0 ? b_id : n_full + q / splits;
  const int c_begin = (int)((int64_t)nck_all * part / nparts);
  const int c_end = (int)((int64_t)nck_all * (part + 1) / nparts);  // this part's chunks
  segment(t, c_begin, c_end, part > 0 ? (q / splits) * (splits - 1) + part - 1 : -1);
}

// ---------------------------------------------------------------------------
// Pass 1, float64 variant (SURF): D[i][j] = sum_f |x'_if - x'_jf| in float64
// ---------------------------------------------------------------------------
// SURF's neighbourhood test compares the float32-rounded distance with a
// float32 sequential mean (SURF.py:158-176), so its distances must round to
// exactly the reference's float32 values; integer quantisation cannot
// promise that, float64 accumulation of float64 diffs can (error ~1e-16).
// x' = (x - min) * recip in float64 (feature-major), discrete columns hold
// category codes.  Same 128x128 tile / 8x8-per-lane layout as k_dist; each
// 16-feature panel is 16 KB (one k-row = one 1 KB global_load_lds_dwordx4).
// 512 lanes per tile: lane (tx, ty) = (tid % 32, tid / 32) owns rows
// {ty*4 + r, 64 + ty*4 + r} x cols {tx*4 + c} (8 x 4 float64 accumulators).
// D += the K-split partials of the split tiles n_full + blockIdx.x (compact
// blocks, tile-local layout T[b][a]), both halves in the full layout
// (integer-valued doubles: exact in any order).  Workgroup (x, y) adds the
// 1024 elements [1024 y, 1024 y + 1024) of tile x, four per lane, so the
// loads of all parts are in flight together.
constexpr int kMergeSlices = kTile * kTile / 1024;
__global__ __launch_bounds__(256) void k_dist_merge(double* __restrict__ D,
                                                   const double* __restrict__ Dpart, int nparts,
                                                   const int2* __restrict__ tiles, int64_t n_full,
                                                   int64_t n_pad, int tiled, int2 win) {
  const int64_t t = n_full + blockIdx.x;
  const int2 tl = tiles[t];
  const int64_t i0 = (int64_t)tl.x * kTile, j0 = (int64_t)tl.y * kTile;
  const double* __restrict__ part = Dpart + (int64_t)blockIdx.x * nparts * kTile * kTile;
  int64_t at[4];
  double v[4];
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const int e = blockIdx.y * 1024 + k * 256 + threadIdx.x;
    at[k] = d_rd(tiled, win, n_pad, t, i0, j0, e % kTile, e / kTile);  // (i0 + a, j0 + b)
    v[k] = D[at[k]];
  }
  for (int s = 0; s < nparts; s++) {
    const double* __restrict__ ps = part + (int64_t)s * kTile * kTile + blockIdx.y * 1024 + threadIdx.x;
#pragma unroll
    for (int k = 0; k < 4; k++) v[k] += ps[k * 256];
  }
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const int e = blockIdx.y * 1024 + k * 256 + threadIdx.x;
    D[at[k]] = v[k];
    // full layout: the other half too where `at` was row j0 + b and row
    // i0 + a is stored (a diagonal tile's `at` covers both halves)
    if (!tiled && tl.x != tl.y && d_row_in(win, j0 + e / kTile) && d_row_in(win, i0 + e % kTile))
      D[(i0 + e % kTile) * n_pad + j0 + e / kTile] = v[k];
  }
}

template <bool DISC>
__device__ __forceinline__ void dist_chunk_f64(const double* __restrict__ A,
                                               const double* __restrict__ B, int tx, int ty,
                                               double (&acc)[8][8]) {
#pragma unroll 2
  for (int k = 0; k < kBK64; k++) {
    const double4 a0 = *(const double4*)&A[k * kTile + ty * 4];
    const double4 a1 = *(const double4*)&A[k * kTile + 64 + ty * 4];
    const double4 b0 = *(const double4*)&B[k * kTile + tx * 4];
    const double4 b1 = *(const double4*)&B[k * kTile + 64 + tx * 4];
    const double av[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
    const double bv[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
#pragma unroll
    for (int r = 0; r < 8; r++)
#pragma unroll
      for (int c = 0; c < 8; c++)
        // codes are small integers: [a != b] == min(|a - b|, 1) without lane masks
        acc[r][c] += DISC ? __builtin_fmin(__builtin_fabs(av[r] - bv[c]), 1.0)
                          : __builtin_fabs(av[r] - bv[c]);
  }
}

// SURF pass 1 in float64 (SURF.py:153-156 arithmetic): one 128x128 tile per
// 256-thread workgroup, 8x8 pairs per lane (the lane layout of k_dist), so a
// k-step reads 128 B of LDS per lane for 64 pair-feature evaluations (8 x 4
// per lane read 96 B for 32 and left the LDS near its bandwidth).
__global__ __launch_bounds__(256, 2) void k_dist_f64(const double* __restrict__ xT, int64_t n_pad,
                                                     int nck_cont, int nck_disc,
                                                     const int2* __restrict__ tiles, int2 win,
                                                     double* __restrict__ D) {
  __shared__ __attribute__((aligned(16))) double ldsA0[kBK64 * kTile], ldsB0[kBK64 * kTile];
  __shared__ __attribute__((aligned(16))) double ldsA1[kBK64 * kTile], ldsB1[kBK64 * kTile];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int2 tl = tiles[blockIdx.x];
  const int64_t i0 = (int64_t)tl.x * kTile, j0 = (int64_t)tl.y * kTile;
  const int tx = tid & 15, ty = tid >> 4;
  double acc[8][8];
#pragma unroll
  for (int r = 0; r < 8; r++)
#pragma unroll
    for (int c = 0; c < 8; c++) acc[r][c] = 0.0;
  // 4 waves; instruction s of wave w moves k-row (kBK64/4)w+s (1 KB): lane
  // l -> doubles 2l, 2l+1 of that row
  constexpr int kRows = kBK64 / 4;
  auto stage = [&](double* la, double* lb, int ck) {
    const int64_t k0 = (int64_t)ck * kBK64;
#pragma unroll
    for (int s = 0; s < kRows; s++) {
      const int krow = wave * kRows + s;
      const double* ga = xT + (k0 + krow) * n_pad + i0 + 2 * lane;
      const double* gb = xT + (k0 + krow) * n_pad + j0 + 2 * lane;
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)ga,
                                       (__attribute__((address_space(3))) void*)(la + krow * kTile),
                                       16, 0, 0);
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)gb,
                                       (__attribute__((address_space(3))) void*)(lb + krow * kTile),
                                       16, 0, 0);
    }
  };
  // continuous then discrete chunks, one instantiation per loop (see k_dist)
  auto run = [&](auto disc_tag, int c0, int c1) {
    constexpr bool DISC = decltype(disc_tag)::value;
    if (c0 >= c1) return;
    stage(ldsA0, ldsB0, c0);
    __syncthreads();
    for (int ck = c0; ck < c1; ck += 2) {
      if (ck + 1 < c1) stage(ldsA1, ldsB1, ck + 1);
      dist_chunk_f64<DISC>(ldsA0, ldsB0, tx, ty, acc);
      __syncthreads();
      if (ck + 1 < c1) {
        if (ck + 2 < c1) stage(ldsA0, ldsB0, ck + 2);
        dist_chunk_f64<DISC>(ldsA1, ldsB1, tx, ty, acc);
        __syncthreads();
      }
    }
  };
  run(std::false_type{}, 0, nck_cont);
  run(std::true_type{}, nck_cont, nck_cont + nck_disc);
#pragma unroll
  for (int r = 0; r < 8; r++) {
    const int64_t i = i0 + ty * 4 + (r & 3) + (r >> 2) * 64;
    if (!d_row_in(win, i)) continue;
    double* row = D + i * n_pad + j0 + tx * 4;
    *(double2*)(row + 0) = make_double2(acc[r][0], acc[r][1]);
    *(double2*)(row + 2) = make_double2(acc[r][2], acc[r][3]);
    *(double2*)(row + 64) = make_double2(acc[r][4], acc[r][5]);
    *(double2*)(row + 66) = make_double2(acc[r][6], acc[r][7]);
  }
  if (tl.x != tl.y) {
#pragma unroll
    for (int c = 0; c < 8; c++) {
      const int64_t j = j0 + tx * 4 + (c & 3) + (c >> 2) * 64;
      if (!d_row_in(win, j)) continue;
      double* row = D + j * n_pad + i0 + ty * 4;
      *(double2*)(row + 0) = make_double2(acc[0][c], acc[1][c]);
      *(double2*)(row + 2) = make_double2(acc[2][c], acc[3][c]);
      *(double2*)(row + 64) = make_double2(acc[4][c], acc[5][c]);
      *(double2*)(row + 66) = make_double2(acc[6][c], acc[7][c]);
    }
  }
}

// x (float64, row-major) -> xT64 (float64, feature-major: scaled values or
// category codes) + xs (float32 pass-2 operands).
__global__ __launch_bounds__(256) void k_quantize_f64(
    const double* __restrict__ x, int64_t n, int64_t n_pad, int64_t p_in, int64_t PW, int64_t pc,
    const int64_t* __restrict__ src_col, const double* __restrict__ off,
    const double* __restrict__ scl, const int64_t* __restrict__ dtab_off,
    const double* __restrict__ dtab, double* __restrict__ xT, float* __restrict__ xs) {
  __shared__ double tile[64][65];
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const int64_t c0 = (int64_t)blockIdx.x * 64, i0 = (int64_t)blockIdx.y * 64;
  const int64_t c = c0 + tx;
  const int64_t col = src_col[c];
  for (int r = ty; r < 64; r += 4) {
    const int64_t i = i0 + r;
    double v = 0.0;
    if (i < n && col >= 0) {
      const double xv = x[i * p_in + col];
      if (c < pc) {
        v = __dmul_rn(__dadd_rn(xv, -off[c]), scl[c]);
      } else {
        int64_t lo = dtab_off[c], hi = dtab_off[c + 1] - 1;
        while (lo < hi) {
          const int64_t mid = (lo + hi) >> 1;
          if (dtab[mid] < xv) lo = mid + 1;
          else hi = mid;
        }
        v = (double)(lo - dtab_off[c]);
      }
    }
    xs[i * PW + c] = (float)v;
    tile[r][tx] = v;
  }
  __syncthreads();
  for (int r = ty; r < 64; r += 4) xT[(c0 + r) * n_pad + i0 + tx] = tile[tx][r];
}

// ---------------------------------------------------------------------------
// MultiSURF row statistics, thresholds and neighbour counts
// ---------------------------------------------------------------------------
// Per-row distance moments from the owned tiles only (tiled D: MultiSURF).
// One workgroup per owned tile t, the 128 x 128 block T_t[b][a] = D(i0 + a,
// j0 + b) read once, coalesced, in 8 chunks of 16 b-rows: thread tid keeps
// row i0 + (tid % 128)'s sums over its half of the b's (combined in a fixed
// order at the end); off the diagonal each chunk is also staged in LDS,
// where 8 lanes per b sum the chunk's 16 columns over a (shuffle-reduced in
// a fixed order) -> part[t][256]: [0, 128) rows i0 + a, [128, 256) rows
// j0 + b.  k_rowstats_reduce adds a row's tile partials in tile order
// (deterministic) and appends this rank's mean correction: rowstats[3i] =
// sum D, [3i+1] = sum D^2, [3i+2] = corr share.
__global__ __launch_bounds__(256) void k_tile_rowstats(const double* __restrict__ D, int64_t n,
                                                       const int2* __restrict__ tiles,
                                                       double2* __restrict__ part) {
  __shared__ double chunk[16][kTile + 1];
  __shared__ double2 red[kTile];
  __shared__ double2 cols[kTile];
  const int2 tl = tiles[blockIdx.x];
  const int64_t i0 = (int64_t)tl.x * kTile, j0 = (int64_t)tl.y * kTile;
  const double* T = D + (int64_t)blockIdx.x * kTile * kTile;
  const int tid = threadIdx.x;
  const int a = tid & (kTile - 1), h = tid >> 7;
  const bool diag = tl.x == tl.y;
  const bool a_in = i0 + a < n;
  double s1 = 0.0, s2 = 0.0;
  for (int k = 0; k < kTile / 16; k++) {
    double v[8];
#pragma unroll
    for (int u = 0; u < 8; u++) v[u] = T[(16 * k + h + 2 * u) * kTile + a];  // b = 16k + h + 2u
#pragma unroll
    for (int u = 0; u < 8; u++) {
      const int64_t o = j0 + 16 * k + h + 2 * u;
      const double d = (a_in && o < n && o != i0 + a) ? v[u] : 0.0;
      s1 += d;
      s2 += d * d;
    }
    if (!diag) {
#pragma unroll
      for (int u = 0; u < 8; u++) chunk[h + 2 * u][a] = a_in ? v[u] : 0.0;
      __syncthreads();
      if (tid < 128) {
        const int bl = tid >> 3, q = tid & 7;
        double c1 = 0.0, c2 = 0.0;
#pragma unroll
        for (int e = 0; e < 16; e++) {
          const double d = chunk[bl][16 * q + e];
          c1 += d;
          c2 += d * d;
        }
#pragma unroll
        for (int o = 4; o > 0; o >>= 1) {
          c1 += __shfl_xor(c1, o);
          c2 += __shfl_xor(c2, o);
        }
        if (q == 0) cols[16 * k + bl] = make_double2(c1, c2);
      }
      __syncthreads();
    }
  }
  if (h == 1) red[a] = make_double2(s1, s2);
  __syncthreads();
  double2 out;
  if (tid < kTile) {
    const double2 o = red[a];
    out = make_double2(s1 + o.x, s2 + o.y);
  } else {
    const int b = tid - kTile;
    out = (!diag && j0 + b < n) ? cols[b] : make_double2(0.0, 0.0);
  }
  part[(int64_t)blockIdx.x * 256 + tid] = out;
}

__global__ void k_rowstats_reduce(const double2* __restrict__ part, int64_t n, int64_t nb,
                                  int rank, int world, const double* __restrict__ corr,
                                  double* __restrict__ rowstats) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const int64_t b = i / kTile, r = i % kTile;
  double s1 = 0.0, s2 = 0.0;
  for (int64_t a = 0; a < nb; a++) {
    const int64_t lo = a < b ? a : b, hi = a < b ? b : a;
    const int64_t t = tile_linear(nb, lo, hi);
    if (t % world != rank) continue;
    // tile (b, a >= b): row block b are its rows; tile (a < b, b): its columns
    const double2 v = part[(t / world) * 256 + (a >= b ? r : kTile + r)];
    s1 += v.x;
    s2 += v.y;
  }
  rowstats[3 * i] = s1;
  rowstats[3 * i + 1] = s2;
  rowstats[3 * i + 2] = corr[i];
}

// MultiSURF threshold (integer units): the quantised mean corrected by
// corr[i]/(n-1), minus half the quantised spread (MultiSURF.py:193-196).
__global__ void k_thr_ms(const double* __restrict__ rowstats, int64_t n,
                         double* __restrict__ thr) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const double nm1 = (double)(n - 1);
  const double mu = rowstats[3 * i] / nm1;
  double var = rowstats[3 * i + 1] / nm1 - mu * mu;
  if (var < 0.0) var = 0.0;
  thr[i] = (mu - rowstats[3 * i + 2] / nm1) - 0.5 * __builtin_sqrt(var);
}

// SURF: avg_i = float32 sequential sum over j (self included, D_ii = 0) of
// the float32 distance row, / (n - 1) in float64 (SURF.py:146-163).  One
// wave per 64 focal rows: 64 x 64 blocks of the rows are staged through LDS
// with coalesced row-segment loads (a row plan stores only its own rows, so
// the symmetric column cannot be read instead), then lane r adds its row's 64
// values in j order -- the float32 sum stays strictly sequential in j, the
// reference's order.
__global__ __launch_bounds__(64) void k_surf_avg(const double* __restrict__ D, int64_t n,
                                                 int64_t n_pad, double inv_sc, int64_t r_lo,
                                                 int64_t r_hi, double* __restrict__ avg) {
  __shared__ float blk[64][65];
  const int lane = threadIdx.x;
  const int64_t row0 = r_lo + (int64_t)blockIdx.x * 64;
  const int64_t nrows = r_hi - row0 < 64 ? r_hi - row0 : 64;
  float s = 0.0f;
  for (int64_t j0 = 0; j0 < n; j0 += 64) {
    const int64_t j = j0 + lane;
#pragma unroll 8
    for (int r = 0; r < 64; r++) {
      float v = 0.0f;
      if (r < nrows && j < n) v = (float)(D[(row0 + r) * n_pad + j] * inv_sc);
      blk[r][lane] = v;
    }
    __syncthreads();
    const int cnt = n - j0 < 64 ? (int)(n - j0) : 64;
    for (int c = 0; c < cnt; c++) s += blk[lane][c];
    __syncthreads();
  }
  if (lane < nrows) avg[row0 + lane] = (double)s / (double)(n - 1);
}

// Flagged pairs are collected per workgroup in LDS and appended to the
// global list with one atomic per workgroup (a single global counter hit by
// every wave that flags a pair serialises in L2).  Overflow of the LDS
// buffer falls back to direct appends.
constexpr int kPairBuf = 1024;
struct PairBuf {
  int2 v[kPairBuf];
  unsigned int n;
  unsigned long long base;
};
__device__ __forceinline__ void pairbuf_init(PairBuf& pb) {
  if (threadIdx.x == 0) pb.n = 0u;
  __syncthreads();
}
__device__ __forceinline__ void pairbuf_add(PairBuf& pb, int64_t i, int64_t j,
                                            int2* __restrict__ list, int64_t cap,
                                            unsigned long long* __restrict__ count) {
  const unsigned int s = atomicAdd(&pb.n, 1u);
  if (s < (unsigned)kPairBuf) {
    pb.v[s] = make_int2((int)i, (int)j);
  } else {
    const unsigned long long k = atomicAdd(count, 1ull);
    if ((int64_t)k < cap) list[k] = make_int2((int)i, (int)j);
  }
}
__device__ __forceinline__ void pairbuf_flush(PairBuf& pb, int2* __restrict__ list, int64_t cap,
                                              unsigned long long* __restrict__ count) {
  __syncthreads();
  const unsigned int m = pb.n < (unsigned)kPairBuf ? pb.n : (unsigned)kPairBuf;
  if (m == 0u) return;
  if (threadIdx.x == 0) pb.base = atomicAdd(count, (unsigned long long)m);
  __syncthreads();
  for (unsigned int t = threadIdx.x; t < m; t += blockDim.x) {
    const unsigned long long k = pb.base + t;
    if ((int64_t)k < cap) list[k] = pb.v[t];
  }
}

// Ambiguous pairs of the owned tiles: the quantised distance lies within the
// error band of either endpoint's threshold, so the near/far decision could
// differ from the reference's.  They are appended to `list` (capacity cap,
// *count may exceed it: the host then grows the list and re-runs).
// MultiSURF compares D (integer units) with thr; SURF compares the float32
// distance with the float64 mean, the band widened by 4 float32 ulps of it.
__global__ __launch_bounds__(256) void k_flag_pairs(const double* __restrict__ D, int64_t n,
                                                    int64_t n_pad, int tiled, int2 win,
                                                    const int2* __restrict__ tiles,
                                                    const double* __restrict__ thr, int algo,
                                                    double inv_sc, double delta,
                                                    int2* __restrict__ list, int64_t cap,
                                                    unsigned long long* __restrict__ count) {
  __shared__ PairBuf pb;
  pairbuf_init(pb);
  const int2 tl = tiles[blockIdx.x];
  const int64_t i0 = (int64_t)tl.x * kTile, j0 = (int64_t)tl.y * kTile;
  for (int e = threadIdx.x; e < kTile * kTile; e += 256) {
    const int jj = e / kTile, ii = e % kTile;
    const int64_t i = i0 + ii, j = j0 + jj;
    bool amb = false;
    if (!(i < n && j < n && (tl.x < tl.y || ii < jj))) {
    } else if (algo == ALGO_MULTISURF) {
      const double d = D[d_rd(tiled, win, n_pad, blockIdx.x, i0, j0, ii, jj)];
      amb = __builtin_fabs(d - thr[i]) < delta || __builtin_fabs(d - thr[j]) < delta;
    } else {
      const double df = D[d_rd(tiled, win, n_pad, blockIdx.x, i0, j0, ii, jj)] * inv_sc;
      const float ai = (float)thr[i], aj = (float)thr[j];
      const double bi = delta + 4.0 * ((double)__uint_as_float(__float_as_uint(ai) + 1u) - (double)ai);
      const double bj = delta + 4.0 * ((double)__uint_as_float(__float_as_uint(aj) + 1u) - (double)aj);
      amb = __builtin_fabs(df - thr[i]) < bi || __builtin_fabs(df - thr[j]) < bj;
    }
    if (amb) pairbuf_add(pb, i, j, list, cap, count);
  }
  pairbuf_flush(pb, list, cap, count);
}

// Where a refined pair's distance goes.  Full layout: D[i][j] and D[j][i].
// Tiled (tw.x = tile rows nb, tw.y = world): pair i < j lives in the owned
// tile of blocks (i / 128, j / 128), the (linear / world)-th tile this rank
// owns (round-robin ownership, owned_tiles); a diagonal tile holds both
// halves.
__device__ __forceinline__ void store_pair(double* __restrict__ D, int64_t n_pad, int2 tw, int2 win,
                                           int2 pr, double v) {
  if (tw.x == 0) {  // full layout: both halves, where their rows are stored
    if (d_row_in(win, pr.x)) D[(int64_t)pr.x * n_pad + pr.y] = v;
    if (d_row_in(win, pr.y)) D[(int64_t)pr.y * n_pad + pr.x] = v;
    return;
  }
  if (pr.x > pr.y) pr = make_int2(pr.y, pr.x);
  const int64_t I = pr.x / kTile, J = pr.y / kTile;  // I <= J
  const int64_t t = tile_linear(tw.x, I, J) / tw.y;
  const int a = pr.x - (int)(I * kTile), b = pr.y - (int)(J * kTile);
  D[(t * kTile + b) * kTile + a] = v;
  if (I == J) D[(t * kTile + a) * kTile + b] = v;
}

// Exact thresholds for the rows that need them (MultiSURF, plan_select).  A
// refined pair compares the reference's own distance with our threshold,
// and that threshold is not the reference's: the mean is exact (the
// correction), but the spread comes from the quantised second moments, off
// by ~(band / 12) / sqrt(n - 1) integer units (the rounding of one pair's
// distance averaged over a row).  A refined pair whose exact distance lies
// within thr_tol of an endpoint's threshold could therefore still be
// decided differently (VERDICT r3 missing #1's decision-level bar: uniform
// noise, n = 16384, one row of 16384).  Those rows are flagged here; if no
// more than exact_thr_rows(n) are, their thresholds are recomputed from exact
// distances to every other sample (k_row_exact_parts / k_row_exact_thr:
// the reference's sum_j D_ij and sum_j D_ij^2, MultiSURF.py:174-196) before
// any pair is counted.  A rank fixes the rows its own refined pairs flag:
// a pair far from a threshold is decided alike by both values, so ranks
// that keep the quantised value for a row decide their pairs correctly too.
__device__ __forceinline__ void mark_uncertain(int2 pr, double v, const double* __restrict__ thr,
                                               double thr_tol, unsigned int* __restrict__ unc) {
  if (__builtin_fabs(v - thr[pr.x]) < thr_tol) unc[pr.x] = 1u;
  if (__builtin_fabs(v - thr[pr.y]) < thr_tol) unc[pr.y] = 1u;
}

// The flagged rows in index order (the first max_rows of them) and their
// count: one 1024-thread workgroup, a contiguous index range per thread.
__global__ __launch_bounds__(1024) void k_unc_compact(const unsigned int* __restrict__ unc,
                                                      int64_t n, int max_rows,
                                                      int32_t* __restrict__ rows,
                                                      int32_t* __restrict__ nrows) {
  __shared__ int part[1024];
  const int t = threadIdx.x;
  const int64_t per = (n + 1023) / 1024;
  const int64_t a = t * per, b = a + per < n ? a + per : n;
  int c = 0;
  for (int64_t i = a; i < b; i++) c += unc[i] != 0u;
  part[t] = c;
  __syncthreads();
  for (int o = 1; o < 1024; o <<= 1) {  // inclusive scan
    const int v = t >= o ? part[t - o] : 0;
    __syncthreads();
    part[t] += v;
    __syncthreads();
  }
  int pos = part[t] - c;
  for (int64_t i = a; i < b; i++)
    if (unc[i] != 0u) {
      if (pos < max_rows) rows[pos] = (int32_t)i;
      pos++;
    }
  if (t == 1023) *nrows = part[1023];
}

// Exact row moments of the flagged rows: grid (chunks of kExChunk = 4
// samples j -- many workgroups even for one flagged row: the loop is
// latency-bound --, groups of 8 flagged rows); the group's slots take
// rows[8 g + k] when the count allows the fix (slots past the count repeat
// the group's last row and are discarded).  The 4 waves split the features
// (wave w, lane l: features w * 64 + l + 256 k), so each wave's chain of
// dependent loads is p / 256 long, not p / 64 as when a wave walked every
// feature of its own samples (cfg2: 0.39 ms for one flagged row).  Per
// feature k_exact_pairs' arithmetic (float32 |a - b| * recip, a float64
// sum); each of the 12 row values per feature is read once for 32
// pair-features, so X streams once per 8 flagged rows.  Each pair's lane sums
// are reduced across the wave, the 4 waves' sums added in a fixed order in
// LDS, and D_ij, D_ij^2 summed in j order (j != i) into
// parts[8 g + k][chunk].
constexpr int kExRows = 8, kExJ = 4, kExChunk = kExJ;
template <typename T>
__global__ __launch_bounds__(256) void k_row_exact_parts(
    const T* __restrict__ x, int64_t n, int64_t p_in, int64_t pc, int64_t PC, int64_t pd,
    const int64_t* __restrict__ src_col, const double* __restrict__ scl,
    const int32_t* __restrict__ rows, const int32_t* __restrict__ nrows, int max_rows,
    double2* __restrict__ parts) {
  __shared__ double wd[4][kExRows][kExJ];
  const int cnt = *nrows;
  const int g = blockIdx.y;
  if (cnt > max_rows || g * kExRows >= cnt) return;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int nr = cnt - g * kExRows < kExRows ? cnt - g * kExRows : kExRows;
  int64_t ri[kExRows];
#pragma unroll
  for (int k = 0; k < kExRows; k++) ri[k] = rows[g * kExRows + (k < nr ? k : nr - 1)];
  const int64_t j0 = (int64_t)blockIdx.x * kExChunk;
  int64_t jj[kExJ];
#pragma unroll
  for (int m = 0; m < kExJ; m++) jj[m] = j0 + m < n ? j0 + m : n - 1;
  double acc[kExRows][kExJ];
#pragma unroll
  for (int k = 0; k < kExRows; k++)
#pragma unroll
    for (int m = 0; m < kExJ; m++) acc[k][m] = 0.0;
  const int c0 = wave * 64 + lane;
#pragma unroll 2
  for (int64_t c = c0; c < pc; c += 256) {
    const int64_t col = src_col[c];
    T a[kExRows], b[kExJ];
#pragma unroll
    for (int k = 0; k < kExRows; k++) a[k] = x[ri[k] * p_in + col];
#pragma unroll
    for (int m = 0; m < kExJ; m++) b[m] = x[jj[m] * p_in + col];
    if (sizeof(T) == 4) {
      const float r = (float)scl[c];
#pragma unroll
      for (int k = 0; k < kExRows; k++)
#pragma unroll
        for (int m = 0; m < kExJ; m++)
          acc[k][m] += (double)(__builtin_fabsf((float)a[k] - (float)b[m]) * r);
    } else {
      const double r = scl[c];
#pragma unroll
      for (int k = 0; k < kExRows; k++)
#pragma unroll
        for (int m = 0; m < kExJ; m++)
          acc[k][m] += __builtin_fabs((double)a[k] - (double)b[m]) * r;
    }
  }
  for (int64_t c = PC + c0; c < PC + pd; c += 256) {
    const int64_t col = src_col[c];
#pragma unroll
    for (int k = 0; k < kExRows; k++)
#pragma unroll
      for (int m = 0; m < kExJ; m++)
        acc[k][m] += (x[ri[k] * p_in + col] != x[jj[m] * p_in + col]) ? 1.0 : 0.0;
  }
#pragma unroll
  for (int k = 0; k < kExRows; k++)
#pragma unroll
    for (int m = 0; m < kExJ; m++) {
      double v = acc[k][m];
      for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
      if (lane == 0) wd[wave][k][m] = v;
    }
  __syncthreads();
  if (threadIdx.x < nr) {
    const int k = threadIdx.x;
    const int64_t i = rows[g * kExRows + k];
    double s1 = 0.0, s2 = 0.0;
#pragma unroll
    for (int m = 0; m < kExJ; m++) {
      const double d = (wd[0][k][m] + wd[1][k][m]) + (wd[2][k][m] + wd[3][k][m]);
      const int64_t j = j0 + m;
      if (j < n && j != i) {
        s1 += d;
        s2 += d * d;
      }
    }
    parts[(int64_t)(g * kExRows + k) * gridDim.x + blockIdx.x] = make_double2(s1, s2);
  }
}

// thr[rows[s]] from the chunk partials (fixed order), in integer units.
__global__ __launch_bounds__(64) void k_row_exact_thr(const double2* __restrict__ parts,
                                                      int64_t nchunk, const int32_t* __restrict__ rows,
                                                      const int32_t* __restrict__ nrows,
                                                      int max_rows, int64_t n, double sc,
                                                      double* __restrict__ thr) {
  const int cnt = *nrows;
  const int slot = blockIdx.x;
  if (cnt > max_rows || slot >= cnt) return;
  const int lane = threadIdx.x;
  double s1 = 0.0, s2 = 0.0;
  for (int64_t c = lane; c < nchunk; c += 64) {
    const double2 v = parts[(int64_t)slot * nchunk + c];
    s1 += v.x;
    s2 += v.y;
  }
  for (int o = 32; o > 0; o >>= 1) {
    s1 += __shfl_xor(s1, o);
    s2 += __shfl_xor(s2, o);
  }
  if (lane == 0) thr[rows[slot]] = multisurf_threshold(s1, s2, n) * sc;
}

// Reference-exact distance of each listed pair: sum_f diff_f(i, j) in
// float64 with diff_f computed exactly as the reference kernels do
// (MultiSURF.py:184-187 / ReliefF.py:151-154 in float32, SURF.py:153-156 in
// float64).  One wave per pair, lanes stride the permuted feature columns;
// the result (in integer units) overwrites both D[i][j] and D[j][i].
template <typename T>
__global__ __launch_bounds__(256) void k_exact_pairs(
    const T* __restrict__ x, int64_t p_in, int64_t pc, int64_t PC, int64_t pd,
    const int64_t* __restrict__ src_col, const double* __restrict__ scl, double sc,
    const int2* __restrict__ list, const unsigned long long* __restrict__ count, int64_t cap,
    int64_t n_pad, int2 tw, int2 win, int mark_f32, double* __restrict__ D,
    float* __restrict__ Dk, const double* __restrict__ thr, double thr_tol,
    unsigned int* __restrict__ unc) {
  const int lane = threadIdx.x & 63;
  const int64_t wave = ((int64_t)blockIdx.x * 256 + threadIdx.x) >> 6;
  const int64_t nw = ((int64_t)gridDim.x * 256) >> 6;
  const int64_t total = (int64_t)*count < cap ? (int64_t)*count : cap;
  for (int64_t k = wave; k < total; k += nw) {
    const int2 pr = list[k];
    const T* xi = x + (int64_t)pr.x * p_in;
    const T* xj = x + (int64_t)pr.y * p_in;
    double acc = 0.0;
    // 4 features per lane per step: the column indices, then all 8 values,
    // are requested before any is used (the row reads are latency-bound)
    constexpr int kU = 4;
    for (int64_t c0 = lane; c0 < pc; c0 += 64 * kU) {
      int64_t col[kU];
      T a[kU], b[kU];
#pragma unroll
      for (int u = 0; u < kU; u++) col[u] = c0 + 64 * u < pc ? src_col[c0 + 64 * u] : -1;
#pragma unroll
      for (int u = 0; u < kU; u++) {
        a[u] = col[u] >= 0 ? xi[col[u]] : (T)0;
        b[u] = col[u] >= 0 ? xj[col[u]] : (T)0;
      }
#pragma unroll
      for (int u = 0; u < kU; u++) {
        if (col[u] < 0) break;
        const int64_t c = c0 + 64 * u;
        if (sizeof(T) == 4) {
          const float dv = __builtin_fabsf((float)a[u] - (float)b[u]) * (float)scl[c];
          acc += (double)dv;
        } else {
          acc += __builtin_fabs((double)a[u] - (double)b[u]) * scl[c];
        }
      }
    }
    for (int64_t c = PC + lane; c < PC + pd; c += 64) {
      const int64_t col = src_col[c];
      acc += (xi[col] != xj[col]) ? 1.0 : 0.0;
    }
    for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
    if (lane == 0) {
      // MultiSURF: exact distance in integer units.  ReliefF (mark_f32): the
      // reference's float32 key, stored negated so k_rf_select knows it is
      // exact (a zero key is stored as +0, never -0, whose bits would sort last).
      if (Dk != nullptr) {  // ReliefF float keys (full layout): the key itself
        const float kf = (float)acc;
        if (d_row_in(win, pr.x)) Dk[(int64_t)pr.x * n_pad + pr.y] = kf;
        if (d_row_in(win, pr.y)) Dk[(int64_t)pr.y * n_pad + pr.x] = kf;
      } else {
        const double v = mark_f32 ? (acc > 0.0 ? -(double)(float)acc : 0.0) : acc * sc;
        store_pair(D, n_pad, tw, win, pr, v);
        if (unc != nullptr) mark_uncertain(pr, v, thr, thr_tol, unc);
      }
    }
  }
}

// k_exact_pairs for the common layout -- every kept feature continuous, in
// input order (src_col = identity), float32 X with a 16-byte row pitch --
// reading both rows as float4 (16 B per lane, 4 KB per wave per row and
// step, 8 loads in flight per lane) instead of a column-indexed dword
// gather.  Same arithmetic per feature: f32 |a - b| * f32 recip, summed in
// f64.  The list is sorted by (i, j), so consecutive waves share row i
// through L2; row j is the HBM read.
__global__ __launch_bounds__(256) void k_exact_pairs_rows(
    const float* __restrict__ x, int64_t p, const float* __restrict__ scl32, double sc,
    const int2* __restrict__ list, const unsigned long long* __restrict__ count, int64_t cap,
    int64_t n_pad, int2 tw, int2 win, double* __restrict__ D, const double* __restrict__ thr,
    double thr_tol, unsigned int* __restrict__ unc) {
  const int lane = threadIdx.x & 63;
  const int64_t wave = ((int64_t)blockIdx.x * 256 + threadIdx.x) >> 6;
  const int64_t nw = ((int64_t)gridDim.x * 256) >> 6;
  const int64_t total = (int64_t)*count < cap ? (int64_t)*count : cap;
  const int64_t p4 = p / 4;
  const float4* __restrict__ s4 = (const float4*)scl32;
  for (int64_t k = wave; k < total; k += nw) {
    const int2 pr = list[k];
    const float4* __restrict__ xi = (const float4*)(x + (int64_t)pr.x * p);
    const float4* __restrict__ xj = (const float4*)(x + (int64_t)pr.y * p);
    double acc = 0.0;
    constexpr int kU = 4;
    for (int64_t c0 = lane; c0 < p4; c0 += 64 * kU) {
      float4 a[kU], b[kU], w[kU];
#pragma unroll
      for (int u = 0; u < kU; u++) {
        const int64_t c = c0 + 64 * u;
        const bool in = c < p4;
        a[u] = in ? xi[c] : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        b[u] = in ? xj[c] : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        w[u] = in ? s4[c] : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
      }
#pragma unroll
      for (int u = 0; u < kU; u++) {
        acc += (double)(__builtin_fabsf(a[u].x - b[u].x) * w[u].x);
        acc += (double)(__builtin_fabsf(a[u].y - b[u].y) * w[u].y);
        acc += (double)(__builtin_fabsf(a[u].z - b[u].z) * w[u].z);
        acc += (double)(__builtin_fabsf(a[u].w - b[u].w) * w[u].w);
      }
    }
    for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
    if (lane == 0) {
      store_pair(D, n_pad, tw, win, pr, acc * sc);
      if (unc != nullptr) mark_uncertain(pr, acc * sc, thr, thr_tol, unc);
    }
  }
}

// Band calibration (calibrate_band): for each sampled pair, the quantised
// distance's error against the reference's arithmetic, err = sum over the
// continuous kept features of |q_i - q_j| - SC * f32(|x_i - x_j| * recip),
// for the 16-bit scale (.x) and the 32-bit scale (.y).  q is formed exactly
// as k_quantize forms it; discrete features contribute no error.  One wave
// per pair, fixed-order reduction (every rank computes the same values).
template <typename T>
__global__ __launch_bounds__(256) void k_calib(
    const T* __restrict__ x, int64_t p_in, int64_t pc, const int64_t* __restrict__ src_col,
    const double* __restrict__ off, const double* __restrict__ qs16,
    const double* __restrict__ qs32, const float* __restrict__ scl32, double sc16, double sc32,
    const int2* __restrict__ pairs, int64_t npairs, double2* __restrict__ err) {
  const int lane = threadIdx.x & 63;
  const int64_t k = ((int64_t)blockIdx.x * 256 + threadIdx.x) >> 6;
  if (k >= npairs) return;
  const int2 pr = pairs[k];
  const T* xi = x + (int64_t)pr.x * p_in;
  const T* xj = x + (int64_t)pr.y * p_in;
  double e16 = 0.0, e32 = 0.0;
  for (int64_t c = lane; c < pc; c += 64) {
    const int64_t col = src_col[c];
    const double a = (double)xi[col], b = (double)xj[col];
    const double ua = __dadd_rn(a, -off[c]), ub = __dadd_rn(b, -off[c]);
    const uint32_t qa16 = (uint32_t)__dadd_rn(__dmul_rn(ua, qs16[c]), 0.5);
    const uint32_t qb16 = (uint32_t)__dadd_rn(__dmul_rn(ub, qs16[c]), 0.5);
    const uint32_t qa32 = (uint32_t)__dadd_rn(__dmul_rn(ua, qs32[c]), 0.5);
    const uint32_t qb32 = (uint32_t)__dadd_rn(__dmul_rn(ub, qs32[c]), 0.5);
    const double ref = (double)(__builtin_fabsf((float)a - (float)b) * scl32[c]);
    e16 += (qa16 > qb16 ? (double)(qa16 - qb16) : (double)(qb16 - qa16)) - sc16 * ref;
    e32 += (qa32 > qb32 ? (double)(qa32 - qb32) : (double)(qb32 - qa32)) - sc32 * ref;
  }
  for (int o = 32; o > 0; o >>= 1) {
    e16 += __shfl_xor(e16, o);
    e32 += __shfl_xor(e32, o);
  }
  if (lane == 0) err[k] = make_double2(e16, e32);
}

// Near hit / miss counts over the owned tiles (D now exact for ambiguous
// pairs): counts[2i], counts[2i+1].
__global__ __launch_bounds__(256) void k_tile_counts(const double* __restrict__ D, int64_t n,
                                                     const int2* __restrict__ tiles,
                                                     const int32_t* __restrict__ lab,
                                                     const double* __restrict__ thr,
                                                     double* __restrict__ counts) {
  // Near hits / misses over the owned tiles (tiled D, exact for ambiguous
  // pairs by now), same lane layout as k_tile_rowstats; counts are integers,
  // so the atomic adds and the wave reductions are exact in any order
  // (counts zeroed by the caller).
  const int2 tl = tiles[blockIdx.x];
  const int64_t i0 = (int64_t)tl.x * kTile, j0 = (int64_t)tl.y * kTile;
  const double* T = D + (int64_t)blockIdx.x * kTile * kTile;
  const int tid = threadIdx.x;
  if (tid < kTile) {
    const int a = tid;
    const int64_t self = i0 + a;
    if (self >= n) return;
    const double t = thr[self];
    const int32_t ls = lab[self];
    double h = 0.0, m = 0.0;
    for (int b0 = 0; b0 < kTile; b0 += 8) {
      bool near[8];  // 8 loads in flight per step
#pragma unroll
      for (int u = 0; u < 8; u++) {
        const int64_t o = j0 + b0 + u;
        const double v = T[(b0 + u) * kTile + a];
        near[u] = (o < n) & (o != self) & (v < t);
      }
#pragma unroll
      for (int u = 0; u < 8; u++) {
        if (near[u]) {
          if (lab[j0 + b0 + u] == ls) h += 1.0;
          else m += 1.0;
        }
      }
    }
    if (h != 0.0) atomicAdd(&counts[2 * self], h);
    if (m != 0.0) atomicAdd(&counts[2 * self + 1], m);
    return;
  }
  if (tl.x == tl.y) return;
  // columns: row j0 + b over the tile's rows, one b per step (contiguous
  // T_t[b][0..127]), wave-reduced; lane b % 64 keeps column b's counts
  const int lane = tid & 63, w2 = (tid >> 6) - 2;
  const bool in0 = i0 + lane < n, in1 = i0 + 64 + lane < n;
  const int32_t l0 = in0 ? lab[i0 + lane] : -1, l1 = in1 ? lab[i0 + 64 + lane] : -1;
  double h = 0.0, m = 0.0;
  for (int k = 0; k < 64; k++) {
    const int b = 64 * w2 + k;
    const int64_t self = j0 + b;
    if (self >= n) break;  // uniform across the wave
    const double t = thr[self];
    const int32_t ls = lab[self];
    const double v0 = T[b * kTile + lane], v1 = T[b * kTile + 64 + lane];
    const bool n0 = in0 && v0 < t, n1 = in1 && v1 < t;
    double hh = (n0 && l0 == ls ? 1.0 : 0.0) + (n1 && l1 == ls ? 1.0 : 0.0);
    double mm = (n0 && l0 != ls ? 1.0 : 0.0) + (n1 && l1 != ls ? 1.0 : 0.0);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      hh += __shfl_xor(hh, o);
      mm += __shfl_xor(mm, o);
    }
    if (lane == k) {
      h = hh;
      m = mm;
    }
  }
  const int64_t self = j0 + 64 * w2 + lane;
  if (self < n) {
    if (h != 0.0) atomicAdd(&counts[2 * self], h);
    if (m != 0.0) atomicAdd(&counts[2 * self + 1], m);
  }
}

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
  double wi, wj;
  if (algo == ALGO_MULTISURF) {
    wi = multisurf_weight(d < thr[i], hit, use_star, counts[2 * i], counts[2 * i + 1]);
    wj = multisurf_weight(d < thr[j], hit, use_star, counts[2 * j], counts[2 * j + 1]);
  } else {  // SURF: float32 distance against the float64 mean
    const double df = (double)(float)(d * inv_sc);
    wi = surf_weight(df < thr[i], hit, use_star);
    wj = surf_weight(df < thr[j], hit, use_star);
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
constexpr int kSWaves = 16;
// entries a tile's streams may hold: 16 streams x 8 columns x 128 rows (both halves)
constexpr int kStreamEntries = (kTile / kSWaves) * kTile;
// floats past xs's last spare row that a pass-2 B-row read may touch (the
// widest feature block of k_score_sparse2)
constexpr int64_t kXsSlack = 512;

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
constexpr int kXcds = 8;
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
  out[o] = (q[0] + q[1]) + (q[2] + q[3]);
}

// ---------------------------------------------------------------------------
// ReliefF: per-row k-nearest selection per class (radix select on the
// float32 distance bits, index order among equal keys) and neighbour update
// ---------------------------------------------------------------------------
// The key of j is the reference's float32 distance row (ReliefF.py:149-155):
// float32(D_ij / SC) from the quantised distance, or the exact reference key
// where k_exact_pairs stored one.  ReliefF plans store these keys directly
// (Dk, float32: k_dist's epilogue forms them, k_rf_select overwrites the
// refined ones); rf_key forms them from a float64 D (negative = exact key),
// the layout of the other plans.
__device__ __forceinline__ uint32_t rf_key(double d, double inv_sc) {
  return __float_as_uint(d < 0.0 ? (float)(-d) : (float)(d * inv_sc));
}

// One workgroup per focal row.  For each class c the k_c-th smallest key T_c
// is found digit by digit (a 10-bit LDS histogram right below the row's
// common key bits, then a ranked gather of the chosen bucket, or 8-bit
// passes when the bucket is big) -> tkey[i][c], and tneed[i][c] = how many
// keys equal to T_c belong to the k_c nearest (0 when the class is taken
// whole).  With x (continuous features), the candidates within the band of
// their class's T_c get the reference's exact keys in the kernel and T_c is
// re-selected among them (see the refinement below).  Every key < T_c (index
// order) and then the first tneed keys == T_c (index order) go to nbr (rows
// where more keys equal T_c than are needed are re-ordered the reference's
// way by k_rf_ties), and teq[i][c] counts the keys equal to T_c.
// The keys are ReliefF's float32 distances as the plan stores them (Dk:
// k_dist's epilogue writes them, this kernel the refined ones).  STAGE: the
// row and its class codes are staged in LDS (n <= 32768); else read from HBM
// on every sweep (256 threads per row).
// (Per-phase clock stamps of round 3's profiling build: DESIGN.md, Kernels.)
template <bool STAGE>
__global__ __launch_bounds__(1024) void k_rf_select(
    const float* __restrict__ Dk, int n, int64_t n_pad, const int32_t* __restrict__ lab,
    const uint8_t* __restrict__ lab8, const int64_t* __restrict__ class_count, int n_classes,
    int k, int64_t row0, uint32_t* __restrict__ tkey, int32_t* __restrict__ tneed,
    int32_t* __restrict__ teq, int32_t* __restrict__ nbr, int32_t* __restrict__ nfound,
    double band_abs, double band_rel, int fcap, unsigned long long* __restrict__ count,
    const float* __restrict__ x, int64_t p_in, int pc, int PC, int pd,
    const int64_t* __restrict__ src_col, const double* __restrict__ scl, int xlds) {
  // Dynamic LDS: hist[C][1024 (C <= 8) or 256]; STAGE: the row's keys and
  // class codes by quads of samples (16-byte aligned); xlds floats of exact-
  // key buffer after them.  Per-class state lives in static LDS.
  extern __shared__ __align__(16) uint32_t sh[];
  const int C = n_classes;
  const int nbins1 = C <= 8 ? 1024 : 256;
  const int nq = (n + 3) >> 2;
  uint32_t* hist = sh;
  uint32_t* keys = sh + C * nbins1;             // STAGE: [4 nq]
  uint8_t* labs = (uint8_t*)(keys + 4 * nq);    // STAGE: [4 nq]
  const int i = (int)(row0 + blockIdx.x);
  const int tid = threadIdx.x, nt = blockDim.x, nwaves = nt >> 6;
  const int wave = tid >> 6, lane = tid & 63;
  const int li = lab[i];
  float* __restrict__ rowk = const_cast<float*>(Dk) + (int64_t)i * n_pad;
  // the focal sample's own key and the padding after n read as kNone: above
  // every finite key, and (its bit 31 set) never equal to an active class's
  // prefix at any digit, so the sweeps need no index test
  constexpr uint32_t kNone = 0xFFFFFFFFu;
  __shared__ uint32_t prefix[64], need[64], pm[64], lcnt[64], bcount[64], gcnt[64];
  __shared__ uint2 kband[64];  // exact-key band per class: [klo, klo + kn)
  __shared__ uint8_t done[64];
  __shared__ uint32_t red_or[16], red_and[16], kor_s, kand_s;
  __shared__ int n_ex, nflag, any_big;

  // xbuf (exact keys of the listed candidates): [x_i | scales | columns |
  // candidate rows ...] at the continuous columns, pc floats each
  float* xbuf = nullptr;
  if (x != nullptr && xlds > 0) {
    const uintptr_t base = STAGE ? (uintptr_t)(labs + 4 * nq) : (uintptr_t)keys;
    xbuf = (float*)((base + 15) & ~(uintptr_t)15);
  }
  const int xb_rows = xbuf != nullptr && pc > 0 ? xlds / pc - 3 : 0;
  const bool xst = xb_rows >= 1;
  int* xcol = xst ? (int*)(xbuf + 2 * pc) : nullptr;
  const float* __restrict__ xi = x != nullptr ? x + (int64_t)i * p_in : nullptr;

  // Quad q (samples 4q..4q+3): keys and class codes
  auto load_quad = [&](int q, uint32_t (&kv)[4], uint32_t& lb) {
    if (STAGE) {
      const uint4 v = ((const uint4*)keys)[q];
      kv[0] = v.x, kv[1] = v.y, kv[2] = v.z, kv[3] = v.w;
      lb = ((const uint32_t*)labs)[q];
    } else {
      const float4 v = ((const float4*)rowk)[q];
      kv[0] = __float_as_uint(v.x), kv[1] = __float_as_uint(v.y);
      kv[2] = __float_as_uint(v.z), kv[3] = __float_as_uint(v.w);
      lb = ((const uint32_t*)lab8)[q];
#pragma unroll
      for (int e = 0; e < 4; e++)
        if (4 * q + e >= n || 4 * q + e == i) kv[e] = kNone;
    }
  };
  // Order-free sweep over the row, two quads per thread in flight: the
  // per-class value arr[c] of every sample is loaded before any test (the
  // sweeps are latency- and issue-bound: no per-sample branches or waits),
  // then fn(j, c, key, arr[c]).
  auto sweep = [&](const auto* arr, auto&& fn) {
    for (int q0 = tid; q0 < nq; q0 += 2 * nt) {
      const int q1 = q0 + nt < nq ? q0 + nt : nq - 1;
      uint32_t kv[2][4], lb[2];
      load_quad(q0, kv[0], lb[0]);
      load_quad(q1, kv[1], lb[1]);
      int cv[2][4];
      auto av = arr[0];
      decltype(av) pv[2][4];
#pragma unroll
      for (int h = 0; h < 2; h++)
#pragma unroll
        for (int e = 0; e < 4; e++) {
          cv[h][e] = (int)((lb[h] >> (8 * e)) & 0xFFu);
          pv[h][e] = arr[cv[h][e]];
        }
#pragma unroll
      for (int e = 0; e < 4; e++) fn(4 * q0 + e, cv[0][e], kv[0][e], pv[0][e]);
      if (q0 + nt < nq) {
#pragma unroll
        for (int e = 0; e < 4; e++) fn(4 * q1 + e, cv[1][e], kv[1][e], pv[1][e]);
      }
    }
  };

  // The reference's float32 key of pair (i, jj), wave-wide (every lane gets
  // it): k_exact_pairs<float>'s sum term by term in its order (lane l sums
  // columns l, l+64, ... in f64, then the discrete mismatches, then the
  // xor-shuffle tree); the unroll only batches the loads.
  auto exact_key = [&](int jj) -> double {
    const float* __restrict__ xj = x + (int64_t)jj * p_in;
    double acc = 0.0;
    constexpr int kUe = 8;
    for (int c0 = lane; c0 < pc; c0 += 64 * kUe) {
      int64_t col[kUe];
      float av[kUe], bv[kUe], sv[kUe];
#pragma unroll
      for (int u = 0; u < kUe; u++) {
        const int c = c0 + 64 * u < pc ? c0 + 64 * u : pc - 1;
        col[u] = src_col[c];
        sv[u] = (float)scl[c];
      }
#pragma unroll
      for (int u = 0; u < kUe; u++) {
        av[u] = xi[col[u]];
        bv[u] = xj[col[u]];
      }
#pragma unroll
      for (int u = 0; u < kUe; u++)
        if (c0 + 64 * u < pc) acc += (double)(__builtin_fabsf(av[u] - bv[u]) * sv[u]);
    }
    for (int c = PC + lane; c < PC + pd; c += 64) {
      const int64_t cl = src_col[c];
      acc += (xi[cl] != xj[cl]) ? 1.0 : 0.0;
    }
    for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
    return acc;
  };
  // stores pair (i, jj)'s exact key into the row (LDS or HBM); its bits
  auto store_key = [&](int jj, double acc) -> uint32_t {
    const uint32_t v = __float_as_uint((float)acc);  // acc >= 0: +0 at worst
    if (STAGE) keys[jj] = v;
    else rowk[jj] = (float)acc;
    return v;
  };

  // 1. The row.  Key range: bits above the highest bit in which two keys
  // differ are common to all of them, so the radix passes start below it (a
  // row's distances share their float exponent or nearly).  The exact-key
  // buffer's fixed rows (x_i, scales, columns) load under the row's read:
  // column indices first, the keys, then x_i at those columns.
  uint32_t kor = 0u, kand = 0xFFFFFFFFu;
  if (STAGE) {
    // one round trip: 8 quads per thread cover n <= 32768 (STAGE's range)
    constexpr int kQ = 8;
    int scol[2] = {0, 0};
    float ssc[2] = {0.0f, 0.0f}, sxi[2] = {0.0f, 0.0f};
    if (xst) {
#pragma unroll
      for (int s = 0; s < 2; s++) {
        const int c = tid + s * nt < pc ? tid + s * nt : pc - 1;
        scol[s] = (int)src_col[c];
        ssc[s] = (float)scl[c];
      }
    }
    uint4 kq[kQ];
    uint32_t lq[kQ];
#pragma unroll
    for (int u = 0; u < kQ; u++) {
      const int q = tid + u * nt < nq ? tid + u * nt : nq - 1;
      kq[u] = ((const uint4*)rowk)[q];
      lq[u] = ((const uint32_t*)lab8)[q];
    }
    if (xst) {
#pragma unroll
      for (int s = 0; s < 2; s++) sxi[s] = xi[scol[s]];
    }
#pragma unroll
    for (int u = 0; u < kQ; u++) {
      const int q = tid + u * nt;
      if (q >= nq) continue;
      uint32_t kv[4] = {kq[u].x, kq[u].y, kq[u].z, kq[u].w};
#pragma unroll
      for (int e = 0; e < 4; e++) {
        const int j = 4 * q + e;
        if (j >= n || j == i) {
          kv[e] = kNone;
        } else {
          kor |= kv[e];
          kand &= kv[e];
        }
      }
      ((uint4*)keys)[q] = make_uint4(kv[0], kv[1], kv[2], kv[3]);
      ((uint32_t*)labs)[q] = lq[u];
    }
    if (xst) {
#pragma unroll
      for (int s = 0; s < 2; s++) {
        const int c = tid + s * nt;
        if (c < pc) xbuf[c] = sxi[s], xbuf[pc + c] = ssc[s], xcol[c] = scol[s];
      }
    }
  } else {
    for (int q = tid; q < nq; q += nt) {
      uint32_t kv[4], lb;
      load_quad(q, kv, lb);
#pragma unroll
      for (int e = 0; e < 4; e++)
        if (kv[e] != kNone) kor |= kv[e], kand &= kv[e];
    }
  }
  if (xst) {  // the columns past 2 per thread
    for (int c = tid + (STAGE ? 2 * nt : 0); c < pc; c += nt) {
      const int col = (int)src_col[c];
      xbuf[c] = xi[col];
      xbuf[pc + c] = (float)scl[c];
      xcol[c] = col;
    }
  }
  for (int o = 32; o > 0; o >>= 1) {
    kor |= __shfl_xor(kor, o);
    kand &= __shfl_xor(kand, o);
  }
  if (lane == 0) red_or[wave] = kor, red_and[wave] = kand;
  __syncthreads();
  if (tid == 0) {
    uint32_t o = 0u, a = 0xFFFFFFFFu;
    for (int w = 0; w < nwaves; w++) o |= red_or[w], a &= red_and[w];
    kor_s = o, kand_s = a, n_ex = 0;
  }

  // 2. Selection.  x != null: round 0 selects on the quantised keys, the
  // candidates within the band of their class's k-th key get the reference's
  // keys (3.), and the exact k-th keys follow from them; round 1 (a second
  // selection over the row) only for rows with over fcap candidates.
  const int rounds = x != nullptr ? 2 : 1;
  for (int round = 0; round < rounds; round++) {
    __syncthreads();
    const uint32_t kor_r = kor_s, kand_r = kand_s;
    const uint32_t diff = kor_r & ~kand_r;  // bits that are not common
    const int top = diff ? 31 - __builtin_clz(diff) : 0;  // <= 30: keys are >= 0
    // pass 1 takes the WB bits [lo1, top] right below the common prefix;
    // 10-bit digits when the histograms fit (C <= 8), else 8
    const int wb = C <= 8 ? 10 : 8;
    const int lo1 = top - (wb - 1) > 0 ? top - (wb - 1) : 0;
    const uint32_t common = top >= 31 ? 0u : (kand_r & ~(0xFFFFFFFFu >> (31 - top)));
    for (int c = tid; c < C; c += nt) {
      const int64_t members = class_count[c] - (c == li ? 1 : 0);
      const int64_t kc = members < k ? members : k;
      // need = rank (1-based) of the wanted key inside the current bucket;
      // kc == members: take everything (T = kNone, nothing equal needed)
      prefix[c] = kc == members ? kNone : common;
      need[c] = kc == members ? 0u : (uint32_t)kc;
      done[c] = 0;
    }
    // One pass: histogram of the digit [lo, hi) of the keys whose bits >= hi
    // match their class's prefix, then per class (one wave each) the bucket
    // holding the need-th key, by a wave prefix sum over the bins.  done[c]:
    // class c's k-th key is final (the small-bucket gather leaves need[c] as
    // a rank among the keys EQUAL to it, which a further pass must not reuse).
    // pm[c]: the prefix to match, kNone for classes not in the pass.
    auto radix_pass = [&](int lo, int hi) {
      const int nbins = 1 << (hi - lo);
      const uint32_t dmask = (uint32_t)nbins - 1u;
      __syncthreads();
      for (int e = tid; e < C * nbins; e += nt) hist[e] = 0;
      for (int c = tid; c < C; c += nt) pm[c] = (need[c] != 0 && !done[c]) ? prefix[c] : kNone;
      __syncthreads();
      sweep(pm, [&](int, int c, uint32_t key, uint32_t P) {
        if ((key >> hi) == (P >> hi)) atomicAdd(&hist[c * nbins + ((key >> lo) & dmask)], 1u);
      });
      __syncthreads();
      const int bpl = (nbins + 63) >> 6;  // bins per lane
      for (int c = wave; c < C; c += nwaves) {
        const uint32_t nd = need[c];
        if (nd == 0 || done[c]) continue;
        const uint32_t* hc = hist + c * nbins;
        const int b0 = lane * bpl;
        // the lane's bins in registers (bpl <= 16), loaded together
        uint32_t hv[16], tot = 0u;
#pragma unroll
        for (int q = 0; q < 16; q++) {
          const int b = b0 + q < nbins ? b0 + q : nbins - 1;
          hv[q] = hc[b];
        }
#pragma unroll
        for (int q = 0; q < 16; q++) {
          if (q >= bpl || b0 + q >= nbins) hv[q] = 0u;
          tot += hv[q];
        }
        uint32_t incl = tot;
        for (int o = 1; o < 64; o <<= 1) {
          const uint32_t t = __shfl_up(incl, o);
          if (lane >= o) incl += t;
        }
        // the first lane whose inclusive sum reaches nd owns the bucket
        const uint64_t m = __ballot(incl >= nd);
        const int owner = (int)__builtin_ctzll(m);
        if (lane == owner) {
          uint32_t cum = incl - tot, bsel = (uint32_t)b0, bc = 0u;
          bool found = false;
#pragma unroll
          for (int q = 0; q < 16; q++) {
            if (!found && q < bpl) {
              if (q == bpl - 1 || cum + hv[q] >= nd) {
                found = true;
                bsel = (uint32_t)(b0 + q);
                bc = hv[q];
              } else {
                cum += hv[q];
              }
            }
          }
          prefix[c] |= bsel << lo;
          need[c] = nd - cum;
          bcount[c] = bc;
        }
      }
      __syncthreads();
    };
    radix_pass(lo1, top + 1);
    if (lo1 > 0) {
      // Small buckets (<= 64 keys: the common case, the k nearest sit in the
      // sparse low tail) finish in one gather: the bucket's keys go to a list
      // (in the histogram space, free now) and the need-th smallest is found
      // by ranking.  Classes with bigger buckets (ties, discrete data)
      // continue with 8-bit passes below lo1.
      uint32_t* list = hist;  // [class][64]
      if (tid == 0) any_big = 0;
      __syncthreads();
      for (int c = tid; c < C; c += nt) {
        gcnt[c] = 0u;
        if (need[c] != 0 && bcount[c] > 64u) any_big = 1;
        pm[c] = (need[c] != 0 && bcount[c] <= 64u) ? prefix[c] : kNone;
      }
      __syncthreads();
      sweep(pm, [&](int, int c, uint32_t key, uint32_t P) {
        if ((key >> lo1) == (P >> lo1)) {
          // (a class outside the gather can take the kNone keys: at most 4)
          const uint32_t slot = atomicAdd(&gcnt[c], 1u);
          if (slot < 64u) list[c * 64 + slot] = key;
        }
      });
      __syncthreads();
      for (int c = wave; c < C; c += nwaves) {
        const uint32_t nd = need[c], m = bcount[c];
        if (nd == 0 || m > 64u) continue;
        const uint32_t v = lane < (int)m ? list[c * 64 + lane] : kNone;
        uint32_t nlt = 0u, nle = 0u;
        for (uint32_t q = 0; q < m; q++) {
          const uint32_t w = list[c * 64 + q];
          nlt += w < v;
          nle += w <= v;
        }
        // the need-th smallest: nlt < nd <= nle (ties: one owner per value)
        const bool own = lane < (int)m && nlt < nd && nd <= nle;
        const uint64_t mo = __ballot(own);
        if (mo != 0ull && lane == (int)__builtin_ctzll(mo)) {
          prefix[c] = v;
          need[c] = nd - nlt;
          done[c] = 1;
        }
      }
      __syncthreads();
      if (any_big)
        for (int hi = lo1; hi > 0; hi -= 8) radix_pass(hi - 8 > 0 ? hi - 8 : 0, hi);
    }
    if (round + 1 >= rounds) break;

    // 3. Exact keys.  The band |key - T| <= band_abs + band_rel * T (in f64)
    // is, for float keys, an interval of key bits [klo, klo + kn): found per
    // class from the f64 bounds rounded to float, then stepped to the exact
    // edges (a step or two), so the sweep tests two integers.  Candidates go
    // to a list (j | class << 26); the keys of a class below the band are
    // counted (lcnt: they stay below the exact T).  The listed keys get the
    // reference's keys, spread over the waves, and the exact k-th key of
    // class c is the (kc - lcnt[c])-th smallest listed key of c.  More than
    // fcap candidates (ties, discrete-heavy rows): the general route, exact
    // keys in chunk order and a second selection over the row.
    constexpr int kFCap = 256;
    uint32_t* fl = hist;  // [kFCap] entries, [kFCap] exact keys
    for (int c = tid; c < C; c += nt) {
      lcnt[c] = 0u;
      uint2 kb = make_uint2(0u, 0u);
      if (need[c] != 0) {
        const uint32_t P = prefix[c];
        const double T = (double)__uint_as_float(P);
        const double B = band_abs + band_rel * T;
        auto in_band = [&](uint32_t f) { return fabs((double)__uint_as_float(f) - T) <= B; };
        const double lo_d = T - B, hi_d = T + B;
        uint32_t a = lo_d <= 0.0 ? 0u : __float_as_uint((float)lo_d);
        if (a > P) a = P;
        while (a > 0u && in_band(a - 1u)) a--;
        while (!in_band(a)) a++;
        uint32_t b = __float_as_uint((float)hi_d);
        if (b < P) b = P;
        if (b > 0x7F7FFFFFu) b = 0x7F7FFFFFu;
        while (b < 0x7F7FFFFFu && in_band(b + 1u)) b++;
        while (!in_band(b)) b--;
        kb = make_uint2(a, b - a + 1u);
      }
      kband[c] = kb;
    }
    if (tid == 0) nflag = 0;
    __syncthreads();
    sweep(kband, [&](int j, int c, uint32_t key, uint2 kb) {
      if (key - kb.x < kb.y) {
        const int slot = atomicAdd(&nflag, 1);
        if (slot < kFCap) fl[slot] = (uint32_t)j | ((uint32_t)c << 26);
      } else if (key < kb.x) {
        atomicAdd(&lcnt[c], 1u);
      }
    });
    __syncthreads();
    const int F = nflag;
    if (F == 0) break;  // nothing near any k-th key: round 0's keys are final
    if (F <= (fcap < kFCap ? fcap : kFCap)) {
      if (xst) {
        // batches of xb_rows candidates gathered at the staged columns
        for (int e0 = 0; e0 < F; e0 += xb_rows) {
          const int nb = F - e0 < xb_rows ? F - e0 : xb_rows;
          const int tot = nb * pc;
          for (int t0 = tid; t0 < tot; t0 += 4 * nt) {
            float v[4];
#pragma unroll
            for (int u = 0; u < 4; u++) {
              const int t = t0 + u * nt < tot ? t0 + u * nt : tot - 1;
              const int q = t / pc, c = t - q * pc;
              const int jr = (int)(fl[e0 + q] & ((1u << 26) - 1u));
              v[u] = x[(int64_t)jr * p_in + xcol[c]];
            }
#pragma unroll
            for (int u = 0; u < 4; u++)
              if (t0 + u * nt < tot) xbuf[3 * pc + t0 + u * nt] = v[u];
          }
          __syncthreads();
          for (int q = wave; q < nb; q += nwaves) {
            const int e = e0 + q;
            const int jj = (int)(fl[e] & ((1u << 26) - 1u));
            const float* xr = xbuf + (3 + q) * pc;
            double acc = 0.0;
            for (int c = lane; c < pc; c += 64)
              acc += (double)(__builtin_fabsf(xbuf[c] - xr[c]) * xbuf[pc + c]);
            for (int c = PC + lane; c < PC + pd; c += 64) {
              const int64_t cl = src_col[c];
              acc += (xi[cl] != x[(int64_t)jj * p_in + cl]) ? 1.0 : 0.0;
            }
            for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
            if (lane == 0) fl[kFCap + e] = store_key(jj, acc);
          }
          __syncthreads();
        }
      } else {
        for (int e = wave; e < F; e += nwaves) {
          const int jj = (int)(fl[e] & ((1u << 26) - 1u));
          const double acc = exact_key(jj);
          if (lane == 0) fl[kFCap + e] = store_key(jj, acc);
        }
        __syncthreads();
      }
      for (int c = wave; c < C; c += nwaves) {
        if (need[c] == 0) continue;
        const int64_t members = class_count[c] - (c == li ? 1 : 0);
        const uint32_t kc = (uint32_t)(members < k ? members : k);
        const uint32_t r = kc - lcnt[c];  // 1-based rank among c's listed keys
        for (int e0 = 0; e0 < F; e0 += 64) {
          const int e = e0 + lane;
          bool own = false;
          uint32_t v = 0u, nlt = 0u, nle = 0u;
          if (e < F && (int)(fl[e] >> 26) == c) {
            v = fl[kFCap + e];
            for (int q = 0; q < F; q++) {
              if ((int)(fl[q] >> 26) != c) continue;
              const uint32_t w = fl[kFCap + q];
              nlt += w < v;
              nle += w <= v;
            }
            own = nlt < r && r <= nle;
          }
          const uint64_t mo = __ballot(own);
          if (mo != 0ull) {
            if (lane == (int)__builtin_ctzll(mo)) {
              prefix[c] = v;
              need[c] = r - nlt;
            }
            break;
          }
        }
      }
      if (tid == 0) n_ex = F;
      __syncthreads();
      break;
    }
    // general route: every candidate of a wave's chunk, in ballot order
    const int chunk_e = (n + nwaves - 1) / nwaves;
    const int jb_e = wave * chunk_e, je_e = jb_e + chunk_e < n ? jb_e + chunk_e : n;
    int n_local = 0;
    for (int j0 = jb_e; j0 < je_e; j0 += 64) {
      const int j = j0 + lane;
      bool flag = false;
      if (j < je_e && j != i) {
        const int c = STAGE ? (int)labs[j] : (int)lab8[j];
        const uint32_t key = STAGE ? keys[j] : __float_as_uint(rowk[j]);
        const uint2 kb = kband[c];
        flag = key - kb.x < kb.y;
      }
      uint64_t m = __ballot(flag);
      while (m != 0ull) {
        const int jj = j0 + __builtin_ctzll(m);
        m &= m - 1ull;
        const double acc = exact_key(jj);
        if (lane == 0) {
          const uint32_t v = store_key(jj, acc);
          atomicOr(&kor_s, v);
          atomicAnd(&kand_s, v);
        }
        n_local++;
      }
    }
    if (lane == 0 && n_local != 0) atomicAdd(&n_ex, n_local);
    __threadfence_block();
  }  // rounds
  __syncthreads();
  if (tid == 0 && count != nullptr && n_ex != 0) atomicAdd(count, (unsigned long long)n_ex);
  for (int c = tid; c < C; c += nt) {
    tkey[(int64_t)i * C + c] = prefix[c];
    tneed[(int64_t)i * C + c] = (int32_t)need[c];
  }

  // 4. Ordered collection over all waves: wave w takes the contiguous chunk
  // [j_w, j_w+1) of the row.  Pass 1 counts, per class, the keys below the
  // k-th key T and the keys equal to it in the chunk, and lists them (j
  // order, by ballot compaction) in the wave's slice of the histogram space;
  // a scan over the waves turns the counts into each wave's output offsets
  // and the number of equal keys before its chunk (only the first need[c]
  // equal keys in j order are taken, as the reference's stable order among
  // ties at this stage).  Pass 2 writes from the lists, or sweeps the chunk
  // again when a list overflowed (ties).  Groups of 4 x 64 keys with no key
  // <= T of its class (nearly all: k per class in a row of n) are skipped
  // on one ballot.  Per-wave counters [wave][class] and the lists reuse the
  // histogram space.
  uint32_t* cnt_lt = hist;
  uint32_t* cnt_eq = hist + 16 * C;
  uint32_t* off_lt = hist + 32 * C;
  uint32_t* off_eq = hist + 48 * C;
  const int lcap = (C * nbins1 - 64 * C) / 16;  // list entries per wave (>= 60)
  uint32_t* wl = hist + 64 * C + wave * lcap;
  __shared__ int ovf;
  const int chunk = (n + nwaves - 1) / nwaves;
  const int jb = wave * chunk, je = jb + chunk < n ? jb + chunk : n;
  const uint64_t below = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  for (int c = lane; c < C; c += 64) cnt_lt[wave * C + c] = cnt_eq[wave * C + c] = 0u;
  if (tid == 0) ovf = 0;
  __syncthreads();
  constexpr int kCU = 4;
  auto classify = [&](int j0, int (&cv)[kCU], bool (&lt)[kCU], bool (&eq)[kCU]) -> bool {
    uint32_t kv[kCU], tv[kCU];
#pragma unroll
    for (int u = 0; u < kCU; u++) {
      const int j = j0 + 64 * u + lane;
      const int jc = j < je ? j : je - 1;  // unconditional loads
      cv[u] = STAGE ? (int)labs[jc] : (int)lab8[jc];
      kv[u] = STAGE ? keys[jc] : __float_as_uint(rowk[jc]);
    }
#pragma unroll
    for (int u = 0; u < kCU; u++) tv[u] = prefix[cv[u]];
    bool any = false;
#pragma unroll
    for (int u = 0; u < kCU; u++) {
      const int j = j0 + 64 * u + lane;
      const bool ok = j < je && j != i;
      lt[u] = ok && kv[u] < tv[u];
      eq[u] = ok && kv[u] == tv[u];
      any |= lt[u] | eq[u];
    }
    return __ballot(any) != 0ull;
  };
  // the classes present among the wave's flagged lanes (bit c), wave-wide
  auto classes_of = [&](bool f, int c) {
    uint64_t cm = f ? (1ull << c) : 0ull;
    for (int o = 32; o > 0; o >>= 1) cm |= __shfl_xor(cm, o);
    return cm;
  };
  // pass-1 counts of one batch of 64 keys (lane 0 keeps the wave's counters)
  auto tally = [&](bool l, bool e, int c) {
    for (uint64_t cm = classes_of(l || e, c); cm != 0ull; cm &= cm - 1ull) {
      const int cc = __builtin_ctzll(cm);
      const uint32_t nl = (uint32_t)__popcll(__ballot(l && c == cc));
      const uint32_t ne = (uint32_t)__popcll(__ballot(e && c == cc));
      if (lane == 0) cnt_lt[wave * C + cc] += nl, cnt_eq[wave * C + cc] += ne;
    }
  };
  // pass-2 writes of one batch of 64 keys in j order (running slots in
  // off_lt / off_eq, lane 0 advances them)
  auto emit = [&](bool l, bool e, int c, int j) {
    for (uint64_t cm = classes_of(l || e, c); cm != 0ull; cm &= cm - 1ull) {
      const int cc = __builtin_ctzll(cm);
      const bool lc = l && c == cc, ec = e && c == cc;
      const uint64_t mlt = __ballot(lc), meq = __ballot(ec);
      const uint32_t rl = off_lt[wave * C + cc], re = off_eq[wave * C + cc];
      int32_t* out = nbr + ((int64_t)i * C + cc) * k;
      if (lc) out[rl + __popcll(mlt & below)] = j;
      if (ec) {
        const uint32_t r = re + (uint32_t)__popcll(meq & below);
        if (r < need[cc]) out[cnt_lt[cc] + r] = j;
      }
      if (lane == 0) {
        off_lt[wave * C + cc] = rl + (uint32_t)__popcll(mlt);
        off_eq[wave * C + cc] = re + (uint32_t)__popcll(meq);
      }
    }
  };
  int nlist = 0;  // wave-uniform
  for (int j0 = jb; j0 < je; j0 += 64 * kCU) {
    int cv[kCU];
    bool lt[kCU], eq[kCU];
    if (!classify(j0, cv, lt, eq)) continue;
#pragma unroll
    for (int u = 0; u < kCU; u++) {
      const bool h = lt[u] || eq[u];
      const uint64_t mh = __ballot(h);
      if (mh == 0ull) continue;
      tally(lt[u], eq[u], cv[u]);
      const int slot = nlist + (int)__popcll(mh & below);
      if (h && slot < lcap)
        wl[slot] = (uint32_t)(j0 + 64 * u + lane) | (eq[u] ? 1u << 25 : 0u) |
                   ((uint32_t)cv[u] << 26);
      nlist += (int)__popcll(mh);
    }
  }
  if (lane == 0 && nlist > lcap) ovf = 1;
  __syncthreads();
  // exclusive scans over the waves, per class (one thread per class)
  for (int c = tid; c < C; c += nt) {
    uint32_t a = 0u, b = 0u;
    for (int w = 0; w < nwaves; w++) {
      const uint32_t ca = cnt_lt[w * C + c], cb = cnt_eq[w * C + c];
      off_lt[w * C + c] = a;
      off_eq[w * C + c] = b;
      a += ca;
      b += cb;
    }
    // every key below T is taken; the first need[c] equal keys follow them
    const uint32_t take_eq = b < need[c] ? b : need[c];
    nfound[(int64_t)i * C + c] = (int32_t)(a + take_eq);
    teq[(int64_t)i * C + c] = (int32_t)b;
    cnt_lt[c] = a;  // total below T (base of the equal keys' slots)
  }
  __syncthreads();
  // pass 2: write.  Keys below T keep j order among themselves; equal keys
  // (in j order) follow.
  if (!ovf) {
    for (int e0 = 0; e0 < nlist; e0 += 64) {
      const int e = e0 + lane;
      const uint32_t ent = e < nlist ? wl[e] : 0u;
      const bool iseq = (ent >> 25) & 1u;
      emit(e < nlist && !iseq, e < nlist && iseq, (int)(ent >> 26), (int)(ent & ((1u << 25) - 1u)));
    }
  } else {
    for (int j0 = jb; j0 < je; j0 += 64 * kCU) {
      int cv[kCU];
      bool lt[kCU], eq[kCU];
      if (!classify(j0, cv, lt, eq)) continue;
#pragma unroll
      for (int u = 0; u < kCU; u++) emit(lt[u], eq[u], cv[u], j0 + 64 * u + lane);
    }
  }
}

// Exact reference keys of whole rows (tie rows of a problem with continuous
// features): grid (tie rows, ceil(n / 4)), one wave per (row, j).  With no
// continuous features the quantised keys are already exact and are copied.
template <typename T>
__global__ __launch_bounds__(256) void k_rf_exact_rows(
    const T* __restrict__ x, int64_t n, int64_t p_in, int64_t pc, int64_t PC, int64_t pd,
    const int64_t* __restrict__ src_col, const double* __restrict__ scl,
    const int32_t* __restrict__ rows, const double* __restrict__ D,
    const float* __restrict__ Dk, int64_t n_pad, double inv_sc, float* __restrict__ keys) {
  const int lane = threadIdx.x & 63;
  const int64_t r = blockIdx.x;
  const int64_t i = rows[r];
  const int64_t j = (int64_t)blockIdx.y * 4 + (threadIdx.x >> 6);
  if (j >= n) return;
  float kv;
  if (pc == 0) {
    kv = Dk != nullptr ? Dk[i * n_pad + j] : __uint_as_float(rf_key(D[i * n_pad + j], inv_sc));
  } else {
    const T* xi = x + i * p_in;
    const T* xj = x + j * p_in;
    double acc = 0.0;
    for (int64_t c = lane; c < pc; c += 64) {
      const int64_t col = src_col[c];
      acc += (double)(__builtin_fabsf((float)xi[col] - (float)xj[col]) * (float)scl[c]);
    }
    for (int64_t c = PC + lane; c < PC + pd; c += 64) {
      const int64_t col = src_col[c];
      acc += (xi[col] != xj[col]) ? 1.0 : 0.0;
    }
    for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
    kv = (float)acc;
  }
  if (lane == 0) keys[r * n + j] = (j == i) ? __builtin_inff() : kv;
}

// Rows where more neighbours share a class's k-th distance than are needed:
// replay numba's quicksort over the row's exact keys (numba_argsort_focus)
// and take the tied neighbours in its order (ReliefF.py:157-175).  One
// workgroup (one wave) per row: the lanes stage the row into LDS when it fits
// (8 bytes per sample, n <= 20480) and lane 0 runs the sequential sort there;
// larger rows sort in their global scratch.
constexpr int64_t kTieLdsMaxN = 20480;

// numba_argsort_focus (fs_internal.h) for one wave: same ranges, pivots,
// swaps and result, but each Hoare partition is computed from its stop lists
// instead of element by element.  In numba's loop the m-th swap exchanges
// the m-th "left stop" (ascending position with key >= pivot) with the m-th
// "right stop" (descending position with key <= pivot) of the untouched
// window between the previous pair, and the loop ends at the first m where
// that left stop is not below that right stop; the pivot then goes to the
// m-th left stop, or to the previous right stop when the window has none
// (that position now holds a swapped element >= pivot), or to `high` when no
// swap happened.  A round collects up to 64 stops per side with ballots and
// performs up to 64 swaps at once.  All lanes run the control flow in
// lockstep; bufL/bufR are 64-entry LDS scratch.
template <typename KeyFn>
__device__ int wave_argsort_focus(int64_t len, int32_t* R, KeyFn key, int32_t* bufL,
                                  int32_t* bufR) {
  const int lane = threadIdx.x & 63;
  const uint64_t below = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  auto has_interest = [&](int64_t lo, int64_t hi) {
    for (int64_t t0 = lo; t0 <= hi; t0 += 64) {
      const int64_t t = t0 + lane;
      if (__ballot(t <= hi && R[t] < 0) != 0ull) return true;
    }
    return false;
  };
  // up to 64 stops of one side inside [a, b], in scan order, into buf;
  // returns how many
  auto collect = [&](int64_t a, int64_t b, float pivot, bool left, int32_t* buf) {
    int cnt = 0;
    for (int64_t c0 = 0; cnt < 64 && c0 <= b - a; c0 += 64) {
      const int64_t t = left ? a + c0 + lane : b - c0 - lane;
      bool stop = false;
      if (left ? t <= b : t >= a) {
        const float kv = key(R[t]);
        stop = left ? !(kv < pivot) : !(pivot < kv);
      }
      const uint64_t m = __ballot(stop);
      const int rank = cnt + __popcll(m & below);
      if (stop && rank < 64) buf[rank] = (int32_t)t;
      cnt += __popcll(m);
    }
    __syncthreads();
    return cnt < 64 ? cnt : 64;
  };
  if (len < 2) return 0;
  constexpr int kSmall = 15, kMaxStack = 100;
  __shared__ int64_t st_lo[kMaxStack], st_hi[kMaxStack];
  int ns = 1;
  st_lo[0] = 0;
  st_hi[0] = len - 1;
  __syncthreads();
  while (ns > 0) {
    ns--;
    int64_t low = st_lo[ns], high = st_hi[ns];
    bool live = true;
    while (high - low >= kSmall) {
      const int64_t mid = (low + high) >> 1;
      // median of three and pivot stash: identical on every lane, one writer
      int32_t rl = R[low], rm = R[mid], rh = R[high], tmp;
      if (key(rm) < key(rl)) { tmp = rl; rl = rm; rm = tmp; }
      if (key(rh) < key(rm)) { tmp = rh; rh = rm; rm = tmp; }
      if (key(rm) < key(rl)) { tmp = rl; rl = rm; rm = tmp; }
      const float pivot = key(rm);
      __syncthreads();
      if (lane == 0) {
        R[low] = rl;
        R[mid] = rh;   // stash: R[high] <-> R[mid]
        R[high] = rm;
      }
      __syncthreads();
      // partition [low, high - 1] around pivot
      int64_t a = low, b = high - 1, jprev = high, ifinal = -1;
      while (ifinal < 0) {
        const int cl = collect(a, b, pivot, true, bufL);
        const int cr = collect(a, b, pivot, false, bufR);
        const int64_t Lm = lane < cl ? bufL[lane] : INT64_MAX;
        const int64_t Rm = lane < cr ? bufR[lane] : -1;
        const uint64_t fail = __ballot(!(Lm < Rm));
        const int f = fail ? (int)__builtin_ctzll(fail) : 64;
        // swaps m < f, all positions distinct: read, then write
        int32_t vl = 0, vr = 0;
        if (lane < f) { vl = R[Lm]; vr = R[Rm]; }
        __syncthreads();
        if (lane < f) { R[Lm] = vr; R[Rm] = vl; }
        __syncthreads();
        if (f < 64) {
          const int64_t jlast = f > 0 ? (int64_t)bufR[f - 1] : jprev;
          ifinal = f < cl ? (int64_t)bufL[f] : jlast;
          if (ifinal > jlast) ifinal = jlast;
        } else {
          a = (int64_t)bufL[63] + 1;
          b = (int64_t)bufR[63] - 1;
          jprev = bufR[63];
        }
        __syncthreads();
      }
      const int64_t i = ifinal;
      {
        const int32_t ri = R[i], rh2 = R[high];
        __syncthreads();
        if (lane == 0) { R[i] = rh2; R[high] = ri; }
        __syncthreads();
      }
      int64_t push_lo, push_hi, keep_lo, keep_hi;
      if (high - i > i - low) {
        push_lo = i + 1; push_hi = high; keep_lo = low; keep_hi = i - 1;
      } else {
        push_lo = low; push_hi = i - 1; keep_lo = i + 1; keep_hi = high;
      }
      if (push_hi >= push_lo && has_interest(push_lo, push_hi)) {
        if (ns >= kMaxStack) return -1;
        __syncthreads();
        if (lane == 0) { st_lo[ns] = push_lo; st_hi[ns] = push_hi; }
        __syncthreads();
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
    if (lane == 0) {  // insertion sort [low, high]
      for (int64_t i = low + 1; i <= high; i++) {
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
    __syncthreads();
  }
  return 0;
}

// Tie rows with n <= kTieMwMaxN: one 1024-thread workgroup per row, the
// row's exact keys (float32) and its permutation (16-bit handles: sample
// index | 0x8000 for a tied candidate) in LDS, 6 bytes per sample.  The
// quicksort replay is numba_argsort_focus's, run by 16 waves at once: the
// sub-ranges a partition leaves are disjoint, so the order in which they are
// processed does not change the result.  A wave pops a range from a shared
// queue, partitions it as wave_argsort_focus does (ballot-collected stops,
// up to 64 swaps per step), pushes the larger side when it holds a tied
// candidate and keeps partitioning the smaller, then insertion-sorts it;
// idle waves wait on the queue until it is empty and no wave is busy.
constexpr int64_t kTieMwMaxN = 25000;  // 6 B per sample + 12 KB static LDS
constexpr int kTieQ = 512;

__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

__global__ __launch_bounds__(1024) void k_rf_ties_mw(
    const int32_t* __restrict__ rows, int n, const float* __restrict__ keys_all,
    const float* __restrict__ Dk, int64_t n_pad, const int32_t* __restrict__ lab, int n_classes, int k, const uint32_t* __restrict__ tkey,
    const int32_t* __restrict__ tneed, const int32_t* __restrict__ teq,
    int32_t* __restrict__ nbr, int32_t* __restrict__ scr_all, int coop_min,
    int* __restrict__ status) {
  extern __shared__ __align__(16) uint32_t tie_lds[];
  float* key = (float*)tie_lds;                 // [n] by sample index
  uint16_t* R = (uint16_t*)(key + n);           // [n] the permutation
  __shared__ int q_lo[kTieQ], q_hi[kTieQ];
  __shared__ int q_n, q_busy, q_lock, q_err;
  __shared__ int32_t bufL_all[16][64], bufR_all[16][64];
  const int tid = threadIdx.x, nt = blockDim.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int64_t r = blockIdx.x;
  const int i = rows[r];
  // keys_all: the row's exact keys (k_rf_exact_rows); null: no continuous
  // features, the plan's keys are exact already (the row of Dk)
  const float* kg = keys_all != nullptr ? keys_all + r * n : Dk + (int64_t)i * n_pad;
  const uint32_t* Ti = tkey + (int64_t)i * n_classes;
  const int32_t* need = tneed + (int64_t)i * n_classes;
  const int32_t* eq = teq + (int64_t)i * n_classes;
  for (int j = tid; j < n; j += nt) {
    const float kv = (keys_all == nullptr && j == i) ? __builtin_inff() : kg[j];
    const int c = lab[j];
    key[j] = kv;
    const bool t = j != i && eq[c] > need[c] && __float_as_uint(kv) == Ti[c];
    R[j] = (uint16_t)(j | (t ? 0x8000 : 0));
  }
  // Ranges of at least coop_min samples are partitioned by the whole
  // workgroup first (the top of the tree, where one wave would work alone):
  // the m-th swap of numba's Hoare loop exchanges the m-th left stop
  // (ascending, key >= pivot, `high` included) with the m-th right stop
  // (descending, key <= pivot), and the loop ends at the first m whose left
  // stop has at most m right stops after it; the pivot then goes to
  // min(L_f, R_{f-1}) (R_{-1} = high).  Stops are ranked by a block scan,
  // the right stops' positions pass through `scr` (global, per row), and
  // every swap is done by its left stop's thread.  Smaller ranges go to the
  // per-wave queue below.
  __shared__ int big_lo[64], big_hi[64], big_n;
  __shared__ int sc_a[16], sc_b[16], s_f, s_lf, s_rprev;
  __shared__ float s_pivot;
  int32_t* scr = scr_all + r * n;
  if (tid == 0) {
    q_n = 0;
    big_n = 0;
    if (n >= 2) {
      if (n >= coop_min) big_lo[0] = 0, big_hi[0] = n - 1, big_n = 1;
      else q_lo[0] = 0, q_hi[0] = n - 1, q_n = 1;
    }
    q_busy = 0;
    q_lock = 0;
    q_err = 0;
  }
  __syncthreads();
  {
    auto key_h = [&](uint32_t h) { return key[h & 0x7FFFu]; };
    // exclusive block scan of (a, b) in thread order, and the totals
    auto block_scan2 = [&](int a, int b, int& ea, int& eb, int& ta, int& tb) {
      int ia = a, ib = b;
      for (int o = 1; o < 64; o <<= 1) {
        const int xa = __shfl_up(ia, o), xb = __shfl_up(ib, o);
        if (lane >= o) ia += xa, ib += xb;
      }
      if (lane == 63) sc_a[wave] = ia, sc_b[wave] = ib;
      __syncthreads();
      int pa = 0, pb = 0, sa = 0, sb = 0;
      for (int w = 0; w < (nt >> 6); w++) {
        const int va = sc_a[w], vb = sc_b[w];
        if (w < wave) pa += va, pb += vb;
        sa += va;
        sb += vb;
      }
      ea = pa + ia - a;
      eb = pb + ib - b;
      ta = sa;
      tb = sb;
      __syncthreads();
    };
    while (true) {
      const int nb = big_n;
      if (nb == 0) break;
      const int low = big_lo[nb - 1], high = big_hi[nb - 1];
      const int mid = (low + high) >> 1;
      __syncthreads();
      if (tid == 0) {
        big_n = nb - 1;
        s_f = INT32_MAX;
        // median of three and pivot stash (numba_argsort_focus)
        uint32_t rl = R[low], rm = R[mid], rh = R[high], tmp;
        if (key_h(rm) < key_h(rl)) { tmp = rl; rl = rm; rm = tmp; }
        if (key_h(rh) < key_h(rm)) { tmp = rh; rh = rm; rm = tmp; }
        if (key_h(rm) < key_h(rl)) { tmp = rl; rl = rm; rm = tmp; }
        R[low] = (uint16_t)rl;
        R[mid] = (uint16_t)rh;
        R[high] = (uint16_t)rm;
        s_pivot = key_h(rm);
      }
      __syncthreads();
      const float pivot = s_pivot;
      const int seg = (high - low + nt) / nt;  // <= 32: n <= kTieMwMaxN
      const int s0 = low + tid * seg;
      uint32_t mL = 0u, mR = 0u;
      for (int u = 0; u < seg; u++) {
        const int q = s0 + u;
        if (q > high) break;
        const float kv = key_h(R[q]);
        if (!(kv < pivot)) mL |= 1u << u;
        if (q < high && !(pivot < kv)) mR |= 1u << u;
      }
      int eL, eR, TL, TR;
      block_scan2(__popc(mL), __popc(mR), eL, eR, TL, TR);
      (void)TL;
      // the crossing f: the first left stop (rank m) with after <= m
      for (uint32_t w = mL; w != 0u;) {
        const int u = __builtin_ctz(w);
        w &= w - 1u;
        const int rank = eL + __popc(mL & ((1u << u) - 1u));
        const uint32_t upto = u >= 31 ? 0xFFFFFFFFu : ((2u << u) - 1u);
        const int after = TR - (eR + __popc(mR & upto));
        if (after <= rank) {
          atomicMin(&s_f, rank);
          break;
        }
      }
      __syncthreads();
      const int f = s_f;
      for (uint32_t w = mL; w != 0u;) {
        const int u = __builtin_ctz(w);
        w &= w - 1u;
        if (eL + __popc(mL & ((1u << u) - 1u)) == f) s_lf = s0 + u;
      }
      for (uint32_t w = mR; w != 0u;) {
        const int u = __builtin_ctz(w);
        w &= w - 1u;
        const int d = TR - 1 - (eR + __popc(mR & ((1u << u) - 1u)));
        if (d < f) scr[d] = s0 + u;
        if (d == f - 1) s_rprev = s0 + u;
      }
      __syncthreads();
      for (uint32_t w = mL; w != 0u;) {
        const int u = __builtin_ctz(w);
        w &= w - 1u;
        const int rank = eL + __popc(mL & ((1u << u) - 1u));
        if (rank < f) {
          const int q = s0 + u, q2 = scr[rank];
          const uint16_t a = R[q];
          R[q] = R[q2];
          R[q2] = a;
        }
      }
      __syncthreads();
      const int ip = f > 0 ? (s_lf < s_rprev ? s_lf : s_rprev) : s_lf;
      if (tid == 0) {
        const uint16_t a = R[ip];
        R[ip] = R[high];
        R[high] = a;
      }
      __syncthreads();
      // the two sides: with a tied candidate, back to the big list or to
      // the queue
#pragma unroll
      for (int side = 0; side < 2; side++) {
        const int a = side ? ip + 1 : low, b = side ? high : ip - 1;
        if (b < a) continue;
        const int sg = (b - a + nt) / nt;
        bool any = false;
        for (int u = 0; u < sg; u++) {
          const int q = a + tid * sg + u;
          if (q <= b && (R[q] & 0x8000u)) any = true;
        }
        if (__syncthreads_or(any) && tid == 0) {
          if (b - a + 1 >= coop_min && big_n < 64) {
            big_lo[big_n] = a, big_hi[big_n] = b, big_n++;
          } else if (q_n < kTieQ) {
            q_lo[q_n] = a, q_hi[q_n] = b, q_n++;
          } else {
            q_err = 1;
          }
        }
      }
      __syncthreads();
    }
  }
  {
    int32_t* bufL = bufL_all[wave];
    int32_t* bufR = bufR_all[wave];
    const uint64_t below = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    auto key_h = [&](uint32_t h) { return key[h & 0x7FFFu]; };
    auto lock = [&]() {  // lane 0 only
      while (atomicCAS(&q_lock, 0, 1) != 0) __builtin_amdgcn_s_sleep(2);
      __threadfence_block();
    };
    auto unlock = [&]() {
      __threadfence_block();
      atomicExch(&q_lock, 0);
    };
    auto has_interest = [&](int lo, int hi) {
      for (int t0 = lo; t0 <= hi; t0 += 64) {
        const int t = t0 + lane;
        if (__ballot(t <= hi && (R[t] & 0x8000u)) != 0ull) return true;
      }
      return false;
    };
    // up to 64 stops of one side inside [a, b], in scan order, into buf
    auto collect = [&](int a, int b, float pivot, bool left, int32_t* buf) {
      int cnt = 0;
      for (int c0 = 0; cnt < 64 && c0 <= b - a; c0 += 64) {
        const int t = left ? a + c0 + lane : b - c0 - lane;
        bool stop = false;
        if (left ? t <= b : t >= a) {
          const float kv = key_h(R[t]);
          stop = left ? !(kv < pivot) : !(pivot < kv);
        }
        const uint64_t m = __ballot(stop);
        const int rank = cnt + __popcll(m & below);
        if (stop && rank < 64) buf[rank] = t;
        cnt += __popcll(m);
      }
      wave_sync();
      return cnt < 64 ? cnt : 64;
    };
    auto push = [&](int lo, int hi) {
      if (lane == 0) {
        lock();
        if (q_n < kTieQ) {
          q_lo[q_n] = lo;
          q_hi[q_n] = hi;
          q_n++;
        } else {
          q_err = 1;  // queue overflow
        }
        unlock();
      }
      wave_sync();
    };
    constexpr int kSmall = 15;
    // numba's partition loop from [low, high], keeping the smaller side
    auto chain = [&](int low, int high) {
      while (high - low >= kSmall) {
        const int mid = (low + high) >> 1;
        // median of three and pivot stash: identical on every lane, one writer
        uint32_t rl = R[low], rm = R[mid], rh = R[high], tmp;
        if (key_h(rm) < key_h(rl)) { tmp = rl; rl = rm; rm = tmp; }
        if (key_h(rh) < key_h(rm)) { tmp = rh; rh = rm; rm = tmp; }
        if (key_h(rm) < key_h(rl)) { tmp = rl; rl = rm; rm = tmp; }
        const float pivot = key_h(rm);
        wave_sync();
        if (lane == 0) {
          R[low] = (uint16_t)rl;
          R[mid] = (uint16_t)rh;  // stash: R[high] <-> R[mid]
          R[high] = (uint16_t)rm;
        }
        wave_sync();
        // partition [low, high - 1] around pivot
        int a = low, b = high - 1, jprev = high, ifinal = -1;
        while (ifinal < 0) {
          const int cl = collect(a, b, pivot, true, bufL);
          const int cr = collect(a, b, pivot, false, bufR);
          const int Lm = lane < cl ? bufL[lane] : INT32_MAX;
          const int Rm = lane < cr ? bufR[lane] : -1;
          const uint64_t fail = __ballot(!(Lm < Rm));
          const int f = fail ? (int)__builtin_ctzll(fail) : 64;
          // swaps m < f, all positions distinct: read, then write
          uint16_t vl = 0, vr = 0;
          if (lane < f) { vl = R[Lm]; vr = R[Rm]; }
          wave_sync();
          if (lane < f) { R[Lm] = vr; R[Rm] = vl; }
          wave_sync();
          if (f < 64) {
            const int jlast = f > 0 ? bufR[f - 1] : jprev;
            ifinal = f < cl ? bufL[f] : jlast;
            if (ifinal > jlast) ifinal = jlast;
          } else {
            a = bufL[63] + 1;
            b = bufR[63] - 1;
            jprev = bufR[63];
          }
          wave_sync();
        }
        const int ip = ifinal;
        {
          const uint16_t ri = R[ip], rh2 = R[high];
          wave_sync();
          if (lane == 0) { R[ip] = rh2; R[high] = ri; }
          wave_sync();
        }
        int push_lo, push_hi, keep_lo, keep_hi;
        if (high - ip > ip - low) {
          push_lo = ip + 1; push_hi = high; keep_lo = low; keep_hi = ip - 1;
        } else {
          push_lo = low; push_hi = ip - 1; keep_lo = ip + 1; keep_hi = high;
        }
        if (push_hi >= push_lo && has_interest(push_lo, push_hi)) push(push_lo, push_hi);
        low = keep_lo;
        high = keep_hi;
        if (high < low || !has_interest(low, high)) return;
      }
      if (lane == 0) {  // insertion sort [low, high]
        for (int ii = low + 1; ii <= high; ii++) {
          const uint16_t kk = R[ii];
          const float v = key_h(kk);
          int j = ii;
          while (j > low && v < key_h(R[j - 1])) {
            R[j] = R[j - 1];
            j--;
          }
          R[j] = kk;
        }
      }
      wave_sync();
    };
    // the work queue; a wave waiting more than 2^22 naps (~2 s) gives up
    // (idle waves poll without the lock and take it only to pop or to
    // confirm the end: pollers holding it would starve the busy waves'
    // pushes)
    int spins = 0;
    while (true) {
      int st = 1, lo = 0, hi = 0;
      if (lane == 0) {
        const int qn = *(volatile int*)&q_n, qb = *(volatile int*)&q_busy;
        if (*(volatile int*)&q_err) {
          st = 2;
        } else if (qn > 0 || qb == 0) {
          lock();
          if (q_err) {
            st = 2;
          } else if (q_n > 0) {
            q_n--;
            lo = q_lo[q_n];
            hi = q_hi[q_n];
            q_busy++;
            st = 0;
          } else if (q_busy == 0) {
            st = 2;
          }
          unlock();
        }
      }
      st = __shfl(st, 0);
      lo = __shfl(lo, 0);
      hi = __shfl(hi, 0);
      if (st == 2) break;
      if (st == 1) {
        if (++spins > (1 << 22)) {
          if (lane == 0) atomicExch(&q_err, 2 + (q_busy << 8) + (q_n << 20));  // wait timeout
          break;
        }
        __builtin_amdgcn_s_sleep(8);
        continue;
      }
      chain(lo, hi);
      if (lane == 0) {
        lock();
        q_busy--;
        unlock();
      }
    }
  }
  __syncthreads();
  if (q_err) {
    if (tid == 0) atomicExch(status, q_err);
    return;
  }
  if (wave != 0) return;
  const uint64_t below = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  for (int c = 0; c < n_classes; c++) {
    if (!(eq[c] > need[c])) continue;
    int32_t* out = nbr + ((int64_t)i * n_classes + c) * k;
    const float T = __uint_as_float(Ti[c]);
    int cnt = 0;
    // every key < T of class c, in index order
    for (int j0 = 0; j0 < n; j0 += 64) {
      const int j = j0 + lane;
      const bool take = j < n && j != i && lab[j] == c && key[j] < T;
      const uint64_t m = __ballot(take);
      if (take) out[cnt + __popcll(m & below)] = j;
      cnt += __popcll(m);
    }
    // then the first need[c] tied keys of class c in numba's order
    int left = need[c];
    for (int t0 = 0; t0 < n && left > 0; t0 += 64) {
      const int t = t0 + lane;
      const uint32_t h = t < n ? R[t] : 0u;
      const bool take = (h & 0x8000u) && lab[h & 0x7FFFu] == c;
      const uint64_t m = __ballot(take);
      const int rank = __popcll(m & below);
      if (take && rank < left) out[cnt + rank] = (int32_t)(h & 0x7FFFu);
      const int got = __popcll(m);
      cnt += got < left ? got : left;
      left -= got < left ? got : left;
    }
  }
}

template <bool IN_LDS>
__global__ __launch_bounds__(64) void k_rf_ties(const int32_t* __restrict__ rows, int64_t n,
                                                const float* __restrict__ keys_all,
                                                const int32_t* __restrict__ lab, int n_classes,
                                                int64_t k, const uint32_t* __restrict__ tkey,
                                                const int32_t* __restrict__ tneed,
                                                const int32_t* __restrict__ teq,
                                                int32_t* __restrict__ R_all,
                                                int32_t* __restrict__ nbr,
                                                int* __restrict__ status) {
  extern __shared__ uint32_t tie_lds[];
  __shared__ int sort_rc;
  const int lane = threadIdx.x;
  const int64_t r = blockIdx.x;
  const int64_t i = rows[r];
  const float* key = keys_all + r * n;
  int32_t* R = R_all + r * n;
  if (IN_LDS) {
    float* kl = (float*)tie_lds;
    for (int64_t j = lane; j < n; j += 64) kl[j] = key[j];
    key = kl;
    R = (int32_t*)(tie_lds + n);
  }
  const uint32_t* Ti = tkey + i * n_classes;
  const int32_t* need = tneed + i * n_classes;
  const int32_t* eq = teq + i * n_classes;
  // handle = sample index, sign bit set for a tied candidate (its key equals
  // the k-th key of its class, in a class with more such keys than needed):
  // the sort then tests "interesting" without touching the labels
  for (int64_t j = lane; j < n; j += 64) {
    const int c = lab[j];
    const bool t = j != i && eq[c] > need[c] && __float_as_uint(key[j]) == Ti[c];
    R[j] = (int32_t)((uint32_t)j | (t ? 0x80000000u : 0u));
  }
  __syncthreads();
  // the whole wave sorts (partitions from ballot-collected stop lists)
  {
    __shared__ int32_t bufL[64], bufR[64];
    const int rc = wave_argsort_focus(
        n, R, [&](int32_t h) { return key[h & 0x7FFFFFFF]; }, bufL, bufR);
    if (lane == 0) sort_rc = rc;
  }
  __syncthreads();
  if (sort_rc != 0) {
    if (lane == 0) atomicExch(status, 1);
    return;
  }
  const uint64_t below = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  for (int c = 0; c < n_classes; c++) {
    if (!(eq[c] > need[c])) continue;
    int32_t* out = nbr + (i * n_classes + c) * k;
    const float T = __uint_as_float(Ti[c]);
    int64_t cnt = 0;
    // every key < T of class c, in index order
    for (int64_t j0 = 0; j0 < n; j0 += 64) {
      const int64_t j = j0 + lane;
      const bool take = j < n && j != i && lab[j] == c && key[j] < T;
      const uint64_t m = __ballot(take);
      if (take) out[cnt + __popcll(m & below)] = (int32_t)j;
      cnt += __popcll(m);
    }
    // then the first need[c] tied keys of class c in numba's order
    int64_t left = need[c];
    for (int64_t t0 = 0; t0 < n && left > 0; t0 += 64) {
      const int64_t t = t0 + lane;
      const int32_t h = t < n ? R[t] : 0;
      const bool take = h < 0 && lab[h & 0x7FFFFFFF] == c;
      const uint64_t m = __ballot(take);
      const int64_t rank = __popcll(m & below);
      if (take && rank < left) out[cnt + rank] = h & 0x7FFFFFFF;
      const int64_t got = __popcll(m);
      cnt += got < left ? got : left;
      left -= got < left ? got : left;
    }
  }
}

// acc_f(i) = -sum_hits d / h_found + sum_{c != y_i} (P_c / (1 - P_yi)) sum_misses_c d / k
// (ReliefF.py:177-216) for the focal rows [r_lo, r_hi).  Grid (PW/64, row
// blocks of kRfRows); 4 waves per workgroup, wave w handles rows w, w+4, ...
// of the block.  (64-row blocks: the partials k_reduce then folds are 1/4 of
// 16-row blocks', and the grid still holds ~10^4 workgroups at n = 20000.)
constexpr int64_t kRfRows = 64;
__global__ __launch_bounds__(256) void k_rf_update(const float* __restrict__ xs, int64_t r_lo,
                                                   int64_t r_hi,
                                                   int64_t PW, int64_t PC,
                                                   const int32_t* __restrict__ lab,
                                                   const double* __restrict__ prior,
                                                   int n_classes, int64_t k,
                                                   const int32_t* __restrict__ nbr,
                                                   const int32_t* __restrict__ nfound,
                                                   double* __restrict__ part) {
  __shared__ double red[4][64];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t c = (int64_t)blockIdx.x * 64 + lane;
  const bool disc = (int64_t)blockIdx.x * 64 >= PC;
  double acc = 0.0;
  const int64_t b0 = r_lo + (int64_t)blockIdx.y * kRfRows;
  for (int64_t i = b0 + wave; i < r_hi && i < b0 + kRfRows; i += 4) {
    const int32_t li = lab[i];
    const float a = xs[i * PW + c];
    double denom = 1.0 - prior[li];
    if (denom == 0.0) denom = 1.0;
    for (int cl = 0; cl < n_classes; cl++) {
      const int32_t found = nfound[i * n_classes + cl];
      if (found == 0) continue;
      // The reference scans the full argsort order, in which the focal sample
      // itself (distance inf, last) is taken as a hit whenever its class has
      // fewer than k other members: it adds a zero diff but counts in
      // h_found (ReliefF.py:144-168, 211-212).
      const int64_t h_found = found < k ? (int64_t)found + 1 : k;
      const double wgt = (cl == li) ? -1.0 / (double)h_found : (prior[cl] / denom) / (double)k;
      const int32_t* lst = nbr + (i * n_classes + cl) * k;
      double s = 0.0;
      for (int32_t t = 0; t < found; t++) {
        const float b = xs[(int64_t)lst[t] * PW + c];
        s += disc ? ((a != b) ? 1.0 : 0.0) : (double)__builtin_fabsf(a - b);
      }
      acc += wgt * s;
    }
  }
  red[wave][lane] = acc;
  __syncthreads();
  if (wave == 0)
    part[(int64_t)blockIdx.y * PW + c] = (red[0][lane] + red[1][lane]) + (red[2][lane] + red[3][lane]);
}

// ---------------------------------------------------------------------------
// Host side
// ---------------------------------------------------------------------------
struct Plan {
  Prepared P;
  int device = 0, rank = 0, world = 1;
  int x_is_f64 = 0;
  hipStream_t stream = nullptr;
  bool own_stream = false;
  // MultiSURF's mean correction (k_colrank, k_rowcorr) runs on `side`,
  // forked after k_quantize and joined before k_rowstats_reduce, beside k_dist
  hipStream_t side = nullptr;
  hipEvent_t ev_fork = nullptr, ev_join = nullptr;
  int64_t nb = 0, n_tiles = 0, seg_len = 1, nseg = 1;
  int64_t nsegpart = 1;         // rows of spart (nseg, or 2 * nseg for the v2 sparse pass)
  int ksplit = 1;               // pass-1 K-split parts of the tail tiles (k_dist)
  int64_t kfull = 0;            // tiles k_dist computes whole (the rest are split)
  int use_q16 = 0;              // pass 1 on packed 16-bit continuous operands
  double calib[7] = {0, 0, 0, 0, 1, 0, 0};  // plan_calibration (calibrate_band, row_guard)
  double cal32[2] = {0, 0};     // sampled rms / max error of 32-bit operands (row_guard)
  int64_t c_lo = 0, c_hi = 0;   // this rank's continuous columns of the mean correction
  int64_t r_lo = 0, r_hi = 0;   // focal rows scored by this plan (row sharding)
  double2* rspart = nullptr;    // per owned tile row-moment partials [tiles][256]
  double* Dpart = nullptr;      // (ksplit - 1) partial distance planes
  int key_shift = 8;             // colsort_key shift of the current scale
  void* colsort_scratch = nullptr;  // large-n route of colsort_terms
  size_t colsort_scratch_bytes = 0;
  // device buffers
  void* x = nullptr;
  int64_t* src_col = nullptr;
  int64_t* out_pos = nullptr;
  double *off = nullptr, *qs = nullptr, *scl = nullptr;
  float* scl32 = nullptr;       // scl as float (k_exact_pairs_rows)
  bool rows_direct = false;     // kept features = X's columns, all continuous, f32, 16-B pitch
  int64_t* dtab_off = nullptr;
  double* dtab = nullptr;
  int32_t* lab = nullptr;
  uint8_t* lab8 = nullptr;  // ReliefF: class codes as bytes (zero padding)
  uint32_t* xqT = nullptr;
  float* xs = nullptr;
  float* epsT = nullptr;
  double* corr = nullptr;
  double* corr_part = nullptr;  // [rowcorr_slices][n_pad] k_rowcorr slice partials
  double* xT64 = nullptr;      // SURF: float64 feature-major operands
  double* D = nullptr;
  int tiled = 0;                // D in the tiled layout (MultiSURF; d_at)
  int64_t dplane = 0;           // doubles of one distance plane (D, each Dpart)
  int2 tw = make_int2(0, 0);    // k_exact_pairs' store_pair: (nb, world) when tiled
  int2 win = make_int2(0, 0);   // full layout: rows [win.x, win.y) stored (d_row_in)
  void* D_alloc = nullptr;      // allocation behind D (D itself points at row 0)
  float* Dk = nullptr;          // ReliefF: the float32 keys instead of D (same layout)
  int2* tiles = nullptr;
  double* thr = nullptr;
  float* Wt = nullptr;          // dense pair weights (sparse == 0)
  uint2* ent = nullptr;         // sparse pair-weight streams (sparse == 1)
  unsigned long long* nnz = nullptr;  // non-zero weights of the last pass 2
  bool nnz_valid = false;
  int sparse = 0;               // pass 2 over non-zero weights only
  double* spart = nullptr;       // pass-2 segment partials (own block, shard_segments)
  size_t spart_cap = 0;           // doubles of spart
  // sparse pass-2 schedule (build_sparse_schedule): tile order, segment
  // offsets and the unit tables of the F = 8 / F = 4 launches (own blocks)
  std::vector<int2> h_tiles;      // the owned tiles (host copy of `tiles`)
  int32_t* sched = nullptr;
  int32_t* seg_off = nullptr;
  int2* units8 = nullptr;
  int2* units4 = nullptr;
  size_t sched_cap = 0;           // int32 slots of `sched` + `seg_off` (one block)
  size_t units_cap = 0;           // int2 slots of units8 + units4 (one block)
  int64_t nunits8 = 0, nunits4 = 0, nfb8 = 0, nfb4 = 0, f_tail = 0;
  // exact thresholds of uncertain rows (exact_thresholds)
  unsigned int* unc = nullptr;  // [n_pad] row flags
  int32_t* urows = nullptr;     // [n_pad + 1] flagged rows in index order, then their count
  double2* uparts = nullptr;    // [thr_rows][nchunk] exact row-moment partials
  size_t uparts_cap = 0;        // double2 slots of uparts
  int thr_rows = kExactThrRows; // rows fixed at most: exact_thr_rows(n) (thr_exact_all test hook: all)
  bool thr_all = false;
  int32_t n_exact_thr = 0;      // rows whose threshold the last select recomputed (-1: too many)
  // ambiguous-pair refinement
  int2* list = nullptr;
  int64_t list_cap = 0;
  unsigned long long* list_count = nullptr;
  int64_t n_refined = 0;
  int64_t n_tie_rows = 0;      // ReliefF rows re-ordered by k_rf_ties
  void* sort_scratch = nullptr;  // pair-list sort (fs_sort.hip)
  size_t sort_scratch_bytes = 0;
  // ev[0..1] distance kernel, ev[2..3] score kernel(s) / ReliefF selection +
  // update, ev[4..5] ReliefF's first k_rf_select launch (plan_kernel_ms)
  hipEvent_t ev[6] = {nullptr, nullptr, nullptr, nullptr, nullptr, nullptr};
  std::vector<void*> owned;         // buffers sized by n (live as long as the plan)
  std::vector<void*> owned_layout;  // buffers sized by the feature layout (PW)
  std::vector<void*> scratch;       // buffers of one plan_score call
  std::vector<void*> owned_shard;   // buffers sized by the owned tiles (plan_set_shard)
  int alloc_target = 0;             // dalloc target: 0 owned, 1 owned_layout, 2 scratch, 3 shard
  bool row_mode = false;
  // the row guard's quantised operands and mean correction are the first
  // step's (one plan over every continuous column): pass 1 takes them
  bool corr_ready = false;
  std::vector<char> colmin, colmax; // per input column, x's dtype (device-measured)
  // reference-order accumulation (P.ref_accum, fs_refacc.hip): the kept
  // columns of X (float32 [n_pad][Kp]), their recip / discreteness, the
  // discrete flag of each 256-feature block (layout buffers); MultiSURF's
  // decision masks [n_pad][n_pad / 64][4] (plan buffer) and the per-batch
  // flagged-row counts of exact_thresholds
  float* xk = nullptr;
  int64_t Kp = 0;
  int64_t* kcol = nullptr;
  float* krecip = nullptr;
  uint8_t* kdisc = nullptr;
  uint8_t* kblk = nullptr;
  uint64_t* masks = nullptr;
  int32_t* bcnt = nullptr;
  float* temp = nullptr;        // the reference's temp rows [rows][Kp] (own block)
  size_t temp_cap = 0;
  float* rkeys = nullptr;       // ReliefF neighbour keys (own block)
  size_t rkeys_cap = 0;
  bool ref_seeded = false;      // ReliefF: the column sums continue from the sums buffer
};

// ---------------------------------------------------------------------------
// Device block cache
// ---------------------------------------------------------------------------
// hipMalloc of the ~11 GB a cfg4 plan holds took 190-310 ms per fit on the
// MI355X (fresh pages are mapped on allocation; tools/fit_breakdown.py) --
// more than the scoring.  Blocks that plans and the column statistics free
// are kept per device up to a cap (an eighth of the device's memory;
// FS_DEVICE_CACHE_MB overrides, 0 disables) and handed to the next request
// they cover within 2x, so repeated fits (TuRF refits, CV folds, benchmarks)
// skip the mapping.  A failed hipMalloc releases the device's cache and
// retries; fs_device_cache_release() returns everything.  Callers free a
// block only after the streams that use it are synchronised, and every
// consumer writes or clears what it reads (blocks come back with stale data).
namespace {
struct Block {
  size_t bytes;
  int device;
  bool cached;
};
std::mutex cache_mu;
std::unordered_map<void*, Block> blocks;             // every block handed out or cached
std::multimap<std::pair<int, size_t>, void*> cache;  // (device, bytes) -> cached block
std::map<int, size_t> cache_bytes;

size_t cache_cap(int device) {  // with cache_mu held
  static long long env_mb = -2;
  if (env_mb == -2) {
    const char* e = std::getenv("FS_DEVICE_CACHE_MB");
    env_mb = (e && *e) ? std::max(0LL, std::atoll(e)) : -1;
  }
  if (env_mb >= 0) return (size_t)env_mb << 20;
  static std::map<int, size_t> total;
  auto it = total.find(device);
  if (it == total.end()) {
    size_t t = 0;
    if (hipDeviceTotalMem(&t, device) != hipSuccess) {
      (void)hipGetLastError();
      t = 0;
    }
    it = total.emplace(device, t).first;
  }
  return it->second / 8;
}

void release_device(int device) {  // with cache_mu held; device < 0: all
  for (auto it = cache.begin(); it != cache.end();) {
    if (device >= 0 && it->first.first != device) {
      ++it;
      continue;
    }
    (void)hipFree(it->second);
    blocks.erase(it->second);
    cache_bytes[it->first.first] -= it->first.second;
    it = cache.erase(it);
  }
}
}  // namespace

int dev_alloc(void** out, size_t bytes, int device) {
  if (bytes == 0) bytes = 1;
  std::lock_guard<std::mutex> lk(cache_mu);
  auto it = cache.lower_bound({device, bytes});
  if (it != cache.end() && it->first.first == device && it->first.second <= 2 * bytes) {
    *out = it->second;
    cache_bytes[device] -= it->first.second;
    blocks[it->second].cached = false;
    cache.erase(it);
    return FS_OK;
  }
  hipError_t e = hipMalloc(out, bytes);
  if (e != hipSuccess) {
    (void)hipGetLastError();
    release_device(device);
    e = hipMalloc(out, bytes);
  }
  if (e != hipSuccess) {
    (void)hipGetLastError();
    set_error(std::string("hipMalloc of ") + std::to_string(bytes) +
              " bytes failed: " + hipGetErrorString(e));
    return FS_EOOM;
  }
  blocks[*out] = Block{bytes, device, false};
  return FS_OK;
}

void dev_free(void* p) {
  if (!p) return;
  std::lock_guard<std::mutex> lk(cache_mu);
  auto it = blocks.find(p);
  if (it == blocks.end()) {
    (void)hipFree(p);
    return;
  }
  Block& b = it->second;
  if (!b.cached && cache_bytes[b.device] + b.bytes <= cache_cap(b.device)) {
    b.cached = true;
    cache.emplace(std::make_pair(b.device, b.bytes), p);
    cache_bytes[b.device] += b.bytes;
    return;
  }
  if (!b.cached) {
    blocks.erase(it);
    (void)hipFree(p);
  }
}

// Pinned host blocks (hipHostMalloc) for the float32 copy of X an estimator
// makes: the host threads cast into already-pinned, already-faulted pages and
// the upload of X is a DMA from them (cfg4 fit: the cast of 3.2 GB of
// float64 into fresh pageable pages and the copy through the runtime's
// staging buffers took ~140 ms of a 330 ms fit).  Freed blocks are kept
// (up to kHostCacheBlocks) for the next fit of a similar size (within 2x).
namespace {
constexpr size_t kHostCacheBlocks = 2;
std::mutex host_mu;
std::unordered_map<void*, size_t> host_live;
std::multimap<size_t, void*> host_cache;
}  // namespace

int host_alloc(void** out, size_t bytes) {
  *out = nullptr;
  if (bytes == 0) bytes = 1;
  {
    std::lock_guard<std::mutex> lk(host_mu);
    auto it = host_cache.lower_bound(bytes);
    if (it != host_cache.end() && it->first <= 2 * bytes) {
      *out = it->second;
      host_live[it->second] = it->first;
      host_cache.erase(it);
      return FS_OK;
    }
  }
  void* p = nullptr;
  if (hipHostMalloc(&p, bytes, hipHostMallocDefault) != hipSuccess) {
    (void)hipGetLastError();
    set_error("hipHostMalloc failed");
    return FS_EOOM;
  }
  std::lock_guard<std::mutex> lk(host_mu);
  host_live[p] = bytes;
  *out = p;
  return FS_OK;
}

void host_free(void* p) {
  if (!p) return;
  std::vector<void*> drop;
  {
    std::lock_guard<std::mutex> lk(host_mu);
    auto it = host_live.find(p);
    if (it == host_live.end()) return;
    host_cache.emplace(it->second, p);
    host_live.erase(it);
    while (host_cache.size() > kHostCacheBlocks) {  // keep the largest blocks
      drop.push_back(host_cache.begin()->second);
      host_cache.erase(host_cache.begin());
    }
  }
  for (void* q : drop) (void)hipHostFree(q);
}

void dev_cache_release() {
  {
    std::lock_guard<std::mutex> lk(cache_mu);
    release_device(-1);
  }
  std::vector<void*> drop;
  {
    std::lock_guard<std::mutex> lk(host_mu);
    for (auto& kv : host_cache) drop.push_back(kv.second);
    host_cache.clear();
  }
  for (void* q : drop) (void)hipHostFree(q);
}

// ---------------------------------------------------------------------------
// Staged X: an estimator's fit uploads X once (fs_stage_x) and both the
// column statistics and the scoring plan read that copy; the plan takes its
// own by a device-to-device copy.  The caller keeps the host array unchanged
// until fs_unstage_x.  Saves one host-to-device copy of X per fit (1.6 GB at
// cfg4, 4 GB of float64 at cfg5).
// ---------------------------------------------------------------------------
namespace {
struct Staged {
  const void* host;
  int64_t n, p;
  int f64, device;
  void* dev;
  std::thread::id owner;  // only the staging thread's calls read it (concurrent
                          // fits of one array stage and free their own copies)
  bool borrowed;          // caller-owned device copy (stage_x_device): not freed
};
std::mutex staged_mu;
std::vector<Staged> staged;
}  // namespace

int stage_x(int device, const void* x, int x_is_f64, int64_t n, int64_t p, uint64_t* handle) {
  *handle = 0;
  if (device < 0 || device >= device_count()) {
    set_error("fs_stage_x: device ordinal out of range");
    return FS_ENODEV;
  }
  FS_HIP(hipSetDevice(device));
  const size_t bytes = (size_t)n * p * (x_is_f64 ? 8 : 4);
  void* d = nullptr;
  if (int rc = dev_alloc(&d, bytes, device)) return rc;
  if (hipMemcpy(d, x, bytes, hipMemcpyHostToDevice) != hipSuccess) {
    (void)hipGetLastError();
    dev_free(d);
    set_error("fs_stage_x: host-to-device copy failed");
    return FS_EHIP;
  }
  std::lock_guard<std::mutex> lk(staged_mu);
  staged.push_back(
      Staged{x, n, p, x_is_f64 ? 1 : 0, device, d, std::this_thread::get_id(), false});
  *handle = (uint64_t)(uintptr_t)d;
  return FS_OK;
}

// A device copy the caller already holds (e.g. X assembled on the GPU by an
// all-gather of each rank's rows) registered under the host array's key.
int stage_x_device(int device, const void* x, const void* x_dev, int x_is_f64, int64_t n,
                   int64_t p, uint64_t* handle) {
  *handle = 0;
  if (device < 0 || device >= device_count()) {
    set_error("fs_stage_x_device: device ordinal out of range");
    return FS_ENODEV;
  }
  std::lock_guard<std::mutex> lk(staged_mu);
  for (const Staged& e : staged)
    if (e.dev == x_dev) {
      set_error("fs_stage_x_device: this device buffer is already staged");
      return FS_EINVAL;
    }
  staged.push_back(Staged{x, n, p, x_is_f64 ? 1 : 0, device, const_cast<void*>(x_dev),
                          std::this_thread::get_id(), true});
  *handle = (uint64_t)(uintptr_t)x_dev;
  return FS_OK;
}

// The float64 -> float32 cast of X that validation makes (or, for float32
// X, a copy into pinned memory), fused with its finiteness scan and its
// upload: host threads cast row blocks (32 MB of float32 each) into `out`
// while this thread copies every finished block to the device (pinned
// `out`: a DMA beside the casting of later blocks).  The
// device copy is registered under `out` as fs_stage_x would; without device
// room for it (or with a non-finite value, which validation will reject) the
// cast alone is done and *handle stays 0.  cfg4 (3.2 GB of float64): the cast
// and the 1.6 GB upload overlap instead of following each other.
int stage_x_cast(int device, const void* x, int x_is_f64, int64_t n, int64_t p, int n_jobs,
                 float* out, int* finite, uint64_t* handle) {
  *handle = 0;
  *finite = 1;
  if (device < 0 || device >= device_count()) {
    set_error("fs_stage_x_cast: device ordinal out of range");
    return FS_ENODEV;
  }
  FS_HIP(hipSetDevice(device));
  const int64_t total = n * p;
  void* d = nullptr;
  hipStream_t st = nullptr;
  if (dev_alloc(&d, (size_t)total * sizeof(float), device) != FS_OK ||
      hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess) {
    (void)hipGetLastError();
    if (d) dev_free(d);
    d = nullptr;
    st = nullptr;
  }
  const int64_t blk_rows = std::max<int64_t>(1, (int64_t(8) << 20) / p);
  const int64_t nblk = (n + blk_rows - 1) / blk_rows;
  std::vector<char> done((size_t)nblk, 0);
  std::mutex mu;
  std::condition_variable cv;
  std::atomic<int64_t> next{0};
  std::atomic<int> bad{0};
  auto work = [&]() {
    for (int64_t b = next++; b < nblk; b = next++) {
      const int64_t lo = b * blk_rows * p, hi = std::min(n, (b + 1) * blk_rows) * p;
      uint32_t any = 0;
      if (x_is_f64) {
        const double* xd = (const double*)x;
        for (int64_t i = lo; i < hi; i++) {
          const float v = (float)xd[i];  // round to nearest, as numpy's astype
          out[i] = v;
          uint32_t u;
          std::memcpy(&u, &v, 4);
          any |= (uint32_t)((u & 0x7f800000u) == 0x7f800000u);
        }
      } else {
        const uint32_t* xu = (const uint32_t*)x;
        uint32_t* ou = (uint32_t*)out;
        for (int64_t i = lo; i < hi; i++) {
          const uint32_t u = xu[i];
          ou[i] = u;
          any |= (uint32_t)((u & 0x7f800000u) == 0x7f800000u);
        }
      }
      if (any) bad.store(1, std::memory_order_relaxed);
      {
        std::lock_guard<std::mutex> lk(mu);
        done[(size_t)b] = 1;
      }
      cv.notify_all();
    }
  };
  const int nt = (int)std::max<int64_t>(1, std::min<int64_t>(hardware_threads(n_jobs), nblk));
  std::vector<std::thread> th;
  th.reserve(nt);
  for (int w = 0; w < nt; w++) th.emplace_back(work);
  bool copy_ok = d != nullptr;
  for (int64_t b = 0; b < nblk; b++) {
    {
      std::unique_lock<std::mutex> lk(mu);
      cv.wait(lk, [&] { return done[(size_t)b] != 0; });
    }
    if (!copy_ok) continue;
    const int64_t lo = b * blk_rows * p, hi = std::min(n, (b + 1) * blk_rows) * p;
    if (hipMemcpyAsync((float*)d + lo, out + lo, (size_t)(hi - lo) * sizeof(float),
                       hipMemcpyHostToDevice, st) != hipSuccess) {
      (void)hipGetLastError();
      copy_ok = false;
    }
  }
  for (auto& t : th) t.join();
  if (st) {
    if (hipStreamSynchronize(st) != hipSuccess) {
      (void)hipGetLastError();
      copy_ok = false;
    }
    (void)hipStreamDestroy(st);
  }
  *finite = bad.load() ? 0 : 1;
  if (d && (!copy_ok || !*finite)) {
    dev_free(d);
    d = nullptr;
  }
  if (d) {
    std::lock_guard<std::mutex> lk(staged_mu);
    staged.push_back(Staged{out, n, p, 0, device, d, std::this_thread::get_id(), false});
    *handle = (uint64_t)(uintptr_t)d;
  }
  return FS_OK;
}

int unstage_x(uint64_t handle) {
  void* d = (void*)(uintptr_t)handle;
  bool borrowed = false;
  {
    std::lock_guard<std::mutex> lk(staged_mu);
    auto it = std::find_if(staged.begin(), staged.end(),
                           [&](const Staged& e) { return e.dev == d; });
    if (it == staged.end()) {
      set_error("fs_unstage_x: unknown handle");
      return FS_EINVAL;
    }
    borrowed = it->borrowed;
    staged.erase(it);
  }
  if (!borrowed) dev_free(d);  // every reader synchronised its stream before returning
  return FS_OK;
}

const void* staged_lookup(const void* host, int64_t n, int64_t p, int x_is_f64, int device) {
  std::lock_guard<std::mutex> lk(staged_mu);
  for (const Staged& e : staged)
    if (e.host == host && e.n == n && e.p == p && e.f64 == (x_is_f64 ? 1 : 0) &&
        e.device == device && e.owner == std::this_thread::get_id())
      return e.dev;
  return nullptr;
}

template <typename T>
static int dalloc(Plan* g, T** p, size_t count) {
  void* q = nullptr;
  if (count == 0) count = 1;
  if (int rc = dev_alloc(&q, count * sizeof(T), g->device)) return rc;
  (g->alloc_target == 1   ? g->owned_layout
   : g->alloc_target == 2 ? g->scratch
   : g->alloc_target == 3 ? g->owned_shard
                          : g->owned)
      .push_back(q);
  *p = (T*)q;
  return FS_OK;
}

#define FS_TRY(expr)              \
  do {                            \
    int rc_ = (expr);             \
    if (rc_ != FS_OK) return rc_; \
  } while (0)

template <typename T>
static int h2d(Plan* g, T* dst, const T* src, size_t count) {
  if (count == 0) return FS_OK;
  FS_HIP(hipMemcpyAsync(dst, src, count * sizeof(T), hipMemcpyHostToDevice, g->stream));
  return FS_OK;
}

static int launch_check(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error(std::string("kernel launch failed (") + what + "): " + hipGetErrorString(e));
    return FS_EHIP;
  }
  return FS_OK;
}

void plan_destroy(Plan* g) {
  if (!g) return;
  if (g->stream) (void)hipStreamSynchronize(g->stream);
  trace_mark("kernels (to sync)");
  if (g->side) (void)hipStreamSynchronize(g->side);
  for (void* q : g->owned) dev_free(q);
  for (void* q : g->owned_layout) dev_free(q);
  for (void* q : g->scratch) dev_free(q);
  for (void* q : g->owned_shard) dev_free(q);
  if (g->spart) dev_free(g->spart);
  if (g->temp) dev_free(g->temp);
  if (g->rkeys) dev_free(g->rkeys);
  if (g->sched) dev_free(g->sched);
  if (g->units8) dev_free(g->units8);
  for (auto& e : g->ev)
    if (e) (void)hipEventDestroy(e);
  if (g->ev_fork) (void)hipEventDestroy(g->ev_fork);
  if (g->ev_join) (void)hipEventDestroy(g->ev_join);
  if (g->side) (void)hipStreamDestroy(g->side);
  if (g->own_stream && g->stream) (void)hipStreamDestroy(g->stream);
  delete g;
  trace_mark("plan: free");
}

// Pass-1 K-split: k_dist holds `slots` workgroups on the chip at a time, so
// T tiles take ceil(T / slots) rounds; splitting every tile's feature range
// into S parts evens out the last round when there are few tiles (cfg2: 820
// tiles on 768 slots; one rank of an N-GPU job).  The merge streams (S + 2)
// tile planes (~66.5 / p of the tile's compute time each); S > 1 only when
// the model gains at least 3%.  (Splitting only the last round's tiles was
// measured too: no better than S = 1 at cfg2, profiles/r02/ksplit_sweep.txt.)
static int choose_ksplit(int64_t tiles, int device, int nchunks, int64_t feats) {
  int cus = 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess ||
      cus <= 0) {
    (void)hipGetLastError();
    return 1;
  }
  // workgroups of k_dist resident per CU (3 at 163 VGPRs / 32 KB LDS)
  int per_cu = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_dist, 256, 0) != hipSuccess ||
      per_cu <= 0) {
    (void)hipGetLastError();
    per_cu = 2;
  }
  const double slots = (double)per_cu * cus;
  auto eff = [&](int sp) {
    const double rounds = (double)tiles * sp / slots;
    const double merge = sp > 1 ? (sp + 2) * 66.5 / (double)(feats > 0 ? feats : 1) : 0.0;
    return rounds / std::ceil(rounds) - merge;
  };
  // the S - 1 partial planes may take at most a quarter of the free memory
  size_t free_b = 0, total_b = 0;
  int max_sp = 8;
  const size_t plane_bytes = (size_t)std::max<int64_t>(tiles, 1) * kTile * kTile * sizeof(double);
  if (hipMemGetInfo(&free_b, &total_b) == hipSuccess)
    max_sp = (int)std::min<size_t>(8, 1 + free_b / 4 / plane_bytes);
  else
    (void)hipGetLastError();
  int best = 1;
  double best_eff = eff(1) + 0.03;
  for (int sp = 2; sp <= max_sp && sp <= nchunks; sp++)
    if (eff(sp) > best_eff) {
      best_eff = eff(sp);
      best = sp;
    }
  return best;
}

// 16-bit pass-1 operands (Prepared::q16) halve k_dist.  ReliefF stays exact
// with them (every candidate near a k-th key gets its reference key), so it
// uses them from kQ16MinRowsRF samples on.  MultiSURF's threshold mu - sigma/2
// comes from the quantised row moments: the sigma error grows as 1/SC and the
// score error it causes (pairs decided on the wrong side of a threshold, each
// worth ~1/n^2) falls as ~n^-1.25 -- measured against the 32-bit path: 8.8e-6
// scale-relative at n=5000, 3.9e-6 at 8192, 1.9e-6 at 20000 --
// so MultiSURF takes them only from kQ16MinRowsMS samples on.  MultiSURF*
// is less sensitive (its far misses weigh the pairs between the two
// thresholds both ways): 5.5e-7 at cfg4, 1.5e-6 at cfg5 (n = 10000,
// p = 50000), so it takes them from kQ16MinRowsMSStar on.  FS_Q16=0/1 in
// the environment forces the choice (tests).  SURF has its own float64 pass.
constexpr int64_t kQ16MinRowsRF = 4096, kQ16MinRowsMS = 16384, kQ16MinRowsMSStar = 10000;
static int choose_q16(const Prepared& P) {
  if (P.algo == ALGO_SURF || P.no_q16) return 0;
  // reference-order MultiSURF replays the reference's decisions: 32-bit
  // operands, whose thresholds need exact recomputation on a handful of rows
  if (P.algo == ALGO_MULTISURF && P.ref_accum) return 0;
  const char* env = std::getenv("FS_Q16");
  if (env && *env) return std::atoi(env) != 0 ? 1 : 0;
  const int64_t min_rows = P.algo == ALGO_RELIEFF ? kQ16MinRowsRF
                           : P.use_star           ? kQ16MinRowsMSStar
                                                  : kQ16MinRowsMS;
  return (P.n >= min_rows && P.pc >= kFeatPad) ? 1 : 0;
}

// Pass 2 on the non-zero pair weights only (k_weights_sparse +
// k_score_sparse) or on every pair (k_weights + k_score).  The sparse loop
// costs ~1.7x the dense one per evaluated pair (LDS row gather), so it pays
// below ~58% density.  Measured (tools/bench_configs.py, one MI355X):
// MultiSURF weighs the ~42% of pairs near one of their samples (cfg4 pass 2
// 142 -> 103 ms sparse); MultiSURF* ~62% (cfg5 91 ms dense vs 102 sparse);
// SURF about break-even (cfg5), SURF* weighs nearly every pair.  A
// row-sharded SURF plan zeroes the sides of the samples it does not own, so
// it goes sparse.  FS_SPARSE=0/1 forces either (tests).
static int choose_sparse(const Plan* g, const Prepared& P) {
  if (P.algo == ALGO_RELIEFF) return 0;
  const char* env = std::getenv("FS_SPARSE");
  if (env && *env) return std::atoi(env) != 0 ? 1 : 0;
  if (P.algo == ALGO_MULTISURF) return P.use_star ? 0 : 1;
  return (g->r_hi - g->r_lo < P.n) ? 1 : 0;  // SURF / SURF*: only when row-sharded
}

// Refinement band from measured pairs.  The model band of finalize_scale
// (12 standard deviations of sum_f sign(t_i - t_j)(eps_i - eps_j) for
// independent per-column rounding) does not hold when the rounding errors of
// different columns are correlated: duplicated or collinear columns, or
// columns on one value grid, add their errors up coherently (up to pc units
// instead of ~sqrt(pc/6)).  kCalibPairs sampled pairs (the same on every
// rank: a fixed generator over [0, n)) get their quantised distance error
// against the reference's arithmetic for both operand widths (k_calib).
//  * 16-bit operands are given up (coherence guard) when the measured rms
//    error exceeds kCoherence x the model's standard deviation: with errors
//    that large the quantised threshold mu - sigma/2 drifts as well, and the
//    32-bit operands make every error 256x smaller.  The q16_guard_off test hook keeps them.
//  * The band becomes max(model, 3 max|err| + rms/2): three times the largest
//    sampled error covers the distance error (the model's 12 sigma is ~3.3x
//    the expected maximum of 4096 Gaussian samples), and rms/2 bounds the
//    spread term of the threshold (|sigma_q - sigma| <= rms_j(err_ij)).
// For independent rounding this reproduces the model band (3 x ~3.7 sigma +
// sigma/2 < 12 sigma), so ordinary data keeps its refinement cost.
constexpr double kCoherence = 2.0;

static int calibrate_band(Plan* g) {
  Prepared& Q = g->P;
  g->calib[0] = Q.q16;
  g->calib[1] = g->calib[2] = 0.0;
  g->calib[3] = std::sqrt((double)Q.pc / 6.0 + 1.0);
  g->calib[4] = 1.0;
  g->calib[5] = 0.0;
  g->calib[6] = 0.0;
  if (Q.algo == ALGO_SURF || Q.pc == 0 || Q.n < 2) return FS_OK;
  const int64_t all_pairs = Q.n * (Q.n - 1) / 2;
  const int64_t S = std::min<int64_t>(kCalibPairs, all_pairs);
  std::vector<std::pair<int64_t, int64_t>> smp;
  calib_pairs(Q.n, Q.pc, S, smp);
  std::vector<int2> pr((size_t)S);
  for (int64_t k = 0; k < S; k++) pr[(size_t)k] = make_int2((int)smp[k].first, (int)smp[k].second);
  const int q_now = Q.q16;
  double sc[2];
  for (int w = 0; w < 2; w++) {
    if (set_integer_scale(Q, 1 - w)) return FS_EINVAL;
    sc[w] = Q.SC;
  }
  if (set_integer_scale(Q, q_now)) return FS_EINVAL;
  std::vector<double> qs((size_t)Q.PW * 2, 0.0);
  for (int64_t c = 0; c < Q.pc; c++) {
    qs[(size_t)c] = Q.scale[c] * sc[0];
    qs[(size_t)(Q.PW + c)] = Q.scale[c] * sc[1];
  }
  int2* dpr = nullptr;
  double* dqs = nullptr;
  double2* derr = nullptr;
  int rc = dev_alloc((void**)&dpr, sizeof(int2) * S, g->device);
  if (!rc) rc = dev_alloc((void**)&dqs, sizeof(double) * qs.size(), g->device);
  if (!rc) rc = dev_alloc((void**)&derr, sizeof(double2) * S, g->device);
  std::vector<double2> err((size_t)S);
  if (!rc && (hipMemcpyAsync(dpr, pr.data(), sizeof(int2) * S, hipMemcpyHostToDevice,
                             g->stream) != hipSuccess ||
              hipMemcpyAsync(dqs, qs.data(), sizeof(double) * qs.size(), hipMemcpyHostToDevice,
                             g->stream) != hipSuccess))
    rc = FS_EHIP;
  if (!rc) {
    const unsigned grid = (unsigned)((S + 3) / 4);
    if (g->x_is_f64)
      k_calib<double><<<grid, 256, 0, g->stream>>>((const double*)g->x, Q.p_in, Q.pc, g->src_col,
                                                   g->off, dqs, dqs + Q.PW, g->scl32, sc[0],
                                                   sc[1], dpr, S, derr);
    else
      k_calib<float><<<grid, 256, 0, g->stream>>>((const float*)g->x, Q.p_in, Q.pc, g->src_col,
                                                  g->off, dqs, dqs + Q.PW, g->scl32, sc[0],
                                                  sc[1], dpr, S, derr);
    rc = launch_check("k_calib");
  }
  if (!rc && (hipMemcpyAsync(err.data(), derr, sizeof(double2) * S, hipMemcpyDeviceToHost,
                             g->stream) != hipSuccess ||
              hipStreamSynchronize(g->stream) != hipSuccess))
    rc = FS_EHIP;
  if (dpr) dev_free(dpr);
  if (dqs) dev_free(dqs);
  if (derr) dev_free(derr);
  if (rc) {
    (void)hipGetLastError();
    if (rc == FS_EHIP) set_error("band calibration: HIP call failed");
    return rc;
  }
  double ss[2] = {0.0, 0.0}, mx[2] = {0.0, 0.0};
  for (const double2& e : err) {
    const double v[2] = {e.x, e.y};
    for (int w = 0; w < 2; w++) {
      ss[w] += v[w] * v[w];
      mx[w] = std::max(mx[w], std::fabs(v[w]));
    }
  }
  const double rms[2] = {std::sqrt(ss[0] / (double)S), std::sqrt(ss[1] / (double)S)};
  g->cal32[0] = rms[1];
  g->cal32[1] = mx[1];
  const double sigma = g->calib[3];
  if (Q.q16 && rms[0] > kCoherence * sigma && !test_hooks().q16_guard_off) {
    g->use_q16 = 0;
    g->calib[5] = 1.0;
    if (set_integer_scale(Q, 0)) return FS_EINVAL;
  }
  const int w = Q.q16 ? 0 : 1;
  Q.amb_delta = calibrated_delta(Q.amb_delta_model, Q.SC, rms[w], mx[w]);
  g->calib[0] = Q.q16;
  g->calib[1] = rms[w];
  g->calib[2] = mx[w];
  g->calib[4] = Q.amb_delta / Q.amb_delta_model;
  if (trace_on()) {
    char msg[256];
    snprintf(msg, sizeof msg,
             "calibrate: rms16 %.1f max16 %.1f rms32 %.1f max32 %.1f model sigma %.1f -> q16 %d, "
             "band x%.2f",
             rms[0], mx[0], rms[1], mx[1], sigma, Q.q16, g->calib[4]);
    trace_mark(msg);
  }
  return FS_OK;
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
//  * block = one group x kSchedFb feature blocks x both halves (<= 32
//    units, one per CU of an XCD), dealt to the XCD with the least work so
//    far (workgroup w runs on XCD w % 8; each XCD's list is padded with
//    empty units to the longest).
// Concurrent units then share their B rows through the XCD's L2 (kSchedRows
// row blocks x 2 halves read each) and their entry streams (kSchedFb
// feature blocks read each).
constexpr int kSchedRows = 8;
constexpr int kSchedFb = 16 / kSchedRows;

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
static int shard_segments(Plan* g) {
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

// Mean-correction terms of the continuous columns [c_lo, c_hi) on stream s
// (fs_colsort.hip); the large-n route's scratch is kept with the plan.
// out[i] = the mean correction of row i over columns [c_lo, c_hi) from the
// terms in epsT (k_rowcorr over column slices, then their fixed-order sum).
static int run_rowcorr(Plan* g, int64_t c_lo, int64_t c_hi, double* out, hipStream_t st) {
  const Prepared& Q = g->P;
  const int sl = rowcorr_slices(Q.n_pad, c_hi - c_lo);
  k_rowcorr<<<dim3((unsigned)(Q.n_pad / 64), (unsigned)sl), 1024, 0, st>>>(g->epsT, Q.n_pad, c_lo,
                                                                          c_hi, g->corr_part);
  FS_TRY(launch_check("k_rowcorr"));
  k_rowcorr_sum<<<(unsigned)((Q.n + 255) / 256), 256, 0, st>>>(g->corr_part, sl, Q.n, Q.n_pad, out);
  return launch_check("k_rowcorr_sum");
}

static int run_colsort(Plan* g, int64_t c_lo, int64_t c_hi, hipStream_t s) {
  const Prepared& Q = g->P;
  if (c_hi <= c_lo) return FS_OK;
  {
    const size_t need = colsort_scratch_bytes(Q.n, c_hi - c_lo);
    if (need == 0) {
      set_error("mean correction: column sort scratch query failed");
      return FS_EHIP;
    }
    if (need > g->colsort_scratch_bytes) {
      const int tgt = g->alloc_target;
      g->alloc_target = 0;
      char* p = nullptr;
      const int rc = dalloc(g, &p, need);
      g->alloc_target = tgt;
      if (rc) return rc;
      g->colsort_scratch = p;
      g->colsort_scratch_bytes = need;
    }
  }
  return colsort_terms(g->xqT, g->epsT, Q.n, Q.n_pad, c_lo, c_hi, Q.q16, g->key_shift,
                       g->colsort_scratch, g->colsort_scratch_bytes, s)
             ? FS_EHIP
             : FS_OK;
}

// Per-row coherence guard of the 16-bit pass 1 (VERDICT r2 next #1c).  The
// sampled calibration above sees a few rows whose every feature rounds the
// same way only by chance, and even a band that covers their pair errors
// cannot fix what those errors do to the OTHER rows' thresholds: row j's
// sigma comes from its quantised second moment, to which a coherent row k
// adds ~2 b_k (D_jk - mu_j) -- large when k sits far from everyone (at the
// column minima), so every threshold moves the same way and the score
// errors add up over rows (tests/test_gpu_rowcoherent.py: 4 such rows of
// 16384 gave 3.3e-5).  The mean correction (k_colrank / k_rowcorr) measures
// each row's bias directly: corr_k = sum_j err_kj, and for independent
// rounding b_k = corr_k / (n - 1) has standard deviation sqrt(pc / 36).  So
// once per feature layout, before any step, the correction is computed over
// all continuous columns on the 16-bit operands; a row beyond 12 standard
// deviations turns the 16-bit operands off (32-bit: 256x smaller errors).
// Every rank computes the same full correction, so every rank decides alike.
// ~5 ms per fit at cfg4, none per step; the q16_guard_off test hook disables it.
static int row_guard(Plan* g) {
  Prepared& Q = g->P;
  if (!Q.q16 || Q.pc == 0 || Q.n < 2 || Q.algo == ALGO_SURF || test_hooks().q16_guard_off)
    return FS_OK;
  // a plan over every continuous column (one rank, one shard) keeps the
  // guard's work for its first pass 1: operands, terms and the correction
  // itself (g->corr) are what that pass would compute again
  const bool reuse = g->c_lo == 0 && g->c_hi == Q.pc;
  double* corr = g->corr;
  if (!reuse) FS_TRY(dev_alloc((void**)&corr, sizeof(double) * Q.n_pad, g->device));
  dim3 gq((unsigned)(Q.PW / 64), (unsigned)(Q.n_pad / 64));
  int rc = FS_OK;
  if (g->x_is_f64)
    k_quantize<double><<<gq, 256, 0, g->stream>>>(
        (const double*)g->x, Q.n, Q.n_pad, Q.p_in, Q.PW, Q.PC, Q.q16, Q.pc, g->src_col, g->off,
        g->qs, g->scl, g->dtab_off, g->dtab, Q.disc_bits, 0, Q.pc, g->xqT, g->xs, g->epsT);
  else
    k_quantize<float><<<gq, 256, 0, g->stream>>>(
        (const float*)g->x, Q.n, Q.n_pad, Q.p_in, Q.PW, Q.PC, Q.q16, Q.pc, g->src_col, g->off,
        g->qs, g->scl, g->dtab_off, g->dtab, Q.disc_bits, 0, Q.pc, g->xqT, g->xs, g->epsT);
  rc = launch_check("k_quantize (row guard)");
  if (!rc) {
    rc = run_colsort(g, 0, Q.pc, g->stream);
  }
  if (!rc) {
    rc = run_rowcorr(g, 0, Q.pc, corr, g->stream);
  }
  std::vector<double> h((size_t)Q.n);
  if (!rc && (hipMemcpyAsync(h.data(), corr, sizeof(double) * Q.n, hipMemcpyDeviceToHost,
                             g->stream) != hipSuccess ||
              hipStreamSynchronize(g->stream) != hipSuccess)) {
    (void)hipGetLastError();
    set_error("row guard: device-to-host copy failed");
    rc = FS_EHIP;
  }
  if (!reuse) dev_free(corr);
  if (rc) return rc;
  double worst = 0.0;
  for (double c : h) worst = std::max(worst, std::fabs(c) / (double)(Q.n - 1));
  const double limit = 12.0 * std::sqrt((double)Q.pc / 36.0 + 1.0);
  g->calib[6] = worst / limit;
  if (worst > limit) {
    g->use_q16 = 0;
    g->calib[5] = 2.0;
    if (set_integer_scale(Q, 0)) return FS_EINVAL;
    Q.amb_delta = calibrated_delta(Q.amb_delta_model, Q.SC, g->cal32[0], g->cal32[1]);
    g->calib[0] = 0.0;
    g->calib[1] = g->cal32[0];
    g->calib[2] = g->cal32[1];
    g->calib[4] = Q.amb_delta / Q.amb_delta_model;
  } else {
    g->corr_ready = reuse;
  }
  if (trace_on()) {
    char msg[160];
    snprintf(msg, sizeof msg, "row guard: max |row bias| %.1f (limit %.1f) -> q16 %d", worst,
             limit, Q.q16);
    trace_mark(msg);
  }
  return FS_OK;
}

// Feature-layout part of a plan: everything sized by the kept features
// (permutation tables, quantised operands, pass-2 partials), rebuilt when
// the plan is re-targeted to another feature subset (fs_plan_set_features).
// Reference-order accumulation (P.ref_accum): the kept columns of X in kept
// order, 256-padded (xk), with each kept feature's float32 recip and
// discreteness as the reference's kernels read them (MultiSURF.py:184-187,
// ReliefF.py:151-154), and a flag per 256-feature block that holds a
// discrete one.  Layout buffers: rebuilt with the feature subset.
static int ref_layout(Plan* g) {
  const Prepared& Q = g->P;
  if (g->x_is_f64) {
    set_error("reference-order accumulation needs float32 X (MultiSURF / ReliefF)");
    return FS_ENOTSUP;
  }
  g->Kp = (Q.n_kept + 255) / 256 * 256;
  std::vector<float> rec((size_t)g->Kp, 0.0f);
  std::vector<uint8_t> dsc((size_t)g->Kp, 0), blk((size_t)(g->Kp / 256), 0);
  for (int64_t k = 0; k < Q.n_kept; k++) {
    const int64_t col = Q.kept_col[k];
    rec[k] = Q.recip_in[col];
    dsc[k] = Q.disc_in[col] ? 1 : 0;
    if (dsc[k]) blk[k / 256] = 1;
  }
  g->alloc_target = 1;
  int rc;
  if ((rc = dalloc(g, &g->xk, (size_t)Q.n_pad * g->Kp)) || (rc = dalloc(g, &g->kcol, Q.n_kept)) ||
      (rc = dalloc(g, &g->krecip, g->Kp)) || (rc = dalloc(g, &g->kdisc, g->Kp)) ||
      (rc = dalloc(g, &g->kblk, g->Kp / 256))) {
    g->alloc_target = 0;
    return rc;
  }
  g->alloc_target = 0;
  if ((rc = h2d(g, g->kcol, Q.kept_col.data(), Q.n_kept)) ||
      (rc = h2d(g, g->krecip, rec.data(), rec.size())) ||
      (rc = h2d(g, g->kdisc, dsc.data(), dsc.size())) ||
      (rc = h2d(g, g->kblk, blk.data(), blk.size())))
    return rc;
  rc = refacc::gather_kept((const float*)g->x, Q.n, Q.n_pad, Q.p_in, g->kcol, Q.n_kept, g->Kp,
                           g->xk, g->stream);
  if (rc == FS_OK) FS_HIP(hipStreamSynchronize(g->stream));  // host vectors above
  return rc;
}

// Rows exact_thresholds fixes per select, from the current layout's feature
// count (both backends use exact_thr_rows(n, pc + pd) of the layout in use,
// a TuRF refit with fewer features may fix more rows); the
// partials buffer grows with it.
static int size_exact_rows(Plan* g) {
  const Prepared& Q = g->P;
  if (Q.algo != ALGO_MULTISURF) return FS_OK;
  g->thr_rows = (int)(g->thr_all ? Q.n : exact_thr_rows(Q.n, Q.pc + Q.pd));
  const int64_t nchunk = (Q.n + kExChunk - 1) / kExChunk;
  const size_t need = (size_t)g->thr_rows * nchunk;
  if (need <= g->uparts_cap) return FS_OK;
  if (g->uparts) {
    g->owned.erase(std::remove(g->owned.begin(), g->owned.end(), (void*)g->uparts),
                   g->owned.end());
    dev_free(g->uparts);
    g->uparts = nullptr;
  }
  FS_TRY(dalloc(g, &g->uparts, need));
  g->uparts_cap = need;
  return FS_OK;
}

static int plan_layout(Plan* g) {
  Prepared& Q = g->P;
  g->corr_ready = false;
  FS_HIP(hipStreamSynchronize(g->stream));
  if (g->side) FS_HIP(hipStreamSynchronize(g->side));
  for (void* q : g->owned_layout) dev_free(q);
  g->owned_layout.clear();
  int rc;
  Q.q16 = g->use_q16;
  if (!Q.ranges_ready) {
    // continuous column ranges, measured on the device once per plan
    const size_t esz = g->x_is_f64 ? 8 : 4;
    if (g->colmin.empty()) {
      g->colmin.resize((size_t)Q.p_in * esz);
      g->colmax.resize((size_t)Q.p_in * esz);
      if ((rc = column_minmax(g->x, g->x_is_f64, Q.n, Q.p_in, g->colmin.data(), g->colmax.data(),
                              g->stream))) {
        g->colmin.clear();
        return rc;
      }
      trace_mark("plan: device ranges");
    }
    std::vector<double> cmin((size_t)Q.pc), cmax((size_t)Q.pc);
    for (int64_t c = 0; c < Q.pc; c++) {
      const int64_t col = Q.src_col[c];
      cmin[c] = g->x_is_f64 ? ((const double*)g->colmin.data())[col]
                            : (double)((const float*)g->colmin.data())[col];
      cmax[c] = g->x_is_f64 ? ((const double*)g->colmax.data())[col]
                            : (double)((const float*)g->colmax.data())[col];
    }
    if (finalize_scale(Q, cmin.data(), cmax.data())) return FS_EINVAL;
  } else if (set_integer_scale(Q, Q.q16)) {
    // the integer scale of the operand width in use (a plan switched to
    // 32-bit operands by plan_decision_guard keeps its ranges)
    return FS_EINVAL;
  }
  g->key_shift = colsort_key_shift(Q.qmax);
  g->alloc_target = 1;
  rc = FS_OK;
  if ((rc = dalloc(g, &g->src_col, Q.PW)) || (rc = dalloc(g, &g->out_pos, Q.PW)) ||
      (rc = dalloc(g, &g->off, Q.PW)) || (rc = dalloc(g, &g->qs, Q.PW)) ||
      (rc = dalloc(g, &g->scl, Q.PW)) || (rc = dalloc(g, &g->scl32, Q.PW)) ||
      (rc = dalloc(g, &g->dtab_off, Q.PW + 1)) ||
      (rc = dalloc(g, &g->dtab, Q.dtab.size())) ||
      // xs: two spare rows (the pass-2 B prefetch runs up to two rows past a
      // tile) plus kXsSlack floats: the asm loop of a last, partial feature
      // block reads a whole block width of each B row, past the end of the
      // last row when PW is narrower than the block
      (rc = dalloc(g, &g->xs, (size_t)(Q.n_pad + 2) * Q.PW + kXsSlack))) {
  } else if (Q.algo == ALGO_SURF) {
    rc = dalloc(g, &g->xT64, (size_t)Q.PW * Q.n_pad);
  } else if ((rc = dalloc(g, &g->xqT, (size_t)Q.PW * Q.n_pad)) == FS_OK) {
    rc = dalloc(g, &g->epsT, (size_t)Q.PW * Q.n_pad);
  }
  g->alloc_target = 0;
  if (rc) return rc;
  if ((rc = shard_segments(g))) return rc;
  std::vector<double> qs(Q.PW, 0.0);
  for (int64_t c = 0; c < Q.PW; c++) qs[c] = Q.scale[c] * Q.SC;
  std::vector<float> scl32(Q.PW, 0.0f);
  for (int64_t c = 0; c < Q.PW; c++) scl32[c] = (float)Q.scale[c];
  g->rows_direct = !g->x_is_f64 && Q.pd == 0 && Q.pc == Q.p_in && Q.p_in % 4 == 0;
  for (int64_t c = 0; g->rows_direct && c < Q.pc; c++) g->rows_direct = Q.src_col[c] == c;
  if ((rc = h2d(g, g->src_col, Q.src_col.data(), Q.PW)) ||
      (rc = h2d(g, g->out_pos, Q.out_pos.data(), Q.PW)) ||
      (rc = h2d(g, g->off, Q.offset.data(), Q.PW)) || (rc = h2d(g, g->qs, qs.data(), Q.PW)) ||
      (rc = h2d(g, g->scl, Q.scale.data(), Q.PW)) ||
      (rc = h2d(g, g->scl32, scl32.data(), Q.PW)) ||
      (rc = h2d(g, g->dtab_off, Q.dtab_off.data(), Q.PW + 1)) ||
      (rc = h2d(g, g->dtab, Q.dtab.data(), Q.dtab.size())))
    return rc;
  if ((rc = size_exact_rows(g))) return rc;
  if (Q.ref_accum && Q.algo != ALGO_SURF && (rc = ref_layout(g))) return rc;
  if ((rc = calibrate_band(g))) return rc;
  if ((rc = row_guard(g))) return rc;
  if (g->calib[5] != 0.0) {
    // the coherence guard switched to 32-bit operands: new scale and sort key
    for (int64_t c = 0; c < Q.PW; c++) qs[c] = Q.scale[c] * Q.SC;
    g->key_shift = colsort_key_shift(Q.qmax);
    if ((rc = h2d(g, g->qs, qs.data(), Q.PW))) return rc;
  }
  FS_HIP(hipStreamSynchronize(g->stream));
  return FS_OK;
}

// Everything sized by the plan's owned tiles: the tile list, the distance
// planes (tiled for MultiSURF: one 128 x 128 block per tile), the K-split,
// row-moment partials and the pass-2 weights.  Called by plan_create and
// again by plan_set_shard, which frees the previous shard's buffers first.
static int setup_shard(Plan* g, const std::vector<int32_t>& bi, const std::vector<int32_t>& bj) {
  const Prepared& Q = g->P;
  g->n_tiles = (int64_t)bi.size();
  std::vector<int2> tl(g->n_tiles);
  for (int64_t t = 0; t < g->n_tiles; t++) tl[t] = make_int2(bi[t], bj[t]);
  g->h_tiles = tl;
  // MultiSURF reads distances only inside owned tiles: tiled layout, one
  // 128 x 128 block per owned tile (half the full matrix at world 1, 1/N of
  // the tiles per rank).  ReliefF / SURF select neighbours over whole rows.
  g->tiled = (Q.algo == ALGO_MULTISURF && !g->row_mode) ? 1 : 0;
  // ReliefF / SURF: the rows of the plan's focal 128-sample blocks only
  // (d_row_in): a whole fit holds n_pad^2, one rank of an N-way row split or
  // one row panel (rows_run_panels) its share
  if (g->tiled) {
    g->win = make_int2(0, 0);
  } else {
    const int64_t w0 = g->row_mode ? g->r_lo / kTile * kTile : 0;
    const int64_t w1 = g->row_mode ? std::min<int64_t>(Q.n_pad, (g->r_hi + kTile - 1) / kTile * kTile)
                                   : Q.n_pad;
    g->win = make_int2((int)w0, (int)std::max(w0, w1));
  }
  g->dplane = g->tiled ? std::max<int64_t>(g->n_tiles, 1) * kTile * kTile
                       : std::max<int64_t>((int64_t)(g->win.y - g->win.x), 1) * Q.n_pad;
  g->tw = g->tiled ? make_int2((int)g->nb, g->world) : make_int2(0, 0);
  // pass-1 chunk count and the per-tile work in feature units of 32-bit SAD
  const int64_t rows_q = (g->use_q16 ? Q.PC / 2 : Q.PC) + Q.PD;
  g->ksplit = choose_ksplit(g->n_tiles, g->device, (int)(rows_q / kBKQ),
                            (g->use_q16 ? Q.pc / 2 : Q.pc) + Q.pd);
  if (test_hooks().ksplit >= 1) g->ksplit = (int)std::min<int64_t>(16, test_hooks().ksplit);
  if (Q.algo == ALGO_SURF) g->ksplit = 1;  // k_dist_f64 has no K-split
  // ReliefF stores float32 keys (Dk), formed in k_dist's epilogue from whole
  // tiles: no K-split (partial sums cannot be keyed before they are added)
  const bool dkeys = Q.algo == ALGO_RELIEFF;
  if (dkeys) g->ksplit = 1;
  g->kfull = g->ksplit > 1 ? 0 : g->n_tiles;  // k_dist can split only a tail; all or none here
  g->alloc_target = 3;
  int rc = FS_OK;
  g->Dk = nullptr;
  if ((rc = dkeys ? dalloc(g, (float**)&g->D_alloc, (size_t)g->dplane)
                  : dalloc(g, (double**)&g->D_alloc, (size_t)g->dplane)) ||
      (dkeys ? (g->Dk = (float*)g->D_alloc - (int64_t)g->win.x * Q.n_pad, g->D = nullptr)
             : (g->D = (double*)g->D_alloc - (g->tiled ? 0 : (int64_t)g->win.x * Q.n_pad)),
       false) ||
      (rc = dalloc(g, &g->tiles, g->n_tiles)) ||
      (rc = dalloc(g, &g->rspart, (size_t)std::max<int64_t>(g->n_tiles, 1) * 256))) {
  } else if (Q.algo != ALGO_RELIEFF && !g->sparse) {
    rc = dalloc(g, &g->Wt, (size_t)(g->n_tiles + 1) * kTile * kTile);
  } else if (g->sparse) {
    // One spare tile: k_score_sparse prefetches two groups past the end of a
    // stream.  Zeroed once, so such reads (and stream tails never written)
    // hold in-range row offsets.
    const size_t count = (size_t)(g->n_tiles + 1) * kSWaves * kStreamEntries;
    if (!(rc = dalloc(g, &g->ent, count)) && !(rc = dalloc(g, &g->nnz, 1)) &&
        hipMemsetAsync(g->ent, 0, sizeof(uint2) * count, g->stream) != hipSuccess)
      rc = FS_EHIP;
  }
  if (!rc && g->ksplit > 1)
    rc = dalloc(g, &g->Dpart,
                (size_t)(g->n_tiles - g->kfull) * (g->ksplit - 1) * kTile * kTile);
  g->alloc_target = 0;
  if (rc) return rc;
  g->nnz_valid = false;
  return h2d(g, g->tiles, tl.data(), g->n_tiles);
}

int plan_set_shard(Plan* g, int rank, int world) {
  if (g->P.algo != ALGO_MULTISURF || g->row_mode) {
    set_error("tile shards of a plan are MultiSURF-only");
    return FS_EINVAL;
  }
  if (world < 1 || rank < 0 || rank >= world) {
    set_error("invalid shard rank/world");
    return FS_EINVAL;
  }
  FS_HIP(hipSetDevice(g->device));
  FS_HIP(hipStreamSynchronize(g->stream));
  if (g->side) FS_HIP(hipStreamSynchronize(g->side));
  for (void* q : g->owned_shard) dev_free(q);
  g->owned_shard.clear();
  g->D = g->Dpart = nullptr;
  g->D_alloc = nullptr;
  g->Wt = nullptr;
  g->ent = nullptr;
  g->tiles = nullptr;
  g->rspart = nullptr;
  g->nnz = nullptr;
  g->rank = rank;
  g->world = world;
  std::vector<int32_t> bi, bj;
  owned_tiles(g->nb, rank, world, bi, bj);
  FS_TRY(setup_shard(g, bi, bj));
  return shard_segments(g);  // pass-2 segments and this shard's mean-correction columns
}

int plan_create(Plan** out, const Prepared& P, const void* x, int x_is_f64, int device,
                int rank, int world, uint64_t stream, int64_t r_lo, int64_t r_hi) {
  *out = nullptr;
  const int ndev = device_count();
  if (ndev <= 0) {
    set_error("backend='gpu' requested but no HIP device is visible");
    return FS_ENODEV;
  }
  if (device < 0 || device >= ndev) {
    set_error("device ordinal out of range");
    return FS_EINVAL;
  }
  if (world < 1 || rank < 0 || rank >= world) {
    set_error("invalid rank/world");
    return FS_EINVAL;
  }
  if (P.n >= (1 << 20)) {  // k_colrank's packed histogram; D alone would be 8 TB
    set_error("the GPU backend supports fewer than 2^20 samples");
    return FS_ENOTSUP;
  }
  const bool row_mode = r_hi >= 0;
  if (row_mode && !(0 <= r_lo && r_lo <= r_hi && r_hi <= P.n)) {
    set_error("row range outside [0, n)");
    return FS_EINVAL;
  }
  FS_HIP(hipSetDevice(device));
  Plan* g = new Plan();
  g->P = P;
  g->device = device;
  g->rank = rank;
  g->world = world;
  g->x_is_f64 = x_is_f64;
  if (stream) {
    g->stream = (hipStream_t)(uintptr_t)stream;
  } else {
    if (hipStreamCreateWithFlags(&g->stream, hipStreamNonBlocking) != hipSuccess) {
      delete g;
      set_error("hipStreamCreate failed");
      return FS_EHIP;
    }
    g->own_stream = true;
  }
  auto fail = [&](int rc) {
    plan_destroy(g);
    return rc;
  };
  for (auto& e : g->ev)
    if (hipEventCreate(&e) != hipSuccess) return fail(FS_EHIP);
  if (hipStreamCreateWithFlags(&g->side, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreateWithFlags(&g->ev_fork, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&g->ev_join, hipEventDisableTiming) != hipSuccess)
    return fail(FS_EHIP);
  const Prepared& Q = g->P;
  g->nb = Q.n_pad / kTile;
  std::vector<int32_t> bi, bj;
  if (row_mode) {
    g->r_lo = r_lo;
    g->r_hi = r_hi;
    if (r_hi > r_lo) row_tiles(g->nb, r_lo / kTile, (r_hi + kTile - 1) / kTile, bi, bj);
  } else {
    g->r_lo = 0;
    g->r_hi = Q.n;
    owned_tiles(g->nb, rank, world, bi, bj);
  }
  g->row_mode = row_mode;
  // (ReliefF refines in k_rf_select and uses only the counter)
  g->list_cap = Q.algo == ALGO_RELIEFF ? 1 : std::max<int64_t>(1 << 16, Q.n * 64);
  g->use_q16 = choose_q16(Q);
  const size_t xbytes = (size_t)Q.n * Q.p_in * (x_is_f64 ? 8 : 4);
  int rc;
  trace_mark("plan: host setup");
  if ((rc = dalloc(g, (char**)&g->x, xbytes)) || (rc = dalloc(g, &g->lab, Q.n_pad)) ||
      (rc = dalloc(g, &g->corr, Q.n_pad)) ||
      (rc = dalloc(g, &g->corr_part, (int64_t)kRowcorrMaxSlices * Q.n_pad)) ||
      (rc = dalloc(g, &g->thr, Q.n_pad)) ||
      (rc = dalloc(g, &g->list, g->list_cap)) || (rc = dalloc(g, &g->list_count, 1)))
    return fail(rc);
  if (Q.algo == ALGO_MULTISURF) {
    // test hook: every row's threshold from exact distances (the machinery
    // of exact_thresholds checked on all rows against the oracle's)
    g->thr_all = test_hooks().thr_exact_all != 0;
    // thr_rows and uparts: size_exact_rows (plan_layout, per feature layout)
    g->thr_rows = (int)(g->thr_all ? Q.n : exact_thr_rows(Q.n, Q.pc + Q.pd));
    if ((rc = dalloc(g, &g->unc, Q.n_pad)) || (rc = dalloc(g, &g->urows, Q.n_pad + 1)))
      return fail(rc);
    // reference-order accumulation: the decision masks (n_pad^2 / 2 bytes)
    // and exact_thresholds' batch counts (every flagged row is fixed, in
    // batches of thr_rows)
    if (Q.ref_accum &&
        ((rc = dalloc(g, &g->masks, (size_t)Q.n_pad * (Q.n_pad / 64) * 4)) ||
         (rc = dalloc(g, &g->bcnt, (size_t)(Q.n / std::max(g->thr_rows, 1) + 2)))))
      return fail(rc);
  }
  g->sparse = choose_sparse(g, Q);
  if ((rc = setup_shard(g, bi, bj))) return fail(rc);
  trace_mark("plan: hipMalloc");
  std::vector<int32_t> lab(Q.n_pad, -1);
  std::copy(Q.labels.begin(), Q.labels.end(), lab.begin());
  const void* sx = staged_lookup(x, Q.n, Q.p_in, x_is_f64, g->device);
  if (sx && hipMemcpyAsync(g->x, sx, xbytes, hipMemcpyDeviceToDevice, g->stream) != hipSuccess) {
    (void)hipGetLastError();
    set_error("plan: device-to-device copy of the staged X failed");
    return fail(FS_EHIP);
  }
  if ((!sx && (rc = h2d(g, (char*)g->x, (const char*)x, xbytes))) ||
      (rc = h2d(g, g->lab, lab.data(), Q.n_pad)))
    return fail(rc);
  if (Q.algo == ALGO_RELIEFF) {
    std::vector<uint8_t> lab8((size_t)Q.n_pad + 16, 0);
    for (int64_t j = 0; j < Q.n; j++) lab8[j] = (uint8_t)Q.labels[j];
    if ((rc = dalloc(g, &g->lab8, lab8.size())) || (rc = h2d(g, g->lab8, lab8.data(), lab8.size())))
      return fail(rc);
  }
  if ((rc = plan_layout(g))) return fail(rc);
  trace_mark("plan: H2D + layout");
  *out = g;
  return FS_OK;
}

int plan_set_features(Plan* g, const Prepared& P) {
  FS_HIP(hipSetDevice(g->device));
  g->P = P;
  return plan_layout(g);
}

// quantize (+ mean correction terms) and pass 1 (distance tiles)
static int run_quantize_dist(Plan* g) {
  const Prepared& Q = g->P;
  FS_HIP(hipSetDevice(g->device));
  dim3 gq((unsigned)(Q.PW / 64), (unsigned)(Q.n_pad / 64));
  if (Q.algo == ALGO_SURF) {
    k_quantize_f64<<<gq, 256, 0, g->stream>>>((const double*)g->x, Q.n, Q.n_pad, Q.p_in, Q.PW,
                                              Q.pc, g->src_col, g->off, g->scl, g->dtab_off,
                                              g->dtab, g->xT64, g->xs);
    FS_TRY(launch_check("k_quantize_f64"));
    if (g->n_tiles > 0) {
      FS_HIP(hipEventRecord(g->ev[0], g->stream));
      k_dist_f64<<<(unsigned)g->n_tiles, 256, 0, g->stream>>>(
          g->xT64, Q.n_pad, (int)(Q.PC / kBK64), (int)(Q.PD / kBK64), g->tiles, g->win, g->D);
      FS_TRY(launch_check("k_dist_f64"));
      FS_HIP(hipEventRecord(g->ev[1], g->stream));
    }
    return FS_OK;
  }
  const bool reuse = g->corr_ready && Q.algo == ALGO_MULTISURF;
  g->corr_ready = false;  // later steps quantise again (the terms overwrote epsT)
  if (reuse) {
    // the row guard's operands and correction (row_guard): nothing to redo
    FS_HIP(hipEventRecord(g->ev_join, g->stream));
  } else if (g->x_is_f64) {
    k_quantize<double><<<gq, 256, 0, g->stream>>>(
        (const double*)g->x, Q.n, Q.n_pad, Q.p_in, Q.PW, Q.PC, Q.q16, Q.pc, g->src_col, g->off,
        g->qs, g->scl, g->dtab_off, g->dtab, Q.disc_bits, g->c_lo, g->c_hi, g->xqT, g->xs,
        g->epsT);
  } else {
    k_quantize<float><<<gq, 256, 0, g->stream>>>(
        (const float*)g->x, Q.n, Q.n_pad, Q.p_in, Q.PW, Q.PC, Q.q16, Q.pc, g->src_col, g->off,
        g->qs, g->scl, g->dtab_off, g->dtab, Q.disc_bits, g->c_lo, g->c_hi, g->xqT, g->xs,
        g->epsT);
  }
  if (!reuse) FS_TRY(launch_check("k_quantize"));
  if (Q.algo == ALGO_MULTISURF && !reuse) {
    // mean correction of this rank's feature share (summed across ranks
    // with the row moments), on the side stream beside k_dist: it reads
    // xqT as k_dist does and writes only epsT / corr, which k_dist leaves
    // alone; plan_pass1 joins it before k_rowstats_reduce reads corr
    // (the side stream won the A/B against running it before k_dist at cfg4
    // and cfg2: profiles/r02/ksplit_sweep2.txt).  The correction runs for
    // both operand widths: with 32-bit operands a row's mean error is tiny
    // for independent rounding, but columns on a shared value grid round
    // coherently and heavy-tailed columns crowd most samples into a few
    // quanta, and both move the thresholds (intgrid, n = 3000: 2.2e-5
    // without it; lognormal: VERDICT r3 missing #1).
    FS_HIP(hipEventRecord(g->ev_fork, g->stream));
    FS_HIP(hipStreamWaitEvent(g->side, g->ev_fork, 0));
    FS_TRY(run_colsort(g, g->c_lo, g->c_hi, g->side));
    FS_TRY(run_rowcorr(g, g->c_lo, g->c_hi, g->corr, g->side));
    FS_HIP(hipEventRecord(g->ev_join, g->side));
  }
  if (g->n_tiles > 0) {
    FS_HIP(hipEventRecord(g->ev[0], g->stream));
    const int64_t n_split = g->ksplit > 1 ? g->n_tiles - g->kfull : 0;
    const int64_t n_full = g->n_tiles - n_split;
    const int nck = (int)((Q.q16 ? Q.PC / 2 : Q.PC) / kBKQ), nckd = (int)(Q.PD / kBKQ);
    {
      k_dist<<<(unsigned)(n_full + n_split * g->ksplit), 256, 0, g->stream>>>(
          g->xqT, Q.n_pad, nck, nckd, Q.SCu, Q.q16, g->tiles, n_full, g->ksplit, g->tiled,
          g->win, g->D, g->Dpart, g->Dk, 1.0 / Q.SC);
      FS_TRY(launch_check("k_dist"));
      if (n_split > 0) {
        k_dist_merge<<<dim3((unsigned)n_split, kMergeSlices), 256, 0, g->stream>>>(
            g->D, g->Dpart, g->ksplit - 1, g->tiles, n_full, Q.n_pad, g->tiled, g->win);
        FS_TRY(launch_check("k_dist_merge"));
      }
    }
    FS_HIP(hipEventRecord(g->ev[1], g->stream));
  }
  return FS_OK;
}

// Order the first `count` pairs of g->list by (i, j) (see fs_sort.hip).
static int sort_pair_list(Plan* g, int64_t count) {
  if (count < 2) return FS_OK;
  const size_t need = pair_sort_scratch_bytes(count);
  if (need == 0) {
    set_error("pair list sort: temporary storage query failed");
    return FS_EHIP;
  }
  if (need > g->sort_scratch_bytes) {
    char* p = nullptr;
    FS_TRY(dalloc(g, &p, need + need / 4));
    g->sort_scratch = p;
    g->sort_scratch_bytes = need + need / 4;
  }
  return sort_pairs(g->list, count, g->sort_scratch, g->sort_scratch_bytes, g->stream) == 0
             ? FS_OK
             : FS_EHIP;
}

// Flag the ambiguous pairs of the owned tiles and recompute them exactly.
// One host round trip reads the pair count (to grow the list if needed).
static int refine_pairs(Plan* g, int algo, double delta, double thr_tol = 0.0,
                        unsigned int* unc = nullptr) {
  const Prepared& Q = g->P;
  g->n_refined = 0;
  if (g->n_tiles == 0) return FS_OK;
  for (int attempt = 0; attempt < 2; attempt++) {
    FS_HIP(hipMemsetAsync(g->list_count, 0, sizeof(unsigned long long), g->stream));
    k_flag_pairs<<<(unsigned)g->n_tiles, 256, 0, g->stream>>>(
        g->D, Q.n, Q.n_pad, g->tiled, g->win, g->tiles, g->thr, algo, 1.0 / Q.SC, delta, g->list,
        g->list_cap, g->list_count);
    FS_TRY(launch_check("k_flag_pairs"));
    unsigned long long cnt = 0;
    FS_HIP(hipMemcpyAsync(&cnt, g->list_count, sizeof(cnt), hipMemcpyDeviceToHost, g->stream));
    FS_HIP(hipStreamSynchronize(g->stream));
    if ((int64_t)cnt <= g->list_cap) {
      g->n_refined = (int64_t)cnt;
      break;
    }
    g->list_cap = (int64_t)cnt + cnt / 4;
    FS_TRY(dalloc(g, &g->list, g->list_cap));
  }
  if (g->n_refined == 0) return FS_OK;
  FS_TRY(sort_pair_list(g, g->n_refined));
  const unsigned grid = (unsigned)std::min<int64_t>((g->n_refined + 3) / 4, 8192);
  if (g->rows_direct && !test_hooks().exact_gather)
    k_exact_pairs_rows<<<grid, 256, 0, g->stream>>>((const float*)g->x, Q.p_in, g->scl32, Q.SC,
                                                    g->list, g->list_count, g->list_cap, Q.n_pad,
                                                    g->tw, g->win, g->D, g->thr, thr_tol, unc);
  else if (g->x_is_f64)
    k_exact_pairs<double><<<grid, 256, 0, g->stream>>>(
        (const double*)g->x, Q.p_in, Q.pc, Q.PC, Q.pd, g->src_col, g->scl, Q.SC, g->list,
        g->list_count, g->list_cap, Q.n_pad, g->tw, g->win, 0, g->D, nullptr, g->thr, thr_tol,
        unc);
  else
    k_exact_pairs<float><<<grid, 256, 0, g->stream>>>(
        (const float*)g->x, Q.p_in, Q.pc, Q.PC, Q.pd, g->src_col, g->scl, Q.SC, g->list,
        g->list_count, g->list_cap, Q.n_pad, g->tw, g->win, 0, g->D, nullptr, g->thr, thr_tol,
        unc);
  return launch_check("k_exact_pairs");
}

// MultiSURF thresholds from exact distances for the rows a refined pair
// sits too close to (mark_uncertain, k_row_exact_*), when at most
// g->thr_rows of them are flagged -- on 32-bit operands a handful per fit;
// on 16-bit operands there can be thousands, and the post-scoring decision
// check (q16_decision_risk) stays in charge.  Runs between refine_pairs and
// the neighbour counts; the count is read back once (the fix's row count is
// reported by fs_plan_info-style diagnostics: g->n_exact_thr).
// Reference-order accumulation: every flagged row, in batches of thr_rows
// (the count is read back once; the decisions are then the reference's
// wherever its arithmetic is replayed exactly).
static int exact_thresholds_all(Plan* g) {
  const Prepared& Q = g->P;
  const int64_t nchunk = (Q.n + kExChunk - 1) / kExChunk;
  const int B = std::max(g->thr_rows, 1);
  const unsigned ngroups = (unsigned)((B + kExRows - 1) / kExRows);
  k_unc_compact<<<1, 1024, 0, g->stream>>>(g->unc, Q.n, (int)Q.n, g->urows, g->urows + Q.n);
  FS_TRY(launch_check("k_unc_compact"));
  int32_t cnt = 0;
  FS_HIP(hipMemcpyAsync(&cnt, g->urows + Q.n, sizeof(cnt), hipMemcpyDeviceToHost, g->stream));
  FS_HIP(hipStreamSynchronize(g->stream));
  g->n_exact_thr = cnt;
  if (cnt == 0) return FS_OK;
  const int nbatch = (cnt + B - 1) / B;
  std::vector<int32_t> bc((size_t)nbatch);
  for (int b = 0; b < nbatch; b++) bc[b] = std::min(B, cnt - b * B);
  FS_TRY(h2d(g, g->bcnt, bc.data(), bc.size()));
  for (int b = 0; b < nbatch; b++) {
    const int32_t* rows = g->urows + (int64_t)b * B;
    k_row_exact_parts<float><<<dim3((unsigned)nchunk, ngroups), 256, 0, g->stream>>>(
        (const float*)g->x, Q.n, Q.p_in, Q.pc, Q.PC, Q.pd, g->src_col, g->scl, rows, g->bcnt + b,
        B, g->uparts);
    FS_TRY(launch_check("k_row_exact_parts"));
    k_row_exact_thr<<<(unsigned)B, 64, 0, g->stream>>>(g->uparts, nchunk, rows, g->bcnt + b, B,
                                                        Q.n, Q.SC, g->thr);
    FS_TRY(launch_check("k_row_exact_thr"));
  }
  FS_HIP(hipStreamSynchronize(g->stream));  // bc
  if (trace_on()) {
    char msg[128];
    snprintf(msg, sizeof msg, "select: %d rows near a refined pair (exact thresholds, all)", cnt);
    trace_mark(msg);
  }
  return FS_OK;
}

static int exact_thresholds(Plan* g) {
  const Prepared& Q = g->P;
  if (Q.ref_accum && !g->thr_all) return exact_thresholds_all(g);
  const int64_t nchunk = (Q.n + kExChunk - 1) / kExChunk;
  const unsigned ngroups = (unsigned)((g->thr_rows + kExRows - 1) / kExRows);
  if (g->thr_all) {  // test hook: flag every row
    std::vector<int32_t> all((size_t)Q.n + 1);
    for (int64_t i = 0; i < Q.n; i++) all[i] = (int32_t)i;
    all[Q.n] = (int32_t)Q.n;
    FS_TRY(h2d(g, g->urows, all.data(), all.size()));  // rows, then the count at thr_rows = n
  } else {
    k_unc_compact<<<1, 1024, 0, g->stream>>>(g->unc, Q.n, g->thr_rows, g->urows,
                                             g->urows + g->thr_rows);
    FS_TRY(launch_check("k_unc_compact"));
  }
  const int32_t* nrows = g->urows + g->thr_rows;
  if (g->x_is_f64)
    k_row_exact_parts<double><<<dim3((unsigned)nchunk, ngroups), 256, 0, g->stream>>>(
        (const double*)g->x, Q.n, Q.p_in, Q.pc, Q.PC, Q.pd, g->src_col, g->scl, g->urows, nrows,
        g->thr_rows, g->uparts);
  else
    k_row_exact_parts<float><<<dim3((unsigned)nchunk, ngroups), 256, 0, g->stream>>>(
        (const float*)g->x, Q.n, Q.p_in, Q.pc, Q.PC, Q.pd, g->src_col, g->scl, g->urows, nrows,
        g->thr_rows, g->uparts);
  FS_TRY(launch_check("k_row_exact_parts"));
  k_row_exact_thr<<<(unsigned)g->thr_rows, 64, 0, g->stream>>>(g->uparts, nchunk, g->urows, nrows,
                                                               g->thr_rows, Q.n, Q.SC, g->thr);
  FS_TRY(launch_check("k_row_exact_thr"));
  if (trace_on()) {
    int32_t cnt = 0;
    FS_HIP(hipMemcpyAsync(&cnt, nrows, sizeof(cnt), hipMemcpyDeviceToHost, g->stream));
    FS_HIP(hipStreamSynchronize(g->stream));
    g->n_exact_thr = cnt <= g->thr_rows ? cnt : -1;
    char msg[128];
    snprintf(msg, sizeof msg, "select: %d rows near a refined pair (%s)", cnt,
             cnt <= g->thr_rows ? "exact thresholds" : "too many: quantised thresholds kept");
    trace_mark(msg);
  }
  return FS_OK;
}

// Pair weights of the owned tiles in the form pass 2 reads (dense or sparse).
static int run_weights(Plan* g, const double* counts, int algo, double inv_sc) {
  const Prepared& Q = g->P;
  if (g->n_tiles == 0) return FS_OK;
  if (g->sparse) {
    FS_HIP(hipMemsetAsync(g->nnz, 0, sizeof(unsigned long long), g->stream));
    g->nnz_valid = true;
    k_weights_sparse2<<<(unsigned)g->n_tiles, 64 * kSWaves, 0, g->stream>>>(
        g->D, Q.n, Q.n_pad, g->tiled, g->win, g->tiles, g->thr, g->lab, counts, algo,
        Q.use_star, inv_sc, g->r_lo, g->r_hi, g->ent, g->nnz);
    return launch_check("k_weights_sparse2");
  }
  k_weights<<<(unsigned)g->n_tiles, 256, 0, g->stream>>>(g->D, Q.n, Q.n_pad, g->tiled, g->win,
                                                         g->tiles,
                                                         g->thr,
                                                         g->lab, counts, algo, Q.use_star, inv_sc,
                                                         g->r_lo, g->r_hi, g->Wt);
  return launch_check("k_weights");
}

static int run_pass2(Plan* g, double* scores_dev) {
  const Prepared& Q = g->P;
  const int64_t nfb = (Q.PW + 127) / 128;
  FS_HIP(hipMemsetAsync(scores_dev, 0, sizeof(double) * Q.n_kept, g->stream));
  if (g->n_tiles == 0) return FS_OK;
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
                                                                   g->out_pos, scores_dev);
  return launch_check("k_reduce");
}

int plan_pass1(Plan* g, double* rowstats) {
  const Prepared& Q = g->P;
  FS_TRY(run_quantize_dist(g));
  if (g->n_tiles > 0) {
    k_tile_rowstats<<<(unsigned)g->n_tiles, 256, 0, g->stream>>>(g->D, Q.n, g->tiles, g->rspart);
    FS_TRY(launch_check("k_tile_rowstats"));
  }
  FS_HIP(hipStreamWaitEvent(g->stream, g->ev_join, 0));  // corr (side stream)
  k_rowstats_reduce<<<(unsigned)((Q.n + 255) / 256), 256, 0, g->stream>>>(
      g->rspart, Q.n, g->nb, g->rank, g->world, g->corr, rowstats);
  FS_TRY(launch_check("k_rowstats_reduce"));
  if (g->own_stream) FS_HIP(hipStreamSynchronize(g->stream));
  return FS_OK;
}

int plan_select(Plan* g, const double* rowstats, double* counts) {
  const Prepared& Q = g->P;
  FS_HIP(hipSetDevice(g->device));
  k_thr_ms<<<(unsigned)((Q.n + 255) / 256), 256, 0, g->stream>>>(rowstats, Q.n, g->thr);
  FS_TRY(launch_check("k_thr_ms"));
  // a threshold's error in integer units: about the band's sigma (band / 12)
  // over sqrt(n - 1) (exact_thresholds); 12 of those plus 2 units of slack
  const double band = Q.amb_delta * Q.SC;
  const double thr_tol = band / std::sqrt((double)std::max<int64_t>(Q.n - 1, 1)) + 2.0;
  FS_HIP(hipMemsetAsync(g->unc, 0, sizeof(unsigned int) * Q.n_pad, g->stream));
  FS_TRY(refine_pairs(g, ALGO_MULTISURF, band, thr_tol, g->unc));
  FS_TRY(exact_thresholds(g));
  FS_HIP(hipMemsetAsync(counts, 0, sizeof(double) * 2 * Q.n, g->stream));
  if (g->n_tiles > 0) {
    k_tile_counts<<<(unsigned)g->n_tiles, 256, 0, g->stream>>>(g->D, Q.n, g->tiles, g->lab,
                                                               g->thr, counts);
    FS_TRY(launch_check("k_tile_counts"));
  }
  if (g->own_stream) FS_HIP(hipStreamSynchronize(g->stream));
  return FS_OK;
}

// Reference-order pass 2 (P.ref_accum), split at the point where every
// owned tile's decisions are known: ref_masks writes the masks of the
// current shard's tiles; ref_chains, once every tile of the triangle has
// written its masks, runs the chains of the focal rows [r_lo, r_hi) and the
// float32 column sums into scores[n_kept] (as doubles; the reference's
// float32 sums, not yet divided by n).
static int ref_masks(Plan* g) {
  const Prepared& Q = g->P;
  return refacc::multisurf_masks(g->D, Q.n, Q.n_pad, g->tiles, g->n_tiles, g->thr, g->lab,
                                 Q.use_star, g->masks, g->stream);
}

// temp[rows][Kp] (float32 rows of the reference's temp matrix), kept between
// steps and grown on demand.
static int ref_temp(Plan* g, int64_t rows, float** out) {
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

static int ref_chains(Plan* g, const double* counts, double* scores) {
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

int plan_pass2(Plan* g, const double* counts, double* scores) {
  const Prepared& Q = g->P;
  FS_HIP(hipSetDevice(g->device));
  if (Q.ref_accum) {
    if (g->world > 1) {
      set_error("reference-order accumulation: pass 2 needs every pair tile's decisions in one "
                "plan (world 1; the one-shot calls shard internally)");
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

int plan_set_rows(Plan* g, int64_t r_lo, int64_t r_hi) {
  if (g->P.algo != ALGO_MULTISURF) {
    set_error("focal-row slices of a plan are MultiSURF-only (ReliefF / SURF: row plans)");
    return FS_EINVAL;
  }
  g->r_lo = r_lo;
  g->r_hi = r_hi;
  return FS_OK;
}

int plan_info(const Plan* g, int64_t* tiles, double* pfe, int64_t* refined) {
  if (tiles) *tiles = g->n_tiles;
  if (pfe) {
    // pairs visited by both passes (diagonal tiles count their full 128x128
    // pass-1 work) x real features
    *pfe = 2.0 * (double)g->n_tiles * kTile * kTile * (double)(g->P.pc + g->P.pd);
  }
  if (refined) *refined = g->n_refined;
  return FS_OK;
}

int plan_calibration(const Plan* g, double* out) {
  for (int k = 0; k < 7; k++) out[k] = g->calib[k];
  out[7] = g->P.SC;
  return FS_OK;
}

int plan_weighted_pairs(Plan* g, int64_t* pairs) {
  *pairs = -1;
  if (!g->sparse || !g->nnz_valid) return FS_OK;
  FS_HIP(hipSetDevice(g->device));
  unsigned long long v = 0;
  FS_HIP(hipMemcpyAsync(&v, g->nnz, sizeof(v), hipMemcpyDeviceToHost, g->stream));
  FS_HIP(hipStreamSynchronize(g->stream));
  *pairs = (int64_t)v;
  return FS_OK;
}

double plan_kernel_ms(const Plan* g, int which) {
  float ms = -1.0f;
  if (which < 0 || which > 2) return -1.0;
  hipEvent_t a = g->ev[2 * which], b = g->ev[2 * which + 1];
  if (hipEventSynchronize(b) != hipSuccess || hipEventElapsedTime(&ms, a, b) != hipSuccess) {
    (void)hipGetLastError();
    return -1.0;
  }
  return (double)ms;
}

// ---- one-shot runs --------------------------------------------------------

static int finish_scores(Plan* g, double* scores_dev, float* scores_out) {
  const Prepared& Q = g->P;
  std::vector<double> h(Q.n_kept);
  FS_HIP(hipMemcpyAsync(h.data(), scores_dev, sizeof(double) * Q.n_kept, hipMemcpyDeviceToHost,
                        g->stream));
  FS_HIP(hipStreamSynchronize(g->stream));
  for (int64_t k = 0; k < Q.n_kept; k++) scores_out[k] = (float)(h[k] / (double)Q.n);
  return FS_OK;
}

// Tile shards a device needs for a MultiSURF job of `world` ranks: the
// tile-sized buffers (~260 KB per tile: the tiled distance block, the
// pass-2 weight streams, partials) of a rank's 1/world of the n_pad^2/2/128^2
// tiles, against the free device memory left after the per-sample buffers
// (X, quantised operands, pass-2 operands, correction terms: ~16 n PW
// bytes) and a 15% reserve.  1 when everything fits; FS_SHARDS forces it.
int multisurf_shards(const Prepared& P, int device, int world, int share) {
  if (const char* e = std::getenv("FS_SHARDS"))
    if (std::atoi(e) >= 1) return std::atoi(e);
  size_t free_b = 0, total_b = 0;
  if (hipSetDevice(device) != hipSuccess || hipMemGetInfo(&free_b, &total_b) != hipSuccess) {
    (void)hipGetLastError();
    return 1;
  }
  const int64_t nb = P.n_pad / kTile;
  const double tiles = (double)nb * (nb + 1) / 2.0 / (double)std::max(world, 1);
  const double per_tile = 2.0 * kTile * kTile * 8.0 + 8.0 * kTile * 256.0 / 2.0;
  const double fixed = 16.0 * (double)P.n_pad * (double)P.PW + 8.0 * (double)P.n * 64.0;
  const double avail = 0.85 * (double)free_b / (double)std::max(share, 1) - fixed;
  if (avail <= 0.0) return 1;  // not even the samples fit: let the allocation report it
  const double v = std::ceil(tiles * per_tile / avail);
  return (int)std::max(1.0, std::min(v, 4096.0));
}

// One MultiSURF scoring pass on a single device in V tile shards (V > 1 when
// the tile buffers of the whole triangle exceed the device: n beyond HBM).
// The distances of a shard are recomputed in each of the three rounds (row
// moments; thresholds -> refinement -> neighbour counts; weights -> pass 2),
// because no shard's distances are kept while another shard runs: 3x the
// pass-1 work for O(n p + n^2 / V) device memory.  The reference streams
// each focal sample's distance row the same way (MultiSURF.py:174-214).
// V == 1 is the plain pass1 / select / pass2 sequence.
static int run_multisurf_shards(Plan* g, int shards, int rank, int world, double* rs, double* cnt,
                                double* sc) {
  const Prepared& Q = g->P;
  if (shards <= 1) {
    FS_TRY(plan_pass1(g, rs));
    FS_TRY(plan_select(g, rs, cnt));
    return plan_pass2(g, cnt, sc);
  }
  double *rs_v = nullptr, *cnt_v = nullptr, *sc_v = nullptr;
  FS_TRY(dalloc(g, &rs_v, 3 * Q.n));
  FS_TRY(dalloc(g, &cnt_v, 2 * Q.n));
  FS_TRY(dalloc(g, &sc_v, Q.n_kept));
  const int W = world * shards;
  auto add = [&](double* dst, const double* src, int64_t count, bool first) -> int {
    if (first)
      return hipMemcpyAsync(dst, src, sizeof(double) * count, hipMemcpyDeviceToDevice,
                            g->stream) == hipSuccess
                 ? FS_OK
                 : FS_EHIP;
    k_accumulate<<<(unsigned)((count + 255) / 256), 256, 0, g->stream>>>(dst, src, count);
    return launch_check("k_accumulate");
  };
  for (int v = 0; v < shards; v++) {  // round 1: row moments
    FS_TRY(plan_set_shard(g, rank + world * v, W));
    FS_TRY(plan_pass1(g, rs_v));
    FS_TRY(add(rs, rs_v, 3 * Q.n, v == 0));
  }
  for (int v = 0; v < shards; v++) {  // round 2: thresholds, refinement, counts
    FS_TRY(plan_set_shard(g, rank + world * v, W));
    FS_TRY(plan_pass1(g, rs_v));
    FS_TRY(plan_select(g, rs, cnt_v));
    FS_TRY(add(cnt, cnt_v, 2 * Q.n, v == 0));
  }
  if (Q.ref_accum) {
    // reference order: every shard's decisions into the masks, then the
    // chains of all focal rows once (one device holds the whole job here)
    if (world != 1) {
      set_error("reference-order accumulation: one device per job in the one-shot calls");
      return FS_ENOTSUP;
    }
    for (int v = 0; v < shards; v++) {
      FS_TRY(plan_set_shard(g, rank + world * v, W));
      FS_TRY(plan_pass1(g, rs_v));
      FS_TRY(plan_select(g, rs, cnt_v));
      FS_TRY(ref_masks(g));
    }
    return ref_chains(g, cnt, sc);
  }
  for (int v = 0; v < shards; v++) {  // round 3: weights, pass 2
    FS_TRY(plan_set_shard(g, rank + world * v, W));
    FS_TRY(plan_pass1(g, rs_v));
    FS_TRY(plan_select(g, rs, cnt_v));
    FS_TRY(plan_pass2(g, cnt, sc_v));
    FS_TRY(add(sc, sc_v, Q.n_kept, v == 0));
  }
  return FS_OK;
}

// Decision risk of a MultiSURF score vector computed with 16-bit pass-1
// operands.  Their thresholds mu - sigma/2 take mu exactly (the quantised row
// sums minus the exact mean correction, fs_colsort.hip) but sigma from the
// quantised second moment: with pair errors e_ij of std sqrt(pc/6) quanta,
// independent of D_ij, sigma_q - sigma = cov_j(D_ij - mu_i, e_ij) / sigma_i
// has std ~ sqrt(pc/6) / sqrt(n) quanta, so T_i errs by about half that
// (kQ16ThrErr keeps a factor 2 of margin: sqrt(pc/6 + 1) / sqrt(n)).  Every
// pair whose exact distance lies between the two thresholds is decided
// differently from MultiSURF.py:193-217.  Row i holds ~ n * phi(1/2) / sigma_i
// such pairs per quantum of T error (Gaussian row distances, phi(1/2) =
// 0.352); each moves one sample across its near boundary, changing the row's
// hit or miss average by ~ dbar / m_i (m_i = the smaller of its near hit /
// miss counts, dbar the mean per-feature diff from the rows' mean distances,
// x2 for the features above the mean), i.e. the final score (divided by n)
// by dbar / (n m_i).  With random signs the expected score error is
// sqrt(sum_i flips_i * effect_i^2); the risk is that over max |score|.
// Measured against the oracle (tests/test_gpu_families.py): uniform noise
// with unrelated labels, n = 16384, is signal-free and trips it; cfg4
// (make_classification) does not.  Above kQ16MaxRisk a MultiSURF plan
// re-scores on 32-bit operands (plan_decision_guard).
constexpr double kQ16MaxRisk = 5e-6;
static thread_local double g_last_risk = -1.0;
static thread_local int g_last_rerun = 0;

static double q16_decision_risk(const Prepared& P, const double* rs, const double* cnt,
                                const double* sums) {
  const double n = (double)P.n, nm1 = n - 1.0;
  double smax = 0.0;
  for (int64_t k = 0; k < P.n_kept; k++)
    smax = std::max(smax, (double)std::fabs((float)(sums[k] / n)));
  const double nfeat = (double)(P.pc + P.pd);
  if (n < 3.0 || nfeat <= 0.0 || P.SC <= 0.0) return 0.0;
  if (smax <= 0.0) return HUGE_VAL;
  const double thr_err = std::sqrt((double)P.pc / 6.0 + 1.0) / std::sqrt(n);
  double mu_sum = 0.0;
  for (int64_t i = 0; i < P.n; i++) mu_sum += (rs[3 * i] - rs[3 * i + 2]) / nm1;
  const double dbar = 2.0 * mu_sum / n / (P.SC * nfeat);
  double acc = 0.0;
  for (int64_t i = 0; i < P.n; i++) {
    const double mu = rs[3 * i] / nm1, var = rs[3 * i + 1] / nm1 - mu * mu;
    if (!(var > 0.0)) continue;
    const double flips = n * 0.352 * thr_err / std::sqrt(var);
    const double m = std::max(1.0, std::min(cnt[2 * i], cnt[2 * i + 1]));
    const double eff = dbar / (n * m);
    acc += flips * eff * eff;
  }
  return std::sqrt(acc) / smax;
}

// After a MultiSURF step with 16-bit operands: the decision risk from the
// step's exchange vectors (rowstats[3n], counts[2n], score sums[n_kept],
// device memory, summed over every rank and shard -- so every rank computes
// the same risk and decides alike).  Above kQ16MaxRisk the plan is switched
// to 32-bit operands for good (its layout and shard rebuilt; X stays on the
// device) and *switched = 1: the caller runs the step again.  risk = -1 when
// there is nothing to check (32-bit operands, MultiSURF*, FS_Q16 forcing).
int plan_decision_guard(Plan* g, const double* rowstats, const double* counts,
                        const double* sums, double* risk, int* switched) {
  *risk = -1.0;
  *switched = 0;
  const Prepared& Q = g->P;
  const char* force = std::getenv("FS_Q16");
  if (Q.algo != ALGO_MULTISURF || !g->use_q16 || Q.use_star || (force && *force)) return FS_OK;
  // a focal-row slice holds only its rows' partial sums: as the one-shot
  // slice calls (multisurf_rows, a partial multisurf_run_devices), no check
  // (max |score| of a partial sum would inflate the risk)
  if (g->r_lo != 0 || g->r_hi != Q.n) return FS_OK;
  FS_HIP(hipSetDevice(g->device));
  std::vector<double> h((size_t)(5 * Q.n + Q.n_kept));
  FS_HIP(hipMemcpyAsync(h.data(), rowstats, sizeof(double) * 3 * Q.n, hipMemcpyDeviceToHost,
                        g->stream));
  FS_HIP(hipMemcpyAsync(h.data() + 3 * Q.n, counts, sizeof(double) * 2 * Q.n,
                        hipMemcpyDeviceToHost, g->stream));
  FS_HIP(hipMemcpyAsync(h.data() + 5 * Q.n, sums, sizeof(double) * Q.n_kept,
                        hipMemcpyDeviceToHost, g->stream));
  FS_HIP(hipStreamSynchronize(g->stream));
  *risk = q16_decision_risk(Q, h.data(), h.data() + 3 * Q.n, h.data() + 5 * Q.n);
  if (!(*risk > kQ16MaxRisk)) return FS_OK;
  trace_mark("multisurf: 16-bit decision risk above bound, 32-bit operands");
  g->use_q16 = 0;
  g->P.no_q16 = 1;
  FS_TRY(plan_layout(g));
  FS_TRY(plan_set_shard(g, g->rank, g->world));
  *switched = 1;
  return FS_OK;
}

int multisurf_last_guard(double* risk, int* rerun) {
  if (risk) *risk = g_last_risk;
  if (rerun) *rerun = g_last_rerun;
  return FS_OK;
}

int multisurf_run(const Prepared& P, const void* x, int device, float* scores_out) {
  Plan* g = nullptr;
  g_last_risk = -1.0;
  g_last_rerun = 0;
  const int shards = multisurf_shards(P, device, 1);
  FS_TRY(plan_create(&g, P, x, 0, device, 0, shards, 0));
  double *rs = nullptr, *cnt = nullptr, *sc = nullptr;
  int rc, switched = 0;
  double risk = -1.0;
  if ((rc = dalloc(g, &rs, 3 * P.n)) || (rc = dalloc(g, &cnt, 2 * P.n)) ||
      (rc = dalloc(g, &sc, P.n_kept)) || (rc = run_multisurf_shards(g, shards, 0, 1, rs, cnt, sc)) ||
      (rc = plan_decision_guard(g, rs, cnt, sc, &risk, &switched)) ||
      (switched && (rc = run_multisurf_shards(g, shards, 0, 1, rs, cnt, sc))) ||
      (rc = finish_scores(g, sc, scores_out))) {
    plan_destroy(g);
    return rc;
  }
  g_last_risk = risk;
  g_last_rerun = switched;
  plan_destroy(g);
  return FS_OK;
}

static int copy_sums(Plan* g, const double* sums_dev, double* sums_out) {
  FS_HIP(hipMemcpyAsync(sums_out, sums_dev, sizeof(double) * g->P.n_kept, hipMemcpyDeviceToHost,
                        g->stream));
  FS_HIP(hipStreamSynchronize(g->stream));
  return FS_OK;
}

int multisurf_rows(const Prepared& P, const void* x, int device, int64_t r_lo, int64_t r_hi,
                   double* sums_out) {
  Plan* g = nullptr;
  const int shards = multisurf_shards(P, device, 1);
  FS_TRY(plan_create(&g, P, x, 0, device, 0, shards, 0));
  double *rs = nullptr, *cnt = nullptr, *sc = nullptr;
  int rc;
  if ((rc = plan_set_rows(g, r_lo, r_hi)) || (rc = dalloc(g, &rs, 3 * P.n)) ||
      (rc = dalloc(g, &cnt, 2 * P.n)) || (rc = dalloc(g, &sc, P.n_kept)) ||
      (rc = run_multisurf_shards(g, shards, 0, 1, rs, cnt, sc)) ||
      (rc = copy_sums(g, sc, sums_out))) {
    plan_destroy(g);
    return rc;
  }
  plan_destroy(g);
  return FS_OK;
}

// SURF score sums of the plan's focal rows into sums_dev[n_kept].
static int plan_score_surf(Plan* g, double* sums_dev) {
  const Prepared& Q = g->P;
  int rc = run_quantize_dist(g);  // float64 distances, real units
  if (rc == FS_OK && g->r_hi > g->r_lo) {
    k_surf_avg<<<(unsigned)((g->r_hi - g->r_lo + 63) / 64), 64, 0, g->stream>>>(
        g->D, Q.n, Q.n_pad, 1.0, g->r_lo, g->r_hi, g->thr);
    rc = launch_check("k_surf_avg");
  }
  if (rc == FS_OK) rc = run_weights(g, nullptr, ALGO_SURF, 1.0);
  if (rc == FS_OK) rc = run_pass2(g, sums_dev);
  return rc;
}

// Rows per panel of a ReliefF / SURF one-shot call: a plan stores the
// distance rows of its focal blocks (d_row_in), ~n_pad * 8 bytes per row plus
// its share of the pass-2 weights and selection scratch (~n_pad * 16 more),
// beside the per-sample buffers (X, the quantised and pass-2 operands:
// ~20 n_pad PW bytes).  Focal ranges whose rows exceed 80% of the free
// device memory are scored in panels of whole 128-sample blocks, one plan
// each, and their sums added -- the reference streams each focal sample's
// distance row the same way (ReliefF.py:143-157, SURF.py:139-163).
// The row_panel test hook forces the panel height.
static int64_t row_panel_rows(const Prepared& P, int device, int64_t rows) {
  if (const int64_t e = test_hooks().row_panel; e >= 1)
    return std::max<int64_t>(kTile, e / kTile * kTile);
  size_t free_b = 0, total_b = 0;
  if (hipSetDevice(device) != hipSuccess || hipMemGetInfo(&free_b, &total_b) != hipSuccess) {
    (void)hipGetLastError();
    return rows;
  }
  const double fixed = 20.0 * (double)P.n_pad * (double)P.PW + 8.0 * (double)P.n * (double)P.p_in;
  // a stored row of D (8 bytes per sample; ReliefF's float32 keys 4) plus
  // the per-row scratch
  const double per_row = (P.algo == ALGO_RELIEFF ? 20.0 : 24.0) * (double)P.n_pad;
  const double avail = 0.8 * (double)free_b - fixed;
  if (avail <= per_row * kTile) return kTile;  // let the allocation report it
  const int64_t fit = (int64_t)(avail / per_row) / kTile * kTile;
  return std::max<int64_t>(kTile, std::min<int64_t>(fit, (rows + kTile - 1) / kTile * kTile));
}

// Score [r_lo, r_hi) in panels of `panel` rows (block-aligned), summing the
// panels' float64 sums in panel order.
template <typename Fn>
static int run_panels(const Prepared& P, int64_t r_lo, int64_t r_hi, int64_t panel,
                      double* sums_out, Fn&& one) {
  std::fill(sums_out, sums_out + P.n_kept, 0.0);
  std::vector<double> part((size_t)P.n_kept);
  for (int64_t lo = r_lo; lo < r_hi;) {
    const int64_t hi = std::min(r_hi, (lo / kTile * kTile) + panel);
    FS_TRY(one(lo, hi, part.data()));
    for (int64_t k = 0; k < P.n_kept; k++) sums_out[k] += part[k];
    lo = hi;
  }
  return FS_OK;
}

static int surf_run_one(const Prepared& P, const void* x, int device, int64_t r_lo, int64_t r_hi,
                        double* sums_out);
static int relieff_run_one(const Prepared& P, const void* x, int device, int64_t r_lo,
                           int64_t r_hi, double* sums_out, const double* seed = nullptr);

int surf_run(const Prepared& P, const void* x, int device, int64_t r_lo, int64_t r_hi,
             double* sums_out) {
  const int64_t panel = row_panel_rows(P, device, r_hi - r_lo);
  if (r_hi - r_lo <= panel) return surf_run_one(P, x, device, r_lo, r_hi, sums_out);
  return run_panels(P, r_lo, r_hi, panel, sums_out, [&](int64_t lo, int64_t hi, double* o) {
    return surf_run_one(P, x, device, lo, hi, o);
  });
}

int relieff_run(const Prepared& P, const void* x, int device, int64_t r_lo, int64_t r_hi,
                double* sums_out) {
  const int64_t panel = row_panel_rows(P, device, r_hi - r_lo);
  if (r_hi - r_lo <= panel) return relieff_run_one(P, x, device, r_lo, r_hi, sums_out);
  if (P.ref_accum) {
    // one float32 column sum over all panels, each continuing the last
    std::vector<double> prev((size_t)P.n_kept, 0.0);
    for (int64_t lo = r_lo; lo < r_hi;) {
      const int64_t hi = std::min(r_hi, (lo / kTile * kTile) + panel);
      FS_TRY(relieff_run_one(P, x, device, lo, hi, sums_out, lo == r_lo ? nullptr : prev.data()));
      std::copy(sums_out, sums_out + P.n_kept, prev.begin());
      lo = hi;
    }
    return FS_OK;
  }
  return run_panels(P, r_lo, r_hi, panel, sums_out, [&](int64_t lo, int64_t hi, double* o) {
    return relieff_run_one(P, x, device, lo, hi, o);
  });
}

static int surf_run_one(const Prepared& P, const void* x, int device, int64_t r_lo, int64_t r_hi,
                        double* sums_out) {
  Plan* g = nullptr;
  FS_TRY(plan_create(&g, P, x, 1, device, 0, 1, 0, r_lo, r_hi));
  double* sc = nullptr;
  int rc = dalloc(g, &sc, g->P.n_kept);
  if (rc == FS_OK) rc = plan_score_surf(g, sc);
  if (rc == FS_OK) rc = copy_sums(g, sc, sums_out);
  plan_destroy(g);
  return rc;
}

// ReliefF neighbour selection on the resident distances: quantised keys,
// exact reference keys for every candidate near a class's k-th key, exact
// selection, then numba's quicksort order for rows with ties at the k-th key.
static int relieff_select(Plan* g, const int64_t* dcc, int32_t* nbr, int32_t* nfound) {
  const Prepared& Q = g->P;
  const int C = Q.n_classes;
  const int64_t k = Q.k_neighbors, n = Q.n;
  const int64_t r_lo = g->r_lo, nr_own = g->r_hi - g->r_lo;  // focal rows of this plan
  const double inv_sc = 1.0 / Q.SC;
  if (nr_own <= 0) return FS_OK;
  uint32_t* tkey = nullptr;
  int32_t *tneed = nullptr, *teq = nullptr;
  g->alloc_target = 2;  // per-call temporaries
  FS_TRY(dalloc(g, &tkey, (size_t)n * C));
  FS_TRY(dalloc(g, &tneed, (size_t)n * C));
  FS_TRY(dalloc(g, &teq, (size_t)n * C));
  g->alloc_target = 0;
  // histograms: 1024 bins per class for n_classes <= 8 (10-bit first digit);
  // staged rows: 4 B of key + 1 B of class code per sample (by quads), for
  // n <= 32768 (one round trip of 8 quads per thread)
  const size_t shbytes = (size_t)C * (C <= 8 ? 1024 : 256) * 4;
  const size_t nq = (size_t)(n + 3) / 4;
  const size_t shstage = shbytes + nq * 20;
  // (k_rf_select's static LDS, 2.2 KB, comes out of the same 160 KB)
  constexpr size_t kSelLds = 157 * 1024;
  const bool stage = n <= 32768 && shstage <= kSelLds;
  // the rest of the 160 KB: the exact keys' gather buffer (x_i, the scales,
  // the column indices and at least one candidate row at the continuous
  // columns), else none (the unstaged kernel keeps to 40 KB: four
  // workgroups per CU)
  size_t shsel = stage ? shstage : shbytes;
  int xlds = 0;
  const size_t lds_cap = stage ? kSelLds : 40 * 1024;
  const size_t lds_left = lds_cap > shsel + 16 ? lds_cap - 16 - shsel : 0;
  if (Q.pc > 0 && lds_left / 4 >= (size_t)Q.pc * 4) xlds = (int)(lds_left / 4);
  if (const int64_t v = test_hooks().rf_xlds; v >= 0) {  // tests: a cap in floats
    if (v < xlds) xlds = v >= 4 * Q.pc ? (int)v : 0;
  }
  if (xlds) shsel += 16 + (size_t)xlds * 4;
  if (shsel > 64 * 1024) {
    if (stage)
      FS_HIP(hipFuncSetAttribute((const void*)k_rf_select<true>,
                                 hipFuncAttributeMaxDynamicSharedMemorySize, (int)shsel));
    else
      FS_HIP(hipFuncSetAttribute((const void*)k_rf_select<false>,
                                 hipFuncAttributeMaxDynamicSharedMemorySize, (int)shsel));
  }
  // band of the exact-key refinement (quantisation error + float32 rounding)
  const double band_abs = 2.0 * Q.amb_delta, band_rel = 2.0 * 1.2e-7;
  // One launch: selection on the quantised keys, the reference's keys for
  // the candidates inside the band around each k-th key (computed in the
  // kernel, k_exact_pairs' arithmetic), the exact k-th keys, ordered
  // collection.
  // Continuous features only need the exact keys (discrete distances are
  // exact integers already).
  const float* xk = Q.pc > 0 ? (const float*)g->x : nullptr;
  // candidates listed in LDS per row (above: the general route); the rf_fcap
  // test hook lowers it (0 forces the general route)
  int fcap = 256;
  if (test_hooks().rf_fcap >= 0) fcap = (int)std::min<int64_t>(256, test_hooks().rf_fcap);
  FS_HIP(hipMemsetAsync(g->list_count, 0, sizeof(unsigned long long), g->stream));
  FS_HIP(hipEventRecord(g->ev[4], g->stream));
  if (stage)
    k_rf_select<true><<<(unsigned)nr_own, 1024, shsel, g->stream>>>(
        g->Dk, (int)n, Q.n_pad, g->lab, g->lab8, dcc, C, (int)k, r_lo, tkey, tneed, teq, nbr,
        nfound, band_abs, band_rel, fcap, g->list_count, xk, Q.p_in, (int)Q.pc, (int)Q.PC,
        (int)Q.pd, g->src_col, g->scl, xlds);
  else
    k_rf_select<false><<<(unsigned)nr_own, 256, shsel, g->stream>>>(
        g->Dk, (int)n, Q.n_pad, g->lab, g->lab8, dcc, C, (int)k, r_lo, tkey, tneed, teq, nbr,
        nfound, band_abs, band_rel, fcap, g->list_count, xk, Q.p_in, (int)Q.pc, (int)Q.PC,
        (int)Q.pd, g->src_col, g->scl, xlds);
  FS_TRY(launch_check("k_rf_select"));
  FS_HIP(hipEventRecord(g->ev[5], g->stream));
  // exact keys computed (list_count), read with the tie counts below
  unsigned long long ex_cnt = 0;
  FS_HIP(hipMemcpyAsync(&ex_cnt, g->list_count, sizeof(ex_cnt), hipMemcpyDeviceToHost, g->stream));
  // 4. rows with more neighbours at the k-th key than needed
  std::vector<int32_t> hneed((size_t)nr_own * C), heq((size_t)nr_own * C);
  FS_HIP(hipMemcpyAsync(hneed.data(), tneed + r_lo * C, hneed.size() * 4, hipMemcpyDeviceToHost,
                        g->stream));
  FS_HIP(hipMemcpyAsync(heq.data(), teq + r_lo * C, heq.size() * 4, hipMemcpyDeviceToHost,
                        g->stream));
  FS_HIP(hipStreamSynchronize(g->stream));
  g->n_refined = (int64_t)ex_cnt;
  std::vector<int32_t> tie_rows;
  for (int64_t r = 0; r < nr_own; r++)
    for (int c = 0; c < C; c++)
      if (hneed[r * C + c] > 0 && heq[r * C + c] > hneed[r * C + c]) {
        tie_rows.push_back((int32_t)(r_lo + r));
        break;
      }
  g->n_tie_rows = (int64_t)tie_rows.size();
  if (tie_rows.empty()) return FS_OK;
  // n <= kTieMwMaxN: 16 waves per row, the row in LDS (6 B per sample)
  const bool mw = n <= kTieMwMaxN && !test_hooks().ties_1w;  // ties_1w: tests
  const size_t mw_lds = ((size_t)n * 6 + 15) & ~(size_t)15;
  int coop_min = 2048;  // ranges the whole workgroup partitions (ties_coop: tests)
  if (test_hooks().ties_coop > 0) coop_min = (int)std::max<int64_t>(16, test_hooks().ties_coop);
  // per-row scratch: exact keys (unless all-discrete under mw) and the
  // one-wave replay's permutation; batches bounded to ~512 MB of it
  const bool need_keys = !(mw && Q.pc == 0);
  // (mw: the cooperative partitions' scratch; else the permutation)
  const int64_t row_bytes = (need_keys ? 4 * n : 0) + 4 * n;
  const int64_t batch = std::max<int64_t>(
      1, std::min<int64_t>((int64_t)tie_rows.size(),
                           row_bytes > 0 ? (int64_t)(512ll << 20) / row_bytes : INT64_MAX));
  int32_t *drows = nullptr, *R = nullptr;
  float* keys = nullptr;
  int* status = nullptr;
  g->alloc_target = 2;
  FS_TRY(dalloc(g, &drows, (size_t)batch));
  FS_TRY(dalloc(g, &R, (size_t)batch * n));
  if (need_keys) FS_TRY(dalloc(g, &keys, (size_t)batch * n));
  FS_TRY(dalloc(g, &status, 1));
  g->alloc_target = 0;
  FS_HIP(hipMemsetAsync(status, 0, sizeof(int), g->stream));
  if (mw)
    FS_HIP(hipFuncSetAttribute((const void*)k_rf_ties_mw,
                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)mw_lds));
  else if (n <= kTieLdsMaxN)
    FS_HIP(hipFuncSetAttribute((const void*)k_rf_ties<true>,
                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)(8 * n)));
  for (int64_t r0 = 0; r0 < (int64_t)tie_rows.size(); r0 += batch) {
    const int64_t nr = std::min<int64_t>(batch, (int64_t)tie_rows.size() - r0);
    FS_TRY(h2d(g, drows, tie_rows.data() + r0, (size_t)nr));
    // (all-discrete: the multi-wave replay reads the plan's keys, exact
    // already, straight from Dk)
    if (need_keys) {
      k_rf_exact_rows<float><<<dim3((unsigned)nr, (unsigned)((n + 3) / 4)), 256, 0, g->stream>>>(
          (const float*)g->x, n, Q.p_in, Q.pc, Q.PC, Q.pd, g->src_col, g->scl, drows, g->D,
          g->Dk, Q.n_pad, inv_sc, keys);
      FS_TRY(launch_check("k_rf_exact_rows"));
    }
    if (mw)
      k_rf_ties_mw<<<(unsigned)nr, 1024, mw_lds, g->stream>>>(
          drows, (int)n, need_keys ? keys : nullptr, g->Dk, Q.n_pad, g->lab, C, (int)k, tkey,
          tneed, teq, nbr, R, coop_min, status);
    else if (n <= kTieLdsMaxN)
      k_rf_ties<true><<<(unsigned)nr, 64, (size_t)8 * n, g->stream>>>(
          drows, n, keys, g->lab, C, k, tkey, tneed, teq, R, nbr, status);
    else
      k_rf_ties<false><<<(unsigned)nr, 64, 0, g->stream>>>(drows, n, keys, g->lab, C, k, tkey,
                                                           tneed, teq, R, nbr, status);
    FS_TRY(launch_check("k_rf_ties"));
  }
  int hstatus = 0;
  FS_HIP(hipMemcpyAsync(&hstatus, status, sizeof(int), hipMemcpyDeviceToHost, g->stream));
  FS_HIP(hipStreamSynchronize(g->stream));
  if (hstatus != 0) {
    set_error(hstatus == 1 ? "ReliefF tie ordering: quicksort stack overflow"
                           : ("ReliefF tie ordering: work queue stalled (status " +
                              std::to_string(hstatus) + ")").c_str());
    return FS_EHIP;
  }
  return FS_OK;
}

// ReliefF score sums of the plan's focal rows into sums_dev[n_kept]:
// pass 1, neighbour selection, then the neighbour-gather update.
static int plan_score_relieff(Plan* g, double* sums_dev) {
  const Prepared& Q = g->P;
  const int C = Q.n_classes;
  const int64_t k = Q.k_neighbors;
  std::vector<int64_t> cc(C, 0);
  for (int64_t i = 0; i < Q.n; i++) cc[Q.labels[i]]++;
  std::vector<double> prior(Q.class_prior);
  double *dprior = nullptr, *part = nullptr;
  int64_t* dcc = nullptr;
  int32_t *nbr = nullptr, *nfound = nullptr;
  const int64_t nrb = std::max<int64_t>(1, (g->r_hi - g->r_lo + kRfRows - 1) / kRfRows);
  int rc;
  g->alloc_target = 2;  // per-call buffers
  rc = dalloc(g, &dprior, C);
  if (rc == FS_OK) rc = dalloc(g, &part, (size_t)nrb * Q.PW);
  if (rc == FS_OK) rc = dalloc(g, &dcc, C);
  if (rc == FS_OK) rc = dalloc(g, &nbr, (size_t)Q.n * C * std::max<int64_t>(k, 1));
  if (rc == FS_OK) rc = dalloc(g, &nfound, (size_t)Q.n * C);
  g->alloc_target = 0;
  if (rc || (rc = h2d(g, dcc, cc.data(), C)) || (rc = h2d(g, dprior, prior.data(), C)) ||
      (rc = run_quantize_dist(g)))
    return rc;
  FS_HIP(hipEventRecord(g->ev[2], g->stream));
  if ((rc = relieff_select(g, dcc, nbr, nfound))) return rc;
  if (trace_on()) {
    (void)hipStreamSynchronize(g->stream);
    std::fprintf(stderr, "[fs_trace] relieff: %lld exact pairs, %lld tie rows\n",
                 (long long)g->n_refined, (long long)g->n_tie_rows);
  }
  if (Q.ref_accum) {
    // the reference's order (fs_refacc.hip): neighbour lists in argsort
    // order, float32 temp rows, float32 sequential column sums, continuing
    // from the previous row panel's sums when seeded (relieff_run)
    const int64_t rows = g->r_hi - g->r_lo;
    const size_t nkeys = (size_t)std::max<int64_t>(rows * C * std::max<int64_t>(k, 1), 1);
    if (nkeys > g->rkeys_cap) {
      if (g->rkeys) dev_free(g->rkeys);
      g->rkeys = nullptr;
      g->rkeys_cap = 0;
      void* p = nullptr;
      FS_TRY(dev_alloc(&p, nkeys * sizeof(float), g->device));
      g->rkeys = (float*)p;
      g->rkeys_cap = nkeys;
    }
    float* temp = nullptr;
    FS_TRY(ref_temp(g, rows, &temp));
    FS_TRY(refacc::relieff_rows(g->xk, g->Kp, g->krecip, g->kdisc, Q.n_kept, g->lab, dprior, C, k,
                                nbr, nfound, g->r_lo, g->r_hi, g->rkeys, temp, g->stream));
    FS_HIP(hipEventRecord(g->ev[3], g->stream));
    if (!g->ref_seeded) FS_HIP(hipMemsetAsync(sums_dev, 0, sizeof(double) * Q.n_kept, g->stream));
    if (rows <= 0) return FS_OK;
    return refacc::column_sums(temp, rows, g->Kp, Q.n_kept, g->ref_seeded ? sums_dev : nullptr,
                                sums_dev, g->stream);
  }
  k_rf_update<<<dim3((unsigned)(Q.PW / 64), (unsigned)nrb), 256, 0, g->stream>>>(
      g->xs, g->r_lo, g->r_hi, Q.PW, Q.PC, g->lab, dprior, C, k, nbr, nfound, part);
  FS_TRY(launch_check("k_rf_update"));
  FS_HIP(hipEventRecord(g->ev[3], g->stream));
  FS_HIP(hipMemsetAsync(sums_dev, 0, sizeof(double) * Q.n_kept, g->stream));
  k_reduce<<<(unsigned)((Q.PW + 63) / 64), 1024, 0, g->stream>>>(part, nrb, Q.PW, g->out_pos,
                                                                   sums_dev);
  return launch_check("k_reduce");
}

static int relieff_run_one(const Prepared& P, const void* x, int device, int64_t r_lo,
                           int64_t r_hi, double* sums_out, const double* seed) {
  if (P.n_classes > 64) {
    set_error("GPU ReliefF supports at most 64 classes");
    return FS_ENOTSUP;
  }
  Plan* g = nullptr;
  FS_TRY(plan_create(&g, P, x, 0, device, 0, 1, 0, r_lo, r_hi));
  double* sc = nullptr;
  int rc = dalloc(g, &sc, g->P.n_kept);
  if (rc == FS_OK && seed) {
    // reference order, a later row panel: the float32 column sums go on
    // from the previous panels' (ReliefF.py:219-220 is one sequential sum)
    g->ref_seeded = true;
    rc = h2d(g, sc, seed, (size_t)g->P.n_kept);
  }
  if (rc == FS_OK) rc = plan_score_relieff(g, sc);
  if (rc == FS_OK) rc = copy_sums(g, sc, sums_out);
  plan_destroy(g);
  return rc;
}

// ReliefF / SURF plans (resident scoring, fs_plan_score): float64 score sums
// of the plan's focal rows into device memory; per-call buffers are freed
// before returning.
int plan_score(Plan* g, double* sums_dev) {
  FS_HIP(hipSetDevice(g->device));
  int rc;
  if (g->P.algo == ALGO_RELIEFF) {
    if (g->P.n_classes > 64) {
      set_error("GPU ReliefF supports at most 64 classes");
      return FS_ENOTSUP;
    }
    rc = plan_score_relieff(g, sums_dev);
  } else if (g->P.algo == ALGO_SURF) {
    rc = plan_score_surf(g, sums_dev);
  } else {
    set_error("fs_plan_score: MultiSURF plans score through pass1 / select / pass2");
    return FS_EINVAL;
  }
  if (hipStreamSynchronize(g->stream) != hipSuccess && rc == FS_OK) rc = FS_EHIP;
  for (void* q : g->scratch) dev_free(q);
  g->scratch.clear();
  return rc;
}

}  // namespace gpu
}  // namespace fs

// ---------------------------------------------------------------------------
// Single-process multi-GPU (the estimators' `devices=`)
// ---------------------------------------------------------------------------
namespace fs {
namespace gpu {

namespace {
// dst[k] = sum over r = 0..N-1, in that order, of parts[r][k]: every device
// sums the gathered vectors in the same order, so all get bit-identical sums
__global__ void k_rank_sum(double* __restrict__ dst, const double* __restrict__ parts, int N,
                           int64_t len) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= len) return;
  double s = 0.0;
  for (int r = 0; r < N; r++) s += parts[(int64_t)r * len + k];
  dst[k] = s;
}

// Peer access between every pair of distinct devices of a devices= call
// (xGMI copies instead of staging through host memory); once per pair.
void enable_peers(const int* devices, int N) {
  static std::mutex mu;
  static std::vector<std::pair<int, int>> done;
  std::lock_guard<std::mutex> lk(mu);
  for (int a = 0; a < N; a++)
    for (int b = 0; b < N; b++) {
      const int da = devices[a], db = devices[b];
      if (da == db) continue;
      if (std::find(done.begin(), done.end(), std::make_pair(da, db)) != done.end()) continue;
      done.emplace_back(da, db);
      int can = 0;
      if (hipDeviceCanAccessPeer(&can, da, db) == hipSuccess && can && hipSetDevice(da) == hipSuccess)
        (void)hipDeviceEnablePeerAccess(db, 0);
      (void)hipGetLastError();  // already enabled, or no peer path: copies still work
    }
}

// One device thread of a devices= call: its plan's stream, an event per
// exchange, and the thread's view of the group (barrier, every thread's
// send buffer and event).
struct DevGroup {
  int N;
  const int* devices;
  StageBarrier bar;
  std::vector<const void*> send;  // per thread: the buffer its peers copy from
  std::vector<hipEvent_t> ready;  // per thread: recorded once `send` holds the data
  explicit DevGroup(int n, const int* d) : N(n), devices(d), bar(n), send(n), ready(n) {}
};

// Thread r's part of an exchange: thread r's `part` (len doubles, on its
// device, complete once its stream reaches this point) is summed over all
// threads into `out` on every device.  Each stream waits for the peers'
// events and copies their parts into `gather` [N][len] (device to device
// over xGMI; a repeated ordinal copies within the device), then k_rank_sum
// adds them in thread order.  Nothing passes through host memory, and no
// thread waits for another's device work on the host: one barrier makes the
// events and buffers visible.  A part must not be rewritten until every peer
// has copied it: the callers give each exchange its own part buffer, and
// every later write to it is ordered behind the next exchange's waits.
bool exchange_parts(DevGroup& G, int r, hipStream_t st, hipEvent_t ev, const double* part,
                    double* gather, double* out, int64_t len, int& rc) {
  int e = rc;
  if (!e && hipEventRecord(ev, st) != hipSuccess) {
    set_error("multi-device exchange: event record failed");
    e = FS_EHIP;
  }
  G.send[r] = part;
  G.ready[r] = ev;
  if (!G.bar.arrive(e, e ? std::string(fs_last_error()) : std::string())) return false;
  for (int k = 0; k < G.N && !rc; k++) {
    if (hipStreamWaitEvent(st, G.ready[k], 0) != hipSuccess ||
        hipMemcpyPeerAsync(gather + (int64_t)k * len, G.devices[r], G.send[k], G.devices[k],
                           sizeof(double) * len, st) != hipSuccess) {
      (void)hipGetLastError();
      set_error("multi-device exchange: peer copy failed");
      rc = FS_EHIP;
    }
  }
  if (!rc) {
    k_rank_sum<<<(unsigned)((len + 255) / 256), 256, 0, st>>>(out, gather, G.N, len);
    rc = launch_check("k_rank_sum");
  }
  // the peers read G.ready / G.send of this exchange before the next
  // exchange's barrier rewrites them: keep them apart with a second barrier
  return G.bar.arrive(rc, rc ? std::string(fs_last_error()) : std::string());
}

// X on every device of a devices= call, moved over the host link once: thread
// r uploads its 1/N of the rows into a full-size buffer on its device, then
// copies the other threads' row ranges from their devices (xGMI peer copies;
// a repeated ordinal copies within the device).  *buf receives the buffer
// (caller frees it after a barrier that follows the last peer copy).
bool distribute_x(DevGroup& G, int r, const void* x, size_t row_bytes, int64_t n, void** buf,
                  hipStream_t st, hipEvent_t ev, int& rc) {
  const int dev = G.devices[r];
  *buf = nullptr;
  if (!rc) rc = dev_alloc(buf, row_bytes * (size_t)n, dev);
  auto lo = [&](int k) { return n * k / G.N; };
  if (!rc && hipMemcpyAsync((char*)*buf + row_bytes * lo(r), (const char*)x + row_bytes * lo(r),
                            row_bytes * (size_t)(lo(r + 1) - lo(r)), hipMemcpyHostToDevice,
                            st) != hipSuccess) {
    (void)hipGetLastError();
    set_error("multi-device X: host-to-device copy of the row share failed");
    rc = FS_EHIP;
  }
  int e = rc;
  if (!e && hipEventRecord(ev, st) != hipSuccess) e = FS_EHIP;
  G.send[r] = *buf;
  G.ready[r] = ev;
  if (!G.bar.arrive(e, e ? std::string(fs_last_error()) : std::string())) return false;
  for (int k = 0; k < G.N && !rc; k++) {
    if (k == r || lo(k + 1) == lo(k)) continue;
    if (hipStreamWaitEvent(st, G.ready[k], 0) != hipSuccess ||
        hipMemcpyPeerAsync((char*)*buf + row_bytes * lo(k), dev,
                           (const char*)G.send[k] + row_bytes * lo(k), G.devices[k],
                           row_bytes * (size_t)(lo(k + 1) - lo(k)), st) != hipSuccess) {
      (void)hipGetLastError();
      set_error("multi-device X: peer copy failed");
      rc = FS_EHIP;
    }
  }
  if (!rc && hipStreamSynchronize(st) != hipSuccess) {
    (void)hipGetLastError();
    rc = FS_EHIP;
  }
  if (r == 0 && trace_on()) {
    char msg[160];
    snprintf(msg, sizeof msg, "devices: X on %d devices (%.1f MB per device over the host link, "
             "the rest peer-copied)", G.N, (double)row_bytes * (double)(lo(1) - lo(0)) / 1e6);
    trace_mark(msg);
  }
  return G.bar.arrive(rc, rc ? std::string(fs_last_error()) : std::string());
}

// how many of devices[0..N) are `d` (plans sharing a device share its memory)
int ordinal_share(const int* devices, int N, int d) {
  int m = 0;
  for (int k = 0; k < N; k++) m += devices[k] == d;
  return std::max(m, 1);
}
}  // namespace

// MultiSURF over several devices from one process: thread r (devices[r],
// repeats allowed) owns the tiles t with t % (N V) == r + N v of the
// upper triangle -- the partition of parallel.py's one-process-per-GPU path.
// X crosses the host link once (distribute_x: 1/N of the rows per device,
// the rest by peer copies), and the three exchange vectors (row moments,
// neighbour counts, score sums) are summed device-side (exchange_parts: peer
// copies of every thread's part, a fixed-order sum on each device) where the
// multi-process path all-reduces them over RCCL.  V > 1 tile shards per
// device when the largest share exceeds a device's memory (sized with the
// device's memory split between the plans that share it).  Focal samples
// [r_lo, r_hi) as fs_multisurf_score_rows; sums (not / n).
int multisurf_run_devices(const Prepared& P, const void* x, const int* devices, int ndev,
                          int64_t r_lo, int64_t r_hi, double* sums_out) {
  const int N = ndev;
  int V = 1;
  for (int r = 0; r < N; r++)
    V = std::max(V, multisurf_shards(P, devices[r], N, ordinal_share(devices, N, devices[r])));
  const int W = N * V;
  const int64_t n = P.n, nk = P.n_kept;
  enable_peers(devices, N);
  DevGroup G(N, devices);
  std::vector<double> result((size_t)nk);
  const bool whole = r_lo == 0 && r_hi == n;
  if (whole) {
    g_last_risk = -1.0;
    g_last_rerun = 0;
  }
  auto worker = [&](int r) {
    Plan* g = nullptr;
    // per exchange: this thread's part, the gathered parts, the sum
    double *rs_p = nullptr, *cnt_p = nullptr, *sc_p = nullptr, *gath = nullptr;
    double *rs = nullptr, *cnt = nullptr, *sc = nullptr, *tmp = nullptr;
    void* xbuf = nullptr;
    uint64_t staged = 0;
    hipStream_t xs_st = nullptr;
    hipEvent_t evs[4] = {nullptr, nullptr, nullptr, nullptr};
    int rc = hipSetDevice(devices[r]) == hipSuccess ? FS_OK : FS_EHIP;
    for (auto& e : evs)
      if (!rc && hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) rc = FS_EHIP;
    if (!rc && hipStreamCreateWithFlags(&xs_st, hipStreamNonBlocking) != hipSuccess) rc = FS_EHIP;
    bool ok = distribute_x(G, r, x, sizeof(float) * (size_t)P.p_in, n, &xbuf, xs_st, evs[0], rc);
    if (ok && !rc) rc = stage_x_device(devices[r], x, xbuf, 0, n, P.p_in, &staged);
    if (ok && !rc) rc = plan_create(&g, P, x, 0, devices[r], r, W, 0);
    if (staged) unstage_x(staged);
    if (ok && !rc) rc = plan_set_rows(g, r_lo, r_hi);
    const int64_t glen = (int64_t)N * std::max<int64_t>(3 * n, nk);
    if (ok && !rc && ((rc = dalloc(g, &rs_p, 3 * n)) || (rc = dalloc(g, &cnt_p, 2 * n)) ||
                      (rc = dalloc(g, &sc_p, nk)) || (rc = dalloc(g, &rs, 3 * n)) ||
                      (rc = dalloc(g, &cnt, 2 * n)) || (rc = dalloc(g, &sc, nk)) ||
                      (rc = dalloc(g, &gath, glen)) ||
                      (rc = dalloc(g, &tmp, std::max<int64_t>(3 * n, nk)))))
      ;
    // every peer has copied its rows of xbuf (the barrier after the copies)
    // and the plan holds its own copy: free it
    if (xbuf) dev_free(xbuf);
    hipStream_t st = g ? g->stream : nullptr;
    auto exch = [&](int which) {
      double* part = which == 0 ? rs_p : which == 1 ? cnt_p : sc_p;
      double* out = which == 0 ? rs : which == 1 ? cnt : sc;
      const int64_t len = which == 0 ? 3 * n : which == 1 ? 2 * n : nk;
      return exchange_parts(G, r, st, evs[1 + which], part, gath, out, len, rc);
    };
    auto acc = [&](double* dst, const double* src, int64_t len, bool first) -> int {
      if (first)
        return hipMemcpyAsync(dst, src, sizeof(double) * len, hipMemcpyDeviceToDevice, st) ==
                       hipSuccess
                   ? FS_OK
                   : FS_EHIP;
      k_accumulate<<<(unsigned)((len + 255) / 256), 256, 0, st>>>(dst, src, len);
      return launch_check("k_accumulate");
    };
    auto stages = [&]() {
      if (V == 1) {
        if (!rc) rc = plan_pass1(g, rs_p);
        ok = exch(0);
        if (ok && !rc) rc = plan_select(g, rs, cnt_p);
        ok = ok && exch(1);
        if (ok && !rc) rc = plan_pass2(g, cnt, sc_p);
        ok = ok && exch(2);
        return;
      }
      for (int round = 0; round < 3 && ok; round++) {
        for (int v = 0; v < V && !rc; v++) {
          if ((rc = plan_set_shard(g, r + N * v, W))) break;
          if ((rc = plan_pass1(g, tmp))) break;
          if (round == 0) { rc = acc(rs_p, tmp, 3 * n, v == 0); continue; }
          if ((rc = plan_select(g, rs, tmp))) break;
          if (round == 1) { rc = acc(cnt_p, tmp, 2 * n, v == 0); continue; }
          if ((rc = plan_pass2(g, cnt, tmp))) break;
          rc = acc(sc_p, tmp, nk, v == 0);
        }
        ok = exch(round);
      }
    };
    if (ok) stages();
    // the decision check on a whole-range call: every thread holds the same
    // summed vectors, so every thread reaches the same decision
    if (ok && whole) {
      double risk = -1.0;
      int sw = 0;
      if (!rc) rc = plan_decision_guard(g, rs, cnt, sc, &risk, &sw);
      if (r == 0) {
        g_last_risk = risk;
        g_last_rerun = sw;
      }
      ok = G.bar.arrive(rc, rc ? std::string(fs_last_error()) : std::string());
      if (ok && sw) stages();
    }
    if (ok && !rc && r == 0) {
      if (hipMemcpyAsync(result.data(), sc, sizeof(double) * nk, hipMemcpyDeviceToHost, st) !=
              hipSuccess ||
          hipStreamSynchronize(st) != hipSuccess) {
        (void)hipGetLastError();
        set_error("multi-device MultiSURF: device-to-host copy of the sums failed");
        rc = FS_EHIP;
      }
    }
    if (g) plan_destroy(g);
    if (ok) G.bar.arrive(rc, rc ? std::string(fs_last_error()) : std::string());
    // after the final barrier nobody waits on this thread's events any more
    if (xs_st) (void)hipStreamDestroy(xs_st);
    for (auto& e : evs)
      if (e) (void)hipEventDestroy(e);
    return rc;
  };
  std::vector<std::thread> th;
  for (int r = 1; r < N; r++) th.emplace_back(worker, r);
  worker(0);
  for (auto& t : th) t.join();
  if (G.bar.rc() != FS_OK) {
    set_error(G.bar.err().empty() ? std::string("multi-device MultiSURF failed") : G.bar.err());
    return G.bar.rc();
  }
  std::copy(result.begin(), result.end(), sums_out);
  return FS_OK;
}

// ReliefF / SURF over several devices: thread r scores the focal samples of
// its whole 128-sample blocks of [r_lo, r_hi) (parallel.shard_rows) on
// devices[r]; the float64 sums are added on the host in rank order.  Their
// neighbour selection is row-local (ReliefF.py:144-175, SURF.py:146-163),
// so there is no other exchange.
int rows_run_devices(const Prepared& P, const void* x, const int* devices, int ndev,
                     int64_t r_lo, int64_t r_hi, double* sums_out) {
  const int N = ndev;
  const int64_t b0 = r_lo / kTile, b1 = (r_hi + kTile - 1) / kTile, nb = b1 - b0;
  const int x_f64 = P.algo == ALGO_SURF ? 1 : 0;  // SURF's kernel dtype (SURF.py:330-333)
  std::vector<std::vector<double>> parts(N, std::vector<double>(P.n_kept, 0.0));
  enable_peers(devices, N);
  DevGroup G(N, devices);
  auto worker = [&](int r) {
    const int64_t lo = std::max(r_lo, (b0 + nb * r / N) * kTile);
    const int64_t hi = std::min(r_hi, (b0 + nb * (r + 1) / N) * kTile);
    void* xbuf = nullptr;
    uint64_t staged = 0;
    hipStream_t st = nullptr;
    hipEvent_t ev = nullptr;
    int rc = hipSetDevice(devices[r]) == hipSuccess ? FS_OK : FS_EHIP;
    if (!rc && (hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess ||
                hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess))
      rc = FS_EHIP;
    // X once over the host link: 1/N of the rows per device, the rest by
    // peer copies, registered as this thread's staged X for the plans
    const bool ok = distribute_x(G, r, x, (x_f64 ? 8 : 4) * (size_t)P.p_in, P.n, &xbuf, st, ev, rc);
    if (ok && !rc) rc = stage_x_device(devices[r], x, xbuf, x_f64, P.n, P.p_in, &staged);
    if (ok && !rc && hi > lo)
      rc = P.algo == ALGO_RELIEFF ? relieff_run(P, x, devices[r], lo, hi, parts[r].data())
                                  : surf_run(P, x, devices[r], lo, hi, parts[r].data());
    if (staged) unstage_x(staged);
    if (xbuf) dev_free(xbuf);
    if (ok) G.bar.arrive(rc, rc ? std::string(fs_last_error()) : std::string());
    if (st) (void)hipStreamDestroy(st);
    if (ev) (void)hipEventDestroy(ev);
  };
  std::vector<std::thread> th;
  for (int r = 1; r < N; r++) th.emplace_back(worker, r);
  worker(0);
  for (auto& t : th) t.join();
  if (G.bar.rc() != FS_OK) {
    set_error(G.bar.err().empty() ? std::string("multi-device scoring failed") : G.bar.err());
    return G.bar.rc();
  }
  // the row partition's float64 sums, added in thread order (one small
  // vector per device; there is no other exchange)
  std::fill(sums_out, sums_out + P.n_kept, 0.0);
  for (int r = 0; r < N; r++)
    for (int64_t k = 0; k < P.n_kept; k++) sums_out[k] += parts[r][k];
  return FS_OK;
}

}  // namespace gpu
}  // namespace fs
