// fs_pass1.hip -- pass 1: quantisation, the distance tiles, row moments, the mean correction glue, calibration and the row guard; SURF.
// Shared state and helpers: fs_gpu_internal.h.
#include "fs_gpu_internal.h"

namespace fs {
namespace gpu {

// ---------------------------------------------------------------------------
// Quantize: X -> xqT (u32, [PW][n_pad]) and xs (f32, [n_pad][PW]), and
// with a star split (fs_starterm.hip) xs feature-major as well (xsT)
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
    float* __restrict__ epsT, float* __restrict__ xsT) {
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
  float vr[kR];
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
    vr[k] = v;
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
  if (xsT) {  // the pass-2 values transposed through etile
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kR; k++) etile[ty + 4 * k][tx] = vr[k];
    __syncthreads();
    for (int r = ty; r < 64; r += 4) xsT[(c0 + r) * n_pad + i0 + tx] = etile[tx][r];
  }
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
    const double* __restrict__ dtab, double* __restrict__ xT, float* __restrict__ xs,
    float* __restrict__ xsT) {
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
  if (xsT)
    for (int r = ty; r < 64; r += 4) xsT[(c0 + r) * n_pad + i0 + tx] = (float)tile[tx][r];
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

// Band calibration (calibrate_band): for each sampled pair, the quantised
// distance's error against the reference's arithmetic, err = sum over the
// continuous kept features of |q_i - q_j| - SC * f32(|x_i - x_j| * recip),
// for the 16-bit scale (.x) and the 32-bit scale (.y) -- SURF (scl64): the
// float64 terms |x_i - x_j| * recip, .x the continuous part of the distance
// (the float32 rounding the band must resolve, surf_int).  q is formed exactly
// as k_quantize forms it; discrete features contribute no error.  One wave
// per pair, fixed-order reduction (every rank computes the same values).
template <typename T>
__global__ __launch_bounds__(256) void k_calib(
    const T* __restrict__ x, int64_t p_in, int64_t pc, const int64_t* __restrict__ src_col,
    const double* __restrict__ off, const double* __restrict__ qs16,
    const double* __restrict__ qs32, const float* __restrict__ scl32, double sc16, double sc32,
    const double* __restrict__ scl64, const int2* __restrict__ pairs, int64_t npairs,
    double2* __restrict__ err) {
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
    if (scl64) {  // SURF: float64 terms (SURF.py:156); .x = the distance itself
      const double ref = __builtin_fabs(a - b) * scl64[c];
      e16 += ref;
      e32 += (qa32 > qb32 ? (double)(qa32 - qb32) : (double)(qb32 - qa32)) - sc32 * ref;
      continue;
    }
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

// Pass-1 K-split: k_dist holds `slots` workgroups on the chip at a time, so
// T tiles take ceil(T / slots) rounds; splitting every tile's feature range
// into S parts evens out the last round when there are few tiles (cfg2: 820
// tiles on 768 slots; one rank of an N-GPU job).  The merge streams (S + 2)
// tile planes (~66.5 / p of the tile's compute time each); S > 1 only when
// the model gains at least 3%.  (Splitting only the last round's tiles was
// measured too: no better than S = 1 at cfg2, profiles/r02/ksplit_sweep.txt.)
// `beside`: MultiSURF's mean correction runs on the side stream during
// k_dist, and when the tiles fill fewer than two rounds its workgroups take
// the slots a finer split would even out -- cfg2 (820 tiles on 768 slots)
// measured 4.51 / 4.22-4.23 / 4.22 / 4.39 / 4.31 / 4.33 / ~4.4 ms a step at
// S = 1 / 2 / 3 / 4 / 5 / 6 / 8 (the model's pick), so S stops at 3 there
// (profiles/r06/ksplit_ab.txt); SURF's integer route (no correction) keeps
// the model's pick (cfg5s: 182.2 ms at S = 1, 178.1 at the pick).
int choose_ksplit(int64_t tiles, int device, int nchunks, int64_t feats, bool beside) {
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
  if (beside && (double)tiles < 2.0 * slots) max_sp = std::min(max_sp, 3);
  for (int sp = 2; sp <= max_sp && sp <= nchunks; sp++)
    if (eff(sp) > best_eff) {
      best_eff = eff(sp);
      best = sp;
    }
  return best;
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

// SURF (surf_int, fs_surfint.hip): the band of y = D_q / SC from the sampled
// 32-bit errors (.y), and the integer route only while the band stays below
// one float32 ulp of the shorter sampled distances (.x, their 10th
// percentile): beyond it most pairs keep several candidates and the row
// sums stop at ~band / ulp times more pairs, so coherent rounding
// (duplicated or same-grid columns) and few features (the band grows as
// sqrt(pc), the ulp as pc) keep the float64 distances.  The surf_f64 test
// hook forces either route (both give the same float32 distances).
constexpr double kSurfIntMinWork = 5e9;
static int surf_band(Plan* g, const std::vector<double2>& err) {
  Prepared& Q = g->P;
  double ss = 0.0, mx = 0.0;
  std::vector<double> dist;
  dist.reserve(err.size());
  for (const double2& e : err) {
    ss += e.y * e.y;
    mx = std::max(mx, std::fabs(e.y));
    dist.push_back(e.x);
  }
  const double rms = std::sqrt(ss / (double)std::max<size_t>(err.size(), 1));
  Q.amb_delta = calibrated_delta(Q.amb_delta_model, Q.SC, rms, mx);
  double ulp = 0.0;
  if (!dist.empty()) {
    const size_t k = dist.size() / 10;
    std::nth_element(dist.begin(), dist.begin() + k, dist.end());
    const float d10 = (float)dist[k];
    if (d10 > 0.0f) {
      int e = 0;
      (void)std::frexp(d10, &e);
      ulp = std::ldexp(1.0, e - 24);
    }
  }
  // and only where pass 1 is worth the rounds: ~2x the float64 kernel's rate
  // saves ~0.35 ms per 1e10 pair-features, a round of the row sums costs
  // ~0.05 ms
  const double work = 0.5 * (double)Q.n * (double)Q.n * (double)Q.pc;
  if (test_hooks().surf_f64 < 0 && !(Q.amb_delta <= ulp && work >= kSurfIntMinWork))
    g->surf_int = false;
  g->calib[0] = 0.0;
  g->calib[5] = g->surf_int ? 0.0 : 3.0;
  g->calib[1] = rms;
  g->calib[2] = mx;
  g->calib[4] = Q.amb_delta / Q.amb_delta_model;
  if (trace_on()) {
    char msg[256];
    snprintf(msg, sizeof msg,
             "calibrate (SURF): rms32 %.1f max32 %.1f model sigma %.1f, band %.3g, ulp %.3g -> %s",
             rms, mx, g->calib[3], Q.amb_delta, ulp,
             g->surf_int ? "integer distances" : "float64 distances");
    trace_mark(msg);
  }
  return FS_OK;
}

int calibrate_band(Plan* g) {
  Prepared& Q = g->P;
  g->calib[0] = Q.q16;
  g->calib[1] = g->calib[2] = 0.0;
  g->calib[3] = std::sqrt((double)Q.pc / 6.0 + 1.0);
  g->calib[4] = 1.0;
  g->calib[5] = 0.0;
  g->calib[6] = 0.0;
  const bool surf = Q.algo == ALGO_SURF;
  g->surf_int = surf && test_hooks().surf_f64 != 1 && Q.n >= 2;
  if (surf && !g->surf_int) g->calib[5] = 3.0;
  if (Q.pc == 0 || Q.n < 2) return FS_OK;
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
                                                   sc[1], surf ? g->scl : nullptr, dpr, S, derr);
    else
      k_calib<float><<<grid, 256, 0, g->stream>>>((const float*)g->x, Q.p_in, Q.pc, g->src_col,
                                                  g->off, dqs, dqs + Q.PW, g->scl32, sc[0],
                                                  sc[1], nullptr, dpr, S, derr);
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
  if (surf) return surf_band(g, err);
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
// The row guard's decision from the host copy of corr (every continuous
// column): a row whose mean is off by more than the limit keeps 32-bit
// operands (the plan's scale is switched here; the caller re-uploads it).
// MultiSURF* split plans sort each continuous column once for both the mean
// correction and the star sums (fs_colsort.hip k_colsort_star) -- the
// colsort_star test hook 0 keeps the binned correction and a separate sort
static bool colsort_star(const Plan* g) {
  return g->P.algo == ALGO_MULTISURF && g->star_split && test_hooks().colsort_star != 0 &&
         colsort_lds(g->P.n);
}

static int row_guard_decide(Plan* g, const std::vector<double>& h, bool* switched) {
  Prepared& Q = g->P;
  *switched = false;
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
    *switched = true;
  }
  if (trace_on()) {
    char msg[160];
    snprintf(msg, sizeof msg, "row guard: max |row bias| %.1f (limit %.1f) -> q16 %d", worst,
             limit, Q.q16);
    trace_mark(msg);
  }
  return FS_OK;
}

static int copy_corr(Plan* g, const double* corr, std::vector<double>& h) {
  h.resize((size_t)g->P.n);
  if (hipMemcpyAsync(h.data(), corr, sizeof(double) * g->P.n, hipMemcpyDeviceToHost,
                     g->stream) != hipSuccess ||
      hipStreamSynchronize(g->stream) != hipSuccess) {
    (void)hipGetLastError();
    set_error("row guard: device-to-host copy failed");
    return FS_EHIP;
  }
  return FS_OK;
}

int row_guard(Plan* g) {
  Prepared& Q = g->P;
  g->guard_pending = false;
  if (!Q.q16 || Q.pc == 0 || Q.n < 2 || Q.algo == ALGO_SURF || test_hooks().q16_guard_off)
    return FS_OK;
  // a plan over every continuous column (one rank, one shard) keeps the
  // guard's work for its first pass 1: operands, terms and the correction
  // itself (g->corr) are what that pass would compute again
  const bool reuse = g->c_lo == 0 && g->c_hi == Q.pc;
  if (reuse && Q.defer_guard && !Q.ref_accum) {
    // decided after the first pass 1 instead (plan_pass1), whose correction
    // runs beside k_dist on the side stream rather than before it
    g->guard_pending = true;
    return FS_OK;
  }
  double* corr = g->corr;
  if (!reuse) FS_TRY(dev_alloc((void**)&corr, sizeof(double) * Q.n_pad, g->device));
  dim3 gq((unsigned)(Q.PW / 64), (unsigned)(Q.n_pad / 64));
  int rc = FS_OK;
  if (g->x_is_f64)
    k_quantize<double><<<gq, 256, 0, g->stream>>>(
        (const double*)g->x, Q.n, Q.n_pad, Q.p_in, Q.PW, Q.PC, Q.q16, Q.pc, g->src_col, g->off,
        g->qs, g->scl, g->dtab_off, g->dtab, Q.disc_bits, 0, Q.pc, g->xqT, g->xs, g->epsT, g->xsT);
  else
    k_quantize<float><<<gq, 256, 0, g->stream>>>(
        (const float*)g->x, Q.n, Q.n_pad, Q.p_in, Q.PW, Q.PC, Q.q16, Q.pc, g->src_col, g->off,
        g->qs, g->scl, g->dtab_off, g->dtab, Q.disc_bits, 0, Q.pc, g->xqT, g->xs, g->epsT, g->xsT);
  rc = launch_check("k_quantize (row guard)");
  if (!rc) rc = run_colsort(g, 0, Q.pc, g->stream);
  if (!rc) rc = run_rowcorr(g, 0, Q.pc, corr, g->stream);
  std::vector<double> h;
  if (!rc) rc = copy_corr(g, corr, h);
  if (!reuse) dev_free(corr);
  if (rc) return rc;
  bool switched = false;
  FS_TRY(row_guard_decide(g, h, &switched));
  // (a MultiSURF* split plan's steps take their correction from the fused
  // full sort, k_colsort_star: its first step computes it too, so that every
  // step's terms are the same)
  if (!switched) g->corr_ready = reuse && !colsort_star(g);
  return FS_OK;
}

// SURF*'s star-split column terms (fs_starterm.hip) need only the operands
// and the focal rows: on the side stream beside pass 1, joined by run_pass2
// before k_reduce adds them
static int fork_star_terms(Plan* g) {
  FS_HIP(hipEventRecord(g->ev_fork, g->stream));
  FS_HIP(hipStreamWaitEvent(g->side, g->ev_fork, 0));
  FS_TRY(star_terms(g, g->side));
  FS_HIP(hipEventRecord(g->ev_join, g->side));
  return FS_OK;
}

// quantize (+ mean correction terms) and pass 1 (distance tiles)
int run_quantize_dist(Plan* g) {
  const Prepared& Q = g->P;
  FS_HIP(hipSetDevice(g->device));
  dim3 gq((unsigned)(Q.PW / 64), (unsigned)(Q.n_pad / 64));
  if (Q.algo == ALGO_SURF && !g->surf_int) {
    k_quantize_f64<<<gq, 256, 0, g->stream>>>((const double*)g->x, Q.n, Q.n_pad, Q.p_in, Q.PW,
                                              Q.pc, g->src_col, g->off, g->scl, g->dtab_off,
                                              g->dtab, g->xT64, g->xs, g->xsT);
    FS_TRY(launch_check("k_quantize_f64"));
    if (g->star_split) FS_TRY(fork_star_terms(g));
    if (g->n_tiles > 0) {
      FS_HIP(hipEventRecord(g->ev[0], g->stream));
      k_dist_f64<<<(unsigned)g->n_tiles, 256, 0, g->stream>>>(
          g->xT64, Q.n_pad, (int)(Q.PC / kBK64), (int)(Q.PD / kBK64), g->tiles, g->win, g->D);
      FS_TRY(launch_check("k_dist_f64"));
      FS_HIP(hipEventRecord(g->ev[1], g->stream));
    }
    return FS_OK;
  }
  // SURF's integer route (fs_surfint.hip) quantises as MultiSURF does: no
  // mean correction, no K-split, float64 X
  const bool reuse = g->corr_ready && Q.algo == ALGO_MULTISURF;
  // MultiSURF*'s per-sample sums overwrite xsT in place: a pass 1 run again
  // (the deferred row guard's switch to 32-bit operands) quantises only after
  // the previous sums are done with it
  if (g->side2) FS_HIP(hipStreamWaitEvent(g->stream, g->ev_star, 0));
  g->corr_ready = false;  // later steps quantise again (the terms overwrote epsT)
  // quantisation errors for the mean correction (MultiSURF; ReliefF keeps
  // them unused), none on SURF's integer route (no epsT)
  const int64_t eps_lo = Q.algo == ALGO_SURF ? 0 : g->c_lo;
  const int64_t eps_hi = Q.algo == ALGO_SURF ? 0 : g->c_hi;
  if (reuse) {
    // the row guard's operands and correction (row_guard): nothing to redo
    FS_HIP(hipEventRecord(g->ev_join, g->stream));
  } else if (g->x_is_f64) {
    k_quantize<double><<<gq, 256, 0, g->stream>>>(
        (const double*)g->x, Q.n, Q.n_pad, Q.p_in, Q.PW, Q.PC, Q.q16, Q.pc, g->src_col, g->off,
        g->qs, g->scl, g->dtab_off, g->dtab, Q.disc_bits, eps_lo, eps_hi, g->xqT, g->xs,
        g->epsT, g->xsT);
  } else {
    k_quantize<float><<<gq, 256, 0, g->stream>>>(
        (const float*)g->x, Q.n, Q.n_pad, Q.p_in, Q.PW, Q.PC, Q.q16, Q.pc, g->src_col, g->off,
        g->qs, g->scl, g->dtab_off, g->dtab, Q.disc_bits, eps_lo, eps_hi, g->xqT, g->xs,
        g->epsT, g->xsT);
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
    if (colsort_star(g)) {
      // one full sort per column for the correction and the star sums
      if (colsort_star_terms(g->xqT, g->epsT, g->xsT, g->lab, g->out_pos, Q.n_classes, Q.n,
                             Q.n_pad, g->c_lo, g->c_hi, Q.q16, g->key_shift, g->side))
        return FS_EHIP;
    } else {
      FS_TRY(run_colsort(g, g->c_lo, g->c_hi, g->side));
    }
    FS_TRY(run_rowcorr(g, g->c_lo, g->c_hi, g->corr, g->side));
    FS_HIP(hipEventRecord(g->ev_join, g->side));
  }
  if (Q.algo == ALGO_SURF && g->star_split) FS_TRY(fork_star_terms(g));
  if (Q.algo == ALGO_MULTISURF && g->star_split) {
    // MultiSURF*'s per-sample sums over the other classes, on a third stream
    // beside k_dist and the correction (run_weights waits for ev_star): they
    // need only the operands (the counts weigh them in star_reduce)
    FS_HIP(hipEventRecord(g->ev_fork, g->stream));
    FS_HIP(hipStreamWaitEvent(g->side2, g->ev_fork, 0));
    FS_TRY(star_sums(g, g->side2, !(colsort_star(g) && !reuse)));
    FS_HIP(hipEventRecord(g->ev_star, g->side2));
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

int plan_pass1(Plan* g, double* rowstats) {
  const Prepared& Q = g->P;
  FS_TRY(run_quantize_dist(g));
  if (g->n_tiles > 0) {
    k_tile_rowstats<<<(unsigned)g->n_tiles, 256, 0, g->stream>>>(g->D, Q.n, g->tiles, g->rspart);
    FS_TRY(launch_check("k_tile_rowstats"));
  }
  FS_HIP(hipStreamWaitEvent(g->stream, g->ev_join, 0));  // corr (side stream)
  if (g->guard_pending) {
    // the deferred row guard (P.defer_guard): this pass's correction covers
    // every continuous column; a coherent row switches the plan to 32-bit
    // operands and pass 1 runs again on them
    g->guard_pending = false;
    std::vector<double> h;
    FS_TRY(copy_corr(g, g->corr, h));
    bool switched = false;
    FS_TRY(row_guard_decide(g, h, &switched));
    if (switched) {
      FS_TRY(apply_operand_width(g));
      return plan_pass1(g, rowstats);
    }
  }
  k_rowstats_reduce<<<(unsigned)((Q.n + 255) / 256), 256, 0, g->stream>>>(
      g->rspart, Q.n, g->nb, g->rank, g->world, g->corr, rowstats);
  FS_TRY(launch_check("k_rowstats_reduce"));
  if (g->own_stream) FS_HIP(hipStreamSynchronize(g->stream));
  return FS_OK;
}

// SURF score sums of the plan's focal rows into sums_dev[n_kept].
int plan_score_surf(Plan* g, double* sums_dev) {
  const Prepared& Q = g->P;
  int rc = run_quantize_dist(g);  // integer or float64 distances
  if (rc == FS_OK && g->surf_int) {
    // the means, then D as float32 values in real units (plan_kernel_ms 2)
    FS_HIP(hipEventRecord(g->ev[4], g->stream));
    rc = surf_resolve(g);
    FS_HIP(hipEventRecord(g->ev[5], g->stream));
  } else if (rc == FS_OK && g->r_hi > g->r_lo) {
    k_surf_avg<<<(unsigned)((g->r_hi - g->r_lo + 63) / 64), 64, 0, g->stream>>>(
        g->D, Q.n, Q.n_pad, 1.0, g->r_lo, g->r_hi, g->thr);
    rc = launch_check("k_surf_avg");
  }
  if (rc == FS_OK && Q.ref_accum) return surf_ref(g, sums_dev);  // fs_refacc.hip order
  if (rc == FS_OK) rc = run_weights(g, nullptr, ALGO_SURF, 1.0);
  if (rc == FS_OK) rc = run_pass2(g, sums_dev);
  return rc;
}

}  // namespace gpu
}  // namespace fs
