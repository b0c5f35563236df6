// fs_relieff.hip -- ReliefF: k-nearest selection per class and the neighbour update.
// Shared state and helpers: fs_gpu_internal.h.
#include "fs_gpu_internal.h"

namespace fs {
namespace gpu {

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

// Reference order (fs_refacc.hip): runs of equal keys inside a row's
// neighbour lists (sorted by key, then index) put in numba's quicksort order
// (ReliefF.py:157-175 scans the argsort, so its float64 hit / miss sums of
// ReliefF.py:181-207 add tied neighbours in that order).  One wave per row:
// every sample of a run is a focus sample (R's sign bit), wave_argsort_focus
// replays numba's quicksort over the row's exact keys (keys_all, +inf at i),
// the focus samples are collected in their sorted order (ord, per-row
// scratch of C k), and lane 0 re-orders each run by that order.  IN_LDS:
// the keys and R in LDS (8 bytes per sample), else in the global scratch.
template <bool IN_LDS>
__global__ __launch_bounds__(64) void k_rf_ref_ties(
    const int32_t* __restrict__ rows, int64_t n, const float* __restrict__ keys_all, int C,
    int64_t k, int64_t r_lo, int32_t* __restrict__ nbr, const int32_t* __restrict__ nfound,
    const float* __restrict__ lkeys, int32_t* __restrict__ R_all, int32_t* __restrict__ ord_all,
    int* __restrict__ status) {
  extern __shared__ uint32_t tie_lds[];
  __shared__ int sort_rc;
  const int lane = threadIdx.x;
  const int64_t r = blockIdx.x;
  const int64_t i = rows[r];
  const float* key = keys_all + r * n;
  int32_t* R = R_all + r * n;
  int32_t* ord = ord_all + r * C * k;
  if (IN_LDS) {
    float* kl = (float*)tie_lds;
    for (int64_t j = lane; j < n; j += 64) kl[j] = key[j];
    key = kl;
    R = (int32_t*)(tie_lds + n);
  }
  for (int64_t j = lane; j < n; j += 64) R[j] = (int32_t)j;
  __syncthreads();
  // focus samples: the members of a run of equal keys in one list (each
  // sample is in one class's list at most once, so the lanes' stores are to
  // distinct samples)
  for (int64_t e = lane; e < (int64_t)C * k; e += 64) {
    const int64_t c = e / k, t = e % k;
    const int64_t m = nfound[i * C + c];
    if (t >= m) continue;
    const float* K = lkeys + ((i - r_lo) * C + c) * k;
    if ((t > 0 && K[t] == K[t - 1]) || (t + 1 < m && K[t + 1] == K[t])) {
      const int32_t j = nbr[(i * C + c) * k + t];
      R[j] = (int32_t)((uint32_t)j | 0x80000000u);
    }
  }
  __syncthreads();
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
  int64_t cnt = 0;
  for (int64_t t0 = 0; t0 < n; t0 += 64) {
    const int64_t t = t0 + lane;
    const int32_t h = t < n ? R[t] : 0;
    const uint64_t m = __ballot(h < 0);
    if (h < 0) ord[cnt + __popcll(m & below)] = h & 0x7FFFFFFF;
    cnt += __popcll(m);
  }
  __threadfence_block();
  __syncthreads();
  if (lane != 0) return;
  for (int c = 0; c < C; c++) {
    const int64_t m = nfound[i * C + c];
    int32_t* L = nbr + (i * C + c) * k;
    const float* K = lkeys + ((i - r_lo) * C + c) * k;
    for (int64_t s = 0; s < m;) {
      int64_t e = s + 1;
      while (e < m && K[e] == K[s]) e++;
      // insertion sort of L[s, e) by rank in ord
      auto rank = [&](int32_t j) {
        int64_t q = 0;
        while (q < cnt && ord[q] != j) q++;
        return q;
      };
      for (int64_t a = s + 1; a < e; a++) {
        const int32_t v = L[a];
        const int64_t rv = rank(v);
        int64_t b = a;
        while (b > s && rank(L[b - 1]) > rv) {
          L[b] = L[b - 1];
          b--;
        }
        L[b] = v;
      }
      s = e;
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

// Reference order: the rows whose neighbour lists hold runs of equal keys
// (dup, from relieff_order) get those runs in numba's quicksort order
// (k_rf_ref_ties over the row's exact keys) -- when that order can change
// the row's float64 sums at all (k_rf_ref_order_matters): continuous data
// has many rows with float32 key ties among the k nearest, but diffs
// within 2^29 of each other add exactly in any order; an all-discrete
// layout's 0 / 1 diffs always do, so the caller skips it (pc == 0).
static int relieff_ref_ties(Plan* g, int32_t* nbr, const int32_t* nfound, const int32_t* dup) {
  const Prepared& Q = g->P;
  const int C = Q.n_classes;
  const int64_t k = Q.k_neighbors, n = Q.n, rows = g->r_hi - g->r_lo;
  std::vector<int32_t> h((size_t)rows * C);
  FS_HIP(hipMemcpyAsync(h.data(), dup, h.size() * sizeof(int32_t), hipMemcpyDeviceToHost,
                        g->stream));
  FS_HIP(hipStreamSynchronize(g->stream));
  std::vector<int32_t> tie_rows;
  for (int64_t r = 0; r < rows; r++)
    for (int c = 0; c < C; c++)
      if (h[r * C + c]) {
        tie_rows.push_back((int32_t)(g->r_lo + r));
        break;
      }
  const size_t n_tied = tie_rows.size();
  if (tie_rows.empty()) {
    if (trace_on()) std::fprintf(stderr, "[fs_trace] relieff reference order: no tied keys\n");
    return FS_OK;
  }
  int rc;
  if (!test_hooks().rf_ref_replay) {
    // the replay reads the row's n keys (n * n_kept diffs); first drop the
    // rows whose sums come out the same in any order (k_rf_ref_order_matters,
    // C * k * n_kept diffs) -- on continuous data, all of them
    int32_t *crows = nullptr, *matters = nullptr;
    g->alloc_target = 2;
    if ((rc = dalloc(g, &crows, n_tied)) || (rc = dalloc(g, &matters, n_tied))) {
      g->alloc_target = 0;
      return rc;
    }
    g->alloc_target = 0;
    FS_TRY(h2d(g, crows, tie_rows.data(), n_tied));
    FS_TRY(refacc::relieff_order_matters(g->xk, g->Kp, g->krecip, g->kdisc, Q.n_kept, crows,
                                         (int64_t)n_tied, dup, nbr, nfound, g->r_lo, C, k,
                                         matters, g->stream));
    std::vector<int32_t> hm(n_tied);
    FS_HIP(hipMemcpyAsync(hm.data(), matters, n_tied * sizeof(int32_t), hipMemcpyDeviceToHost,
                          g->stream));
    FS_HIP(hipStreamSynchronize(g->stream));
    size_t w = 0;
    for (size_t r = 0; r < n_tied; r++)
      if (hm[r]) tie_rows[w++] = tie_rows[r];
    tie_rows.resize(w);
  }
  if (trace_on())
    std::fprintf(stderr,
                 "[fs_trace] relieff reference order: %zu rows with tied keys, %zu replayed\n",
                 n_tied, tie_rows.size());
  if (tie_rows.empty()) return FS_OK;
  const int64_t row_bytes = 8 * n + 4 * (int64_t)C * k;
  const int64_t batch = std::max<int64_t>(
      1, std::min<int64_t>((int64_t)tie_rows.size(), (int64_t)(512ll << 20) / row_bytes));
  int32_t *drows = nullptr, *R = nullptr, *ord = nullptr;
  float* keys = nullptr;
  int* status = nullptr;
  g->alloc_target = 2;
  if ((rc = dalloc(g, &drows, (size_t)batch)) || (rc = dalloc(g, &R, (size_t)(batch * n))) ||
      (rc = dalloc(g, &keys, (size_t)(batch * n))) ||
      (rc = dalloc(g, &ord, (size_t)(batch * C * k))) || (rc = dalloc(g, &status, 1))) {
    g->alloc_target = 0;
    return rc;
  }
  g->alloc_target = 0;
  FS_HIP(hipMemsetAsync(status, 0, sizeof(int), g->stream));
  // keys and R in LDS (8 B per sample) beside ~2.2 KB of static LDS
  const bool in_lds = 8 * n + 2304 <= 160 * 1024;
  if (in_lds)
    FS_HIP(hipFuncSetAttribute((const void*)k_rf_ref_ties<true>,
                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)(8 * n)));
  for (int64_t r0 = 0; r0 < (int64_t)tie_rows.size(); r0 += batch) {
    const int64_t nr = std::min<int64_t>(batch, (int64_t)tie_rows.size() - r0);
    FS_TRY(h2d(g, drows, tie_rows.data() + r0, (size_t)nr));
    FS_TRY(refacc::relieff_row_keys(g->xk, g->Kp, g->krecip, g->kdisc, Q.n_kept, drows, nr, n,
                                    keys, g->stream));
    if (in_lds)
      k_rf_ref_ties<true><<<(unsigned)nr, 64, (size_t)(8 * n), g->stream>>>(
          drows, n, keys, C, k, g->r_lo, nbr, nfound, g->rkeys, R, ord, status);
    else
      k_rf_ref_ties<false><<<(unsigned)nr, 64, 0, g->stream>>>(drows, n, keys, C, k, g->r_lo, nbr,
                                                              nfound, g->rkeys, R, ord, status);
    FS_TRY(launch_check("k_rf_ref_ties"));
  }
  int hstatus = 0;
  FS_HIP(hipMemcpyAsync(&hstatus, status, sizeof(int), hipMemcpyDeviceToHost, g->stream));
  FS_HIP(hipStreamSynchronize(g->stream));
  if (hstatus != 0) {
    set_error("ReliefF reference order: quicksort stack overflow");
    return FS_EHIP;
  }
  return FS_OK;
}

// ReliefF score sums of the plan's focal rows into sums_dev[n_kept]:
// pass 1, neighbour selection, then the neighbour-gather update.
int plan_score_relieff(Plan* g, double* sums_dev) {
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
    int32_t* dup = nullptr;
    g->alloc_target = 2;
    rc = dalloc(g, &dup, (size_t)std::max<int64_t>(rows * C, 1));
    g->alloc_target = 0;
    FS_TRY(rc);
    FS_TRY(refacc::relieff_order(g->xk, g->Kp, g->krecip, g->kdisc, Q.n_kept, C, k, nbr, nfound,
                                 g->r_lo, g->r_hi, g->rkeys, dup, g->stream));
    if (rows > 0 && k > 1 && Q.pc > 0) FS_TRY(relieff_ref_ties(g, nbr, nfound, dup));
    FS_TRY(refacc::relieff_update(g->xk, g->Kp, g->krecip, g->kdisc, g->lab, dprior, C, k, nbr,
                                  nfound, g->r_lo, g->r_hi, temp, g->stream));
    FS_HIP(hipEventRecord(g->ev[3], g->stream));
    if (g->ref_defer) {  // fs_plan_ref_temp: the column sums come later (plan_ref_sums)
      g->ref_rows = std::max<int64_t>(rows, 0);
      return FS_OK;
    }
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
  return reduce_segments(part, nrb, Q.PW, g->out_pos, sums_dev, g->stream);
}

int relieff_run_one(const Prepared& P, const void* x, int device, int64_t r_lo, int64_t r_hi,
                    double* sums_out, const double* seed) {
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

}  // namespace gpu
}  // namespace fs
