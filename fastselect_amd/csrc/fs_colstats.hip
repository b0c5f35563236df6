// fs_colstats.hip -- per-column statistics of X on the GPU: minimum, maximum
// and the number of distinct values up to a cap.  This is the preprocessing
// every reference fit() runs on the host before scoring
// (MultiSURF.py:141-144,409-420: x.max(0) - x.min(0) and
// np.unique(x[:, f]).size <= discrete_limit; ReliefF.py:366-380;
// SURF.py:347-355), which at BASELINE cfg4/cfg5 costs more host time than the
// GPU scoring itself.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <vector>

#include "../../include/fastselect_amd.h"
#include "fs_internal.h"

namespace fs {
namespace gpu {

namespace {

// Partial min / max over a chunk of rows: lanes = 64 consecutive columns
// (coalesced 256-byte row segments), 4 waves split the chunk's rows.
template <typename T>
__global__ __launch_bounds__(256) void k_colminmax(const T* __restrict__ x, int64_t n, int64_t p,
                                                   int64_t rows_per_chunk, T* __restrict__ pmin,
                                                   T* __restrict__ pmax) {
  __shared__ T smin[4][64], smax[4][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t c = (int64_t)blockIdx.x * 64 + lane;
  const int64_t r0 = (int64_t)blockIdx.y * rows_per_chunk;
  const int64_t r1 = r0 + rows_per_chunk < n ? r0 + rows_per_chunk : n;
  // every chunk has at least one row (r0 < n): start from it
  T lo = 0, hi = 0;
  if (c < p) {
    lo = hi = x[r0 * p + c];
    for (int64_t i = r0 + wave; i < r1; i += 4) {
      const T v = x[i * p + c];
      lo = v < lo ? v : lo;
      hi = v > hi ? v : hi;
    }
  }
  smin[wave][lane] = lo;
  smax[wave][lane] = hi;
  __syncthreads();
  if (wave == 0 && c < p) {
    for (int w = 1; w < 4; w++) {
      lo = smin[w][lane] < lo ? smin[w][lane] : lo;
      hi = smax[w][lane] > hi ? smax[w][lane] : hi;
    }
    pmin[(int64_t)blockIdx.y * p + c] = lo;
    pmax[(int64_t)blockIdx.y * p + c] = hi;
  }
}

template <typename T>
__global__ __launch_bounds__(256) void k_colminmax_reduce(const T* __restrict__ pmin,
                                                          const T* __restrict__ pmax,
                                                          int64_t chunks, int64_t p,
                                                          T* __restrict__ mn, T* __restrict__ mx) {
  const int64_t c = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (c >= p) return;
  T lo = pmin[c], hi = pmax[c];
  for (int64_t k = 1; k < chunks; k++) {
    const T a = pmin[k * p + c], b = pmax[k * p + c];
    lo = a < lo ? a : lo;
    hi = b > hi ? b : hi;
  }
  mn[c] = lo;
  mx[c] = hi;
}

// Distinct values of one column per workgroup, counted exactly up to `cap`
// with an LDS open-addressing hash set of 64-bit keys (the value widened to
// double; -0.0 folded into +0.0 because np.unique treats them as equal).
// As soon as more than `cap` distinct values are seen the column is
// continuous and every thread leaves (continuous columns stop after a few
// hundred rows; only discrete columns are scanned to the end).
constexpr unsigned long long kEmpty = ~0ull;  // a NaN pattern; X is finite

template <typename T>
__global__ __launch_bounds__(256) void k_coldistinct(const T* __restrict__ x, int64_t n, int64_t p,
                                                     int cap, int tbits,
                                                     int64_t* __restrict__ ndistinct) {
  extern __shared__ unsigned long long table[];
  __shared__ int count;
  const int64_t c = blockIdx.x;
  const int tsize = 1 << tbits;
  for (int k = threadIdx.x; k < tsize; k += 256) table[k] = kEmpty;
  if (threadIdx.x == 0) count = 0;
  __syncthreads();
  for (int64_t base = 0; base < n; base += 256) {
    const int seen = count;
    __syncthreads();         // every thread has read `count` before any update
    if (seen > cap) break;   // uniform decision
    const int64_t i = base + threadIdx.x;
    if (i < n) {
      double v = (double)x[i * p + c];
      if (v == 0.0) v = 0.0;
      const unsigned long long key = (unsigned long long)__double_as_longlong(v);
      unsigned h = (unsigned)((key * 0x9E3779B97F4A7C15ull) >> (64 - tbits));
      for (int probe = 0; probe < tsize; probe++) {
        const unsigned long long old = atomicCAS(&table[h], kEmpty, key);
        if (old == kEmpty) {
          atomicAdd(&count, 1);
          break;
        }
        if (old == key) break;
        h = (h + 1) & (tsize - 1);
      }
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) ndistinct[c] = count > cap ? (int64_t)cap + 1 : (int64_t)count;
}

}  // namespace

static void minmax_grid(int64_t n, int64_t& rows_per_chunk, int64_t& nchunks) {
  const int64_t chunks = std::min<int64_t>(std::max<int64_t>(1, n / 64), 256);
  rows_per_chunk = (n + chunks - 1) / chunks;
  nchunks = (n + rows_per_chunk - 1) / rows_per_chunk;
}

static void launch_minmax(const void* dx, int x_is_f64, int64_t n, int64_t p,
                          int64_t rows_per_chunk, int64_t nchunks, void* pmin, void* pmax,
                          void* dmin, void* dmax, hipStream_t s) {
  const dim3 g((unsigned)((p + 63) / 64), (unsigned)nchunks);
  const unsigned gr = (unsigned)((p + 255) / 256);
  if (x_is_f64) {
    k_colminmax<double><<<g, 256, 0, s>>>((const double*)dx, n, p, rows_per_chunk,
                                          (double*)pmin, (double*)pmax);
    k_colminmax_reduce<double><<<gr, 256, 0, s>>>((const double*)pmin, (const double*)pmax,
                                                  nchunks, p, (double*)dmin, (double*)dmax);
  } else {
    k_colminmax<float><<<g, 256, 0, s>>>((const float*)dx, n, p, rows_per_chunk, (float*)pmin,
                                         (float*)pmax);
    k_colminmax_reduce<float><<<gr, 256, 0, s>>>((const float*)pmin, (const float*)pmax,
                                                 nchunks, p, (float*)dmin, (float*)dmax);
  }
}

int column_minmax(const void* dx, int x_is_f64, int64_t n, int64_t p, void* hmin, void* hmax,
                  void* stream) {
  hipStream_t s = (hipStream_t)stream;
  const size_t esz = x_is_f64 ? 8 : 4;
  int64_t rows_per_chunk = 0, nchunks = 0;
  minmax_grid(n, rows_per_chunk, nchunks);
  void* buf = nullptr;  // [nchunks][p] min, [nchunks][p] max, [p] min, [p] max
  const size_t part = (size_t)nchunks * p * esz;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) {
    (void)hipGetLastError();
    set_error("column ranges: hipGetDevice failed");
    return FS_EHIP;
  }
  if (int rc = dev_alloc(&buf, 2 * part + 2 * (size_t)p * esz, dev)) return rc;
  hipError_t e;
  char* b = (char*)buf;
  launch_minmax(dx, x_is_f64, n, p, rows_per_chunk, nchunks, b, b + part, b + 2 * part,
                b + 2 * part + p * esz, s);
  e = hipGetLastError();
  if (e == hipSuccess)
    e = hipMemcpyAsync(hmin, b + 2 * part, (size_t)p * esz, hipMemcpyDeviceToHost, s);
  if (e == hipSuccess)
    e = hipMemcpyAsync(hmax, b + 2 * part + p * esz, (size_t)p * esz, hipMemcpyDeviceToHost, s);
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  dev_free(buf);
  if (e != hipSuccess) {
    (void)hipGetLastError();
    set_error(std::string("column ranges: ") + hipGetErrorString(e));
    return FS_EHIP;
  }
  return FS_OK;
}

int column_stats(const void* x, int x_is_f64, int64_t n, int64_t p, int64_t cap, int device,
                 void* colmin, void* colmax, int64_t* ndistinct) {
  if (device_count() <= 0) {
    set_error("backend='gpu' requested but no HIP device is visible");
    return FS_ENODEV;
  }
  // hash table: at least twice the cap, one key per 8 bytes of LDS
  int tbits = 6;
  while ((1ll << tbits) < 2 * (cap + 1)) tbits++;
  if (tbits > 14) {
    set_error("count_cap above 8191 is not supported by the GPU column statistics");
    return FS_ENOTSUP;
  }
  const size_t esz = x_is_f64 ? 8 : 4;
  int64_t rows_per_chunk = 0, nchunks = 0;
  minmax_grid(n, rows_per_chunk, nchunks);
  void *dx = nullptr, *pmin = nullptr, *pmax = nullptr, *dmin = nullptr, *dmax = nullptr;
  int64_t* dcnt = nullptr;
  hipStream_t s = nullptr;
  int rc = FS_OK;
  auto fail = [&](const char* what, hipError_t e) {
    set_error(std::string(what) + ": " + hipGetErrorString(e));
    (void)hipGetLastError();
    rc = (e == hipErrorOutOfMemory) ? FS_EOOM : FS_EHIP;
  };
  hipError_t e;
  if ((e = hipSetDevice(device)) != hipSuccess) fail("hipSetDevice", e);
  if (rc == FS_OK && (e = hipStreamCreateWithFlags(&s, hipStreamNonBlocking)) != hipSuccess)
    fail("hipStreamCreate", e);
  // a staged copy of x (fs_stage_x) is read in place, else x is uploaded
  const void* sx = staged_lookup(x, n, p, x_is_f64, device);
  if (rc == FS_OK && !sx) rc = dev_alloc((void**)&dx, (size_t)n * p * esz, device);
  if (rc == FS_OK) rc = dev_alloc((void**)&pmin, (size_t)nchunks * p * esz, device);
  if (rc == FS_OK) rc = dev_alloc((void**)&pmax, (size_t)nchunks * p * esz, device);
  if (rc == FS_OK) rc = dev_alloc((void**)&dmin, (size_t)p * esz, device);
  if (rc == FS_OK) rc = dev_alloc((void**)&dmax, (size_t)p * esz, device);
  if (rc == FS_OK) rc = dev_alloc((void**)&dcnt, (size_t)p * 8, device);
  if (rc == FS_OK &&
      !sx && (e = hipMemcpyAsync(dx, x, (size_t)n * p * esz, hipMemcpyHostToDevice, s)) != hipSuccess)
    fail("hipMemcpy H2D", e);
  const void* xd = sx ? sx : dx;
  // a staged copy cast by fs_stage_x_cast knows its extrema already
  const bool known = sx && staged_extrema(sx, colmin, colmax);
  if (rc == FS_OK) {
    const size_t lds = sizeof(unsigned long long) << tbits;
    if (!known)
      launch_minmax(xd, x_is_f64, n, p, rows_per_chunk, nchunks, pmin, pmax, dmin, dmax, s);
    if (x_is_f64)
      k_coldistinct<double><<<(unsigned)p, 256, lds, s>>>((const double*)xd, n, p, (int)cap,
                                                          tbits, dcnt);
    else
      k_coldistinct<float><<<(unsigned)p, 256, lds, s>>>((const float*)xd, n, p, (int)cap, tbits,
                                                         dcnt);
    if ((e = hipGetLastError()) != hipSuccess) fail("column statistics kernels", e);
  }
  if (rc == FS_OK &&
      ((!known &&
        ((e = hipMemcpyAsync(colmin, dmin, (size_t)p * esz, hipMemcpyDeviceToHost, s)) !=
             hipSuccess ||
         (e = hipMemcpyAsync(colmax, dmax, (size_t)p * esz, hipMemcpyDeviceToHost, s)) !=
             hipSuccess)) ||
       (e = hipMemcpyAsync(ndistinct, dcnt, (size_t)p * 8, hipMemcpyDeviceToHost, s)) !=
           hipSuccess))
    fail("hipMemcpy D2H", e);
  if (rc == FS_OK && (e = hipStreamSynchronize(s)) != hipSuccess) fail("column statistics", e);
  if (s) (void)hipStreamSynchronize(s);
  for (void* q : {dx, pmin, pmax, dmin, dmax, (void*)dcnt})
    if (q) dev_free(q);
  if (s) (void)hipStreamDestroy(s);
  return rc;
}

}  // namespace gpu
}  // namespace fs
