// fs_sort.hip -- ordering of the exact-recompute pair lists.
//
// k_flag_pairs / k_rf_flag append pairs (i, j) in whatever order their
// workgroups finish.  Sorting the list by (i, j) (rocPRIM device radix sort
// on 40-bit keys i << 20 | j; the GPU backend keeps n < 2^20) gives
// k_exact_pairs runs of pairs that share row i, which its consecutive waves
// then read once through L2 instead of once per pair, and makes the list
// order deterministic.
#include <hip/hip_runtime.h>

#include <rocprim/device/device_radix_sort.hpp>

#include "fs_internal.h"

namespace fs {
namespace gpu {

namespace {
constexpr int kPairKeyShift = 20;

__global__ void k_pairs_to_keys(const int2* __restrict__ list, int64_t count,
                                unsigned long long* __restrict__ keys) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k < count) {
    const int2 p = list[k];
    keys[k] = ((unsigned long long)(unsigned)p.x << kPairKeyShift) | (unsigned)p.y;
  }
}

__global__ void k_keys_to_pairs(const unsigned long long* __restrict__ keys, int64_t count,
                                int2* __restrict__ list) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k < count) {
    const unsigned long long v = keys[k];
    list[k] = make_int2((int)(v >> kPairKeyShift), (int)(v & ((1ull << kPairKeyShift) - 1ull)));
  }
}
}  // namespace

// the two key arrays, rounded up so the rocPRIM storage after them is
// 256-byte aligned
static size_t keys_bytes(int64_t count) {
  return (2 * (size_t)count * sizeof(unsigned long long) + 255) & ~(size_t)255;
}

size_t pair_sort_scratch_bytes(int64_t count) {
  size_t temp = 0;
  unsigned long long* null_keys = nullptr;
  if (rocprim::radix_sort_keys(nullptr, temp, null_keys, null_keys, (size_t)count, 0,
                               2 * kPairKeyShift) != hipSuccess) {
    (void)hipGetLastError();
    return 0;
  }
  return keys_bytes(count) + ((temp + 255) & ~(size_t)255);
}

int sort_pairs(void* list_v, int64_t count, void* scratch, size_t scratch_bytes, void* stream) {
  int2* list = (int2*)list_v;
  if (count < 2) return 0;
  hipStream_t s = (hipStream_t)stream;
  unsigned long long* keys_in = (unsigned long long*)scratch;
  unsigned long long* keys_out = keys_in + count;
  void* temp = (char*)scratch + keys_bytes(count);
  size_t temp_bytes = scratch_bytes - keys_bytes(count);
  const unsigned grid = (unsigned)((count + 255) / 256);
  k_pairs_to_keys<<<grid, 256, 0, s>>>(list, count, keys_in);
  if (rocprim::radix_sort_keys(temp, temp_bytes, keys_in, keys_out, (size_t)count, 0,
                               2 * kPairKeyShift, s) != hipSuccess) {
    (void)hipGetLastError();
    set_error("pair list sort failed");
    return -1;
  }
  k_keys_to_pairs<<<grid, 256, 0, s>>>(keys_out, count, list);
  if (hipGetLastError() != hipSuccess) {
    set_error("pair list sort: kernel launch failed");
    return -1;
  }
  return 0;
}

}  // namespace gpu
}  // namespace fs
