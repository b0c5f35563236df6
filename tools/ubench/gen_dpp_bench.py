"""Microbenchmark + correctness check of the DPP-broadcast sparse stream
(tools/gen_sparse_asm.py gen_dpp) on synthetic streams.  Writes dpp_bench.hip;
build: hipcc --offload-arch=gfx950 -O3 dpp_bench.hip -o dpp_bench"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from gen_sparse_asm import gen_dpp_macro  # noqa: E402

src = ["#include <hip/hip_runtime.h>", "#include <cstdio>", "#include <cstdlib>", "#include <cstdint>",
       "#include <cmath>", "#include <vector>", "#include <random>",
       '#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)',
       gen_dpp_macro("STREAM"), gen_dpp_macro("STREAM1", plain_fma=True), gen_dpp_macro("STREAM2", no_b=True),
       gen_dpp_macro("STREAM3", no_ds=True), gen_dpp_macro("STREAM4", plain_fma=True, plain_add=True, no_b=True)]
src.append(r'''
constexpr int kTile = 128, kSWaves = 16, kStreamGroups = 128;
template <int V>
__global__ __launch_bounds__(1024) void kern(const uint2* ent, const uint4* cnt, const float* xs, int PW, int ntiles,
                                             int tiles_per_wg, float* out) {
  __shared__ float4 As[kTile * 64];
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  for (int r = wave; r < kTile; r += kSWaves) As[r * 64 + lane] = make_float4(r * 0.01f + lane, r * 0.01f + lane + 1, r * 0.01f + lane + 2, r * 0.01f + lane + 3);
  __syncthreads();
  float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  const uint32_t lane16 = (uint32_t)(uintptr_t)As + lane * 16u, lane4 = lane * 4u, laneoff = (lane & 15) * 8u;
  const uint32_t bstride = kSWaves * PW * 4;
  for (int k = 0; k < tiles_per_wg; k++) {
    const int t = __builtin_amdgcn_readfirstlane((int)((blockIdx.x / 32 * tiles_per_wg + k) % ntiles));
    const int64_t st = (int64_t)t * kSWaves + wave;
    const uint64_t eb = (uint64_t)(uintptr_t)(ent + st * kStreamGroups * 8);
    const uint64_t cb = (uint64_t)(uintptr_t)(cnt + st);
    const uint64_t bp = (uint64_t)(uintptr_t)(xs + (int64_t)wave * PW);
    if (V == 0) STREAM(acc, lane16, lane4, laneoff, eb, cb, bp, bstride);
    if (V == 1) STREAM1(acc, lane16, lane4, laneoff, eb, cb, bp, bstride);
    if (V == 2) STREAM2(acc, lane16, lane4, laneoff, eb, cb, bp, bstride);
    if (V == 3) STREAM3(acc, lane16, lane4, laneoff, eb, cb, bp, bstride);
    if (V == 4) STREAM4(acc, lane16, lane4, laneoff, eb, cb, bp, bstride);
  }
  for (int i = 0; i < 8; i++) out[((size_t)blockIdx.x * 1024 + threadIdx.x) * 8 + i] = acc[i];
}

int main() {
  const int ntiles = 2048, PW = 1024;
  const double dens = 0.42;
  std::mt19937 rng(1);
  std::vector<uint2> ent((size_t)(ntiles + 1) * kSWaves * kStreamGroups * 8, make_uint2(0, 0));
  std::vector<uint4> cnt((size_t)(ntiles + 1) * kSWaves, make_uint4(0, 0, 0, 0));
  std::vector<int64_t> tile_groups(ntiles, 0);
  for (int t = 0; t < ntiles; t++)
    for (int w = 0; w < kSWaves; w++) {
      const int64_t st = (int64_t)t * kSWaves + w;
      uint2* o = &ent[st * kStreamGroups * 8];
      int off = 0, tot = 0;
      uint32_t c03 = 0, c47 = 0;
      for (int m = 0; m < kTile / kSWaves; m++) {
        int c = 0;
        for (int ii = 0; ii < kTile; ii++)
          if (std::uniform_real_distribution<double>(0, 1)(rng) < dens)
            o[off + c++] = make_uint2(ii * 1024u, __builtin_bit_cast(uint32_t, (float)(1 + (ii + m) % 7) * 0.125f));
        int pad = c == 0 ? 8 : (c + 7) / 8 * 8;
        for (int e = c; e < pad; e++) o[off + e] = make_uint2(0, 0);
        off += pad;
        const int ng = pad / 8;
        if (m < 4) c03 |= (uint32_t)ng << (8 * m); else c47 |= (uint32_t)ng << (8 * (m - 4));
        tot += ng;
      }
      cnt[st] = make_uint4(c03, c47, (uint32_t)tot, 0);
      tile_groups[t] += tot;
    }
  uint2* dent; uint4* dcnt; float *dxs, *dout;
  CHK(hipMalloc(&dent, ent.size() * 8)); CHK(hipMemcpy(dent, ent.data(), ent.size() * 8, hipMemcpyHostToDevice));
  CHK(hipMalloc(&dcnt, cnt.size() * 16)); CHK(hipMemcpy(dcnt, cnt.data(), cnt.size() * 16, hipMemcpyHostToDevice));
  // B rows: xs[row][f0 + lane + 64 f] = 0.5 * f (row-independent)
  std::vector<float> hx((size_t)(kTile + 2) * PW);
  for (size_t i = 0; i < hx.size(); i++) hx[i] = 0.5f * (float)((i % PW) / 64 % 4);
  CHK(hipMalloc(&dxs, hx.size() * 4)); CHK(hipMemcpy(dxs, hx.data(), hx.size() * 4, hipMemcpyHostToDevice));
  const int wgs = 4096, tpw = 4;
  CHK(hipMalloc(&dout, (size_t)wgs * 1024 * 8 * 4));
  // correctness on a few workgroups
  kern<0><<<wgs, 1024>>>(dent, dcnt, dxs, PW, ntiles, tpw, dout);
  CHK(hipDeviceSynchronize());
  std::vector<float> ho((size_t)wgs * 1024 * 8);
  CHK(hipMemcpy(ho.data(), dout, ho.size() * 4, hipMemcpyDeviceToHost));
  int bad = 0; double maxrel = 0;
  for (int b = 0; b < wgs; b += 397)
    for (int w = 0; w < kSWaves; w++)
      for (int lane = 0; lane < 64; lane += 7) {
        double want[4] = {0, 0, 0, 0}, got[4] = {0, 0, 0, 0};
        for (int k = 0; k < tpw; k++) {
          const int t = (b / 32 * tpw + k) % ntiles;
          const int64_t st = (int64_t)t * kSWaves + w;
          const uint2* o = &ent[st * kStreamGroups * 8];
          for (int e = 0; e < (int)cnt[st].z * 8; e++) {
            const int r = o[e].x / 1024; const float wt = __builtin_bit_cast(float, o[e].y);
            for (int f = 0; f < 4; f++) want[f] += wt * fabs((r * 0.01f + lane + f) - 0.5 * f);
          }
        }
        const float* g = &ho[((size_t)b * 1024 + w * 64 + lane) * 8];
        for (int f = 0; f < 4; f++) {
          got[f] = (double)g[2 * f] + g[2 * f + 1];
          const double rel = fabs(got[f] - want[f]) / fmax(1.0, fabs(want[f]));
          if (rel > maxrel) maxrel = rel;
          if (rel > 1e-4) { if (bad < 5) printf("mismatch wg %d wave %d lane %d f %d: got %g want %g\n", b, w, lane, f, got[f], want[f]); bad++; }
        }
      }
  printf("check: %s (max rel err %.2e)\n", bad ? "WRONG" : "ok", maxrel);
  fflush(stdout);
  double g_total = 0;
  for (int b = 0; b < wgs; b++) for (int k = 0; k < tpw; k++) g_total += tile_groups[(b / 32 * tpw + k) % ntiles];
  const char* nm[5] = {"dpp stream", "plain fma", "no per-group B", "no LDS reads", "plain fma+add, no B"};
  for (int v = 0; v < 5; v++) {
  auto K = v == 0 ? kern<0> : v == 1 ? kern<1> : v == 2 ? kern<2> : v == 3 ? kern<3> : kern<4>;
  hipEvent_t e0, e1; CHK(hipEventCreate(&e0)); CHK(hipEventCreate(&e1));
  float best = 1e30f;
  for (int rep = 0; rep < 4; rep++) {
    CHK(hipEventRecord(e0));
    K<<<wgs, 1024>>>(dent, dcnt, dxs, PW, ntiles, tpw, dout);
    CHK(hipEventRecord(e1)); CHK(hipEventSynchronize(e1));
    float ms; CHK(hipEventElapsedTime(&ms, e0, e1));
    if (rep && ms < best) best = ms;
  }
  const double valu_ms = g_total * 72 * 2 / 1024.0 / 2.4e9 * 1e3;
  printf("%-22s %8.3f ms   groups %.3g  cycles/group/SIMD %.1f  per entry-feature %.2f  (VALU floor %.3f ms = %.0f%%)\n",
         nm[v], best, g_total, best * 1e-3 * 2.4e9 * 1024 / g_total, best * 1e-3 * 2.4e9 * 1024 / g_total / 32, valu_ms, 100 * valu_ms / best);
  fflush(stdout);
  }
  return 0;
}
''')
open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "dpp_bench.hip"), "w").write("\n".join(src))
