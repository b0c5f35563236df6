"""Microbenchmark + correctness check of the LDS-ring sparse stream
(tools/gen_sparse_asm.py gen_ring) against the scalar-load stream (gen) on
the same synthetic weights.  Writes ring_bench.hip; build:
  hipcc --offload-arch=gfx950 -O3 ring_bench.hip -o ring_bench"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from gen_sparse_asm import gen, gen_ring  # noqa: E402

src = ["#include <hip/hip_runtime.h>", "#include <cstdio>", "#include <cstdlib>", "#include <cstdint>",
       "#include <cmath>", "#include <vector>", "#include <random>",
       '#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)',
       gen_ring("RING"), gen("SMEM")]
src.append(r'''
constexpr int kTile = 128, kSWaves = 16, kStreamDw = 2048;   // 8 KB per stream
template <int V>
__global__ __launch_bounds__(1024) void kern(const uint32_t* ent, const uint4* cnt, const float* xs, int PW,
                                             int ntiles, int tiles_per_wg, float* out) {
  __shared__ float4 As[kTile * 64];
  __shared__ uint32_t ring[kSWaves * 512];
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  for (int r = wave; r < kTile; r += kSWaves) As[r * 64 + lane] = make_float4(r * 0.01f + lane, r * 0.01f + lane + 1, r * 0.01f + lane + 2, r * 0.01f + lane + 3);
  __syncthreads();
  float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  const uint32_t lane16 = (uint32_t)(uintptr_t)As + lane * 16u, lane4 = lane * 4u, laneoff = lane * 16u;
  const uint32_t ringa = (uint32_t)__builtin_amdgcn_readfirstlane((int)((uint32_t)(uintptr_t)ring + wave * 2048u));
  const uint32_t ringv = ringa;
  const uint32_t bstride = kSWaves * PW * 4, ncols = kTile / kSWaves;
  for (int k = 0; k < tiles_per_wg; k++) {
    const int t = __builtin_amdgcn_readfirstlane((int)((blockIdx.x / 32 * tiles_per_wg + k) % ntiles));
    const int64_t st = (int64_t)t * kSWaves + wave;
    const uint64_t eb = (uint64_t)(uintptr_t)(ent + st * kStreamDw);
    const uint64_t cb = (uint64_t)(uintptr_t)(cnt + st);
    const uint64_t bp = (uint64_t)(uintptr_t)(xs + (int64_t)wave * PW);
    if (V == 0) RING(acc, lane16, lane4, laneoff, ringv, ringa, eb, cb, bp, bstride);
    if (V == 1) SMEM(acc, lane16, lane4, eb, bp, bstride, ncols);
  }
  for (int i = 0; i < 8; i++) out[((size_t)blockIdx.x * 1024 + threadIdx.x) * 8 + i] = acc[i];
}

int main() {
  const int ntiles = 2048, PW = 1024;
  const double dens = 0.42;
  std::mt19937 rng(1);
  const size_t total_dw = (size_t)(ntiles + 1) * kSWaves * kStreamDw;
  std::vector<uint32_t> soa(total_dw, 0u), aos(total_dw, 0u);
  std::vector<uint4> cnt((size_t)(ntiles + 1) * kSWaves, make_uint4(0, 0, 0, 0));
  std::vector<int64_t> tile_groups(ntiles, 0);
  std::vector<std::vector<std::pair<int, float>>> lists((size_t)ntiles * kSWaves);
  for (int t = 0; t < ntiles; t++)
    for (int w = 0; w < kSWaves; w++) {
      const int64_t st = (int64_t)t * kSWaves + w;
      uint32_t* S = &soa[st * kStreamDw];
      uint32_t* A = &aos[st * kStreamDw];
      int grp = 0;
      uint32_t c03 = 0, c47 = 0;
      for (int m = 0; m < kTile / kSWaves; m++) {
        std::vector<std::pair<int, float>> col;
        for (int ii = 0; ii < kTile; ii++)
          if (std::uniform_real_distribution<double>(0, 1)(rng) < dens) col.push_back({ii, (float)(2 + (ii + m) % 7) * 0.125f});
        const int ng = col.empty() ? 1 : ((int)col.size() + 7) / 8;
        for (int e = 0; e < ng * 8; e++) {
          const int g = grp + e / 8, q = e % 8;
          const int row = e < (int)col.size() ? col[e].first : 0;
          const float wt = e < (int)col.size() ? col[e].second : 0.0f;
          uint32_t wb = __builtin_bit_cast(uint32_t, wt);
          S[g * 16 + q] = row * 1024u;
          S[g * 16 + 8 + q] = wb;
          A[g * 16 + 2 * q] = row * 1024u;
          A[g * 16 + 2 * q + 1] = (wb & ~1u) | ((e == (ng - 1) * 8) ? 1u : 0u);
        }
        grp += ng;
        if (m < 4) c03 |= (uint32_t)ng << (8 * m); else c47 |= (uint32_t)ng << (8 * (m - 4));
        for (auto& c : col) lists[st].push_back(c);
      }
      cnt[st] = make_uint4(c03, c47, (uint32_t)grp, 0);
      tile_groups[t] += grp;
    }
  uint32_t *dsoa, *daos; uint4* dcnt; float *dxs, *dout;
  CHK(hipMalloc(&dsoa, total_dw * 4)); CHK(hipMemcpy(dsoa, soa.data(), total_dw * 4, hipMemcpyHostToDevice));
  CHK(hipMalloc(&daos, total_dw * 4)); CHK(hipMemcpy(daos, aos.data(), total_dw * 4, hipMemcpyHostToDevice));
  CHK(hipMalloc(&dcnt, cnt.size() * 16)); CHK(hipMemcpy(dcnt, cnt.data(), cnt.size() * 16, hipMemcpyHostToDevice));
  std::vector<float> hx((size_t)(kTile + 2) * PW);
  for (size_t i = 0; i < hx.size(); i++) hx[i] = 0.5f * (float)((i % PW) / 64 % 4);
  CHK(hipMalloc(&dxs, hx.size() * 4)); CHK(hipMemcpy(dxs, hx.data(), hx.size() * 4, hipMemcpyHostToDevice));
  const int wgs = 4096, tpw = 4;
  CHK(hipMalloc(&dout, (size_t)wgs * 1024 * 8 * 4));
  const char* nm[2] = {"lds ring (SoA, LDS-DMA)", "scalar loads (shipped)"};
  double g_total = 0;
  for (int b = 0; b < wgs; b++) for (int k = 0; k < tpw; k++) g_total += tile_groups[(b / 32 * tpw + k) % ntiles];
  for (int v = 0; v < 2; v++) {
    auto K = v == 0 ? kern<0> : kern<1>;
    const uint32_t* E = v == 0 ? dsoa : daos;
    K<<<wgs, 1024>>>(E, dcnt, dxs, PW, ntiles, tpw, dout);
    CHK(hipDeviceSynchronize());
    std::vector<float> ho((size_t)wgs * 1024 * 8);
    CHK(hipMemcpy(ho.data(), dout, ho.size() * 4, hipMemcpyDeviceToHost));
    int bad = 0; double maxrel = 0;
    for (int b = 0; b < wgs; b += 397)
      for (int w = 0; w < kSWaves; w++)
        for (int lane = 0; lane < 64; lane += 7) {
          double want[4] = {0, 0, 0, 0};
          for (int k = 0; k < tpw; k++) {
            const int t = (b / 32 * tpw + k) % ntiles;
            for (auto& c : lists[(int64_t)t * kSWaves + w])
              for (int f = 0; f < 4; f++) want[f] += c.second * fabs((c.first * 0.01f + lane + f) - 0.5 * f);
          }
          const float* g = &ho[((size_t)b * 1024 + w * 64 + lane) * 8];
          for (int f = 0; f < 4; f++) {
            const double got = (double)g[2 * f] + g[2 * f + 1];
            const double rel = fabs(got - want[f]) / fmax(1.0, fabs(want[f]));
            if (rel > maxrel) maxrel = rel;
            if (rel > 1e-4) { if (bad < 5) printf("%s mismatch wg %d wave %d lane %d f %d: got %g want %g\n", nm[v], b, w, lane, f, got, want[f]); bad++; }
          }
        }
    printf("%-26s check: %s (max rel err %.2e)\n", nm[v], bad ? "WRONG" : "ok", maxrel);
    fflush(stdout);
    hipEvent_t e0, e1; CHK(hipEventCreate(&e0)); CHK(hipEventCreate(&e1));
    float best = 1e30f;
    for (int rep = 0; rep < 4; rep++) {
      CHK(hipEventRecord(e0));
      K<<<wgs, 1024>>>(E, dcnt, dxs, PW, ntiles, tpw, dout);
      CHK(hipEventRecord(e1)); CHK(hipEventSynchronize(e1));
      float ms; CHK(hipEventElapsedTime(&ms, e0, e1));
      if (rep && ms < best) best = ms;
    }
    printf("%-26s %8.3f ms   groups %.3g  cycles/group/SIMD %.1f  (VALU floor 160 = %.0f%%)\n", nm[v], best, g_total,
           best * 1e-3 * 2.4e9 * 1024 / g_total, 100 * 160 / (best * 1e-3 * 2.4e9 * 1024 / g_total));
    fflush(stdout);
  }
  return 0;
}
''')
open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "ring_bench.hip"), "w").write("\n".join(src))
