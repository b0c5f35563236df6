"""Microbenchmark: dense pass-2 column step (32 rows in VGPRs x 2 features,
weights in SGPRs) with and without a scalar branch skipping zero-weight rows.
Writes branch_bench.hip; build: hipcc --offload-arch=gfx950 -O3 branch_bench.hip -o branch_bench"""
import os

def column(skip, ws, label):
    L = []
    for r in range(32):
        w = f"s{ws + r}"
        if skip:
            L += [f"s_cmp_lg_u32 {w}, 0", f"s_cbranch_scc0 {label}{r}f"]
        L += [f"v_sub_f32 v{100 + (r % 2) * 2}, v{36 + r}, %[b0]",
              f"v_sub_f32 v{101 + (r % 2) * 2}, v{68 + r}, %[b1]",
              f"v_fma_f32 %[acc{r % 4}], {w}, |v{100 + (r % 2) * 2}|, %[acc{r % 4}]",
              f"v_fma_f32 %[acc{4 + r % 4}], {w}, |v{101 + (r % 2) * 2}|, %[acc{4 + r % 4}]"]
        if skip:
            L.append(f"{label}{r}:")
    return L

def kernel(v):
    skip = v == 1
    init = [f"v_add_f32 v{36 + r}, {float(r)}, %[b0]" for r in range(32)] + \
           [f"v_add_f32 v{68 + r}, {float(r) + 0.5}, %[b1]" for r in range(32)]
    lines = init + ["s_mov_b64 s[34:35], %[wp]", "s_mov_b32 s33, %[ncol]",
                    "s_load_dwordx16 s[36:51], s[34:35], 0x0", "s_load_dwordx16 s[52:67], s[34:35], 0x40",
                    "1:",
                    "s_waitcnt lgkmcnt(0)",
                    "s_add_u32 s34, s34, 0x80", "s_addc_u32 s35, s35, 0",
                    "s_load_dwordx16 s[68:83], s[34:35], 0x0", "s_load_dwordx16 s[84:99], s[34:35], 0x40"]
    # two columns per iteration (ping-pong SGPR sets)
    lines += column(skip, 36, 3)
    lines += ["s_waitcnt lgkmcnt(0)", "s_add_u32 s34, s34, 0x80", "s_addc_u32 s35, s35, 0",
              "s_load_dwordx16 s[36:51], s[34:35], 0x0", "s_load_dwordx16 s[52:67], s[34:35], 0x40"]
    lines += column(skip, 68, 4)
    lines += ["s_sub_u32 s33, s33, 2", "s_cmp_gt_i32 s33, 0", "s_cbranch_scc1 1b", "s_waitcnt lgkmcnt(0)"]
    body = "\n".join(f'      "{l}\\n"' for l in lines)
    vclob = ", ".join(f'"v{i}"' for i in range(36, 104))
    sclob = ", ".join(f'"s{i}"' for i in range(33, 100))
    return f'''
__global__ __launch_bounds__(256) void kern{v}(const float* in, const float* wts, float* out, int ncol) {{
  float acc0 = 0, acc1 = 0, acc2 = 0, acc3 = 0, acc4 = 0, acc5 = 0, acc6 = 0, acc7 = 0;
  const float b0 = in[threadIdx.x & 63], b1 = in[64 + (threadIdx.x & 63)];
  const uint64_t wp = (uint64_t)(uintptr_t)(wts + (size_t)(blockIdx.x % 64) * 32 * 4096);
  asm volatile(
{body}
      : [acc0] "+v"(acc0), [acc1] "+v"(acc1), [acc2] "+v"(acc2), [acc3] "+v"(acc3),
        [acc4] "+v"(acc4), [acc5] "+v"(acc5), [acc6] "+v"(acc6), [acc7] "+v"(acc7)
      : [b0] "v"(b0), [b1] "v"(b1), [wp] "s"(wp), [ncol] "s"(ncol)
      : {vclob}, {sclob}, "scc", "memory");
  out[blockIdx.x * 256 + threadIdx.x] = acc0 + acc1 + acc2 + acc3 + acc4 + acc5 + acc6 + acc7;
}}
'''

src = ['#include <hip/hip_runtime.h>', '#include <cstdio>', '#include <cstdlib>', '#include <cstdint>', '#include <vector>', '#include <random>',
       '#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)']
src += [kernel(0), kernel(1)]
src.append(r'''
int main() {
  const int ncol = 2048, blocks = 256 * 20;
  std::vector<float> w((size_t)64 * 32 * 4096 + 64);
  std::mt19937 rng(1);
  for (auto& x : w) x = std::uniform_real_distribution<float>(0, 1)(rng) < 0.42f ? 0.01f : 0.0f;
  float *din, *dw, *dout;
  CHK(hipMalloc(&din, 512)); CHK(hipMemset(din, 0, 512));
  CHK(hipMalloc(&dw, w.size() * 4)); CHK(hipMemcpy(dw, w.data(), w.size() * 4, hipMemcpyHostToDevice));
  CHK(hipMalloc(&dout, (size_t)blocks * 256 * 4));
  const char* nm[2] = {"dense", "branch-skip zero rows"};
  for (int v = 0; v < 2; v++) {
    auto K = v == 0 ? kern0 : kern1;
    hipEvent_t e0, e1; CHK(hipEventCreate(&e0)); CHK(hipEventCreate(&e1));
    float best = 1e30f;
    for (int rep = 0; rep < 4; rep++) {
      CHK(hipEventRecord(e0)); K<<<blocks, 256>>>(din, dw, dout, ncol);
      CHK(hipEventRecord(e1)); CHK(hipEventSynchronize(e1));
      float ms; CHK(hipEventElapsedTime(&ms, e0, e1)); if (rep && ms < best) best = ms;
    }
    const double rowcols = (double)blocks * 4 * ncol * 32 / 1024.0;   // per SIMD
    printf("%-24s %8.3f ms  %.2f cycles per row-column per SIMD (dense VALU floor 8)\n", nm[v], best, best * 1e-3 * 2.4e9 / rowcols);
    fflush(stdout);
  }
  return 0;
}
''')
open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "branch_bench.hip"), "w").write("\n".join(src))
