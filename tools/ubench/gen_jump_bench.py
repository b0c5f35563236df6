"""Microbenchmark: a pass-2 layout with the focal ROWS in VGPRs (16 rows x 8
features per lane) and a per-entry computed jump (s_setpc_b64) into the code
block of the entry's row, instead of the shipped loop's LDS row read per
entry.  Per entry: 8 v_sub_f32 + 8 v_fma_f32 (no address add, no LDS read)
and 3 SALU (target = table + entry offset, s_setpc).  Blocks are duplicated
per entry position e (its weight SGPR) and row r: 256 blocks of 128 B.

Kernels:
  0 straight   -- the same 16 entries per step as straight-line code (no jumps):
                  the VALU + SALU floor of the block bodies
  1 jump       -- entries dispatched by s_setpc_b64 to random rows
  2 jump+B     -- as 1, plus a B-column reload from LDS (2 ds_read_b128) every
                  8 entries, waited at the next block (a column switch per
                  ~7 entries at 42% density over 16 rows)
Writes jump_bench.hip; build: hipcc --offload-arch=gfx950 -O3 jump_bench.hip -o jump_bench
"""
import os

NE, NR, BLK = 16, 16, 128
ROW0, B0, T0 = 40, 24, 32          # rows v40..v167, B v24..v31, diffs v32..v39
SE = 36                            # working entry set s36..s67, prefetch s68..s99


def block(e, r, kind, pre):
    L = []
    if kind == 2 and e in (0, 8):
        L.append("s_waitcnt lgkmcnt(0)")
    L += [f"v_sub_f32 v{T0 + f}, v{ROW0 + r * 8 + f}, v{B0 + f}" for f in range(8)]
    L += [f"v_fma_f32 %[acc{f}], s{SE + 2 * e + 1}, |v{T0 + f}|, %[acc{f}]" for f in range(8)]
    if kind == 2 and e in (7, 15):
        L += [f"ds_read_b128 v[{B0 + 4}:{B0 + 7}], %[lds_lane] offset:1024",
              f"ds_read_b128 v[{B0}:{B0 + 3}], %[lds_lane]"]
    if e < NE - 1:
        L += [f"s_add_u32 s18, s16, s{SE + 2 * (e + 1)}", "s_addc_u32 s19, s17, 0"]
        if kind != 0:
            L.append("s_setpc_b64 s[18:19]")
    else:
        L.append(f"s_branch {pre}_end")
    return L


def kernel(kind):
    pre = f"jb{kind}"
    lines = ["s_mov_b64 s[20:21], %[ep]", "s_mov_b32 s22, %[nsteps]",
             "s_getpc_b64 s[16:17]", f"{pre}_pc:",
             f"s_add_u32 s16, s16, {pre}_tab-{pre}_pc", "s_addc_u32 s17, s17, 0",
             "s_load_dwordx16 s[68:83], s[20:21], 0x0",
             "s_load_dwordx16 s[84:99], s[20:21], 0x40",
             "s_add_u32 s20, s20, 0x80", "s_addc_u32 s21, s21, 0",
             f"{pre}_top:", "s_waitcnt lgkmcnt(0)"]
    lines += [f"s_mov_b64 s[{SE + 2 * i}:{SE + 2 * i + 1}], s[{68 + 2 * i}:{69 + 2 * i}]" for i in range(16)]
    lines += ["s_load_dwordx16 s[68:83], s[20:21], 0x0",
              "s_load_dwordx16 s[84:99], s[20:21], 0x40",
              "s_add_u32 s20, s20, 0x80", "s_addc_u32 s21, s21, 0"]
    if kind == 0:
        for e in range(NE):
            lines += block(e, e % NR, kind, pre)
    else:
        lines += [f"s_add_u32 s18, s16, s{SE}", "s_addc_u32 s19, s17, 0", "s_setpc_b64 s[18:19]",
                  ".p2align 7", f"{pre}_tab:"]
        for e in range(NE):
            for r in range(NR):
                lines.append(".p2align 7")
                lines += block(e, r, kind, pre)
    if kind == 0:
        lines += [f"{pre}_tab:"]
    lines += [f"{pre}_end:", "s_sub_u32 s22, s22, 1", "s_cmp_gt_u32 s22, 0",
              f"s_cbranch_scc1 {pre}_top", "s_waitcnt vmcnt(0) lgkmcnt(0)"]
    body = "\n".join(f'      "{l}\\n"' for l in lines)
    vclob = ", ".join(f'"v{i}"' for i in range(B0, ROW0 + NR * 8))
    sclob = ", ".join(f'"s{i}"' for i in list(range(16, 23)) + list(range(36, 100)))
    init = "\n".join(
        f'  asm volatile("v_add_f32 v{ROW0 + k}, {float(k % 7) * 0.125}, %0" :: "v"(x) : "v{ROW0 + k}");'
        for k in range(NR * 8))
    initb = "\n".join(f'  asm volatile("v_mov_b32 v{B0 + f}, %0" :: "v"(x) : "v{B0 + f}");' for f in range(8))
    return f'''
__global__ __launch_bounds__(256) void kern{kind}(const uint32_t* ent, const float* in, float* out,
                                                  int nsteps, size_t stream_dw) {{
  __shared__ float lds[2048];
  for (int i = threadIdx.x; i < 2048; i += 256) lds[i] = in[i & 255];
  __syncthreads();
  const float x = in[threadIdx.x & 63];
  float acc0 = 0, acc1 = 0, acc2 = 0, acc3 = 0, acc4 = 0, acc5 = 0, acc6 = 0, acc7 = 0;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint64_t ep = (uint64_t)(uintptr_t)(ent + ((size_t)(blockIdx.x % 64) * 4 + wave) * stream_dw);
  const uint32_t lds_lane = (uint32_t)(uintptr_t)lds + (threadIdx.x & 63) * 16;
{init}
{initb}
  asm volatile(
{body}
      : [acc0] "+v"(acc0), [acc1] "+v"(acc1), [acc2] "+v"(acc2), [acc3] "+v"(acc3),
        [acc4] "+v"(acc4), [acc5] "+v"(acc5), [acc6] "+v"(acc6), [acc7] "+v"(acc7)
      : [ep] "s"(ep), [nsteps] "s"(nsteps), [lds_lane] "v"(lds_lane)
      : {vclob}, {sclob}, "scc", "memory");
  out[blockIdx.x * 256 + threadIdx.x] = acc0 + acc1 + acc2 + acc3 + acc4 + acc5 + acc6 + acc7;
}}
'''


src = ['#include <hip/hip_runtime.h>', '#include <cstdio>', '#include <cstdlib>', '#include <cstdint>',
       '#include <vector>', '#include <random>', '#include <cstring>',
       '#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)']
src += [kernel(0), kernel(1), kernel(2)]
src.append(r'''
int main() {
  const int nsteps = 512, blocks = 256 * 12;
  const size_t stream_dw = (size_t)(nsteps + 2) * 32;   // +2 steps: the prefetch reads one ahead
  std::vector<uint32_t> ent(stream_dw * 256);
  std::mt19937 rng(7);
  for (size_t s = 0; s < 256; s++)
    for (int st = 0; st < nsteps + 2; st++)
      for (int e = 0; e < 16; e++) {
        const uint32_t r = rng() % 16;
        const float w = 1e-3f * (1 + (rng() % 5));
        uint32_t wb; std::memcpy(&wb, &w, 4);
        ent[s * stream_dw + st * 32 + 2 * e] = (uint32_t)((e * 16 + r) * 128);
        ent[s * stream_dw + st * 32 + 2 * e + 1] = wb;
      }
  std::vector<float> in(256);
  for (int i = 0; i < 256; i++) in[i] = 0.001f * i;
  uint32_t* dent; float *din, *dout;
  CHK(hipMalloc(&dent, ent.size() * 4)); CHK(hipMemcpy(dent, ent.data(), ent.size() * 4, hipMemcpyHostToDevice));
  CHK(hipMalloc(&din, 1024)); CHK(hipMemcpy(din, in.data(), 1024, hipMemcpyHostToDevice));
  CHK(hipMalloc(&dout, (size_t)blocks * 256 * 4));
  const char* nm[3] = {"straight (no jumps)", "jump per entry", "jump + B reload / 8"};
  void (*K[3])(const uint32_t*, const float*, float*, int, size_t) = {kern0, kern1, kern2};
  for (int v = 0; v < 3; v++) {
    hipEvent_t e0, e1; CHK(hipEventCreate(&e0)); CHK(hipEventCreate(&e1));
    float best = 1e30f;
    for (int rep = 0; rep < 5; rep++) {
      CHK(hipEventRecord(e0)); K[v]<<<blocks, 256>>>(dent, din, dout, nsteps, stream_dw);
      CHK(hipEventRecord(e1)); CHK(hipEventSynchronize(e1));
      float ms; CHK(hipEventElapsedTime(&ms, e0, e1)); if (rep && ms < best) best = ms;
    }
    std::vector<float> o(256);
    CHK(hipMemcpy(o.data(), dout, 1024, hipMemcpyDeviceToHost));
    const double wave_entries = (double)blocks * 4 * nsteps * 16;
    const double per_simd = wave_entries / 1024.0;
    printf("%-24s %8.3f ms  %.2f cycles per entry per SIMD at 2.4 GHz (VALU floor 32)  chk %g\n",
           nm[v], best, best * 1e-3 * 2.4e9 / per_simd, (double)o[0]);
    fflush(stdout);
  }
  return 0;
}
''')
open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "jump_bench.hip"), "w").write("\n".join(src))
