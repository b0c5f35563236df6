"""Generate gpridx.hip: can pass 2 skip zero pair weights with VGPR-indexed
rows (s_set_gpr_idx_on / s_set_gpr_idx_idx) at the dense VALU rate?

Variants (one wave = 32 rows x 2 features in v[40:103], per pair: 2 v_sub +
2 v_fma, weight in an SGPR):
  0 dense: static row registers, no SALU
  1 idx:   s_set_gpr_idx_idx per pair, src0 of the v_subs indexed
  2 idx + per-2-pairs s_bitcmp1 + s_cbranch_scc1 (never taken)
  3 idx + per-4-pairs s_bitcmp1 + s_cbranch_scc1
  4 idx + 2 extra SALU per pair (SALU issue sensitivity)
(v_movrels_b32 does not exist on gfx950.)
Also checks on the device that the indexed source is v[40 + r] and the
SGPR src0 of the fma is not offset.
"""
PAIRS = 16   # pairs per loop iteration

def body(v):
    L = []
    for k in range(PAIRS):
        r = f"%[r{k % 8}]"
        w = f"%[w{k % 8}]"
        t0, t1 = f"v{104 + 2 * (k % 4)}", f"v{105 + 2 * (k % 4)}"
        a0 = 40 if v in (1, 2, 3, 4) else 40 + (k * 5) % 32
        a1 = 72 if v in (1, 2, 3, 4) else 72 + (k * 5) % 32
        if True:
            if v in (1, 2, 3, 4):
                L.append(f"s_set_gpr_idx_idx {r}")
            L.append(f"v_sub_f32 {t0}, v{a0}, %[b0]")
            L.append(f"v_sub_f32 {t1}, v{a1}, %[b1]")
        L.append(f"v_fma_f32 %[acc{(2*k) % 8}], {w}, |{t0}|, %[acc{(2*k) % 8}]")
        L.append(f"v_fma_f32 %[acc{(2*k+1) % 8}], {w}, |{t1}|, %[acc{(2*k+1) % 8}]")
        if v == 4:
            L.append("s_add_u32 %[cnt], %[cnt], 0")
            L.append("s_add_u32 %[cnt], %[cnt], 0")
        if (v == 2 and k % 2 == 1) or (v == 3 and k % 4 == 3):
            L.append(f"s_bitcmp1_b32 {r}, 31")
            L.append(f"s_cbranch_scc1 9f")
    return L

def kernel(v):
    init = [f"v_add_f32 v{40 + r}, {float(r * 1000)}, %[la]" for r in range(32)]
    init += [f"v_add_f32 v{72 + r}, {float(r * 1000 + 500)}, %[la]" for r in range(32)]
    lines = init
    if v in (1, 2, 3, 4):
        lines.append("s_set_gpr_idx_on %[r0], gpr_idx(SRC0)")
    lines.append("s_mov_b32 %[cnt], %[iters]")
    lines.append("1:")
    lines += body(v)
    lines.append("s_sub_u32 %[cnt], %[cnt], 1")
    lines.append("s_cmp_lg_u32 %[cnt], 0")
    lines.append("s_cbranch_scc1 1b")
    lines.append("9:")
    if v in (1, 2, 3, 4):
        lines.append("s_set_gpr_idx_off")
    asm = "\\n\"\n      \"".join(lines)
    clob = ", ".join(f'"v{i}"' for i in range(40, 112))
    return f'''
__global__ __launch_bounds__(256) void kern{v}(const float* in, const int* rr, float* out, int iters) {{
  float acc0 = 0, acc1 = 0, acc2 = 0, acc3 = 0, acc4 = 0, acc5 = 0, acc6 = 0, acc7 = 0;
  const float la = (float)(threadIdx.x & 63);
  const float b0 = in[0], b1 = in[1];
  int r0 = __builtin_amdgcn_readfirstlane(rr[0]), r1 = __builtin_amdgcn_readfirstlane(rr[1]),
      r2 = __builtin_amdgcn_readfirstlane(rr[2]), r3 = __builtin_amdgcn_readfirstlane(rr[3]),
      r4 = __builtin_amdgcn_readfirstlane(rr[4]), r5 = __builtin_amdgcn_readfirstlane(rr[5]),
      r6 = __builtin_amdgcn_readfirstlane(rr[6]), r7 = __builtin_amdgcn_readfirstlane(rr[7]);
  float w0 = __builtin_amdgcn_readfirstlane(__float_as_int(in[2])), w1 = in[3], w2 = in[4], w3 = in[5],
        w4 = in[6], w5 = in[7], w6 = in[8], w7 = in[9];
  w0 = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(in[2])));
  w1 = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(in[3])));
  w2 = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(in[4])));
  w3 = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(in[5])));
  w4 = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(in[6])));
  w5 = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(in[7])));
  w6 = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(in[8])));
  w7 = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(in[9])));
  int cnt;
  asm volatile(
      "{asm}\\n"
      : [acc0] "+v"(acc0), [acc1] "+v"(acc1), [acc2] "+v"(acc2), [acc3] "+v"(acc3),
        [acc4] "+v"(acc4), [acc5] "+v"(acc5), [acc6] "+v"(acc6), [acc7] "+v"(acc7), [cnt] "=&s"(cnt)
      : [la] "v"(la), [b0] "v"(b0), [b1] "v"(b1), [iters] "s"(iters),
        [r0] "s"(r0), [r1] "s"(r1), [r2] "s"(r2), [r3] "s"(r3), [r4] "s"(r4), [r5] "s"(r5), [r6] "s"(r6), [r7] "s"(r7),
        [w0] "s"(w0), [w1] "s"(w1), [w2] "s"(w2), [w3] "s"(w3), [w4] "s"(w4), [w5] "s"(w5), [w6] "s"(w6), [w7] "s"(w7)
      : {clob}, "scc");
  float* o = out + ((size_t)blockIdx.x * 256 + threadIdx.x) * 8;
  o[0] = acc0; o[1] = acc1; o[2] = acc2; o[3] = acc3; o[4] = acc4; o[5] = acc5; o[6] = acc6; o[7] = acc7;
}}
'''

src = ['#include <hip/hip_runtime.h>', '#include <cstdio>', '#include <cstdlib>', '#include <cmath>', '#include <vector>',
       '#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)']
for v in range(5):
    src.append(kernel(v))
src.append(r'''
typedef void (*K)(const float*, const int*, float*, int);
int main() {
  const int blocks = 256 * 16;
  float *in, *out; int* rr;
  CHK(hipMalloc(&in, 64 * 4)); CHK(hipMalloc(&rr, 64 * 4)); CHK(hipMalloc(&out, (size_t)blocks * 256 * 8 * 4));
  float hin[16] = {0.25f, 0.5f, 1.0f, 2.0f, 4.0f, 8.0f, 16.0f, 32.0f, 64.0f, 128.0f};
  int hr[8] = {3, 7, 11, 0, 31, 19, 5, 26};
  CHK(hipMemcpy(in, hin, sizeof(hin), hipMemcpyHostToDevice));
  CHK(hipMemcpy(rr, hr, sizeof(hr), hipMemcpyHostToDevice));
  K ks[5] = {kern0, kern1, kern2, kern3, kern4};
  const char* nm[5] = {"dense (no SALU)", "idx per pair", "idx + bitcmp/branch per 2 pairs", "idx + bitcmp/branch per 4 pairs", "idx + 2 extra SALU per pair"};
  // correctness: one iteration, one block
  for (int v = 1; v < 5; v++) {
    ks[v]<<<1, 256>>>(in, rr, out, 1);
    CHK(hipDeviceSynchronize());
    std::vector<float> h(256 * 8);
    CHK(hipMemcpy(h.data(), out, h.size() * 4, hipMemcpyDeviceToHost));
    int bad = 0;
    for (int l = 0; l < 64; l++) {
      double acc[8] = {0};
      for (int k = 0; k < 16; k++) {
        int r = hr[k % 8]; double w = hin[2 + k % 8];
        acc[(2 * k) % 8] += w * fabs((r * 1000.0 + l) - hin[0]);
        acc[(2 * k + 1) % 8] += w * fabs((r * 1000.0 + 500 + l) - hin[1]);
      }
      for (int a = 0; a < 8; a++) if (fabs(acc[a] - h[l * 8 + a]) > 1e-3 * fabs(acc[a])) bad++;
    }
    printf("check %-36s %s\n", nm[v], bad ? "WRONG" : "ok");
  }
  const int iters = 4096;
  for (int v = 0; v < 5; v++) {
    hipEvent_t e0, e1; CHK(hipEventCreate(&e0)); CHK(hipEventCreate(&e1));
    float best = 1e30f;
    for (int rep = 0; rep < 4; rep++) {
      CHK(hipEventRecord(e0));
      ks[v]<<<blocks, 256>>>(in, rr, out, iters);
      CHK(hipEventRecord(e1)); CHK(hipEventSynchronize(e1));
      float ms; CHK(hipEventElapsedTime(&ms, e0, e1));
      if (rep && ms < best) best = ms;
    }
    double pairs_per_simd = (double)blocks * 4 * iters * 16 / 1024.0;   // wave-pairs per SIMD
    double valu = 4;
    printf("%-36s %8.3f ms  %.2f cycles/pair/SIMD @2.4GHz (VALU-only floor %.0f)\n", nm[v], best,
           best * 1e-3 * 2.4e9 / pairs_per_simd, valu * 2);
  }
  return 0;
}
''')
open(__file__.replace("gen_gpridx.py", "gpridx.hip"), "w").write("\n".join(src))
