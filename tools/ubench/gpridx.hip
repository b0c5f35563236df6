#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cmath>
#include <vector>
#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

__global__ __launch_bounds__(256) void kern0(const float* in, const int* rr, float* out, int iters) {
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
      "v_add_f32 v40, 0.0, %[la]\n"
      "v_add_f32 v41, 1000.0, %[la]\n"
      "v_add_f32 v42, 2000.0, %[la]\n"
      "v_add_f32 v43, 3000.0, %[la]\n"
      "v_add_f32 v44, 4000.0, %[la]\n"
      "v_add_f32 v45, 5000.0, %[la]\n"
      "v_add_f32 v46, 6000.0, %[la]\n"
      "v_add_f32 v47, 7000.0, %[la]\n"
      "v_add_f32 v48, 8000.0, %[la]\n"
      "v_add_f32 v49, 9000.0, %[la]\n"
      "v_add_f32 v50, 10000.0, %[la]\n"
      "v_add_f32 v51, 11000.0, %[la]\n"
      "v_add_f32 v52, 12000.0, %[la]\n"
      "v_add_f32 v53, 13000.0, %[la]\n"
      "v_add_f32 v54, 14000.0, %[la]\n"
      "v_add_f32 v55, 15000.0, %[la]\n"
      "v_add_f32 v56, 16000.0, %[la]\n"
      "v_add_f32 v57, 17000.0, %[la]\n"
      "v_add_f32 v58, 18000.0, %[la]\n"
      "v_add_f32 v59, 19000.0, %[la]\n"
      "v_add_f32 v60, 20000.0, %[la]\n"
      "v_add_f32 v61, 21000.0, %[la]\n"
      "v_add_f32 v62, 22000.0, %[la]\n"
      "v_add_f32 v63, 23000.0, %[la]\n"
      "v_add_f32 v64, 24000.0, %[la]\n"
      "v_add_f32 v65, 25000.0, %[la]\n"
      "v_add_f32 v66, 26000.0, %[la]\n"
      "v_add_f32 v67, 27000.0, %[la]\n"
      "v_add_f32 v68, 28000.0, %[la]\n"
      "v_add_f32 v69, 29000.0, %[la]\n"
      "v_add_f32 v70, 30000.0, %[la]\n"
      "v_add_f32 v71, 31000.0, %[la]\n"
      "v_add_f32 v72, 500.0, %[la]\n"
      "v_add_f32 v73, 1500.0, %[la]\n"
      "v_add_f32 v74, 2500.0, %[la]\n"
      "v_add_f32 v75, 3500.0, %[la]\n"
      "v_add_f32 v76, 4500.0, %[la]\n"
      "v_add_f32 v77, 5500.0, %[la]\n"
      "v_add_f32 v78, 6500.0, %[la]\n"
      "v_add_f32 v79, 7500.0, %[la]\n"
      "v_add_f32 v80, 8500.0, %[la]\n"
      "v_add_f32 v81, 9500.0, %[la]\n"
      "v_add_f32 v82, 10500.0, %[la]\n"
      "v_add_f32 v83, 11500.0, %[la]\n"
      "v_add_f32 v84, 12500.0, %[la]\n"
      "v_add_f32 v85, 13500.0, %[la]\n"
      "v_add_f32 v86, 14500.0, %[la]\n"
      "v_add_f32 v87, 15500.0, %[la]\n"
      "v_add_f32 v88, 16500.0, %[la]\n"
      "v_add_f32 v89, 17500.0, %[la]\n"
      "v_add_f32 v90, 18500.0, %[la]\n"
      "v_add_f32 v91, 19500.0, %[la]\n"
      "v_add_f32 v92, 20500.0, %[la]\n"
      "v_add_f32 v93, 21500.0, %[la]\n"
      "v_add_f32 v94, 22500.0, %[la]\n"
      "v_add_f32 v95, 23500.0, %[la]\n"
      "v_add_f32 v96, 24500.0, %[la]\n"
      "v_add_f32 v97, 25500.0, %[la]\n"
      "v_add_f32 v98, 26500.0, %[la]\n"
      "v_add_f32 v99, 27500.0, %[la]\n"
      "v_add_f32 v100, 28500.0, %[la]\n"
      "v_add_f32 v101, 29500.0, %[la]\n"
      "v_add_f32 v102, 30500.0, %[la]\n"
      "v_add_f32 v103, 31500.0, %[la]\n"
      "s_mov_b32 %[cnt], %[iters]\n"
      "1:\n"
      "v_sub_f32 v104, v40, %[b0]\n"
      "v_sub_f32 v105, v72, %[b1]\n"
      "v_fma_f32 %[acc0], %[w0], |v104|, %[acc0]\n"
      "v_fma_f32 %[acc1], %[w0], |v105|, %[acc1]\n"
      "v_sub_f32 v106, v45, %[b0]\n"
      "v_sub_f32 v107, v77, %[b1]\n"
      "v_fma_f32 %[acc2], %[w1], |v106|, %[acc2]\n"
      "v_fma_f32 %[acc3], %[w1], |v107|, %[acc3]\n"
      "v_sub_f32 v108, v50, %[b0]\n"
      "v_sub_f32 v109, v82, %[b1]\n"
      "v_fma_f32 %[acc4], %[w2], |v108|, %[acc4]\n"
      "v_fma_f32 %[acc5], %[w2], |v109|, %[acc5]\n"
      "v_sub_f32 v110, v55, %[b0]\n"
      "v_sub_f32 v111, v87, %[b1]\n"
      "v_fma_f32 %[acc6], %[w3], |v110|, %[acc6]\n"
      "v_fma_f32 %[acc7], %[w3], |v111|, %[acc7]\n"
      "v_sub_f32 v104, v60, %[b0]\n"
      "v_sub_f32 v105, v92, %[b1]\n"
      "v_fma_f32 %[acc0], %[w4], |v104|, %[acc0]\n"
      "v_fma_f32 %[acc1], %[w4], |v105|, %[acc1]\n"
      "v_sub_f32 v106, v65, %[b0]\n"
      "v_sub_f32 v107, v97, %[b1]\n"
      "v_fma_f32 %[acc2], %[w5], |v106|, %[acc2]\n"
      "v_fma_f32 %[acc3], %[w5], |v107|, %[acc3]\n"
      "v_sub_f32 v108, v70, %[b0]\n"
      "v_sub_f32 v109, v102, %[b1]\n"
      "v_fma_f32 %[acc4], %[w6], |v108|, %[acc4]\n"
      "v_fma_f32 %[acc5], %[w6], |v109|, %[acc5]\n"
      "v_sub_f32 v110, v43, %[b0]\n"
      "v_sub_f32 v111, v75, %[b1]\n"
      "v_fma_f32 %[acc6], %[w7], |v110|, %[acc6]\n"
      "v_fma_f32 %[acc7], %[w7], |v111|, %[acc7]\n"
      "v_sub_f32 v104, v48, %[b0]\n"
      "v_sub_f32 v105, v80, %[b1]\n"
      "v_fma_f32 %[acc0], %[w0], |v104|, %[acc0]\n"
      "v_fma_f32 %[acc1], %[w0], |v105|, %[acc1]\n"
      "v_sub_f32 v106, v53, %[b0]\n"
      "v_sub_f32 v107, v85, %[b1]\n"
      "v_fma_f32 %[acc2], %[w1], |v106|, %[acc2]\n"
      "v_fma_f32 %[acc3], %[w1], |v107|, %[acc3]\n"
      "v_sub_f32 v108, v58, %[b0]\n"
      "v_sub_f32 v109, v90, %[b1]\n"
      "v_fma_f32 %[acc4], %[w2], |v108|, %[acc4]\n"
      "v_fma_f32 %[acc5], %[w2], |v109|, %[acc5]\n"
      "v_sub_f32 v110, v63, %[b0]\n"
      "v_sub_f32 v111, v95, %[b1]\n"
      "v_fma_f32 %[acc6], %[w3], |v110|, %[acc6]\n"
      "v_fma_f32 %[acc7], %[w3], |v111|, %[acc7]\n"
      "v_sub_f32 v104, v68, %[b0]\n"
      "v_sub_f32 v105, v100, %[b1]\n"
      "v_fma_f32 %[acc0], %[w4], |v104|, %[acc0]\n"
      "v_fma_f32 %[acc1], %[w4], |v105|, %[acc1]\n"
      "v_sub_f32 v106, v41, %[b0]\n"
      "v_sub_f32 v107, v73, %[b1]\n"
      "v_fma_f32 %[acc2], %[w5], |v106|, %[acc2]\n"
      "v_fma_f32 %[acc3], %[w5], |v107|, %[acc3]\n"
      "v_sub_f32 v108, v46, %[b0]\n"
      "v_sub_f32 v109, v78, %[b1]\n"
      "v_fma_f32 %[acc4], %[w6], |v108|, %[acc4]\n"
      "v_fma_f32 %[acc5], %[w6], |v109|, %[acc5]\n"
      "v_sub_f32 v110, v51, %[b0]\n"
      "v_sub_f32 v111, v83, %[b1]\n"
      "v_fma_f32 %[acc6], %[w7], |v110|, %[acc6]\n"
      "v_fma_f32 %[acc7], %[w7], |v111|, %[acc7]\n"
      "s_sub_u32 %[cnt], %[cnt], 1\n"
      "s_cmp_lg_u32 %[cnt], 0\n"
      "s_cbranch_scc1 1b\n"
      "9:\n"
      : [acc0] "+v"(acc0), [acc1] "+v"(acc1), [acc2] "+v"(acc2), [acc3] "+v"(acc3),
        [acc4] "+v"(acc4), [acc5] "+v"(acc5), [acc6] "+v"(acc6), [acc7] "+v"(acc7), [cnt] "=&s"(cnt)
      : [la] "v"(la), [b0] "v"(b0), [b1] "v"(b1), [iters] "s"(iters),
        [r0] "s"(r0), [r1] "s"(r1), [r2] "s"(r2), [r3] "s"(r3), [r4] "s"(r4), [r5] "s"(r5), [r6] "s"(r6), [r7] "s"(r7),
        [w0] "s"(w0), [w1] "s"(w1), [w2] "s"(w2), [w3] "s"(w3), [w4] "s"(w4), [w5] "s"(w5), [w6] "s"(w6), [w7] "s"(w7)
      : "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v48", "v49", "v50", "v51", "v52", "v53", "v54", "v55", "v56", "v57", "v58", "v59", "v60", "v61", "v62", "v63", "v64", "v65", "v66", "v67", "v68", "v69", "v70", "v71", "v72", "v73", "v74", "v75", "v76", "v77", "v78", "v79", "v80", "v81", "v82", "v83", "v84", "v85", "v86", "v87", "v88", "v89", "v90", "v91", "v92", "v93", "v94", "v95", "v96", "v97", "v98", "v99", "v100", "v101", "v102", "v103", "v104", "v105", "v106", "v107", "v108", "v109", "v110", "v111", "scc");
  float* o = out + ((size_t)blockIdx.x * 256 + threadIdx.x) * 8;
  o[0] = acc0; o[1] = acc1; o[2] = acc2; o[3] = acc3; o[4] = acc4; o[5] = acc5; o[6] = acc6; o[7] = acc7;
}


__global__ __launch_bounds__(256) void kern1(const float* in, const int* rr, float* out, int iters) {
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
      "v_add_f32 v40, 0.0, %[la]\n"
      "v_add_f32 v41, 1000.0, %[la]\n"
      "v_add_f32 v42, 2000.0, %[la]\n"
      "v_add_f32 v43, 3000.0, %[la]\n"
      "v_add_f32 v44, 4000.0, %[la]\n"
      "v_add_f32 v45, 5000.0, %[la]\n"
      "v_add_f32 v46, 6000.0, %[la]\n"
      "v_add_f32 v47, 7000.0, %[la]\n"
      "v_add_f32 v48, 8000.0, %[la]\n"
      "v_add_f32 v49, 9000.0, %[la]\n"
      "v_add_f32 v50, 10000.0, %[la]\n"
      "v_add_f32 v51, 11000.0, %[la]\n"
      "v_add_f32 v52, 12000.0, %[la]\n"
      "v_add_f32 v53, 13000.0, %[la]\n"
      "v_add_f32 v54, 14000.0, %[la]\n"
      "v_add_f32 v55, 15000.0, %[la]\n"
      "v_add_f32 v56, 16000.0, %[la]\n"
      "v_add_f32 v57, 17000.0, %[la]\n"
      "v_add_f32 v58, 18000.0, %[la]\n"
      "v_add_f32 v59, 19000.0, %[la]\n"
      "v_add_f32 v60, 20000.0, %[la]\n"
      "v_add_f32 v61, 21000.0, %[la]\n"
      "v_add_f32 v62, 22000.0, %[la]\n"
      "v_add_f32 v63, 23000.0, %[la]\n"
      "v_add_f32 v64, 24000.0, %[la]\n"
      "v_add_f32 v65, 25000.0, %[la]\n"
      "v_add_f32 v66, 26000.0, %[la]\n"
      "v_add_f32 v67, 27000.0, %[la]\n"
      "v_add_f32 v68, 28000.0, %[la]\n"
      "v_add_f32 v69, 29000.0, %[la]\n"
      "v_add_f32 v70, 30000.0, %[la]\n"
      "v_add_f32 v71, 31000.0, %[la]\n"
      "v_add_f32 v72, 500.0, %[la]\n"
      "v_add_f32 v73, 1500.0, %[la]\n"
      "v_add_f32 v74, 2500.0, %[la]\n"
      "v_add_f32 v75, 3500.0, %[la]\n"
      "v_add_f32 v76, 4500.0, %[la]\n"
      "v_add_f32 v77, 5500.0, %[la]\n"
      "v_add_f32 v78, 6500.0, %[la]\n"
      "v_add_f32 v79, 7500.0, %[la]\n"
      "v_add_f32 v80, 8500.0, %[la]\n"
      "v_add_f32 v81, 9500.0, %[la]\n"
      "v_add_f32 v82, 10500.0, %[la]\n"
      "v_add_f32 v83, 11500.0, %[la]\n"
      "v_add_f32 v84, 12500.0, %[la]\n"
      "v_add_f32 v85, 13500.0, %[la]\n"
      "v_add_f32 v86, 14500.0, %[la]\n"
      "v_add_f32 v87, 15500.0, %[la]\n"
      "v_add_f32 v88, 16500.0, %[la]\n"
      "v_add_f32 v89, 17500.0, %[la]\n"
      "v_add_f32 v90, 18500.0, %[la]\n"
      "v_add_f32 v91, 19500.0, %[la]\n"
      "v_add_f32 v92, 20500.0, %[la]\n"
      "v_add_f32 v93, 21500.0, %[la]\n"
      "v_add_f32 v94, 22500.0, %[la]\n"
      "v_add_f32 v95, 23500.0, %[la]\n"
      "v_add_f32 v96, 24500.0, %[la]\n"
      "v_add_f32 v97, 25500.0, %[la]\n"
      "v_add_f32 v98, 26500.0, %[la]\n"
      "v_add_f32 v99, 27500.0, %[la]\n"
      "v_add_f32 v100, 28500.0, %[la]\n"
      "v_add_f32 v101, 29500.0, %[la]\n"
      "v_add_f32 v102, 30500.0, %[la]\n"
      "v_add_f32 v103, 31500.0, %[la]\n"
      "s_set_gpr_idx_on %[r0], gpr_idx(SRC0)\n"
      "s_mov_b32 %[cnt], %[iters]\n"
      "1:\n"
      "s_set_gpr_idx_idx %[r0]\n"
      "v_sub_f32 v104, v40, %[b0]\n"
      "v_sub_f32 v105, v72, %[b1]\n"
      "v_fma_f32 %[acc0], %[w0], |v104|, %[acc0]\n"
      "v_fma_f32 %[acc1], %[w0], |v105|, %[acc1]\n"
      "s_set_gpr_idx_idx %[r1]\n"
      "v_sub_f32 v106, v40, %[b0]\n"
      "v_sub_f32 v107, v72, %[b1]\n"
      "v_fma_f32 %[acc2], %[w1], |v106|, %[acc2]\n"
      "v_fma_f32 %[acc3], %[w1], |v107|, %[acc3]\n"
      "s_set_gpr_idx_idx %[r2]\n"
      "v_sub_f32 v108, v40, %[b0]\n"
      "v_sub_f32 v109, v72, %[b1]\n"
      "v_fma_f32 %[acc4], %[w2], |v108|, %[acc4]\n"
      "v_fma_f32 %[acc5], %[w2], |v109|, %[acc5]\n"
      "s_set_gpr_idx_idx %[r3]\n"
      "v_sub_f32 v110, v40, %[b0]\n"
      "v_sub_f32 v111, v72, %[b1]\n"
      "v_fma_f32 %[acc6], %[w3], |v110|, %[acc6]\n"
      "v_fma_f32 %[acc7], %[w3], |v111|, %[acc7]\n"
      "s_set_gpr_idx_idx %[r4]\n"
      "v_sub_f32 v104, v40, %[b0]\n"
      "v_sub_f32 v105, v72, %[b1]\n"
      "v_fma_f32 %[acc0], %[w4], |v104|, %[acc0]\n"
      "v_fma_f32 %[acc1], %[w4], |v105|, %[acc1]\n"
      "s_set_gpr_idx_idx %[r5]\n"
      "v_sub_f32 v106, v40, %[b0]\n"
      "v_sub_f32 v107, v72, %[b1]\n"
      "v_fma_f32 %[acc2], %[w5], |v106|, %[acc2]\n"
      "v_fma_f32 %[acc3], %[w5], |v107|, %[acc3]\n"
      "s_set_gpr_idx_idx %[r6]\n"
      "v_sub_f32 v108, v40, %[b0]\n"
      "v_sub_f32 v109, v72, %[b1]\n"
      "v_fma_f32 %[acc4], %[w6], |v108|, %[acc4]\n"
      "v_fma_f32 %[acc5], %[w6], |v109|, %[acc5]\n"
      "s_set_gpr_idx_idx %[r7]\n"
      "v_sub_f32 v110, v40, %[b0]\n"
      "v_sub_f32 v111, v72, %[b1]\n"
      "v_fma_f32 %[acc6], %[w7], |v110|, %[acc6]\n"
      "v_fma_f32 %[acc7], %[w7], |v111|, %[acc7]\n"
      "s_set_gpr_idx_idx %[r0]\n"
      "v_sub_f32 v104, v40, %[b0]\n"
      "v_sub_f32 v105, v72, %[b1]\n"
      "v_fma_f32 %[acc0], %[w0], |v104|, %[acc0]\n"
      "v_fma_f32 %[acc1], %[w0], |v105|, %[acc1]\n"
      "s_set_gpr_idx_idx %[r1]\n"
      "v_sub_f32 v106, v40, %[b0]\n"
      "v_sub_f32 v107, v72, %[b1]\n"
      "v_fma_f32 %[acc2], %[w1], |v106|, %[acc2]\n"
      "v_fma_f32 %[acc3], %[w1], |v107|, %[acc3]\n"
      "s_set_gpr_idx_idx %[r2]\n"
      "v_sub_f32 v108, v40, %[b0]\n"
      "v_sub_f32 v109, v72, %[b1]\n"
      "v_fma_f32 %[acc4], %[w2], |v108|, %[acc4]\n"
      "v_fma_f32 %[acc5], %[w2], |v109|, %[acc5]\n"
      "s_set_gpr_idx_idx %[r3]\n"
      "v_sub_f32 v110, v40, %[b0]\n"
      "v_sub_f32 v111, v72, %[b1]\n"
      "v_fma_f32 %[acc6], %[w3], |v110|, %[acc6]\n"
      "v_fma_f32 %[acc7], %[w3], |v111|, %[acc7]\n"
      "s_set_gpr_idx_idx %[r4]\n"
      "v_sub_f32 v104, v40, %[b0]\n"
      "v_sub_f32 v105, v72, %[b1]\n"
      "v_fma_f32 %[acc0], %[w4], |v104|, %[acc0]\n"
      "v_fma_f32 %[acc1], %[w4], |v105|, %[acc1]\n"
      "s_set_gpr_idx_idx %[r5]\n"
      "v_sub_f32 v106, v40, %[b0]\n"
      "v_sub_f32 v107, v72, %[b1]\n"
      "v_fma_f32 %[acc2], %[w5], |v106|, %[acc2]\n"
      "v_fma_f32 %[acc3], %[w5], |v107|, %[acc3]\n"
      "s_set_gpr_idx_idx %[r6]\n"
      "v_sub_f32 v108, v40, %[b0]\n"
      "v_sub_f32 v109, v72, %[b1]\n"
      "v_fma_f32 %[acc4], %[w6], |v108|, %[acc4]\n"
      "v_fma_f32 %[acc5], %[w6], |v109|, %[acc5]\n"
      "s_set_gpr_idx_idx %[r7]\n"
      "v_sub_f32 v110, v40, %[b0]\n"
      "v_sub_f32 v111, v72, %[b1]\n"
      "v_fma_f32 %[acc6], %[w7], |v110|, %[acc6]\n"
      "v_fma_f32 %[acc7], %[w7], |v111|, %[acc7]\n"
      "s_sub_u32 %[cnt], %[cnt], 1\n"
      "s_cmp_lg_u32 %[cnt], 0\n"
      "s_cbranch_scc1 1b\n"
      "9:\n"
      "s_set_gpr_idx_off\n"
      : [acc0] "+v"(acc0), [acc1] "+v"(acc1), [acc2] "+v"(acc2), [acc3] "+v"(acc3),
        [acc4] "+v"(acc4), [acc5] "+v"(acc5), [acc6] "+v"(acc6), [acc7] "+v"(acc7), [cnt] "=&s"(cnt)
      : [la] "v"(la), [b0] "v"(b0), [b1] "v"(b1), [iters] "s"(iters),
        [r0] "s"(r0), [r1] "s"(r1), [r2] "s"(r2), [r3] "s"(r3), [r4] "s"(r4), [r5] "s"(r5), [r6] "s"(r6), [r7] "s"(r7),
        [w0] "s"(w0), [w1] "s"(w1), [w2] "s"(w2), [w3] "s"(w3), [w4] "s"(w4), [w5] "s"(w5), [w6] "s"(w6), [w7] "s"(w7)
      : "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v48", "v49", "v50", "v51", "v52", "v53", "v54", "v55", "v56", "v57", "v58", "v59", "v60", "v61", "v62", "v63", "v64", "v65", "v66", "v67", "v68", "v69", "v70", "v71", "v72", "v73", "v74", "v75", "v76", "v77", "v78", "v79", "v80", "v81", "v82", "v83", "v84", "v85", "v86", "v87", "v88", "v89", "v90", "v91", "v92", "v93", "v94", "v95", "v96", "v97", "v98", "v99", "v100", "v101", "v102", "v103", "v104", "v105", "v106", "v107", "v108", "v109", "v110", "v111", "scc");
  float* o = out + ((size_t)blockIdx.x * 256 + threadIdx.x) * 8;
  o[0] = acc0; o[1] = acc1; o[2] = acc2; o[3] = acc3; o[4] = acc4; o[5] = acc5; o[6] = acc6; o[7] = acc7;
}


__global__ __launch_bounds__(256) void kern2(const float* in, const int* rr, float* out, int iters) {
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
      "v_add_f32 v40, 0.0, %[la]\n"
      "v_add_f32 v41, 1000.0, %[la]\n"
      "v_add_f32 v42, 2000.0, %[la]\n"
      "v_add_f32 v43, 3000.0, %[la]\n"
      "v_add_f32 v44, 4000.0, %[la]\n"
      "v_add_f32 v45, 5000.0, %[la]\n"
      "v_add_f32 v46, 6000.0, %[la]\n"
      "v_add_f32 v47, 7000.0, %[la]\n"
      "v_add_f32 v48, 8000.0, %[la]\n"
      "v_add_f32 v49, 9000.0, %[la]\n"
      "v_add_f32 v50, 10000.0, %[la]\n"
      "v_add_f32 v51, 11000.0, %[la]\n"
      "v_add_f32 v52, 12000.0, %[la]\n"
      "v_add_f32 v53, 13000.0, %[la]\n"
      "v_add_f32 v54, 14000.0, %[la]\n"
      "v_add_f32 v55, 15000.0, %[la]\n"
      "v_add_f32 v56, 16000.0, %[la]\n"
      "v_add_f32 v57, 17000.0, %[la]\n"
      "v_add_f32 v58, 18000.0, %[la]\n"
      "v_add_f32 v59, 19000.0, %[la]\n"
      "v_add_f32 v60, 20000.0, %[la]\n"
      "v_add_f32 v61, 21000.0, %[la]\n"
      "v_add_f32 v62, 22000.0, %[la]\n"
      "v_add_f32 v63, 23000.0, %[la]\n"
      "v_add_f32 v64, 24000.0, %[la]\n"
      "v_add_f32 v65, 25000.0, %[la]\n"
      "v_add_f32 v66, 26000.0, %[la]\n"
      "v_add_f32 v67, 27000.0, %[la]\n"
      "v_add_f32 v68, 28000.0, %[la]\n"
      "v_add_f32 v69, 29000.0, %[la]\n"
      "v_add_f32 v70, 30000.0, %[la]\n"
      "v_add_f32 v71, 31000.0, %[la]\n"
      "v_add_f32 v72, 500.0, %[la]\n"
      "v_add_f32 v73, 1500.0, %[la]\n"
      "v_add_f32 v74, 2500.0, %[la]\n"
      "v_add_f32 v75, 3500.0, %[la]\n"
      "v_add_f32 v76, 4500.0, %[la]\n"
      "v_add_f32 v77, 5500.0, %[la]\n"
      "v_add_f32 v78, 6500.0, %[la]\n"
      "v_add_f32 v79, 7500.0, %[la]\n"
      "v_add_f32 v80, 8500.0, %[la]\n"
      "v_add_f32 v81, 9500.0, %[la]\n"
      "v_add_f32 v82, 10500.0, %[la]\n"
      "v_add_f32 v83, 11500.0, %[la]\n"
      "v_add_f32 v84, 12500.0, %[la]\n"
      "v_add_f32 v85, 13500.0, %[la]\n"
      "v_add_f32 v86, 14500.0, %[la]\n"
      "v_add_f32 v87, 15500.0, %[la]\n"
      "v_add_f32 v88, 16500.0, %[la]\n"
      "v_add_f32 v89, 17500.0, %[la]\n"
      "v_add_f32 v90, 18500.0, %[la]\n"
      "v_add_f32 v91, 19500.0, %[la]\n"
      "v_add_f32 v92, 20500.0, %[la]\n"
      "v_add_f32 v93, 21500.0, %[la]\n"
      "v_add_f32 v94, 22500.0, %[la]\n"
      "v_add_f32 v95, 23500.0, %[la]\n"
      "v_add_f32 v96, 24500.0, %[la]\n"
      "v_add_f32 v97, 25500.0, %[la]\n"
      "v_add_f32 v98, 26500.0, %[la]\n"
      "v_add_f32 v99, 27500.0, %[la]\n"
      "v_add_f32 v100, 28500.0, %[la]\n"
      "v_add_f32 v101, 29500.0, %[la]\n"
      "v_add_f32 v102, 30500.0, %[la]\n"
      "v_add_f32 v103, 31500.0, %[la]\n"
      "s_set_gpr_idx_on %[r0], gpr_idx(SRC0)\n"
      "s_mov_b32 %[cnt], %[iters]\n"
      "1:\n"
      "s_set_gpr_idx_idx %[r0]\n"
      "v_sub_f32 v104, v40, %[b0]\n"
      "v_sub_f32 v105, v72, %[b1]\n"
      "v_fma_f32 %[acc0], %[w0], |v104|, %[acc0]\n"
      "v_fma_f32 %[acc1], %[w0], |v105|, %[acc1]\n"
      "s_set_gpr_idx_idx %[r1]\n"
      "v_sub_f32 v106, v40, %[b0]\n"
      "v_sub_f32 v107, v72, %[b1]\n"
      "v_fma_f32 %[acc2], %[w1], |v106|, %[acc2]\n"
      "v_fma_f32 %[acc3], %[w1], |v107|, %[acc3]\n"
      "s_bitcmp1_b32 %[r1], 31\n"
      "s_cbranch_scc1 9f\n"
      "s_set_gpr_idx_idx %[r2]\n"
      "v_sub_f32 v108, v40, %[b0]\n"
      "v_sub_f32 v109, v72, %[b1]\n"
      "v_fma_f32 %[acc4], %[w2], |v108|, %[acc4]\n"
      "v_fma_f32 %[acc5], %[w2], |v109|, %[acc5]\n"
      "s_set_gpr_idx_idx %[r3]\n"
      "v_sub_f32 v110, v40, %[b0]\n"
      "v_sub_f32 v111, v72, %[b1]\n"
      "v_fma_f32 %[acc6], %[w3], |v110|, %[acc6]\n"
      "v_fma_f32 %[acc7], %[w3], |v111|, %[acc7]\n"
      "s_bitcmp1_b32 %[r3], 31\n"
      "s_cbranch_scc1 9f\n"
      "s_set_gpr_idx_idx %[r4]\n"
      "v_sub_f32 v104, v40, %[b0]\n"
      "v_sub_f32 v105, v72, %[b1]\n"
      "v_fma_f32 %[acc0], %[w4], |v104|, %[acc0]\n"
      "v_fma_f32 %[acc1], %[w4], |v105|, %[acc1]\n"
      "s_set_gpr_idx_idx %[r5]\n"
      "v_sub_f32 v106, v40, %[b0]\n"
      "v_sub_f32 v107, v72, %[b1]\n"
      "v_fma_f32 %[acc2], %[w5], |v106|, %[acc2]\n"
      "v_fma_f32 %[acc3], %[w5], |v107|, %[acc3]\n"
      "s_bitcmp1_b32 %[r5], 31\n"
      "s_cbranch_scc1 9f\n"
      "s_set_gpr_idx_idx %[r6]\n"
      "v_sub_f32 v108, v40, %[b0]\n"
      "v_sub_f32 v109, v72, %[b1]\n"
      "v_fma_f32 %[acc4], %[w6], |v108|, %[acc4]\n"
      "v_fma_f32 %[acc5], %[w6], |v109|, %[acc5]\n"
      "s_set_gpr_idx_idx %[r7]\n"
      "v_sub_f32 v110, v40, %[b0]\n"
      "v_sub_f32 v111, v72, %[b1]\n"
      "v_fma_f32 %[acc6], %[w7], |v110|, %[acc6]\n"
      "v_fma_f32 %[acc7], %[w7], |v111|, %[acc7]\n"
      "s_bitcmp1_b32 %[r7], 31\n"
      "s_cbranch_scc1 9f\n"
      "s_set_gpr_idx_idx %[r0]\n"
      "v_sub_f32 v104, v40, %[b0]\n"
      "v_sub_f32 v105, v72, %[b1]\n"
      "v_fma_f32 %[acc0], %[w0], |v104|, %[acc0]\n"
      "v_fma_f32 %[acc1], %[w0], |v105|, %[acc1]\n"
      "s_set_gpr_idx_idx %[r1]\n"
      "v_sub_f32 v106, v40, %[b0]\n"
      "v_sub_f32 v107, v72, %[b1]\n"
      "v_fma_f32 %[acc2], %[w1], |v106|, %[acc2]\n"
      "v_fma_f32 %[acc3], %[w1], |v107|, %[acc3]\n"
      "s_bitcmp1_b32 %[r1], 31\n"
      "s_cbranch_scc1 9f\n"
      "s_set_gpr_idx_idx %[r2]\n"
      "v_sub_f32 v108, v40, %[b0]\n"
      "v_sub_f32 v109, v72, %[b1]\n"
      "v_fma_f32 %[acc4], %[w2], |v108|, %[acc4]\n"
      "v_fma_f32 %[acc5], %[w2], |v109|, %[acc5]\n"
      "s_set_gpr_idx_idx %[r3]\n"
      "v_sub_f32 v110, v40, %[b0]\n"
      "v_sub_f32 v111, v72, %[b1]\n"
      "v_fma_f32 %[acc6], %[w3], |v110|, %[acc6]\n"
      "v_fma_f32 %[acc7], %[w3], |v111|, %[acc7]\n"
      "s_bitcmp1_b32 %[r3], 31\n"
      "s_cbranch_scc1 9f\n"
      "s_set_gpr_idx_idx %[r4]\n"
      "v_sub_f32 v104, v40, %[b0]\n"
      "v_sub_f32 v105, v72, %[b1]\n"
      "v_fma_f32 %[acc0], %[w4], |v104|, %[acc0]\n"
      "v_fma_f32 %[acc1], %[w4], |v105|, %[acc1]\n"
      "s_set_gpr_idx_idx %[r5]\n"
      "v_sub_f32 v106, v40, %[b0]\n"
      "v_sub_f32 v107, v72, %[b1]\n"
      "v_fma_f32 %[acc2], %[w5], |v106|, %[acc2]\n"
      "v_fma_f32 %[acc3], %[w5], |v107|, %[acc3]\n"
      "s_bitcmp1_b32 %[r5], 31\n"
      "s_cbranch_scc1 9f\n"
      "s_set_gpr_idx_idx %[r6]\n"
      "v_sub_f32 v108, v40, %[b0]\n"
      "v_sub_f32 v109, v72, %[b1]\n"
      "v_fma_f32 %[acc4], %[w6], |v108|, %[acc4]\n"
      "v_fma_f32 %[acc5], %[w6], |v109|, %[acc5]\n"
      "s_set_gpr_idx_idx %[r7]\n"
      "v_sub_f32 v110, v40, %[b0]\n"
      "v_sub_f32 v111, v72, %[b1]\n"
      "v_fma_f32 %[acc6], %[w7], |v110|, %[acc6]\n"
      "v_fma_f32 %[acc7], %[w7], |v111|, %[acc7]\n"
      "s_bitcmp1_b32 %[r7], 31\n"
      "s_cbranch_scc1 9f\n"
      "s_sub_u32 %[cnt], %[cnt], 1\n"
      "s_cmp_lg_u32 %[cnt], 0\n"
      "s_cbranch_scc1 1b\n"
      "9:\n"
      "s_set_gpr_idx_off\n"
      : [acc0] "+v"(acc0), [acc1] "+v"(acc1), [acc2] "+v"(acc2), [acc3] "+v"(acc3),
        [acc4] "+v"(acc4), [acc5] "+v"(acc5), [acc6] "+v"(acc6), [acc7] "+v"(acc7), [cnt] "=&s"(cnt)
      : [la] "v"(la), [b0] "v"(b0), [b1] "v"(b1), [iters] "s"(iters),
        [r0] "s"(r0), [r1] "s"(r1), [r2] "s"(r2), [r3] "s"(r3), [r4] "s"(r4), [r5] "s"(r5), [r6] "s"(r6), [r7] "s"(r7),
        [w0] "s"(w0), [w1] "s"(w1), [w2] "s"(w2), [w3] "s"(w3), [w4] "s"(w4), [w5] "s"(w5), [w6] "s"(w6), [w7] "s"(w7)
      : "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v48", "v49", "v50", "v51", "v52", "v53", "v54", "v55", "v56", "v57", "v58", "v59", "v60", "v61", "v62", "v63", "v64", "v65", "v66", "v67", "v68", "v69", "v70", "v71", "v72", "v73", "v74", "v75", "v76", "v77", "v78", "v79", "v80", "v81", "v82", "v83", "v84", "v85", "v86", "v87", "v88", "v89", "v90", "v91", "v92", "v93", "v94", "v95", "v96", "v97", "v98", "v99", "v100", "v101", "v102", "v103", "v104", "v105", "v106", "v107", "v108", "v109", "v110", "v111", "scc");
  float* o = out + ((size_t)blockIdx.x * 256 + threadIdx.x) * 8;
  o[0] = acc0; o[1] = acc1; o[2] = acc2; o[3] = acc3; o[4] = acc4; o[5] = acc5; o[6] = acc6; o[7] = acc7;
}


__global__ __launch_bounds__(256) void kern3(const float* in, const int* rr, float* out, int iters) {
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
      "v_add_f32 v40, 0.0, %[la]\n"
      "v_add_f32 v41, 1000.0, %[la]\n"
      "v_add_f32 v42, 2000.0, %[la]\n"
      "v_add_f32 v43, 3000.0, %[la]\n"
      "v_add_f32 v44, 4000.0, %[la]\n"
      "v_add_f32 v45, 5000.0, %[la]\n"
      "v_add_f32 v46, 6000.0, %[la]\n"
      "v_add_f32 v47, 7000.0, %[la]\n"
      "v_add_f32 v48, 8000.0, %[la]\n"
      "v_add_f32 v49, 9000.0, %[la]\n"
      "v_add_f32 v50, 10000.0, %[la]\n"
      "v_add_f32 v51, 11000.0, %[la]\n"
      "v_add_f32 v52, 12000.0, %[la]\n"
      "v_add_f32 v53, 13000.0, %[la]\n"
      "v_add_f32 v54, 14000.0, %[la]\n"
      "v_add_f32 v55, 15000.0, %[la]\n"
      "v_add_f32 v56, 16000.0, %[la]\n"
      "v_add_f32 v57, 17000.0, %[la]\n"
      "v_add_f32 v58, 18000.0, %[la]\n"
      "v_add_f32 v59, 19000.0, %[la]\n"
      "v_add_f32 v60, 20000.0, %[la]\n"
      "v_add_f32 v61, 21000.0, %[la]\n"
      "v_add_f32 v62, 22000.0, %[la]\n"
      "v_add_f32 v63, 23000.0, %[la]\n"
      "v_add_f32 v64, 24000.0, %[la]\n"
      "v_add_f32 v65, 25000.0, %[la]\n"
      "v_add_f32 v66, 26000.0, %[la]\n"
      "v_add_f32 v67, 27000.0, %[la]\n"
      "v_add_f32 v68, 28000.0, %[la]\n"
      "v_add_f32 v69, 29000.0, %[la]\n"
      "v_add_f32 v70, 30000.0, %[la]\n"
      "v_add_f32 v71, 31000.0, %[la]\n"
      "v_add_f32 v72, 500.0, %[la]\n"
      "v_add_f32 v73, 1500.0, %[la]\n"
      "v_add_f32 v74, 2500.0, %[la]\n"
      "v_add_f32 v75, 3500.0, %[la]\n"
      "v_add_f32 v76, 4500.0, %[la]\n"
      "v_add_f32 v77, 5500.0, %[la]\n"
      "v_add_f32 v78, 6500.0, %[la]\n"
      "v_add_f32 v79, 7500.0, %[la]\n"
      "v_add_f32 v80, 8500.0, %[la]\n"
      "v_add_f32 v81, 9500.0, %[la]\n"
      "v_add_f32 v82, 10500.0, %[la]\n"
      "v_add_f32 v83, 11500.0, %[la]\n"
      "v_add_f32 v84, 12500.0, %[la]\n"
      "v_add_f32 v85, 13500.0, %[la]\n"
      "v_add_f32 v86, 14500.0, %[la]\n"
      "v_add_f32 v87, 15500.0, %[la]\n"
      "v_add_f32 v88, 16500.0, %[la]\n"
      "v_add_f32 v89, 17500.0, %[la]\n"
      "v_add_f32 v90, 18500.0, %[la]\n"
      "v_add_f32 v91, 19500.0, %[la]\n"
      "v_add_f32 v92, 20500.0, %[la]\n"
      "v_add_f32 v93, 21500.0, %[la]\n"
      "v_add_f32 v94, 22500.0, %[la]\n"
      "v_add_f32 v95, 23500.0, %[la]\n"
      "v_add_f32 v96, 24500.0, %[la]\n"
      "v_add_f32 v97, 25500.0, %[la]\n"
      "v_add_f32 v98, 26500.0, %[la]\n"
      "v_add_f32 v99, 27500.0, %[la]\n"
      "v_add_f32 v100, 28500.0, %[la]\n"
      "v_add_f32 v101, 29500.0, %[la]\n"
      "v_add_f32 v102, 30500.0, %[la]\n"
      "v_add_f32 v103, 31500.0, %[la]\n"
      "s_set_gpr_idx_on %[r0], gpr_idx(SRC0)\n"
      "s_mov_b32 %[cnt], %[iters]\n"
      "1:\n"
      "s_set_gpr_idx_idx %[r0]\n"
      "v_sub_f32 v104, v40, %[b0]\n"
      "v_sub_f32 v105, v72, %[b1]\n"
      "v_fma_f32 %[acc0], %[w0], |v104|, %[acc0]\n"
      "v_fma_f32 %[acc1], %[w0], |v105|, %[acc1]\n"
      "s_set_gpr_idx_idx %[r1]\n"
      "v_sub_f32 v106, v40, %[b0]\n"
      "v_sub_f32 v107, v72, %[b1]\n"
      "v_fma_f32 %[acc2], %[w1], |v106|, %[acc2]\n"
      "v_fma_f32 %[acc3], %[w1], |v107|, %[acc3]\n"
      "s_set_gpr_idx_idx %[r2]\n"
      "v_sub_f32 v108, v40, %[b0]\n"
      "v_sub_f32 v109, v72, %[b1]\n"
      "v_fma_f32 %[acc4], %[w2], |v108|, %[acc4]\n"
      "v_fma_f32 %[acc5], %[w2], |v109|, %[acc5]\n"
      "s_set_gpr_idx_idx %[r3]\n"
      "v_sub_f32 v110, v40, %[b0]\n"
      "v_sub_f32 v111, v72, %[b1]\n"
      "v_fma_f32 %[acc6], %[w3], |v110|, %[acc6]\n"
      "v_fma_f32 %[acc7], %[w3], |v111|, %[acc7]\n"
      "s_bitcmp1_b32 %[r3], 31\n"
      "s_cbranch_scc1 9f\n"
      "s_set_gpr_idx_idx %[r4]\n"
      "v_sub_f32 v104, v40, %[b0]\n"
      "v_sub_f32 v105, v72, %[b1]\n"
      "v_fma_f32 %[acc0], %[w4], |v104|, %[acc0]\n"
      "v_fma_f32 %[acc1], %[w4], |v105|, %[acc1]\n"
      "s_set_gpr_idx_idx %[r5]\n"
      "v_sub_f32 v106, v40, %[b0]\n"
      "v_sub_f32 v107, v72, %[b1]\n"
      "v_fma_f32 %[acc2], %[w5], |v106|, %[acc2]\n"
      "v_fma_f32 %[acc3], %[w5], |v107|, %[acc3]\n"
      "s_set_gpr_idx_idx %[r6]\n"
      "v_sub_f32 v108, v40, %[b0]\n"
      "v_sub_f32 v109, v72, %[b1]\n"
      "v_fma_f32 %[acc4], %[w6], |v108|, %[acc4]\n"
      "v_fma_f32 %[acc5], %[w6], |v109|, %[acc5]\n"
      "s_set_gpr_idx_idx %[r7]\n"
      "v_sub_f32 v110, v40, %[b0]\n"
      "v_sub_f32 v111, v72, %[b1]\n"
      "v_fma_f32 %[acc6], %[w7], |v110|, %[acc6]\n"
      "v_fma_f32 %[acc7], %[w7], |v111|, %[acc7]\n"
      "s_bitcmp1_b32 %[r7], 31\n"
      "s_cbranch_scc1 9f\n"
      "s_set_gpr_idx_idx %[r0]\n"
      "v_sub_f32 v104, v40, %[b0]\n"
      "v_sub_f32 v105, v72, %[b1]\n"
      "v_fma_f32 %[acc0], %[w0], |v104|, %[acc0]\n"
      "v_fma_f32 %[acc1], %[w0], |v105|, %[acc1]\n"
      "s_set_gpr_idx_idx %[r1]\n"
      "v_sub_f32 v106, v40, %[b0]\n"
      "v_sub_f32 v107, v72, %[b1]\n"
      "v_fma_f32 %[acc2], %[w1], |v106|, %[acc2]\n"
      "v_fma_f32 %[acc3], %[w1], |v107|, %[acc3]\n"
      "s_set_gpr_idx_idx %[r2]\n"
      "v_sub_f32 v108, v40, %[b0]\n"
      "v_sub_f32 v109, v72, %[b1]\n"
      "v_fma_f32 %[acc4], %[w2], |v108|, %[acc4]\n"
      "v_fma_f32 %[acc5], %[w2], |v109|, %[acc5]\n"
      "s_set_gpr_idx_idx %[r3]\n"
      "v_sub_f32 v110, v40, %[b0]\n"
      "v_sub_f32 v111, v72, %[b1]\n"
      "v_fma_f32 %[acc6], %[w3], |v110|, %[acc6]\n"
      "v_fma_f32 %[acc7], %[w3], |v111|, %[acc7]\n"
      "s_bitcmp1_b32 %[r3], 31\n"
      "s_cbranch_scc1 9f\n"
      "s_set_gpr_idx_idx %[r4]\n"
      "v_sub_f32 v104, v40, %[b0]\n"
      "v_sub_f32 v105, v72, %[b1]\n"
      "v_fma_f32 %[acc0], %[w4], |v104|, %[acc0]\n"
      "v_fma_f32 %[acc1], %[w4], |v105|, %[acc1]\n"
      "s_set_gpr_idx_idx %[r5]\n"
      "v_sub_f32 v106, v40, %[b0]\n"
      "v_sub_f32 v107, v72, %[b1]\n"
      "v_fma_f32 %[acc2], %[w5], |v106|, %[acc2]\n"
      "v_fma_f32 %[acc3], %[w5], |v107|, %[acc3]\n"
      "s_set_gpr_idx_idx %[r6]\n"
      "v_sub_f32 v108, v40, %[b0]\n"
      "v_sub_f32 v109, v72, %[b1]\n"
      "v_fma_f32 %[acc4], %[w6], |v108|, %[acc4]\n"
      "v_fma_f32 %[acc5], %[w6], |v109|, %[acc5]\n"
      "s_set_gpr_idx_idx %[r7]\n"
      "v_sub_f32 v110, v40, %[b0]\n"
      "v_sub_f32 v111, v72, %[b1]\n"
      "v_fma_f32 %[acc6], %[w7], |v110|, %[acc6]\n"
      "v_fma_f32 %[acc7], %[w7], |v111|, %[acc7]\n"
      "s_bitcmp1_b32 %[r7], 31\n"
      "s_cbranch_scc1 9f\n"
      "s_sub_u32 %[cnt], %[cnt], 1\n"
      "s_cmp_lg_u32 %[cnt], 0\n"
      "s_cbranch_scc1 1b\n"
      "9:\n"
      "s_set_gpr_idx_off\n"
      : [acc0] "+v"(acc0), [acc1] "+v"(acc1), [acc2] "+v"(acc2), [acc3] "+v"(acc3),
        [acc4] "+v"(acc4), [acc5] "+v"(acc5), [acc6] "+v"(acc6), [acc7] "+v"(acc7), [cnt] "=&s"(cnt)
      : [la] "v"(la), [b0] "v"(b0), [b1] "v"(b1), [iters] "s"(iters),
        [r0] "s"(r0), [r1] "s"(r1), [r2] "s"(r2), [r3] "s"(r3), [r4] "s"(r4), [r5] "s"(r5), [r6] "s"(r6), [r7] "s"(r7),
        [w0] "s"(w0), [w1] "s"(w1), [w2] "s"(w2), [w3] "s"(w3), [w4] "s"(w4), [w5] "s"(w5), [w6] "s"(w6), [w7] "s"(w7)
      : "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v48", "v49", "v50", "v51", "v52", "v53", "v54", "v55", "v56", "v57", "v58", "v59", "v60", "v61", "v62", "v63", "v64", "v65", "v66", "v67", "v68", "v69", "v70", "v71", "v72", "v73", "v74", "v75", "v76", "v77", "v78", "v79", "v80", "v81", "v82", "v83", "v84", "v85", "v86", "v87", "v88", "v89", "v90", "v91", "v92", "v93", "v94", "v95", "v96", "v97", "v98", "v99", "v100", "v101", "v102", "v103", "v104", "v105", "v106", "v107", "v108", "v109", "v110", "v111", "scc");
  float* o = out + ((size_t)blockIdx.x * 256 + threadIdx.x) * 8;
  o[0] = acc0; o[1] = acc1; o[2] = acc2; o[3] = acc3; o[4] = acc4; o[5] = acc5; o[6] = acc6; o[7] = acc7;
}


__global__ __launch_bounds__(256) void kern4(const float* in, const int* rr, float* out, int iters) {
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
      "v_add_f32 v40, 0.0, %[la]\n"
      "v_add_f32 v41, 1000.0, %[la]\n"
      "v_add_f32 v42, 2000.0, %[la]\n"
      "v_add_f32 v43, 3000.0, %[la]\n"
      "v_add_f32 v44, 4000.0, %[la]\n"
      "v_add_f32 v45, 5000.0, %[la]\n"
      "v_add_f32 v46, 6000.0, %[la]\n"
      "v_add_f32 v47, 7000.0, %[la]\n"
      "v_add_f32 v48, 8000.0, %[la]\n"
      "v_add_f32 v49, 9000.0, %[la]\n"
      "v_add_f32 v50, 10000.0, %[la]\n"
      "v_add_f32 v51, 11000.0, %[la]\n"
      "v_add_f32 v52, 12000.0, %[la]\n"
      "v_add_f32 v53, 13000.0, %[la]\n"
      "v_add_f32 v54, 14000.0, %[la]\n"
      "v_add_f32 v55, 15000.0, %[la]\n"
      "v_add_f32 v56, 16000.0, %[la]\n"
      "v_add_f32 v57, 17000.0, %[la]\n"
      "v_add_f32 v58, 18000.0, %[la]\n"
      "v_add_f32 v59, 19000.0, %[la]\n"
      "v_add_f32 v60, 20000.0, %[la]\n"
      "v_add_f32 v61, 21000.0, %[la]\n"
      "v_add_f32 v62, 22000.0, %[la]\n"
      "v_add_f32 v63, 23000.0, %[la]\n"
      "v_add_f32 v64, 24000.0, %[la]\n"
      "v_add_f32 v65, 25000.0, %[la]\n"
      "v_add_f32 v66, 26000.0, %[la]\n"
      "v_add_f32 v67, 27000.0, %[la]\n"
      "v_add_f32 v68, 28000.0, %[la]\n"
      "v_add_f32 v69, 29000.0, %[la]\n"
      "v_add_f32 v70, 30000.0, %[la]\n"
      "v_add_f32 v71, 31000.0, %[la]\n"
      "v_add_f32 v72, 500.0, %[la]\n"
      "v_add_f32 v73, 1500.0, %[la]\n"
      "v_add_f32 v74, 2500.0, %[la]\n"
      "v_add_f32 v75, 3500.0, %[la]\n"
      "v_add_f32 v76, 4500.0, %[la]\n"
      "v_add_f32 v77, 5500.0, %[la]\n"
      "v_add_f32 v78, 6500.0, %[la]\n"
      "v_add_f32 v79, 7500.0, %[la]\n"
      "v_add_f32 v80, 8500.0, %[la]\n"
      "v_add_f32 v81, 9500.0, %[la]\n"
      "v_add_f32 v82, 10500.0, %[la]\n"
      "v_add_f32 v83, 11500.0, %[la]\n"
      "v_add_f32 v84, 12500.0, %[la]\n"
      "v_add_f32 v85, 13500.0, %[la]\n"
      "v_add_f32 v86, 14500.0, %[la]\n"
      "v_add_f32 v87, 15500.0, %[la]\n"
      "v_add_f32 v88, 16500.0, %[la]\n"
      "v_add_f32 v89, 17500.0, %[la]\n"
      "v_add_f32 v90, 18500.0, %[la]\n"
      "v_add_f32 v91, 19500.0, %[la]\n"
      "v_add_f32 v92, 20500.0, %[la]\n"
      "v_add_f32 v93, 21500.0, %[la]\n"
      "v_add_f32 v94, 22500.0, %[la]\n"
      "v_add_f32 v95, 23500.0, %[la]\n"
      "v_add_f32 v96, 24500.0, %[la]\n"
      "v_add_f32 v97, 25500.0, %[la]\n"
      "v_add_f32 v98, 26500.0, %[la]\n"
      "v_add_f32 v99, 27500.0, %[la]\n"
      "v_add_f32 v100, 28500.0, %[la]\n"
      "v_add_f32 v101, 29500.0, %[la]\n"
      "v_add_f32 v102, 30500.0, %[la]\n"
      "v_add_f32 v103, 31500.0, %[la]\n"
      "s_set_gpr_idx_on %[r0], gpr_idx(SRC0)\n"
      "s_mov_b32 %[cnt], %[iters]\n"
      "1:\n"
      "s_set_gpr_idx_idx %[r0]\n"
      "v_sub_f32 v104, v40, %[b0]\n"
      "v_sub_f32 v105, v72, %[b1]\n"
      "v_fma_f32 %[acc0], %[w0], |v104|, %[acc0]\n"
      "v_fma_f32 %[acc1], %[w0], |v105|, %[acc1]\n"
      "s_add_u32 %[cnt], %[cnt], 0\n"
      "s_add_u32 %[cnt], %[cnt], 0\n"
      "s_set_gpr_idx_idx %[r1]\n"
      "v_sub_f32 v106, v40, %[b0]\n"
      "v_sub_f32 v107, v72, %[b1]\n"
      "v_fma_f32 %[acc2], %[w1], |v106|, %[acc2]\n"
      "v_fma_f32 %[acc3], %[w1], |v107|, %[acc3]\n"
      "s_add_u32 %[cnt], %[cnt], 0\n"
      "s_add_u32 %[cnt], %[cnt], 0\n"
      "s_set_gpr_idx_idx %[r2]\n"
      "v_sub_f32 v108, v40, %[b0]\n"
      "v_sub_f32 v109, v72, %[b1]\n"
      "v_fma_f32 %[acc4], %[w2], |v108|, %[acc4]\n"
      "v_fma_f32 %[acc5], %[w2], |v109|, %[acc5]\n"
      "s_add_u32 %[cnt], %[cnt], 0\n"
      "s_add_u32 %[cnt], %[cnt], 0\n"
      "s_set_gpr_idx_idx %[r3]\n"
      "v_sub_f32 v110, v40, %[b0]\n"
      "v_sub_f32 v111, v72, %[b1]\n"
      "v_fma_f32 %[acc6], %[w3], |v110|, %[acc6]\n"
      "v_fma_f32 %[acc7], %[w3], |v111|, %[acc7]\n"
      "s_add_u32 %[cnt], %[cnt], 0\n"
      "s_add_u32 %[cnt], %[cnt], 0\n"
      "s_set_gpr_idx_idx %[r4]\n"
      "v_sub_f32 v104, v40, %[b0]\n"
      "v_sub_f32 v105, v72, %[b1]\n"
      "v_fma_f32 %[acc0], %[w4], |v104|, %[acc0]\n"
      "v_fma_f32 %[acc1], %[w4], |v105|, %[acc1]\n"
      "s_add_u32 %[cnt], %[cnt], 0\n"
      "s_add_u32 %[cnt], %[cnt], 0\n"
      "s_set_gpr_idx_idx %[r5]\n"
      "v_sub_f32 v106, v40, %[b0]\n"
      "v_sub_f32 v107, v72, %[b1]\n"
      "v_fma_f32 %[acc2], %[w5], |v106|, %[acc2]\n"
      "v_fma_f32 %[acc3], %[w5], |v107|, %[acc3]\n"
      "s_add_u32 %[cnt], %[cnt], 0\n"
      "s_add_u32 %[cnt], %[cnt], 0\n"
      "s_set_gpr_idx_idx %[r6]\n"
      "v_sub_f32 v108, v40, %[b0]\n"
      "v_sub_f32 v109, v72, %[b1]\n"
      "v_fma_f32 %[acc4], %[w6], |v108|, %[acc4]\n"
      "v_fma_f32 %[acc5], %[w6], |v109|, %[acc5]\n"
      "s_add_u32 %[cnt], %[cnt], 0\n"
      "s_add_u32 %[cnt], %[cnt], 0\n"
      "s_set_gpr_idx_idx %[r7]\n"
      "v_sub_f32 v110, v40, %[b0]\n"
      "v_sub_f32 v111, v72, %[b1]\n"
      "v_fma_f32 %[acc6], %[w7], |v110|, %[acc6]\n"
      "v_fma_f32 %[acc7], %[w7], |v111|, %[acc7]\n"
      "s_add_u32 %[cnt], %[cnt], 0\n"
      "s_add_u32 %[cnt], %[cnt], 0\n"
      "s_set_gpr_idx_idx %[r0]\n"
      "v_sub_f32 v104, v40, %[b0]\n"
      "v_sub_f32 v105, v72, %[b1]\n"
      "v_fma_f32 %[acc0], %[w0], |v104|, %[acc0]\n"
      "v_fma_f32 %[acc1], %[w0], |v105|, %[acc1]\n"
      "s_add_u32 %[cnt], %[cnt], 0\n"
      "s_add_u32 %[cnt], %[cnt], 0\n"
      "s_set_gpr_idx_idx %[r1]\n"
      "v_sub_f32 v106, v40, %[b0]\n"
      "v_sub_f32 v107, v72, %[b1]\n"
      "v_fma_f32 %[acc2], %[w1], |v106|, %[acc2]\n"
      "v_fma_f32 %[acc3], %[w1], |v107|, %[acc3]\n"
      "s_add_u32 %[cnt], %[cnt], 0\n"
      "s_add_u32 %[cnt], %[cnt], 0\n"
      "s_set_gpr_idx_idx %[r2]\n"
      "v_sub_f32 v108, v40, %[b0]\n"
      "v_sub_f32 v109, v72, %[b1]\n"
      "v_fma_f32 %[acc4], %[w2], |v108|, %[acc4]\n"
      "v_fma_f32 %[acc5], %[w2], |v109|, %[acc5]\n"
      "s_add_u32 %[cnt], %[cnt], 0\n"
      "s_add_u32 %[cnt], %[cnt], 0\n"
      "s_set_gpr_idx_idx %[r3]\n"
      "v_sub_f32 v110, v40, %[b0]\n"
      "v_sub_f32 v111, v72, %[b1]\n"
      "v_fma_f32 %[acc6], %[w3], |v110|, %[acc6]\n"
      "v_fma_f32 %[acc7], %[w3], |v111|, %[acc7]\n"
      "s_add_u32 %[cnt], %[cnt], 0\n"
      "s_add_u32 %[cnt], %[cnt], 0\n"
      "s_set_gpr_idx_idx %[r4]\n"
      "v_sub_f32 v104, v40, %[b0]\n"
      "v_sub_f32 v105, v72, %[b1]\n"
      "v_fma_f32 %[acc0], %[w4], |v104|, %[acc0]\n"
      "v_fma_f32 %[acc1], %[w4], |v105|, %[acc1]\n"
      "s_add_u32 %[cnt], %[cnt], 0\n"
      "s_add_u32 %[cnt], %[cnt], 0\n"
      "s_set_gpr_idx_idx %[r5]\n"
      "v_sub_f32 v106, v40, %[b0]\n"
      "v_sub_f32 v107, v72, %[b1]\n"
      "v_fma_f32 %[acc2], %[w5], |v106|, %[acc2]\n"
      "v_fma_f32 %[acc3], %[w5], |v107|, %[acc3]\n"
      "s_add_u32 %[cnt], %[cnt], 0\n"
      "s_add_u32 %[cnt], %[cnt], 0\n"
      "s_set_gpr_idx_idx %[r6]\n"
      "v_sub_f32 v108, v40, %[b0]\n"
      "v_sub_f32 v109, v72, %[b1]\n"
      "v_fma_f32 %[acc4], %[w6], |v108|, %[acc4]\n"
      "v_fma_f32 %[acc5], %[w6], |v109|, %[acc5]\n"
      "s_add_u32 %[cnt], %[cnt], 0\n"
      "s_add_u32 %[cnt], %[cnt], 0\n"
      "s_set_gpr_idx_idx %[r7]\n"
      "v_sub_f32 v110, v40, %[b0]\n"
      "v_sub_f32 v111, v72, %[b1]\n"
      "v_fma_f32 %[acc6], %[w7], |v110|, %[acc6]\n"
      "v_fma_f32 %[acc7], %[w7], |v111|, %[acc7]\n"
      "s_add_u32 %[cnt], %[cnt], 0\n"
      "s_add_u32 %[cnt], %[cnt], 0\n"
      "s_sub_u32 %[cnt], %[cnt], 1\n"
      "s_cmp_lg_u32 %[cnt], 0\n"
      "s_cbranch_scc1 1b\n"
      "9:\n"
      "s_set_gpr_idx_off\n"
      : [acc0] "+v"(acc0), [acc1] "+v"(acc1), [acc2] "+v"(acc2), [acc3] "+v"(acc3),
        [acc4] "+v"(acc4), [acc5] "+v"(acc5), [acc6] "+v"(acc6), [acc7] "+v"(acc7), [cnt] "=&s"(cnt)
      : [la] "v"(la), [b0] "v"(b0), [b1] "v"(b1), [iters] "s"(iters),
        [r0] "s"(r0), [r1] "s"(r1), [r2] "s"(r2), [r3] "s"(r3), [r4] "s"(r4), [r5] "s"(r5), [r6] "s"(r6), [r7] "s"(r7),
        [w0] "s"(w0), [w1] "s"(w1), [w2] "s"(w2), [w3] "s"(w3), [w4] "s"(w4), [w5] "s"(w5), [w6] "s"(w6), [w7] "s"(w7)
      : "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v48", "v49", "v50", "v51", "v52", "v53", "v54", "v55", "v56", "v57", "v58", "v59", "v60", "v61", "v62", "v63", "v64", "v65", "v66", "v67", "v68", "v69", "v70", "v71", "v72", "v73", "v74", "v75", "v76", "v77", "v78", "v79", "v80", "v81", "v82", "v83", "v84", "v85", "v86", "v87", "v88", "v89", "v90", "v91", "v92", "v93", "v94", "v95", "v96", "v97", "v98", "v99", "v100", "v101", "v102", "v103", "v104", "v105", "v106", "v107", "v108", "v109", "v110", "v111", "scc");
  float* o = out + ((size_t)blockIdx.x * 256 + threadIdx.x) * 8;
  o[0] = acc0; o[1] = acc1; o[2] = acc2; o[3] = acc3; o[4] = acc4; o[5] = acc5; o[6] = acc6; o[7] = acc7;
}


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
