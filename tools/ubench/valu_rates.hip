// Microbenchmark: VALU issue rate of the candidate pair-feature instruction
// mixes on gfx950.  Inner loops are inline asm so the instruction count per
// PFE (pair-feature evaluation) is exact; 8 independent accumulators per lane,
// 8 waves per SIMD, no memory traffic in the timed loop.
// Build: hipcc --offload-arch=gfx950 -O3 valu_rates.hip -o valu_rates
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

constexpr int ITERS = 1 << 15;

#define SAD8(b) \
  asm volatile("v_sad_u32 %0, %8, %16, %0\n v_sad_u32 %1, %9, %16, %1\n v_sad_u32 %2, %10, %16, %2\n v_sad_u32 %3, %11, %16, %3\n" \
               "v_sad_u32 %4, %12, %16, %4\n v_sad_u32 %5, %13, %16, %5\n v_sad_u32 %6, %14, %16, %6\n v_sad_u32 %7, %15, %16, %7\n" \
    : "+v"(c0), "+v"(c1), "+v"(c2), "+v"(c3), "+v"(c4), "+v"(c5), "+v"(c6), "+v"(c7) \
    : "v"(a0), "v"(a1), "v"(a2), "v"(a3), "v"(a4), "v"(a5), "v"(a6), "v"(a7), "v"(b))

#define SADX(op, b) \
  asm volatile(op " %0, %8, %16, %0\n " op " %1, %9, %16, %1\n " op " %2, %10, %16, %2\n " op " %3, %11, %16, %3\n" \
               op " %4, %12, %16, %4\n " op " %5, %13, %16, %5\n " op " %6, %14, %16, %6\n " op " %7, %15, %16, %7\n" \
    : "+v"(c0), "+v"(c1), "+v"(c2), "+v"(c3), "+v"(c4), "+v"(c5), "+v"(c6), "+v"(c7) \
    : "v"(a0), "v"(a1), "v"(a2), "v"(a3), "v"(a4), "v"(a5), "v"(a6), "v"(a7), "v"(b))

#define ADD8(op, b) \
  asm volatile(op " %0, %8, %16\n " op " %1, %9, %16\n " op " %2, %10, %16\n " op " %3, %11, %16\n " \
               op " %4, %12, %16\n " op " %5, %13, %16\n " op " %6, %14, %16\n " op " %7, %15, %16\n" \
    : "+v"(c0), "+v"(c1), "+v"(c2), "+v"(c3), "+v"(c4), "+v"(c5), "+v"(c6), "+v"(c7) \
    : "v"(a0), "v"(a1), "v"(a2), "v"(a3), "v"(a4), "v"(a5), "v"(a6), "v"(a7), "v"(b))

template <int MIX>
__global__ void __launch_bounds__(256) kern(const uint32_t* in, uint32_t* out) {
  uint32_t a0 = in[threadIdx.x], a1 = in[threadIdx.x + 1], a2 = in[threadIdx.x + 2], a3 = in[threadIdx.x + 3];
  uint32_t a4 = in[threadIdx.x + 4], a5 = in[threadIdx.x + 5], a6 = in[threadIdx.x + 6], a7 = in[threadIdx.x + 7];
  uint32_t c0 = 0, c1 = 0, c2 = 0, c3 = 0, c4 = 0, c5 = 0, c6 = 0, c7 = 0;
  uint32_t b = in[threadIdx.x + 8];
  uint32_t t0 = 0, t1 = 0, t2 = 0, t3 = 0;
  uint64_t p0 = a0, p1 = a1, p2 = a2, p3 = a3, p4 = a4, p5 = a5, p6 = a6, p7 = a7, pb = b;
  for (int it = 0; it < ITERS; it++) {
    if (MIX == 0) { SAD8(b); SAD8(b); SAD8(b); SAD8(b); }
    if (MIX == 1) { ADD8("v_add_f32", b); ADD8("v_add_f32", b); ADD8("v_add_f32", b); ADD8("v_add_f32", b); }
    if (MIX == 2) { ADD8("v_add_u32", b); ADD8("v_add_u32", b); ADD8("v_add_u32", b); ADD8("v_add_u32", b); }
    if (MIX == 3) { ADD8("v_max_f32", b); ADD8("v_max_f32", b); ADD8("v_max_f32", b); ADD8("v_max_f32", b); }
    if (MIX == 4) {  // f32: t = a - b ; c += |t|  (2 instrs per PFE)
      asm volatile(
        "v_sub_f32 %8, %12, %20\n v_sub_f32 %9, %13, %20\n v_sub_f32 %10, %14, %20\n v_sub_f32 %11, %15, %20\n"
        "v_add_f32 %0, %0, |%8|\n v_add_f32 %1, %1, |%9|\n v_add_f32 %2, %2, |%10|\n v_add_f32 %3, %3, |%11|\n"
        "v_sub_f32 %8, %16, %20\n v_sub_f32 %9, %17, %20\n v_sub_f32 %10, %18, %20\n v_sub_f32 %11, %19, %20\n"
        "v_add_f32 %4, %4, |%8|\n v_add_f32 %5, %5, |%9|\n v_add_f32 %6, %6, |%10|\n v_add_f32 %7, %7, |%11|\n"
        : "+v"(c0), "+v"(c1), "+v"(c2), "+v"(c3), "+v"(c4), "+v"(c5), "+v"(c6), "+v"(c7),
          "+v"(t0), "+v"(t1), "+v"(t2), "+v"(t3)
        : "v"(a0), "v"(a1), "v"(a2), "v"(a3), "v"(a4), "v"(a5), "v"(a6), "v"(a7), "v"(b));
    }
    if (MIX == 5) {  // packed f32 add (2 lane-ops per instr)
      asm volatile(
        "v_pk_add_f32 %0, %0, %8\n v_pk_add_f32 %1, %1, %8\n v_pk_add_f32 %2, %2, %8\n v_pk_add_f32 %3, %3, %8\n"
        "v_pk_add_f32 %4, %4, %8\n v_pk_add_f32 %5, %5, %8\n v_pk_add_f32 %6, %6, %8\n v_pk_add_f32 %7, %7, %8\n"
        : "+v"(p0), "+v"(p1), "+v"(p2), "+v"(p3), "+v"(p4), "+v"(p5), "+v"(p6), "+v"(p7) : "v"(pb));
    }
    if (MIX == 6) { SADX("v_sad_u16", b); SADX("v_sad_u16", b); SADX("v_sad_u16", b); SADX("v_sad_u16", b); }
    if (MIX == 7) { SADX("v_sad_u8", b); SADX("v_sad_u8", b); SADX("v_sad_u8", b); SADX("v_sad_u8", b); }
    if (MIX == 8) { ADD8("v_pk_sub_u16", b); ADD8("v_pk_sub_u16", b); ADD8("v_pk_sub_u16", b); ADD8("v_pk_sub_u16", b); }
    if (MIX == 9) { SADX("v_dot2_u32_u16", b); SADX("v_dot2_u32_u16", b); SADX("v_dot2_u32_u16", b); SADX("v_dot2_u32_u16", b); }
    if (MIX == 10) { SADX("v_sad_hi_u8", b); SADX("v_sad_hi_u8", b); SADX("v_sad_hi_u8", b); SADX("v_sad_hi_u8", b); }
    if (MIX == 11) { SADX("v_mad_u32_u24", b); SADX("v_mad_u32_u24", b); SADX("v_mad_u32_u24", b); SADX("v_mad_u32_u24", b); }
    if (MIX == 12) { ADD8("v_sub_u32", b); ADD8("v_sub_u32", b); ADD8("v_sub_u32", b); ADD8("v_sub_u32", b); }
    if (MIX == 13) { SADX("v_fma_f32", b); SADX("v_fma_f32", b); SADX("v_fma_f32", b); SADX("v_fma_f32", b); }
    b += 1;
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = c0 + c1 + c2 + c3 + c4 + c5 + c6 + c7 + t0 + t1 + t2 + t3 + (uint32_t)(p0 + p1 + p2 + p3 + p4 + p5 + p6 + p7);
}

template <int MIX>
float run(int blocks, uint32_t* in, uint32_t* out) {
  hipEvent_t e0, e1; CHK(hipEventCreate(&e0)); CHK(hipEventCreate(&e1));
  float best = 1e30f;
  for (int rep = 0; rep < 5; rep++) {
    CHK(hipEventRecord(e0));
    kern<MIX><<<blocks, 256>>>(in, out);
    CHK(hipEventRecord(e1)); CHK(hipEventSynchronize(e1));
    float ms; CHK(hipEventElapsedTime(&ms, e0, e1));
    if (rep > 0 && ms < best) best = ms;
  }
  return best;
}

int main() {
  const int blocks = 256 * 8;   // 8 workgroups of 256 per CU -> 8 waves/SIMD
  uint32_t *in, *out;
  CHK(hipMalloc(&in, 4096 * 4)); CHK(hipMalloc(&out, blocks * 256 * 4));
  CHK(hipMemset(in, 1, 4096 * 4));
  // instructions per lane in the timed loop (asm body); loop overhead ~3 scalar/vector instrs per iter
  const double lanes = (double)blocks * 256;
  struct { const char* nm; float ms; double instr_per_iter; } r[14];
  r[0] = {"v_sad_u32", run<0>(blocks, in, out), 32};
  r[1] = {"v_add_f32", run<1>(blocks, in, out), 32};
  r[2] = {"v_add_u32", run<2>(blocks, in, out), 32};
  r[3] = {"v_max_f32", run<3>(blocks, in, out), 32};
  r[4] = {"v_sub_f32 + v_add_f32|abs|", run<4>(blocks, in, out), 16};
  r[5] = {"v_pk_add_f32", run<5>(blocks, in, out), 8};
  r[6] = {"v_sad_u16", run<6>(blocks, in, out), 32};
  r[7] = {"v_sad_u8", run<7>(blocks, in, out), 32};
  r[8] = {"v_pk_sub_u16", run<8>(blocks, in, out), 32};
  r[9] = {"v_dot2_u32_u16", run<9>(blocks, in, out), 32};
  r[10] = {"v_sad_hi_u8", run<10>(blocks, in, out), 32};
  r[11] = {"v_mad_u32_u24", run<11>(blocks, in, out), 32};
  r[12] = {"v_sub_u32", run<12>(blocks, in, out), 32};
  r[13] = {"v_fma_f32", run<13>(blocks, in, out), 32};
  for (int m = 0; m < 14; m++) {
    double winstr = lanes / 64.0 * ITERS * r[m].instr_per_iter;   // wave-instructions
    double per_simd = winstr / 1024.0;
    printf("%-30s %8.3f ms  %8.3f Twave-instr/s  -> %.3f G wave-instr/s/SIMD (cycles/instr at 2.4GHz: %.2f)\n",
           r[m].nm, r[m].ms, winstr / (r[m].ms * 1e-3) / 1e12, per_simd / (r[m].ms * 1e-3) / 1e9,
           2.4e9 / (per_simd / (r[m].ms * 1e-3)));
  }
  return 0;
}
