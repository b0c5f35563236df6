// Semantics check of v_sad_u16 on gfx950: are the 16-bit halves unsigned?
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
__global__ void k(const uint32_t* a, const uint32_t* b, uint32_t* out, int n) {
  int i = threadIdx.x;
  if (i >= n) return;
  uint32_t d;
  asm volatile("v_sad_u16 %0, %1, %2, %3" : "=v"(d) : "v"(a[i]), "v"(b[i]), "v"(7u));
  out[i] = d;
}
int main() {
  const int n = 6;
  uint32_t ha[n] = {0x0000FFFFu, 0xFFFF0000u, 0x80007FFFu, 0x00010002u, 0xFFFFFFFFu, 0x12345678u};
  uint32_t hb[n] = {0x00000000u, 0x00000000u, 0x7FFF8000u, 0x00020001u, 0x00000000u, 0x87654321u};
  uint32_t *da, *db, *dout, hout[n];
  hipMalloc(&da, 4 * n); hipMalloc(&db, 4 * n); hipMalloc(&dout, 4 * n);
  hipMemcpy(da, ha, 4 * n, hipMemcpyHostToDevice); hipMemcpy(db, hb, 4 * n, hipMemcpyHostToDevice);
  k<<<1, 64>>>(da, db, dout, n);
  hipMemcpy(hout, dout, 4 * n, hipMemcpyDeviceToHost);
  for (int i = 0; i < n; i++) {
    uint32_t al = ha[i] & 0xFFFF, ah = ha[i] >> 16, bl = hb[i] & 0xFFFF, bh = hb[i] >> 16;
    uint32_t expect = (al > bl ? al - bl : bl - al) + (ah > bh ? ah - bh : bh - ah) + 7;
    printf("a=%08x b=%08x sad_u16=%u unsigned-expect=%u %s\n", ha[i], hb[i], hout[i], expect,
           hout[i] == expect ? "OK" : "MISMATCH");
  }
  return 0;
}
