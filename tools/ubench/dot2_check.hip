// v_dot2_f32_bf16 / v_dot2_f32_f16 semantics on the device (dev check for the fused bwd_pre D)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstring>
__global__ void k(const uint32_t* a, const uint32_t* b, const float* c, float* out) {
  int i = threadIdx.x;
  float r0, r1;
  asm volatile("v_dot2_f32_bf16 %0, %1, %2, %3" : "=v"(r0) : "v"(a[i]), "v"(b[i]), "v"(c[i]));
  asm volatile("v_dot2_f32_f16 %0, %1, %2, %3" : "=v"(r1) : "v"(a[i]), "v"(b[i]), "v"(c[i]));
  out[2 * i] = r0; out[2 * i + 1] = r1;
}
static float bf(uint16_t u) { uint32_t x = (uint32_t)u << 16; float f; memcpy(&f, &x, 4); return f; }
int main() {
  const int n = 64;
  uint32_t ha[n], hb[n]; float hc[n], ho[2 * n];
  for (int i = 0; i < n; ++i) {
    uint16_t a0 = 0x3f80 + i, a1 = 0x4000 + 3 * i, b0 = 0x3fc0 - i, b1 = 0xbf80 + 2 * i;   // bf16 values
    ha[i] = a0 | ((uint32_t)a1 << 16); hb[i] = b0 | ((uint32_t)b1 << 16); hc[i] = 0.25f * i;
  }
  uint32_t *da, *db; float *dc, *dout;
  hipMalloc(&da, sizeof ha); hipMalloc(&db, sizeof hb); hipMalloc(&dc, sizeof hc); hipMalloc(&dout, sizeof ho);
  hipMemcpy(da, ha, sizeof ha, hipMemcpyHostToDevice); hipMemcpy(db, hb, sizeof hb, hipMemcpyHostToDevice);
  hipMemcpy(dc, hc, sizeof hc, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, da, db, dc, dout);
  hipMemcpy(ho, dout, sizeof ho, hipMemcpyDeviceToHost);
  for (int i = 0; i < 8; ++i) {
    float want = bf(ha[i] & 0xffff) * bf(hb[i] & 0xffff) + bf(ha[i] >> 16) * bf(hb[i] >> 16) + hc[i];
    printf("i=%d bf16 dot2 %.6f want %.6f | lo*lo %.6f hi*hi %.6f c %.3f\n", i, ho[2 * i], want,
           bf(ha[i] & 0xffff) * bf(hb[i] & 0xffff), bf(ha[i] >> 16) * bf(hb[i] >> 16), hc[i]);
  }
  return 0;
}
