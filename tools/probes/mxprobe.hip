#include <hip/hip_runtime.h>
#include <stdio.h>
typedef __attribute__((ext_vector_type(2))) float f2;
typedef __attribute__((ext_vector_type(2))) short s2;
__global__ void k(const float* x, int n, float scale, unsigned* o4, float* r4, unsigned* o8, float* r8) {
  int i = threadIdx.x;
  if (2 * i + 1 >= n) return;
  unsigned p = __builtin_amdgcn_cvt_scalef32_pk_fp4_f32(0u, x[2 * i], x[2 * i + 1], scale, 0);
  o4[i] = p;
  f2 b = __builtin_amdgcn_cvt_scalef32_pk_f32_fp4(p, scale, 0);
  r4[2 * i] = b[0]; r4[2 * i + 1] = b[1];
  s2 q = __builtin_amdgcn_cvt_scalef32_pk_fp8_f32(s2{0, 0}, x[2 * i], x[2 * i + 1], scale, false);
  unsigned u = (unsigned)(unsigned short)q[0] | ((unsigned)(unsigned short)q[1] << 16);
  o8[i] = u;
  f2 c = __builtin_amdgcn_cvt_scalef32_pk_f32_fp8(u, scale, false);
  r8[2 * i] = c[0]; r8[2 * i + 1] = c[1];
}
int main() {
  const int n = 16;
  float hx[n] = {0.f, 0.25f, 0.5f, 0.75f, 1.f, 1.25f, 1.5f, 2.5f, 3.f, 5.f, 6.f, 7.f, -1.f, -3.5f, 100.f, 0.3f};
  float *dx, *r4, *r8; unsigned *o4, *o8;
  hipMalloc(&dx, n * 4); hipMalloc(&r4, n * 4); hipMalloc(&r8, n * 4); hipMalloc(&o4, n * 4); hipMalloc(&o8, n * 4);
  hipMemcpy(dx, hx, n * 4, hipMemcpyHostToDevice);
  for (float scale : {1.f, 2.f, 0.5f}) {
    hipLaunchKernelGGL(k, 1, 8, 0, 0, dx, n, scale, o4, r4, o8, r8);
    float h4[n], h8[n]; unsigned c4[n / 2], c8[n / 2];
    hipMemcpy(h4, r4, n * 4, hipMemcpyDeviceToHost); hipMemcpy(h8, r8, n * 4, hipMemcpyDeviceToHost);
    hipMemcpy(c4, o4, n * 2, hipMemcpyDeviceToHost); hipMemcpy(c8, o8, n * 2, hipMemcpyDeviceToHost);
    printf("scale %g\n", scale);
    for (int i = 0; i < n; ++i) printf("  x=%8.3f fp4code=%02x fp4rt=%8.3f fp8code=%04x fp8rt=%9.4f\n", hx[i],
                                       (c4[i / 2] >> (8 * 0)) & 0xff, h4[i], (c8[i / 2] >> (16 * (i & 1))) & 0xffff, h8[i]);
  }
  return 0;
}
