// Semantics of gfx950 v_cvt_scalef32_pk_fp8_f32 (scale applied as multiply or divide? saturation?)
// against v_cvt_pk_fp8_f32 of explicitly scaled inputs.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef __attribute__((ext_vector_type(2))) short v2s;
__global__ void k(const float* in, const float* sc, unsigned* out, int n) {
  int i = threadIdx.x;
  if (i >= n) return;
  float a = in[i], s = sc[i];
  v2s old = {0, 0};
  v2s r = __builtin_amdgcn_cvt_scalef32_pk_fp8_f32(old, a, -a, s, false);
  unsigned mul = __builtin_amdgcn_cvt_pk_fp8_f32(a * s, -a * s, 0u, false);
  unsigned div = __builtin_amdgcn_cvt_pk_fp8_f32(a / s, -a / s, 0u, false);
  out[3 * i] = (unsigned)__builtin_bit_cast(unsigned, r) & 0xffffu;
  out[3 * i + 1] = mul & 0xffffu;
  out[3 * i + 2] = div & 0xffffu;
}
int main() {
  const int n = 10;
  float in[n] = {1.f, 3.f, 100.f, 448.f, 460.f, 500.f, 1e4f, 0.01f, 200.f, 7.f};
  float sc[n] = {1.f, 2.f, 4.f, 1.f, 1.f, 1.f, 0.0625f, 16.f, 0.5f, 0.25f};
  float *din, *dsc; unsigned* dout; unsigned out[3 * n];
  hipMalloc(&din, sizeof in); hipMalloc(&dsc, sizeof sc); hipMalloc(&dout, sizeof out);
  hipMemcpy(din, in, sizeof in, hipMemcpyHostToDevice); hipMemcpy(dsc, sc, sizeof sc, hipMemcpyHostToDevice);
  k<<<1, 64>>>(din, dsc, dout, n);
  hipMemcpy(out, dout, sizeof out, hipMemcpyDeviceToHost);
  for (int i = 0; i < n; ++i)
    printf("a=%g s=%g  scalef32=%04x  cvt(a*s)=%04x  cvt(a/s)=%04x\n", in[i], sc[i], out[3 * i], out[3 * i + 1], out[3 * i + 2]);
  return 0;
}
