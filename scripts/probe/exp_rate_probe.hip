// Throughput of v_exp_f32 vs v_exp_f16 vs v_exp_f32 on packed halves (gfx950): 8 waves per CU,
// independent chains, cycles per instruction per SIMD from the elapsed time.
#include <hip/hip_runtime.h>
#include <cstdio>
template <int MODE>
__global__ __launch_bounds__(512) void k(float* out, int iters) {
  float a0 = threadIdx.x * 1e-3f, a1 = a0 + 0.1f, a2 = a0 + 0.2f, a3 = a0 + 0.3f;
  _Float16 h0 = (_Float16)a0, h1 = (_Float16)a1, h2 = (_Float16)a2, h3 = (_Float16)a3;
  for (int i = 0; i < iters; ++i) {
    if constexpr (MODE == 0) {
      a0 = __builtin_amdgcn_exp2f(a0) - 1.f; a1 = __builtin_amdgcn_exp2f(a1) - 1.f;
      a2 = __builtin_amdgcn_exp2f(a2) - 1.f; a3 = __builtin_amdgcn_exp2f(a3) - 1.f;
    } else if constexpr (MODE == 1) {
      h0 = (_Float16)(__builtin_amdgcn_exp2f((float)0) * 0) + h0;  // placeholder (overwritten below)
      asm volatile("v_exp_f16 %0, %0\n\tv_exp_f16 %1, %1\n\tv_exp_f16 %2, %2\n\tv_exp_f16 %3, %3" : "+v"(h0), "+v"(h1), "+v"(h2), "+v"(h3));
    } else {
      asm volatile("v_add_f32 %0, 1.0, %0\n\tv_add_f32 %1, 1.0, %1\n\tv_add_f32 %2, 1.0, %2\n\tv_add_f32 %3, 1.0, %3" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3));
    }
  }
  out[blockIdx.x * 512 + threadIdx.x] = a0 + a1 + a2 + a3 + (float)h0 + (float)h1 + (float)h2 + (float)h3;
}
int main() {
  float* d; hipMalloc(&d, 256 * 4 * 512 * 4);
  const int iters = 20000;
  const char* names[3] = {"v_exp_f32", "v_exp_f16", "v_add_f32 (reference)"};
  for (int mode = 0; mode < 3; ++mode) {
    for (int rep = 0; rep < 2; ++rep) {
      hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
      hipEventRecord(e0);
      if (mode == 0) k<0><<<256 * 4, 512>>>(d, iters);
      else if (mode == 1) k<1><<<256 * 4, 512>>>(d, iters);
      else k<2><<<256 * 4, 512>>>(d, iters);
      hipEventRecord(e1); hipEventSynchronize(e1);
      float ms; hipEventElapsedTime(&ms, e0, e1);
      // instructions per SIMD: blocks*8 waves / 1024 SIMDs * iters * 4
      const double per_simd = (256.0 * 4 * 8 / 1024.0) * iters * 4;
      if (rep) printf("%-24s %.3f ms  %.2f cycles/instr/SIMD at 2.4 GHz\n", names[mode], ms, ms * 1e-3 * 2.4e9 / per_simd);
    }
  }
  return 0;
}
