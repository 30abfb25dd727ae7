// Probe: achievable v_mfma_f32_16x16x32_bf16 throughput on the whole chip (8 waves per CU, two per
// SIMD, independent accumulators), alone and with R ds_read_b128 per MFMA from a conflict-free
// lane-linear LDS image — the ceiling the conv / GEMM kernels are measured against.
#include <hip/hip_runtime.h>
#include <cstdio>

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;

template <int R>   // ds_read_b128 per 8 MFMAs (0 = MFMA only)
__global__ __launch_bounds__(512, 1) void mfma_loop(float* out, int iters) {
  __shared__ __attribute__((aligned(16))) unsigned char lds[64 * 1024];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int i = threadIdx.x; i < 64 * 1024 / 4; i += 512) reinterpret_cast<float*>(lds)[i] = 0.001f * (i & 7);
  __syncthreads();
  bf16x8 a, b;
  for (int e = 0; e < 8; ++e) { a[e] = (__bf16)(0.01f * (lane + e)); b[e] = (__bf16)(0.02f * e); }
  f32x4 acc[8];
  for (int j = 0; j < 8; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const unsigned char* base = lds + wave * 8192 + lane * 16;
  for (int it = 0; it < iters; ++it) {
    bf16x8 r[R > 0 ? R : 1];
#pragma unroll
    for (int k = 0; k < R; ++k) r[k] = *reinterpret_cast<const bf16x8*>(base + ((it + k) & 7) * 1024);
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc[j], 0, 0, 0);
#pragma unroll
    for (int k = 0; k < R; ++k) asm volatile("" ::"v"(r[k]));   // the reads must complete, no VALU
  }
  float s = 0.f;
  for (int j = 0; j < 8; ++j) s += acc[j][0] + acc[j][1] + acc[j][2] + acc[j][3];
  if (s == 12345.f) out[threadIdx.x] = s;
}

typedef __attribute__((ext_vector_type(8))) int i32x8;
// the scaled fp8 MFMA of the encoder GEMMs (v_mfma_scale_f32_16x16x128_f8f6f4), unit scales
__global__ __launch_bounds__(512, 1) void mfma_fp8_loop(float* out, int iters) {
  const int lane = threadIdx.x & 63;
  i32x8 a, b;
  for (int e = 0; e < 8; ++e) { a[e] = 0x38383838 + lane; b[e] = 0x30303030 + e; }
  f32x4 acc[8];
  for (int j = 0; j < 8; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int j = 0; j < 8; ++j)
      acc[j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, acc[j], 0, 0, 0, 127, 0, 127);
  }
  float s = 0.f;
  for (int j = 0; j < 8; ++j) s += acc[j][0] + acc[j][1] + acc[j][2] + acc[j][3];
  if (s == 12345.f) out[threadIdx.x] = s;
}

static void run_fp8(int cus, int clk) {
  float* d;
  (void)hipMalloc(&d, 4096);
  const int iters = 10000;
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  mfma_fp8_loop<<<cus, 512>>>(d, 100);
  (void)hipDeviceSynchronize();
  (void)hipEventRecord(e0);
  mfma_fp8_loop<<<cus, 512>>>(d, iters);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms = 0.f;
  (void)hipEventElapsedTime(&ms, e0, e1);
  const double flops = (double)cus * 8 * iters * 8 * (16.0 * 16 * 128 * 2);
  printf("fp8 16x16x128 (scaled): %.3f ms  %.1f TFLOP/s  %.1f cycles per MFMA per SIMD at %.0f MHz\n", ms,
         flops / ms / 1e9, ms * 1e-3 * clk * 1e3 / ((double)iters * 8 * 2), clk / 1e3);
  (void)hipFree(d);
}

template <int R>
static void run(int cus, int clk) {
  float* d;
  (void)hipMalloc(&d, 4096);
  const int iters = 20000;
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  mfma_loop<R><<<cus, 512>>>(d, 100);
  (void)hipDeviceSynchronize();
  (void)hipEventRecord(e0);
  mfma_loop<R><<<cus, 512>>>(d, iters);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms = 0.f;
  (void)hipEventElapsedTime(&ms, e0, e1);
  const double flops = (double)cus * 8 * iters * 8 * (16.0 * 16 * 32 * 2);
  const double cyc_per_mfma = ms * 1e-3 * clk * 1e3 / ((double)iters * 8 * 2);   // per SIMD: 2 waves x 8 MFMAs
  printf("ds_read_b128 per 8 MFMAs %d: %.3f ms  %.1f TFLOP/s  %.1f cycles per MFMA per SIMD at %.0f MHz\n", R, ms,
         flops / ms / 1e9, cyc_per_mfma, clk / 1e3);
  (void)hipFree(d);
}

int main() {
  int dev = 0, cus = 0, clk = 0;
  (void)hipGetDevice(&dev);
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  (void)hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, dev);
  run<0>(cus, clk);
  run<2>(cus, clk);
  run<3>(cus, clk);
  run<4>(cus, clk);
  run<6>(cus, clk);
  run<0>(cus, clk);
  run_fp8(cus, clk);
  run_fp8(cus, clk);
  return 0;
}
