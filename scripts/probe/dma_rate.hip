// Probe: per-CU vector-memory throughput into LDS (buffer_load ... lds, 16 B per lane) and into
// VGPRs (global_load_dwordx4), by outstanding depth per wave, from an L2-resident source (2 MB)
// and from HBM (2 GB).  One 512-thread workgroup per CU (128 KB of LDS pinned), 256 workgroups.
// Every wave streams ITER 1 KB pieces; the LDS form keeps D pieces in flight with a counted
// vmcnt(D - 1) per piece, the VGPR form issues D loads and folds them into a sink.
// Output: GB/s per CU and B/clk/CU at the measured shader clock (s_memtime is a constant 100 MHz
// counter on gfx9: the kernel also records s_memrealtime and s_memtime... here host events only).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef __attribute__((ext_vector_type(4))) unsigned u32x4;

template <int D>
__global__ __launch_bounds__(512, 1) void dma_lds(const unsigned char* src, unsigned long mask, int iter, unsigned* sink) {
  __shared__ __attribute__((aligned(16))) unsigned char lds[8 * 16 * 1024];
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)src, (short)0, 0x7ffffff0, 0x00020000);
  unsigned long base = ((unsigned long)(blockIdx.x * 8 + wave) * iter) << 10;
  unsigned char* slot0 = lds + wave * 16 * 1024;
  for (int i = 0; i < iter; ++i) {
    const unsigned off = (unsigned)(((base + ((unsigned long)i << 10)) & mask) + lane * 16);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(
        r, reinterpret_cast<__attribute__((address_space(3))) void*>(reinterpret_cast<uintptr_t>(slot0 + (i % D) * 1024)),
        16, off, 0, 0, 0);
    if (D > 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(D - 1) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (threadIdx.x == 0 && blockIdx.x == 0) sink[0] = lds[5];
}

template <int D>
__global__ __launch_bounds__(512, 1) void load_vgpr(const unsigned char* src, unsigned long mask, int iter, unsigned* sink) {
  __shared__ unsigned char pin[128 * 1024];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  unsigned long base = ((unsigned long)(blockIdx.x * 8 + wave) * iter) << 10;
  u32x4 acc = {0u, 0u, 0u, 0u};
  for (int i = 0; i < iter; i += D) {
    u32x4 v[D];
#pragma unroll
    for (int d = 0; d < D; ++d)
      v[d] = *reinterpret_cast<const u32x4*>(src + ((base + ((unsigned long)(i + d) << 10)) & mask) + lane * 16);
#pragma unroll
    for (int d = 0; d < D; ++d) acc ^= v[d];
  }
  if (acc[0] == 0x12345678u) { pin[threadIdx.x] = 1; sink[1] = pin[lane]; }
}

template <typename F>
static float run(F launch, int reps) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  launch();
  hipDeviceSynchronize();
  hipEventRecord(a);
  for (int i = 0; i < reps; ++i) launch();
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms = 0;
  hipEventElapsedTime(&ms, a, b);
  return ms / reps;
}

int main() {
  int dev = 0, cus = 0, clk = 0;
  hipGetDevice(&dev);
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, dev);   // kHz
  const size_t big = 2ull << 30;
  unsigned char* src;
  unsigned* sink;
  if (hipMalloc(&src, big) != hipSuccess || hipMalloc(&sink, 64) != hipSuccess) return 1;
  hipMemset(src, 1, big);
  const int grid = cus, iter = 4096;
  const double bytes = (double)grid * 8 * iter * 1024;
  printf("CUs %d, peak clock %.0f MHz, %d x 8 waves x %d KB\n", cus, clk / 1e3, grid, iter);
  for (int hbm = 0; hbm < 2; ++hbm) {
    const unsigned long mask = hbm ? big - 1 : (2ul << 20) - 1;
    const char* where = hbm ? "HBM 2 GB" : "L2  2 MB";
#define LDS_CASE(D)                                                                             \
    {                                                                                           \
      float ms = run([&] { dma_lds<D><<<grid, 512>>>(src, mask, iter, sink); }, 3);            \
      double gbs = bytes / ms / 1e6;                                                            \
      printf("%s lds-dma  depth %2d: %8.1f GB/s chip  %6.1f GB/s/CU  %5.1f B/clk/CU\n", where, D, gbs, gbs / grid, \
             gbs / grid * 1e3 / (clk / 1e3) );                                                   \
    }
    LDS_CASE(1) LDS_CASE(2) LDS_CASE(4) LDS_CASE(8) LDS_CASE(16)
#define VG_CASE(D)                                                                              \
    {                                                                                           \
      float ms = run([&] { load_vgpr<D><<<grid, 512>>>(src, mask, iter, sink); }, 3);          \
      double gbs = bytes / ms / 1e6;                                                            \
      printf("%s vgpr     depth %2d: %8.1f GB/s chip  %6.1f GB/s/CU  %5.1f B/clk/CU\n", where, D, gbs, gbs / grid, \
             gbs / grid * 1e3 / (clk / 1e3));                                                    \
    }
    VG_CASE(1) VG_CASE(2) VG_CASE(4) VG_CASE(8) VG_CASE(16)
  }
  hipFree(src);
  return 0;
}
