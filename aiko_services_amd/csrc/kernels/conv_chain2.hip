// Chained 1x1 convolutions at a ResNet stage-2 bottleneck boundary, weights resident in registers
// (gfx950, wave64, MFMA bf16):
//
//   Y = relu(A . W1^T + b1 + R)     block b's expansion conv3 (K1 = 128 -> N1 = 512, identity R)
//   Z = relu(Y . W2^T + b2)         block b+1's reduction conv1 (K2 = 512 -> N2 = 128)
//
// conv_chain.hip's register-staged design spills at these shapes (W1 and W2 are 128 KB each and
// it re-reads them per tile while holding the next tile's rows in registers).  This kernel turns
// the problem around:
//   * the workgroup's 8 waves hold ALL of W1 and W2 in registers for the whole (persistent)
//     launch: wave w keeps W1 rows 64 w .. 64 w + 63 (16 fragments) and W2 rows 16 w .. 16 w + 15
//     (16 fragments) — 256 KB of weights = exactly the CU's 8 x 64 x 128 VGPRs — so the steady
//     state moves only activations;
//   * both GEMMs are transposed (C^T = W . X^T: weights on the MFMA A side), so each lane's
//     accumulators are consecutive output CHANNELS of one pixel and the epilogues go straight
//     to memory (16-byte Y stores after one v_permlane16_swap per fp32 pair, 8-byte Z stores);
//   * the next 64-pixel tile's A rows and residual rows stream into the other half of a double
//     buffered LDS image by buffer_load ... lds while the current tile computes (160 KB: 2 x 16 KB
//     A + 2 x 64 KB R/Y); the residual tile is overwritten in place by Y, which is then GEMM2's
//     B operand, so Y is written to HBM once and never read back.
// Per tile: 10 LDS-DMA issues and 12 stores per thread; the loop waits with a counted
// `s_waitcnt vmcnt(12)` (this tile's DMAs are older than the previous tile's stores) and raw
// s_barriers — no __syncthreads() while DMAs are in flight.
#include <hip/hip_runtime.h>

#include "common.h"

namespace aiko {

namespace chain2 {
constexpr int BM = 64;
constexpr uint32_t kRecords = 0x7ffffff0u;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* base) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)kRecords, 0x00020000);
}

__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t r, uint32_t voff, void* lds) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(
      r, reinterpret_cast<__attribute__((address_space(3))) void*>(reinterpret_cast<uintptr_t>(lds)), 16,
      voff, 0, 0, 0);
}
}  // namespace chain2

template <int K1, int N1, int N2>
__global__ __launch_bounds__(512, 2) void conv_chain2_kernel(
    const bf16_t* __restrict__ A, const bf16_t* __restrict__ W1, const float* __restrict__ b1,
    const bf16_t* __restrict__ R, bf16_t* __restrict__ Y, const bf16_t* __restrict__ W2,
    const float* __restrict__ b2, bf16_t* __restrict__ Z, int M) {
  using namespace chain2;
  constexpr int NW = 8;
  constexpr int AROW = K1 * 2, YROW = N1 * 2;           // row bytes
  constexpr int A_BYTES = BM * AROW, Y_BYTES = BM * YROW;
  constexpr int ACH = AROW / 16;                          // 16-B chunks per A row
  static_assert(ACH == 16 && YROW == 1024, "stage-2 geometry: 256-B A rows, 1-KB Y rows");
  constexpr int A_DMA = A_BYTES / (64 * 16) / NW;         // A DMA instructions per wave (2)
  constexpr int Y_DMA = BM / NW;                          // R rows per wave, one DMA each (8)
  constexpr int CW1 = N1 / NW, NI1 = CW1 / 16, KS1 = K1 / 32;   // 64 channels, 4 blocks, 4 k-steps
  constexpr int CW2 = N2 / NW, NI2 = CW2 / 16, KS2 = N1 / 32;   // 16 channels, 1 block, 16 k-steps
  constexpr int MI = BM / 16;
  static_assert(NI1 % 2 == 0 && NI2 == 1, "shapes");
  constexpr int NP1 = NI1 / 2;
  constexpr int STORES = MI * NP1 + MI * NI2;             // per thread per tile (Y 16 B, Z 8 B)
  __shared__ __attribute__((aligned(16))) unsigned char smem[2 * A_BYTES + 2 * Y_BYTES];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int fr = lane & 15, fq = lane >> 4;
  const int coff = ((fq & 1) << 4) | ((fq >> 1) << 3);     // channel offset after the pair swap
  const int ntiles = M / BM;

  // ---- resident weights and biases
  bf16x8 w1f[NI1][KS1], w2f[KS2];
#pragma unroll
  for (int j = 0; j < NI1; ++j)
#pragma unroll
    for (int ks = 0; ks < KS1; ++ks)
      w1f[j][ks] = *reinterpret_cast<const bf16x8*>(W1 + (long)(CW1 * wave + 16 * j + fr) * K1 + 32 * ks + 8 * fq);
#pragma unroll
  for (int ks = 0; ks < KS2; ++ks)
    w2f[ks] = *reinterpret_cast<const bf16x8*>(W2 + (long)(CW2 * wave + fr) * N1 + 32 * ks + 8 * fq);
  float bias1[NP1][8], bias2[4];
#pragma unroll
  for (int q = 0; q < NP1; ++q) {
    const f32x4 u = *reinterpret_cast<const f32x4*>(b1 + CW1 * wave + 32 * q + coff);
    const f32x4 v = *reinterpret_cast<const f32x4*>(b1 + CW1 * wave + 32 * q + coff + 4);
    bias1[q][0] = u[0]; bias1[q][1] = u[1]; bias1[q][2] = u[2]; bias1[q][3] = u[3];
    bias1[q][4] = v[0]; bias1[q][5] = v[1]; bias1[q][6] = v[2]; bias1[q][7] = v[3];
  }
  {
    const f32x4 u = *reinterpret_cast<const f32x4*>(b2 + CW2 * wave + 4 * fq);
    bias2[0] = u[0]; bias2[1] = u[1]; bias2[2] = u[2]; bias2[3] = u[3];
  }

  const __amdgpu_buffer_rsrc_t ra = rsrc(A), rr = rsrc(R);
  // DMA geometry: A instruction j of this wave fills rows 4 (2 w + j) .. +3 (lane: row + (l >> 4),
  // position l & 15, source chunk position ^ (row & 15)); R instruction i fills row 8 w + i
  // (lane: position l, source chunk l ^ (row & 15)).  Logical chunk c of row r sits at c ^ (r & 15).
  auto issue = [&](int tile, int buf) {
    const uint32_t m0 = (uint32_t)tile * BM;
    unsigned char* As = smem + buf * A_BYTES;
    unsigned char* Ys = smem + 2 * A_BYTES + buf * Y_BYTES;
#pragma unroll
    for (int j = 0; j < A_DMA; ++j) {
      const int row0 = 4 * (A_DMA * wave + j);
      const int row = row0 + (lane >> 4);
      const uint32_t off = (m0 + row) * (uint32_t)AROW + (uint32_t)(((lane & 15) ^ (row & 15)) << 4);
      dma16(ra, off, As + row0 * AROW);
    }
#pragma unroll
    for (int i = 0; i < Y_DMA; ++i) {
      const int row = Y_DMA * wave + i;
      const uint32_t off = (m0 + row) * (uint32_t)YROW + (uint32_t)((lane ^ (row & 15)) << 4);
      dma16(rr, off, Ys + row * YROW);
    }
  };

  int tile = blockIdx.x;
  if (tile < ntiles) issue(tile, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // weights, biases and tile 0 landed
  int buf = 0;
  for (; tile < ntiles; tile += gridDim.x, buf ^= 1) {
    // this tile's DMAs are older than the previous tile's STORES stores: retire them, then
    // publish to the workgroup (this barrier also ends every read of the other buffers)
    asm volatile("s_waitcnt vmcnt(%0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::"n"(STORES) : "memory");
    const int next = tile + gridDim.x;
    if (next < ntiles) issue(next, buf ^ 1);
    const long m0 = (long)tile * BM;
    const unsigned char* As = smem + buf * A_BYTES;
    unsigned char* Ys = smem + 2 * A_BYTES + buf * Y_BYTES;

    // ---- GEMM1 + epilogue 1 in two 32-pixel halves (bounds the live accumulators to 32 VGPRs
    // beside the 128 of resident weights): Y^T[64 w + 16 j + 4 fq + e][32 h + 16 i + fr]
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      constexpr int MH = MI / 2;
      f32x4 acc[NI1][MH];
#pragma unroll
      for (int j = 0; j < NI1; ++j)
#pragma unroll
        for (int i = 0; i < MH; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < KS1; ++ks) {
        bf16x8 xf[MH];
#pragma unroll
        for (int i = 0; i < MH; ++i)
          xf[i] = *reinterpret_cast<const bf16x8*>(As + (16 * (MH * h + i) + fr) * AROW + (((4 * ks + fq) ^ fr) << 4));
#pragma unroll
        for (int i = 0; i < MH; ++i)
#pragma unroll
          for (int j = 0; j < NI1; ++j)
            acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w1f[j][ks], xf[i], acc[j][i], 0, 0, 0);
      }
      // epilogue 1: Y = relu(acc + b1 + R), in place of R in LDS and to HBM
#pragma unroll
      for (int i = 0; i < MH; ++i) {
        const int row = 16 * (MH * h + i) + fr;
#pragma unroll
        for (int q = 0; q < NP1; ++q) {
          f32x4 lo = acc[2 * q][i], hi = acc[2 * q + 1][i];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const auto s = __builtin_amdgcn_permlane16_swap(__float_as_uint(lo[e]), __float_as_uint(hi[e]), false, false);
            lo[e] = __uint_as_float(s[0]);
            hi[e] = __uint_as_float(s[1]);
          }
          const int ch = CW1 * wave + 32 * q + coff;
          u32x4* slot = reinterpret_cast<u32x4*>(Ys + row * YROW + (((ch >> 3) ^ fr) << 4));
          const u32x4 r = *slot;
          u32x4 o;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float a = fmaxf((e < 2 ? lo[2 * e] : hi[2 * e - 4]) + bias1[q][2 * e] + __uint_as_float(r[e] << 16), 0.f);
            const float b = fmaxf((e < 2 ? lo[2 * e + 1] : hi[2 * e - 3]) + bias1[q][2 * e + 1] +
                                  __uint_as_float(r[e] & 0xffff0000u), 0.f);
            o[e] = pack2(a, b);
          }
          *slot = o;
          *reinterpret_cast<u32x4*>(Y + (m0 + row) * N1 + ch) = o;
        }
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");   // Y tile complete in LDS

    // ---- GEMM2: Z^T[16 w + 4 fq + e][16 i + fr] over K2 = N1
    f32x4 acc2[MI];
#pragma unroll
    for (int i = 0; i < MI; ++i) acc2[i] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < KS2; ++ks) {
      bf16x8 yf[MI];
#pragma unroll
      for (int i = 0; i < MI; ++i)
        yf[i] = *reinterpret_cast<const bf16x8*>(Ys + (16 * i + fr) * YROW + (((4 * ks + fq) ^ fr) << 4));
#pragma unroll
      for (int i = 0; i < MI; ++i) acc2[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w2f[ks], yf[i], acc2[i], 0, 0, 0);
    }
    // ---- epilogue 2: Z = relu(acc2 + b2), 4 channels (8 B) per lane and pixel
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      const int row = 16 * i + fr;
      uint2 o;
      o.x = pack2(fmaxf(acc2[i][0] + bias2[0], 0.f), fmaxf(acc2[i][1] + bias2[1], 0.f));
      o.y = pack2(fmaxf(acc2[i][2] + bias2[2], 0.f), fmaxf(acc2[i][3] + bias2[3], 0.f));
      *reinterpret_cast<uint2*>(Z + (m0 + row) * N2 + CW2 * wave + 4 * fq) = o;
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

}  // namespace aiko

// Y = relu(A W1^T + b1 + R) [M, 512], Z = relu(Y W2^T + b2) [M, 128]; A [M, 128]; M % 64 == 0;
// every operand < 2^31 bytes (32-bit buffer offsets).
extern "C" int aiko_conv_chain2(const void* A, const void* W1, const float* b1, const void* R, void* Y,
                                const void* W2, const float* b2, void* Z, int M, int K1, int N1, int N2,
                                int grid, hipStream_t stream) {
  using namespace aiko;
  if (M <= 0 || M % chain2::BM || K1 != 128 || N1 != 512 || N2 != 128) return -1;
  if ((long)M * N1 * 2 >= 0x7fffff00L) return -1;
  const int ntiles = M / chain2::BM;
  if (grid <= 0) grid = 256;
  if (grid > ntiles) grid = ntiles;
  hipLaunchKernelGGL((conv_chain2_kernel<128, 512, 128>), dim3(grid), dim3(512), 0, stream,
                     static_cast<const bf16_t*>(A), static_cast<const bf16_t*>(W1), b1,
                     static_cast<const bf16_t*>(R), static_cast<bf16_t*>(Y), static_cast<const bf16_t*>(W2),
                     b2, static_cast<bf16_t*>(Z), M);
  return (int)hipGetLastError();
}
