// 3x3 / stride 1 / pad 1 convolution with an LDS-resident input patch (tuner variant 10):
// ResNet stage 1 (56 x 56, 64 -> 64 channels).
//
// As an implicit GEMM every input pixel of a 3x3 conv is fetched nine times (once per tap), and
// with only 64 output channels each fetched byte feeds just 64 MACs: the conv_buf / conv_wide
// kernels move ~10x the layer's HBM bytes through L2 -> LDS and top out near 80 us at B=256.
// Here a workgroup owns TH = 8 output rows of one image and stages the (TH + 2) x (W + 2) input
// patch ONCE per 32-channel half (two halves per tile, double-buffered by buffer_load ... lds);
// the nine taps are nine shifted reads of the same LDS image.  The weights (72 KB, 9 taps x 64 x
// 64) stay in LDS for the whole persistent launch, pre-packed on the host in MFMA fragment order
// (tap, half, 16-channel block, lane) so every A-fragment read is one lane-linear ds_read_b128.
//
// LDS image of a half patch: pixel q = patch_row * PW + patch_col, 64 B (32 channels) per pixel,
// PW = W + 8.  16-byte slot k of pixel q holds source chunk k ^ (((q >> 2) & 1) << 1): together
// with the row pitch W + 8 (a row wrap moves q by 8) this makes the B-fragment reads of every tap
// shift conflict-free under ds_read_b128's lane groups (checked exhaustively; PMC: 0 conflicts).
// W is a template constant with PW % 8 == 0, so a tap's row shift never changes the swizzle: each
// lane precomputes one LDS address per (pixel block, column shift) and every patch read of the
// steady state is that VGPR plus an immediate offset (a first version computing the address per
// read issued 7 VALU per MFMA and was VALU-bound: 68-77 us).
//
// Product transposed (weights on the MFMA A side) as conv_wide.hip: one v_permlane16_swap per
// fp32 pair gives each lane 8 consecutive output channels of one pixel -> one 16-B store, issued
// as a buffer store so masked pixels (image / tile edges) become dropped out-of-range stores and
// every thread issues the same count (the loop's counted vmcnt relies on it).
#include <hip/hip_runtime.h>

#include "common.h"

namespace aiko {

namespace patch {
constexpr int C = 64, TH = 8, PWMAX = 64;
constexpr int HALF_BYTES = (TH + 2) * PWMAX * 64;         // 40 KB per half-patch buffer
constexpr int W_BYTES = 9 * 2 * 4 * 1024;                 // weight image: 72 KB
constexpr int P_DMA = HALF_BYTES / 1024 / 8;              // DMA instructions per wave per half (5)
constexpr int W_DMA = W_BYTES / 1024 / 8;                 // 9
constexpr uint32_t kOOB = 0x80000000u;
constexpr uint32_t kRecords = 0x7ffffff0u;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* base) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)kRecords, 0x00020000);
}
__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t r, uint32_t voff, void* lds) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(
      r, reinterpret_cast<__attribute__((address_space(3))) void*>(reinterpret_cast<uintptr_t>(lds)), 16,
      voff, 0, 0, 0);
}
}  // namespace patch

template <int W>
__global__ __launch_bounds__(512, 2) void conv3x3_patch_kernel(
    const bf16_t* __restrict__ x, const bf16_t* __restrict__ wimg, const float* __restrict__ bias,
    bf16_t* __restrict__ y, int B, int H, int ldy, int act) {
  using namespace patch;
  constexpr int PW = W + 8;
  constexpr int MIW = (TH * W + 63) / 64;                  // 16-pixel blocks per wave (W 56: 7, 40: 5, 24: 3)
  static_assert(PW % 8 == 0 && PW <= PWMAX, "patch pitch");
  // LDS: [half-patch 0 | half-patch 1 | weights]: patch reads take immediate offsets < 64 KB
  __shared__ __attribute__((aligned(16))) unsigned char smem[2 * HALF_BYTES + W_BYTES];
  unsigned char* Wl = smem + 2 * HALF_BYTES;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 1, wc = wave & 1;                 // pixel group (4), channel half (2)
  const int fr = lane & 15, fq = lane >> 4;
  const int coff = ((fq & 1) << 4) | ((fq >> 1) << 3);
  const int tiles_per_img = (H + TH - 1) / TH;
  const int ntiles = B * tiles_per_img;
  const __amdgpu_buffer_rsrc_t rx = rsrc(x), rw = rsrc(wimg), ry = rsrc(y);

  // ---- patch DMA geometry (fixed across tiles): instruction k of this wave covers pixels
  // 16 (8 k + wave) .. +15; lane -> pixel q, slot l & 3, source chunk slot ^ swz(q)
  int p_rel[P_DMA];        // byte offset of the source pixel relative to the tile's (oh0, 0) pixel
  int p_row[P_DMA];        // patch row (ih = oh0 - 1 + row), or -1: padding column / beyond patch
#pragma unroll
  for (int k = 0; k < P_DMA; ++k) {
    const int q = 16 * (8 * k + wave) + (lane >> 2);
    const int pr = q / PW, pc = q - pr * PW;
    const int c = (lane & 3) ^ (((q >> 2) & 1) << 1);
    const bool col_ok = pc >= 1 && pc <= W && pr < TH + 2;
    p_row[k] = col_ok ? pr : -1;
    p_rel[k] = ((pr - 1) * W + (pc - 1)) * (C * 2) + c * 16;
  }
  auto issue = [&](int tile, int half) {
    const int img = tile / tiles_per_img;
    const int oh0 = (tile - img * tiles_per_img) * TH;
    const int base = (img * H + oh0) * W * (C * 2) + half * 64;
    unsigned char* P = smem + half * HALF_BYTES;
#pragma unroll
    for (int k = 0; k < P_DMA; ++k) {
      const int ih = oh0 - 1 + p_row[k];
      const bool ok = p_row[k] >= 0 && ih >= 0 && ih < H;
      dma16(rx, ok ? (uint32_t)(base + p_rel[k]) : kOOB, P + (8 * k + wave) * 1024);
    }
  };

  // ---- per-lane output pixels: block i of group wr -> p = (7 wr + i) 16 + fr (a pixel past the
  // tile reads patch pixel 0 and its store is dropped).  addr[i][s]: LDS byte address of the
  // pixel's tap-(0, s) input chunk; tap (r, s) adds the immediate r PW 64.
  int addr[MIW][3];
  int prel[MIW];
#pragma unroll
  for (int i = 0; i < MIW; ++i) {
    const int p = (MIW * wr + i) * 16 + fr;
    const bool valid = p < TH * W;
    const int ohl = p / W, ow = p - ohl * W;
    const int q0 = valid ? ohl * PW + ow : 0;
#pragma unroll
    for (int s = 0; s < 3; ++s) {
      const int q = q0 + s;
      addr[i][s] = q * 64 + ((fq ^ (((q >> 2) & 1) << 1)) << 4);
    }
    prel[i] = valid ? p : -1;
  }
  float bb[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) bb[e] = bias ? bias[32 * wc + coff + e] : 0.f;
  const int wbase = (2 * wc) * 1024 + lane * 16;           // this wave's first weight block, lane slot

  int tile = blockIdx.x;
  // weights once per workgroup, then the first half patch
#pragma unroll
  for (int k = 0; k < W_DMA; ++k) dma16(rw, (uint32_t)((8 * k + wave) * 1024 + lane * 16), Wl + (8 * k + wave) * 1024);
  if (tile < ntiles) issue(tile, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

  for (; tile < ntiles; tile += gridDim.x) {
    f32x4 acc[2][MIW];
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int i = 0; i < MIW; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      // h = 0: this half's DMAs are older than the previous tile's MIW stores; h = 1: nothing younger
      if (h == 0)
        asm volatile("s_waitcnt vmcnt(%0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::"n"(MIW) : "memory");
      else
        asm volatile("s_waitcnt vmcnt(0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      if (h == 0) {
        issue(tile, 1);
      } else if (tile + (int)gridDim.x < ntiles) {
        issue(tile + gridDim.x, 0);
      }
      const unsigned char* P = smem + h * HALF_BYTES;
#pragma unroll
      for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int s = 0; s < 3; ++s) {
          const int t = 3 * r + s;
          const unsigned char* wp = Wl + (t * 2 + h) * 4096 + wbase;
          const bf16x8 wf0 = *reinterpret_cast<const bf16x8*>(wp);
          const bf16x8 wf1 = *reinterpret_cast<const bf16x8*>(wp + 1024);
#pragma unroll
          for (int i = 0; i < MIW; ++i) {
            const bf16x8 xf = *reinterpret_cast<const bf16x8*>(P + addr[i][s] + r * PW * 64);
            acc[0][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf0, xf, acc[0][i], 0, 0, 0);
            acc[1][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf1, xf, acc[1][i], 0, 0, 0);
          }
        }
    }
    // ---- epilogue: 8 consecutive channels of one pixel per lane and block, one 16-B store
    const int img = tile / tiles_per_img;
    const int oh0 = (tile - img * tiles_per_img) * TH;
    const int pix0 = (img * H + oh0) * W;
    const int valid_px = min(TH, H - oh0) * W;
#pragma unroll
    for (int i = 0; i < MIW; ++i) {
      f32x4 lo = acc[0][i], hi = acc[1][i];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const auto sw = __builtin_amdgcn_permlane16_swap(__float_as_uint(lo[e]), __float_as_uint(hi[e]), false, false);
        lo[e] = __uint_as_float(sw[0]);
        hi[e] = __uint_as_float(sw[1]);
      }
      float v[8] = {lo[0] + bb[0], lo[1] + bb[1], lo[2] + bb[2], lo[3] + bb[3],
                    hi[0] + bb[4], hi[1] + bb[5], hi[2] + bb[6], hi[3] + bb[7]};
      if (act == 1) {
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = fmaxf(v[e], 0.f);
      } else if (act == 2) {
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = silu(v[e]);
      }
      u32x4 o;
#pragma unroll
      for (int e = 0; e < 4; ++e) o[e] = pack2(v[2 * e], v[2 * e + 1]);
      const bool ok = prel[i] >= 0 && prel[i] < valid_px;
      const uint32_t off = ok ? (uint32_t)(((pix0 + prel[i]) * ldy + 32 * wc + coff) * 2) : kOOB;
      __builtin_amdgcn_raw_buffer_store_b128(o, ry, off, 0, 0);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

}  // namespace aiko

// x: [B, H, W, 64] bf16 contiguous; wimg: [9][2][4][64][8] bf16 fragment image (ops.conv.patch_weight);
// y: [B, H, W, >= 64] with pixel pitch ldy.  W in {56, 40, 24} (compile-time patch pitch); every byte
// offset < 2^31.
extern "C" int aiko_conv3x3_patch(const void* x, const void* wimg, const float* bias, void* y, int B, int H,
                                  int W, int ldy, int act, int grid, hipStream_t stream) {
  using namespace aiko;
  if (H < 1 || B < 1 || ldy < 64 || ldy % 8) return -1;
  const int ntiles = B * ((H + patch::TH - 1) / patch::TH);
  if (grid <= 0) grid = 256;
  if (grid > ntiles) grid = ntiles;
  auto xp = static_cast<const bf16_t*>(x);
  auto wp = static_cast<const bf16_t*>(wimg);
  auto yp = static_cast<bf16_t*>(y);
  if (W == 56)
    hipLaunchKernelGGL(conv3x3_patch_kernel<56>, dim3(grid), dim3(512), 0, stream, xp, wp, bias, yp, B, H, ldy, act);
  else if (W == 40)
    hipLaunchKernelGGL(conv3x3_patch_kernel<40>, dim3(grid), dim3(512), 0, stream, xp, wp, bias, yp, B, H, ldy, act);
  else if (W == 24)
    hipLaunchKernelGGL(conv3x3_patch_kernel<24>, dim3(grid), dim3(512), 0, stream, xp, wp, bias, yp, B, H, ldy, act);
  else
    return -1;
  return (int)hipGetLastError();
}
