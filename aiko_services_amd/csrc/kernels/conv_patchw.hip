// 3x3 / stride 1 / pad 1 convolution over a row patch with STREAMED weights (tuner variant 16):
// ResNet stage 2 (28 x 28, 128 -> 128 channels, M = B * 784).
//
// As an implicit GEMM (conv_wide.hip) every K block re-gathers a 256-pixel x 64-channel slab for
// one tap: the nine taps of a channel block fetch nine shifted copies of the same pixels, so a
// 128 x 128 tile moves ~15 KB of L2 -> LDS traffic per MFLOP and the layer sits at ~1.05 PFLOP/s
// (PMC: 0.31 MFMA busy, 35 % of wave time in s_waitcnt).  Here a workgroup owns TH = 14 output
// rows of one image (392 pixels x all 128 output channels) and stages the (TH + 2) x (W + 4) input
// patch ONCE per 32-channel chunk; the nine taps are nine shifted reads of that LDS image (the
// conv_patch.hip layout: 64 B per pixel, 16-B slot k of pixel q holds source chunk
// k ^ (((q >> 2) & 1) << 1), row pitch PW = 32 so a row shift keeps the swizzle).  The 295 KB of
// weights cannot stay resident, so they stream through an 8-slot ring of 8 KB (chunk, tap) blocks
// pre-packed on the host in MFMA fragment order ([chunk][tap][16-channel block][lane][8]: every
// A-fragment read is one lane-linear ds_read_b128) — nine slots, slot = tap, six blocks ahead.  Per (chunk, tap) step a
// CU moves 8 KB of weights + 1/9 of a 32 KB patch (~3.7 KB / MFLOP, a quarter of the implicit
// GEMM's) for 28 MFMAs per wave.
// Measured (MI355X, B=320, scripts/layer_bench.py b4.conv2): 85.3 us against 85.9 us for the best
// implicit-GEMM tile (variant 9) — 2.5x fewer L2 requests (PMC TCP_TCC_READ_REQ 2.6e6 vs 6.6e6) but
// the same ~0.38 MFMA busy and ~42 % of wave time in s_waitcnt (21 % LDS bank-conflict cycles on
// the patch reads), so the layer is not L2-bound either; a tuner candidate.
//
// One DMA stream per workgroup, one barrier per filter row (three taps: a barrier per tap cost
// ~40 % of wave time in waits): patch chunk c + 1 is issued at the first row of chunk c, weight
// blocks g + 6 .. g + 8 at the group of steps g .. g + 2; items past the walk are issued with out-of-range offsets and stores of
// masked pixels go to an out-of-range offset, so every wave issues the same op sequence and each
// `s_waitcnt vmcnt(N)` is the exact count of ops younger than the awaited weight block (compile-
// time tables below; the first tile's first steps are the only non-steady ones).  Persistent:
// workgroup g walks tiles g, g + G, ...
// Product transposed (weights on the MFMA A side) as conv_wide.hip: each lane ends with 8
// consecutive output channels of one pixel -> bias, ReLU, one 16-B store.
#include <cstdlib>
#include <utility>

#include "common.h"

namespace aiko {

namespace patchw {
constexpr int C = 128, N = 128, TH = 14;
constexpr int NCH = C / 32;                               // 32-channel chunks
constexpr int STEPS = NCH * 9;                            // (chunk, tap) steps per tile
constexpr int GS = 3;                                     // steps per barrier: one filter row
constexpr int GROUPS = STEPS / GS;                        // 12 per tile
constexpr int PROWS = TH + 2;
constexpr int W_BYTES = N * 32 * 2;                       // 8 KB per (chunk, tap) weight block
constexpr int NWS = 9, LW = NWS - GS;                     // weight slot = tap; blocks g + 6 .. g + 8 issued at g
constexpr int MI = 7;                                     // 16-pixel blocks per wave (4 x 98 = 392)
constexpr int NST = MI * 2;                               // stores per wave per tile
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
template <typename F, int... I>
__device__ __forceinline__ void static_for_impl(F&& f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
template <int Nn, typename F>
__device__ __forceinline__ void static_for(F&& f) {   // f(integral_constant<0>) .. f(<Nn - 1>)
  static_for_impl(f, std::make_integer_sequence<int, Nn>{});
}
template <int Nn>
__device__ __forceinline__ void vm_barrier() {
  asm volatile("s_waitcnt vmcnt(%0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::"n"(Nn) : "memory");
}

// Issue order per wave: prologue = patch chunk 0 (P_OPS), then weight blocks 0 .. LW - 1; group
// q (steps 3q .. 3q + 2, s = 3q % STEPS) issues [patch of the next chunk if s % 9 == 0: P_OPS]
// [weight blocks 3q + LW .. 3q + LW + 2: 1 op each] and, after its MFMAs when it ends a tile, the
// tile's NST stores.  young(q) = ops issued after weight block 3q + 2 (the group's last) and before
// group q's wait.
template <int P_OPS>
__host__ __device__ constexpr int young(int q) {
  const int blk = GS * q + GS - 1;
  int cnt = 0;
  bool on = false;
  for (int i = 0; i < LW; ++i) {                          // prologue weight blocks
    if (on) cnt += 1;
    if (i == blk) on = true;
  }
  for (int h = 0; h < q; ++h) {
    const int s = (GS * h) % STEPS;
    if (on && s % 9 == 0) cnt += P_OPS;
    for (int j = 0; j < GS; ++j) {
      if (on) cnt += 1;
      if (GS * h + LW + j == blk) on = true;
    }
    if (on && s + GS == STEPS) cnt += NST;
  }
  return cnt;
}
}  // namespace patchw

// PW: patch row pitch in pixels (a multiple of 8, >= W + 2, so a filter-row shift keeps the slot
// swizzle): 32 (default) or 40 (AIKO_PATCHW_PW=40: measured 92.0 vs 85.3 us).
template <int W, int PW>
__global__ __launch_bounds__(512, 1) void conv3x3_patchw_kernel(
    const bf16_t* __restrict__ x, const bf16_t* __restrict__ wimg, const float* __restrict__ bias,
    bf16_t* __restrict__ y, int B, int H, int ldx, int ldy, int act) {
  using namespace patchw;
  constexpr int P_BYTES = PROWS * PW * 64;                // one patch chunk (32 / 40 KB)
  static_assert(P_BYTES % 8192 == 0, "whole DMA ops per wave");
  constexpr int P_OPS = P_BYTES / 1024 / 8;               // patch DMA ops per thread (4 / 5)
  static_assert(PW % 8 == 0 && W + 2 <= PW && MI * 16 * 4 >= TH * W && (MI - 1) * 16 * 4 < TH * W, "tile geometry");
  static_assert(2 * P_BYTES + NWS * W_BYTES + N * 4 <= 160 * 1024, "LDS");
  constexpr int WPX = TH * W / 4;                         // output pixels per wave group (98)
  __shared__ __attribute__((aligned(16))) unsigned char smem[2 * P_BYTES + NWS * W_BYTES + N * 4];
  unsigned char* const Wl = smem + 2 * P_BYTES;
  float* const s_bias = reinterpret_cast<float*>(Wl + NWS * W_BYTES);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 1, wc = wave & 1;                // pixel group (4), channel half (2)
  const int fr = lane & 15, fq = lane >> 4;
  const int coff = ((fq & 1) << 4) | ((fq >> 1) << 3);
  const int tiles_per_img = (H + TH - 1) / TH;
  const int ntiles = B * tiles_per_img;
  const int G = gridDim.x;
  const int lid = blockIdx.x;
  const int my_tiles = lid < ntiles ? (ntiles - 1 - lid) / G + 1 : 0;
  if (my_tiles == 0) return;
  const __amdgpu_buffer_rsrc_t rx = rsrc(x), rw = rsrc(wimg), ry = rsrc(y);

  // ---- patch DMA: op k of this wave covers patch pixels 16 (8 k + wave) .. + 15, lane -> pixel
  // q (row q / PW, column q % PW = image column + 1), 16-B slot lane & 3 = source chunk
  // (lane & 3) ^ swz(q); the geometry is recomputed per issue (every 9 steps) to save VGPRs
  auto issue_patch = [&](int k_tile, int chunk, auto buf_tag) {   // k_tile may run past the walk
    constexpr int BUF = decltype(buf_tag)::value;
    unsigned char* P = smem + BUF * P_BYTES;
    const bool live = k_tile < my_tiles;
    const int tile = lid + k_tile * G;
    const int img = live ? tile / tiles_per_img : 0;
    const int oh0 = live ? (tile - img * tiles_per_img) * TH : 0;
    const int base = (img * H + oh0) * W * ldx * 2 + chunk * 64;
#pragma unroll
    for (int k = 0; k < P_OPS; ++k) {
      const int q = 16 * (8 * k + wave) + (lane >> 2);
      const int pr = q / PW, pc = q % PW;
      const int c = (lane & 3) ^ (((q >> 2) & 1) << 1);
      const int ih = oh0 - 1 + pr;
      const bool ok = live && pc >= 1 && pc <= W && ih >= 0 && ih < H;
      const int rel = ((pr - 1) * W + (pc - 1)) * ldx * 2 + c * 16;
      dma16(rx, ok ? (uint32_t)(base + rel) : kOOB, P + (8 * k + wave) * 1024);
    }
  };
  auto issue_w = [&](int item, bool live) {               // weight block item = chunk * 9 + tap, slot = tap
    dma16(rw, live ? (uint32_t)(item * W_BYTES + (wave * 64 + lane) * 16) : kOOB,
          Wl + (item % 9) * W_BYTES + wave * 1024);
  };

  // ---- per-lane output pixels: block i of group wr -> tile pixel p = 98 wr + 16 i + fr (past the
  // group's 98: masked, its store dropped).  addr[i]: LDS byte offset of the pixel's tap-(0, 0)
  // input slot; tap (r, s) reads pixel q0 + s, i.e. addr + 64 s with the slot swizzle of q0 + s:
  // bit 5 of the offset flips where ((q0 + s) >> 2) & 1 differs from (q0 >> 2) & 1 — bit i + 5 of
  // sflip[s - 1] for block i — and tap row r adds the immediate r * PW * 64.  (Holding all three
  // offsets per block cost 14 VGPRs more and spilled 5 dwords, reloaded every tile.)
  int addr[MI];
  int sflip[2] = {0, 0};
#pragma unroll
  for (int i = 0; i < MI; ++i) {
    const int pl = 16 * i + fr;
    const int p = WPX * wr + pl;
    const int ohl = p / W, ow = p - ohl * W;
    const int q0 = pl < WPX ? ohl * PW + ow : 0;
    addr[i] = q0 * 64 + ((fq ^ (((q0 >> 2) & 1) << 1)) << 4);
#pragma unroll
    for (int s = 1; s < 3; ++s) sflip[s - 1] |= ((((q0 + s) ^ q0) >> 2) & 1) << (i + 5);
  }
  // bias into LDS (visible after the first group's barrier; read only by the epilogues)
  if (tid < N) s_bias[tid] = bias ? bias[tid] : 0.f;

  // prologue: patch chunk 0 of the first tile, weight blocks 0 .. LW - 1
  issue_patch(0, 0, std::integral_constant<int, 0>{});
  static_for<LW>([&](auto i_tag) { issue_w(decltype(i_tag)::value, true); });

  f32x4 acc[4][MI];
  // group q of tile k: steps S0 .. S0 + 2 = (chunk CH, filter row TR, taps 0 .. 2)
  auto group = [&](int k, auto q_tag) {
    constexpr int Q = decltype(q_tag)::value;
    constexpr int S0 = GS * Q, CH = S0 / 9, TR = (S0 % 9) / 3;
    constexpr int YH = young<P_OPS>(Q), YS = young<P_OPS>(GROUPS + Q);   // first tile / steady state
    if (GS * Q + GS - 1 < LW && k == 0) vm_barrier<YH>();
    else vm_barrier<YS>();
    if constexpr (S0 % 9 == 0) {                           // next chunk's patch into the other buffer
      if constexpr (CH + 1 < NCH) issue_patch(k, CH + 1, std::integral_constant<int, (CH + 1) & 1>{});
      else issue_patch(k + 1, 0, std::integral_constant<int, 0>{});
    }
#pragma unroll
    for (int j = 0; j < GS; ++j) {                         // weight blocks g + LW .. g + LW + 2
      const int nxt = S0 + LW + j;
      issue_w(nxt % STEPS, k + nxt / STEPS < my_tiles);
    }
    const unsigned char* P = smem + (CH & 1) * P_BYTES + TR * PW * 64;
    // opaque per group: keeps the compiler from hoisting the tap-1/2 offsets out of the tile loop
    // (14 more live VGPRs, i.e. the spill this layout removes)
    int sf[2] = {sflip[0], sflip[1]};
    asm volatile("" : "+v"(sf[0]), "+v"(sf[1]));
#pragma unroll
    for (int ts = 0; ts < GS; ++ts) {
      if (ts) __builtin_amdgcn_sched_barrier(0);          // keep the next tap's fragment loads from piling up
      const unsigned char* Wp = Wl + (3 * TR + ts) * W_BYTES + (4 * wc) * 1024 + lane * 16;
      bf16x8 wf[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) wf[j] = *reinterpret_cast<const bf16x8*>(Wp + j * 1024);
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        const int a = ts == 0 ? addr[i] : (addr[i] ^ ((sf[ts - 1] >> i) & 32)) + 64 * ts;
        const bf16x8 xf = *reinterpret_cast<const bf16x8*>(P + a);
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[j], xf, acc[j][i], 0, 0, 0);
      }
    }
  };
  for (int k = 0; k < my_tiles; ++k) {
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int i = 0; i < MI; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};
    static_for<GROUPS>([&](auto q_tag) { group(k, q_tag); });
    // ---- epilogue: 8 consecutive channels of one pixel per lane and block pair, 16-B stores
    const int t = lid + k * G;
    const int img = t / tiles_per_img;
    const int oh0 = (t - img * tiles_per_img) * TH;
    const int pix0 = (img * H + oh0) * W;
    const int valid_px = min(TH, H - oh0) * W;
#pragma unroll
    for (int i = 0; i < MI; ++i) {
#pragma unroll
      for (int pp = 0; pp < 2; ++pp) {
        f32x4 lo = acc[2 * pp][i], hi = acc[2 * pp + 1][i];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const auto sw = __builtin_amdgcn_permlane16_swap(__float_as_uint(lo[e]), __float_as_uint(hi[e]), false, false);
          lo[e] = __uint_as_float(sw[0]);
          hi[e] = __uint_as_float(sw[1]);
        }
        const f32x4 b0 = *reinterpret_cast<const f32x4*>(s_bias + 64 * wc + 32 * pp + coff);
        const f32x4 b1 = *reinterpret_cast<const f32x4*>(s_bias + 64 * wc + 32 * pp + coff + 4);
        float v[8] = {lo[0] + b0[0], lo[1] + b0[1], lo[2] + b0[2], lo[3] + b0[3],
                      hi[0] + b1[0], hi[1] + b1[1], hi[2] + b1[2], hi[3] + b1[3]};
        if (act == 1) {
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] = fmaxf(v[e], 0.f);
        }
        u32x4 o;
#pragma unroll
        for (int e = 0; e < 4; ++e) o[e] = pack2(v[2 * e], v[2 * e + 1]);
        const int pl = 16 * i + fr, p = WPX * wr + pl;
        const bool ok = pl < WPX && p < valid_px;
        const uint32_t off = ok ? (uint32_t)(((pix0 + p) * ldy + 64 * wc + 32 * pp + coff) * 2) : kOOB;
        __builtin_amdgcn_raw_buffer_store_b128(o, ry, off, 0, 0);
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");        // DMAs into LDS land before the workgroup ends
}

}  // namespace aiko

// x: [B, H, W, >= 128] bf16 (pixel pitch ldx, 16-B aligned); wimg: [4][9][8][64][8] bf16 fragment
// image (ops.conv.patchw_weight); y: [B, H, W, >= 128] with pixel pitch ldy.  W = 28 (compile-time
// patch pitch); every byte offset < 2^31.  ``grid``: persistent workgroups (<= 0: one per CU).
extern "C" int aiko_conv3x3_patchw(const void* x, const void* wimg, const float* bias, void* y, int B, int H,
                                   int W, int ldx, int ldy, int act, int grid, hipStream_t stream) {
  using namespace aiko;
  if (H < 1 || B < 1 || ldx < 128 || ldx % 8 || ldy < 128 || ldy % 8 || (act != 0 && act != 1)) return -1;
  const int ntiles = B * ((H + patchw::TH - 1) / patchw::TH);
  if (grid <= 0) {
    int dev = 0, cus = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) cus = 256;
    grid = cus;
  }
  if (grid > ntiles) grid = ntiles;
  auto xp = static_cast<const bf16_t*>(x);
  auto wp = static_cast<const bf16_t*>(wimg);
  auto yp = static_cast<bf16_t*>(y);
  static const int pw = [] {
    const char* e = getenv("AIKO_PATCHW_PW");
    return e && e[0] == '4' ? 40 : 32;
  }();
  if (W != 28) return -1;
  if (pw == 32)
    hipLaunchKernelGGL((conv3x3_patchw_kernel<28, 32>), dim3(grid), dim3(512), 0, stream, xp, wp, bias, yp, B, H, ldx,
                       ldy, act);
  else
    hipLaunchKernelGGL((conv3x3_patchw_kernel<28, 40>), dim3(grid), dim3(512), 0, stream, xp, wp, bias, yp, B, H, ldx,
                       ldy, act);
  return (int)hipGetLastError();
}
