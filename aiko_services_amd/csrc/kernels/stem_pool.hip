// Fused ResNet stem: 7x7/s2 conv (+ folded BN bias) + ReLU + 3x3/s2/p1 max-pool in one kernel.
//
// Unfused, the stem writes a [B, 112, 112, 64] bf16 tensor (411 MB at B=256) that the max-pool
// reads straight back: ~0.8 GB of HBM traffic for a 103 MB result, and the stem's N=64 GEMM
// with K padded 147 -> 256 ran at ~376 TFLOP/s (280 us + 127 us for the pool on MI355X).  Here
// each workgroup owns an 8 x 14 tile of POOLED pixels of one image, i.e. a 17 x 29 region of
// stem pixels (10 % halo recompute), and never writes the stem activation to HBM:
//
//  1. the input patch the region needs — 39 rows x 64 pixels x 4 channels of the zero-bordered
//     preprocess buffer, 20 KB — is loaded into LDS once; the folded weights [7][64][32] (28 KB)
//     too, 16-byte chunks XOR-swizzled by (channel >> 2) so fragment reads are conflict-free;
//  2. MFMA v_mfma_f32_16x16x32_bf16 with channels as the A rows and stem pixels as the B
//     columns: one K=32 step is exactly one filter row (8 pixels x 4 channels; pixel 7 and
//     channel 3 carry zero weights), so a B fragment is 16 contiguous bytes of one patch row —
//     an implicit GEMM with no im2col at all (stride 2 = 16-byte steps between pixels).
//     Each of the 4 waves computes 128 stem pixels x 64 channels (8 x 4 accumulator tiles);
//  3. epilogue: bias + ReLU, stem pixels outside the image forced to 0 (ReLU output >= 0, so 0
//     is a valid -inf for the pool), 4 channels packed per 8-byte LDS write into the stem tile
//     [512 px][64 ch] (aliasing the patch/weights), chunks XOR-swizzled by (pixel & 15);
//  4. 3x3/s2 max over the LDS tile, 8 channels (16 B) per thread, coalesced 16-byte stores.
//
// Rounding is identical to the unfused path: the stem value is rounded to bf16 before the max.
#include "common.h"

namespace aiko {

namespace {

constexpr int kTPH = 8, kTPW = 14;                     // pooled tile
constexpr int kSRH = 2 * kTPH + 1, kSRW = 2 * kTPW + 1;  // stem region 17 x 29
constexpr int kNPix = kSRH * kSRW;                      // 493 stem pixels
constexpr int kPatchH = 2 * (kSRH - 1) + 7;             // 39 input rows
constexpr int kPatchW = 2 * (kSRW - 1) + 8;             // 64 input pixels
constexpr int kPatchRowB = kPatchW * 8;                 // 512 B per patch row
constexpr int kPatchB = kPatchH * kPatchRowB;           // 19968 B
constexpr int kWB = 7 * 64 * 64;                        // 28672 B of weights
constexpr int kSB = 512 * 128;                          // stem tile, 128 B per pixel
constexpr int kLdsB = (kPatchB + kWB) > kSB ? (kPatchB + kWB) : kSB;
static_assert(kNPix <= 512, "4 waves x 128 pixels");

struct StemPoolParams {
  const bf16_t* x;      // [B, Hp, Wp, 4]
  const bf16_t* w;      // [64, 256]  K = r * 32 + pixel * 4 + channel
  const float* bias;    // [64]
  bf16_t* y;            // [B, Hm, Wm, ldy]
  int B, Hp, Wp, Ho, Wo, Hm, Wm, ldy, tiles_h, tiles_w;
};

__global__ __launch_bounds__(256, 2) void stem_pool_kernel(StemPoolParams p) {
  __shared__ __attribute__((aligned(16))) unsigned char smem[kLdsB];
  unsigned char* patch = smem;
  unsigned char* wl = smem + kPatchB;
  unsigned char* st = smem;                             // stem tile, after the MFMAs

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int per_img = p.tiles_h * p.tiles_w;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int img = bid / per_img;
  const int t = bid - img * per_img;
  const int ty = t / p.tiles_w, tx = t - ty * p.tiles_w;
  const int py0 = ty * kTPH, px0 = tx * kTPW;
  const int sy0 = 2 * py0 - 1, sx0 = 2 * px0 - 1;      // stem region origin
  const int gy0 = 2 * sy0, gx0 = 2 * sx0;               // patch origin in the padded buffer

  // ---- 1. patch + weights -> LDS ----
  const bf16_t* ximg = p.x + (size_t)img * p.Hp * p.Wp * 4;
  for (int i = tid; i < kPatchH * (kPatchW / 2); i += 256) {
    const int r = i / (kPatchW / 2), c = i - r * (kPatchW / 2);
    const int gy = gy0 + r, gx = gx0 + 2 * c;
    u32x4 v = {0u, 0u, 0u, 0u};
    if ((unsigned)gy < (unsigned)p.Hp && gx >= 0 && gx + 1 < p.Wp)
      v = *reinterpret_cast<const u32x4*>(ximg + ((size_t)gy * p.Wp + gx) * 4);
    *reinterpret_cast<u32x4*>(patch + r * kPatchRowB + c * 16) = v;
  }
  for (int i = tid; i < 7 * 64 * 4; i += 256) {
    const int r = i >> 8, o = (i >> 2) & 63, q = i & 3;
    const u32x4 v = *reinterpret_cast<const u32x4*>(p.w + o * 256 + r * 32 + q * 8);
    *reinterpret_cast<u32x4*>(wl + ((r * 64 + o) * 4 + (q ^ ((o >> 2) & 3))) * 16) = v;
  }
  __syncthreads();

  // ---- 2. MFMA: channels (A rows) x stem pixels (B columns), one filter row per K step ----
  const int fr = lane & 15, fq = lane >> 4;
  int b_off[8];
#pragma unroll
  for (int nb = 0; nb < 8; ++nb) {
    int n = wave * 128 + nb * 16 + fr;
    if (n >= kNPix) n = 0;                               // dummy column, result discarded
    const int ly = n / kSRW, lx = n - ly * kSRW;
    b_off[nb] = 2 * ly * kPatchRowB + (2 * lx) * 8 + fq * 16;
  }
  int a_off[4];
#pragma unroll
  for (int mb = 0; mb < 4; ++mb) {
    const int o = mb * 16 + fr;
    a_off[mb] = (o * 4 + (fq ^ ((o >> 2) & 3))) * 16;
  }
  f32x4 acc[4][8];
#pragma unroll
  for (int mb = 0; mb < 4; ++mb)
#pragma unroll
    for (int nb = 0; nb < 8; ++nb) acc[mb][nb] = f32x4{0.f, 0.f, 0.f, 0.f};

#pragma unroll
  for (int r = 0; r < 7; ++r) {
    bf16x8 af[4];
#pragma unroll
    for (int mb = 0; mb < 4; ++mb)
      af[mb] = *reinterpret_cast<const bf16x8*>(wl + r * 64 * 64 + a_off[mb]);
#pragma unroll
    for (int nb = 0; nb < 8; ++nb) {
      const bf16x8 bfr = *reinterpret_cast<const bf16x8*>(patch + r * kPatchRowB + b_off[nb]);
#pragma unroll
      for (int mb = 0; mb < 4; ++mb)
        acc[mb][nb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[mb], bfr, acc[mb][nb], 0, 0, 0);
    }
  }
  float bias[4][4];
#pragma unroll
  for (int mb = 0; mb < 4; ++mb) {
    const f32x4 b = *reinterpret_cast<const f32x4*>(p.bias + mb * 16 + fq * 4);
    bias[mb][0] = b[0]; bias[mb][1] = b[1]; bias[mb][2] = b[2]; bias[mb][3] = b[3];
  }
  __syncthreads();                                       // patch/weights dead: reuse as stem tile

  // ---- 3. bias + ReLU -> bf16 stem tile in LDS ----
#pragma unroll
  for (int nb = 0; nb < 8; ++nb) {
    const int n = wave * 128 + nb * 16 + fr;
    if (n >= kNPix) continue;
    const int ly = n / kSRW, lx = n - ly * kSRW;
    const bool valid = (unsigned)(sy0 + ly) < (unsigned)p.Ho && (unsigned)(sx0 + lx) < (unsigned)p.Wo;
#pragma unroll
    for (int mb = 0; mb < 4; ++mb) {
      float v[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = valid ? fmaxf(acc[mb][nb][e] + bias[mb][e], 0.f) : 0.f;
      const int c = mb * 4 + fq;                         // 8-byte chunk (4 channels)
      uint2 o2;
      o2.x = pack2(v[0], v[1]);
      o2.y = pack2(v[2], v[3]);
      *reinterpret_cast<uint2*>(st + n * 128 + ((c ^ (n & 15)) * 8)) = o2;
    }
  }
  __syncthreads();

  // ---- 4. 3x3/s2 max-pool from LDS, 8 channels per item ----
  for (int it = tid; it < kTPH * kTPW * 8; it += 256) {
    const int pp = it >> 3, g = it & 7;
    const int py = pp / kTPW, px = pp - py * kTPW;
    const int gy = py0 + py, gx = px0 + px;
    if (gy >= p.Hm || gx >= p.Wm) continue;
    float m[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) m[e] = 0.f;
#pragma unroll
    for (int dy = 0; dy < 3; ++dy)
#pragma unroll
      for (int dx = 0; dx < 3; ++dx) {
        const int n = (2 * py + dy) * kSRW + 2 * px + dx;
        const int s = n & 15;
        u32x4 v = *reinterpret_cast<const u32x4*>(st + n * 128 + ((g ^ (s >> 1)) * 16));
        if (s & 1) v = u32x4{v[2], v[3], v[0], v[1]};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          m[2 * e] = fmaxf(m[2 * e], __uint_as_float(v[e] << 16));
          m[2 * e + 1] = fmaxf(m[2 * e + 1], __uint_as_float(v[e] & 0xffff0000u));
        }
      }
    u32x4 o;
#pragma unroll
    for (int e = 0; e < 4; ++e) o[e] = pack2(m[2 * e], m[2 * e + 1]);
    *reinterpret_cast<u32x4*>(p.y + ((size_t)(img * p.Hm + gy) * p.Wm + gx) * p.ldy + g * 8) = o;
  }
}

}  // namespace

}  // namespace aiko

// x: zero-bordered stem input [B, Hp, Wp, 4] bf16 (image at (3, 3)); w: packed stem weights
// [64, 256] (make_stem_spec: 7 filter rows x 8 pixels x 4 channels, K padded to 256); y: pooled
// [B, Hm, Wm, >= 64] (pixel pitch ldy).  Host preconditions (binding): Cout 64, 7x7/s2 stem,
// Hp >= 2 * Ho + 5, Wp >= 2 * Wo + 6, Hm/Wm = pool(Ho/Wo), 16-byte alignment.
extern "C" int aiko_stem_pool(const void* x, const void* w, const float* bias, void* y, int B, int Hp,
                              int Wp, int Ho, int Wo, int Hm, int Wm, int ldy, hipStream_t stream) {
  using namespace aiko;
  StemPoolParams p;
  p.x = static_cast<const bf16_t*>(x);
  p.w = static_cast<const bf16_t*>(w);
  p.bias = bias;
  p.y = static_cast<bf16_t*>(y);
  p.B = B; p.Hp = Hp; p.Wp = Wp; p.Ho = Ho; p.Wo = Wo; p.Hm = Hm; p.Wm = Wm; p.ldy = ldy;
  p.tiles_h = (Hm + kTPH - 1) / kTPH;
  p.tiles_w = (Wm + kTPW - 1) / kTPW;
  const long grid = (long)B * p.tiles_h * p.tiles_w;
  if (grid <= 0 || grid > 0x7fffffffL) return -1;
  stem_pool_kernel<<<dim3((unsigned)grid), dim3(256), 0, stream>>>(p);
  return (int)hipGetLastError();
}
