// YOLOv8's first two convolutions in ONE launch (gfx950, MFMA bf16): the letterboxed uint8 frame
// -> stem (3x3 / 2, 3 -> 16, SiLU, /255 folded into the epilogue) -> l1 (3x3 / 2, 16 -> 32, SiLU).
//
// Unfused, the stem writes a0 [B, 320, 320, 16] (210 MB at B = 64) and l1 reads it back: the two
// launches (stem_fast_kernel ~60 us, the narrow l1 conv ~88 us at B = 64) are bound by those
// bytes.  Here a workgroup owns an 8 x 32 tile of l1 outputs and keeps everything it needs in LDS:
//   1. the frame tile (35 canvas rows x 136 columns, raw 0..255 values as bf16, 4 per pixel —
//      exactly stem_fast_kernel's fill: 4-pixel groups from three dword loads, letterbox bars at
//      the raw fill value, zeros outside the canvas);
//   2. the a0 tile (17 x 65 stem outputs, the l1 tile's receptive field): two 16x16x32 MFMAs per
//      16 stem pixels (two taps per 32-deep K half, as the stem kernel), then fma(acc, 1/255,
//      bias) and SiLU; a0 pixels outside the 320 x 320 map are zero (l1's padding);
//   3. l1 transposed (weights on the MFMA A side, 16 output channels x 32 K = two taps of 16
//      channels, K padded to 5 chunks with zero weights): every lane ends with 4 consecutive
//      channels of one a1 pixel — bias, SiLU and an 8-byte store.
// The a0 halo (17 x 65 for 16 x 64 new stem outputs, ~8 %) is recomputed per tile; a0 never
// reaches HBM.  Measured (MI355X, B = 64, 480 x 640): 153 us against 60 + 88 us for the stem kernel
// and the tuned l1 conv — each tile's three phases form a serial latency chain (fill, two barriers)
// that the saved a0 traffic does not pay for; opt-in (models/yolov8.py AIKO_STEM_L1=1).  Reference call site: the detector's preprocess + first layers,
// /root/reference/src/aiko_services/examples/yolo/yolo.py:56-87 (Ultralytics model).
#include <cstdint>

#include "common.h"

namespace aiko {

namespace sl {
constexpr int TH = 8, TW = 32;               // a1 outputs per tile
constexpr int AH = 2 * TH + 1, AW = 2 * TW + 1;   // a0 tile (17 x 65)
constexpr int AP = 66;                       // a0 tile pixel pitch per row (16 channels, 32 B each)
constexpr int FH = 2 * AH + 1;               // frame tile rows (35)
constexpr int FG = 34, FW = 4 * FG;          // frame tile 4-pixel groups / columns (136)
constexpr int NT = 512;                      // 8 waves: the three phases are latency chains, not throughput
}  // namespace sl

__global__ __launch_bounds__(512) void stem_l1_kernel(const uint8_t* __restrict__ in, bf16_t* __restrict__ out,
                                                      const bf16_t* __restrict__ w0, const float* __restrict__ b0,
                                                      const bf16_t* __restrict__ w1, int k1,
                                                      const float* __restrict__ b1, int Hin, int Win, int Hc, int Wc,
                                                      int off_t, int off_l, float fill_raw, float inv_std, int H0,
                                                      int W0, int H1, int W1, int ldo) {
  using namespace sl;
  __shared__ __attribute__((aligned(16))) uint32_t ftile[FH * FW * 2];      // [35][136] x 4 bf16
  __shared__ __attribute__((aligned(16))) bf16_t atile[AH * AP * 16];       // [17][66] x 16 bf16
  const int tid = threadIdx.x, b = blockIdx.z, lane = tid & 63, wave = tid >> 6;
  const int fr = lane & 15, fq = lane >> 4;
  const int oy1 = blockIdx.y * TH, ox1 = blockIdx.x * TW;
  const int y0a = 2 * oy1 - 1, x0a = 2 * ox1 - 1;        // a0 tile origin
  const int rt0 = 4 * oy1 - 3, ct0 = 4 * ox1 - 8;         // frame tile origin (canvas; ct0 4-aligned)

  // ---- 1. frame tile
  const uint8_t* img = in + (long)b * Hin * Win * 3;
  const uint32_t f2 = pack2(fill_raw, fill_raw), fb = f2 & 0xffffu;
  // all of this thread's group loads are issued before any is converted (a loop that waits for
  // each group's three dwords in turn exposes the memory latency once per group)
  constexpr int FT = (FH * FG + NT - 1) / NT;
  uint32_t wd[FT][3];
  int kind[FT];                                                // 0: zero padding, 1: frame, 2: fill
#pragma unroll
  for (int u = 0; u < FT; ++u) {
    const int task = tid + NT * u;
    const int ty = task / FG, gi = task - ty * FG;
    const int yc = rt0 + ty, xc = ct0 + 4 * gi;
    kind[u] = 0;
    wd[u][0] = wd[u][1] = wd[u][2] = 0u;
    if (task < FH * FG && yc >= 0 && yc < Hc && xc >= 0 && xc < Wc) {
      const int yo = yc - off_t, xo = xc - off_l;
      if ((unsigned)yo < (unsigned)Hin && (unsigned)xo < (unsigned)Win) {
        const uint32_t* src = reinterpret_cast<const uint32_t*>(img + ((long)yo * Win + xo) * 3);
        wd[u][0] = src[0];
        wd[u][1] = src[1];
        wd[u][2] = src[2];
        kind[u] = 1;
      } else {
        kind[u] = 2;
      }
    }
  }
#pragma unroll
  for (int u = 0; u < FT; ++u) {
    const int task = tid + NT * u;
    if (task >= FH * FG) break;
    const int ty = task / FG, gi = task - ty * FG;
    u32x4 lo = {0u, 0u, 0u, 0u}, hi = {0u, 0u, 0u, 0u};      // outside the canvas: zero padding
    if (kind[u] == 1) {
      float c[12];
#pragma unroll
      for (int j = 0; j < 12; ++j) c[j] = (float)((wd[u][j >> 2] >> (8 * (j & 3))) & 0xFFu);
      lo = u32x4{pack2(c[0], c[1]), pack2(c[2], 0.f), pack2(c[3], c[4]), pack2(c[5], 0.f)};
      hi = u32x4{pack2(c[6], c[7]), pack2(c[8], 0.f), pack2(c[9], c[10]), pack2(c[11], 0.f)};
    } else if (kind[u] == 2) {                                 // letterbox bar (raw fill value)
      lo = u32x4{f2, fb, f2, fb};
      hi = lo;
    }
    uint32_t* dst = ftile + 2 * (ty * FW + 4 * gi);
    *reinterpret_cast<u32x4*>(dst) = lo;
    *reinterpret_cast<u32x4*>(dst + 4) = hi;
  }
  __syncthreads();

  // ---- 2. a0 tile: (row ry, 16-pixel block cb) items, two MFMAs each
  {
    int toff[2][2];
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int t = 2 * (fq + 4 * kk) + h;
        toff[kk][h] = t < 9 ? (t / 3) * FW + (t % 3) : -1;
      }
    bf16x8 wa[2];
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) wa[kk] = *reinterpret_cast<const bf16x8*>(w0 + (long)fr * 64 + 8 * (fq + 4 * kk));
    float cb[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) cb[e] = b0[4 * fq + e];
    constexpr int NCB = (AW + 15) / 16;                        // 5 pixel blocks per a0 row
#pragma unroll 2
    for (int item = wave; item < AH * NCB; item += NT / 64) {
      const int ry = item / NCB, j = 16 * (item - ry * NCB) + fr;
      const int jc = j < AW ? j : AW - 1;                      // (lanes past the tile re-read a valid pixel)
      // a0 (ry, j) takes canvas rows 2 ry + dy and columns 2 j + 5 + dx of the frame tile
      const int base = 2 * ry * FW + 2 * jc + 5;
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        uint2 p0 = {0u, 0u}, p1 = {0u, 0u};
        if (toff[kk][0] >= 0) p0 = *reinterpret_cast<const uint2*>(ftile + 2 * (base + toff[kk][0]));
        if (toff[kk][1] >= 0) p1 = *reinterpret_cast<const uint2*>(ftile + 2 * (base + toff[kk][1]));
        const u32x4 pv = {p0.x, p0.y, p1.x, p1.y};
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa[kk], __builtin_bit_cast(bf16x8, pv), acc, 0, 0, 0);
      }
      const int ya = y0a + ry, xa = x0a + j;
      const bool inside = ya >= 0 && ya < H0 && xa >= 0 && xa < W0;
      float v[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = inside ? silu(fmaf(acc[e], inv_std, cb[e])) : 0.f;
      if (j < AW)
        *reinterpret_cast<uint2*>(atile + (ry * AP + j) * 16 + 4 * fq) = make_uint2(pack2(v[0], v[1]), pack2(v[2], v[3]));
    }
  }
  __syncthreads();

  // ---- 3. l1: 16 pixel fragments (8 rows x 2 halves) x 2 channel blocks, K = 5 chunks of two taps
  constexpr int KQ = 5;
  bf16x8 wf[2][KQ];
#pragma unroll
  for (int nb = 0; nb < 2; ++nb)
#pragma unroll
    for (int q = 0; q < KQ; ++q) wf[nb][q] = *reinterpret_cast<const bf16x8*>(w1 + (long)(16 * nb + fr) * k1 + 32 * q + 8 * fq);
  f32x4 cb1[2];
#pragma unroll
  for (int nb = 0; nb < 2; ++nb) cb1[nb] = *reinterpret_cast<const f32x4*>(b1 + 16 * nb + 4 * fq);
  for (int item = wave; item < TH * 2; item += NT / 64) {
    const int ly = item >> 1, lx = 16 * (item & 1) + fr;
    f32x4 acc[2] = {cb1[0], cb1[1]};
#pragma unroll
    for (int q = 0; q < KQ; ++q) {
      int t = 2 * q + (fq >> 1);
      t = t < 9 ? t : 8;                                      // tap 9: zero weights, any finite pixel
      const int dy = t / 3, dx = t - 3 * dy;
      const bf16x8 xf = *reinterpret_cast<const bf16x8*>(atile + ((2 * ly + dy) * AP + 2 * lx + dx) * 16 + 8 * (fq & 1));
#pragma unroll
      for (int nb = 0; nb < 2; ++nb) acc[nb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[nb][q], xf, acc[nb], 0, 0, 0);
    }
    const int oy = oy1 + ly, ox = ox1 + lx;
    if (oy < H1 && ox < W1) {
#pragma unroll
      for (int nb = 0; nb < 2; ++nb) {
        const f32x4 a = acc[nb];
        *reinterpret_cast<uint2*>(out + (((long)b * H1 + oy) * W1 + ox) * ldo + 16 * nb + 4 * fq) =
            make_uint2(pack2(silu(a[0]), silu(a[1])), pack2(silu(a[2]), silu(a[3])));
      }
    }
  }
}

}  // namespace aiko

// frames u8 [B, Hin, Win, 3] (placed at (off_t, off_l) of an Hc x Wc canvas, fill_raw outside)
// -> a1 [B, H1, W1, ldo] (32 channels): stem w0 [16, 64] (k = (r * 3 + s) * 4 + c, the direct-stem
// layout), l1 w1 [32, k1] (k = tap * 16 + c, k1 >= 160).  H0 x W0 = the stem's output size.
extern "C" int aiko_stem_l1(const void* in, void* out, const void* w0, const float* b0, const void* w1, int k1,
                            const float* b1, int B, int Hin, int Win, int Hc, int Wc, int off_t, int off_l,
                            float fill_raw, float inv_std, int H0, int W0, int H1, int W1, int ldo, hipStream_t stream) {
  using namespace aiko;
  if (B <= 0 || B > 65535 || k1 < 160 || ldo % 4 || off_l % 4 || Win % 4 || Wc % 4 || 2 * H1 != H0 || 2 * W1 != W0 ||
      2 * H0 != Hc || 2 * W0 != Wc)
    return -1;
  const dim3 grid((W1 + sl::TW - 1) / sl::TW, (H1 + sl::TH - 1) / sl::TH, B);
  stem_l1_kernel<<<grid, sl::NT, 0, stream>>>(static_cast<const uint8_t*>(in), static_cast<bf16_t*>(out),
                                              static_cast<const bf16_t*>(w0), b0, static_cast<const bf16_t*>(w1), k1, b1,
                                              Hin, Win, Hc, Wc, off_t, off_l, fill_raw, inv_std, H0, W0, H1, W1, ldo);
  return (int)hipGetLastError();
}
