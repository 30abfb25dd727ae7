// Memory-bound vision kernels for gfx950: frame pre-processing, pooling, classifier head.
// All NHWC, bf16 activations, 16-byte vectorised where the layout allows (Guideline 13).
#include <type_traits>

#include "common.h"

namespace aiko {

// ---------------------------------------------------------------------------------------------
// uint8 RGB frames [B, Hin, Win, 3] -> bf16 [B, Hp, Wp, 4] normalised ((x/255 - mean) / std).
// The padded buffer holds a "canvas" of Hc x Wc at offset (pad_t, pad_l) — everything outside
// it is zero (the first conv's zero padding).  Inside the canvas the frame, bilinearly resized
// to (Ho, Wo) (half-pixel centres, like cv2.INTER_LINEAR), sits at (off_t, off_l); the rest of
// the canvas is the constant colour ``fill`` (letterbox bars, e.g. 114 for YOLO).  The 4th
// channel is zero.  ResNet: canvas == image, YOLO: 640x640 canvas with an aspect-preserving
// image.  One thread per padded output pixel (8-byte store): the buffer never needs a memset.
// (x / 255 - mean) / std — one definition, so the unfused pre-processing and the fused stem
// round identically
__device__ __forceinline__ void normalize3(const float c[3], float m0, float m1, float m2, float is0,
                                           float is1, float is2, float& v0, float& v1, float& v2) {
  v0 = (c[0] * (1.f / 255.f) - m0) * is0;
  v1 = (c[1] * (1.f / 255.f) - m1) * is1;
  v2 = (c[2] * (1.f / 255.f) - m2) * is2;
}

// the canvas colour of one pixel (image bilinearly resized into the canvas, ``fill`` around it),
// normalised; shared by the pre-processing kernel and the fused YOLO stem
__device__ __forceinline__ void pre_pixel(const uint8_t* __restrict__ in, int b, int Hin, int Win, int Ho,
                                          int Wo, int off_t, int off_l, int yc, int xc, float fill,
                                          float m0, float m1, float m2, float is0, float is1, float is2,
                                          int bgr, float& v0, float& v1, float& v2) {
  const int yo = yc - off_t, xo = xc - off_l;
  float c[3] = {fill, fill, fill};
  if (yo >= 0 && yo < Ho && xo >= 0 && xo < Wo) {
    if (Hin == Ho && Win == Wo) {
      const uint8_t* px = in + (((long)b * Hin + yo) * Win + xo) * 3;
      c[0] = px[0]; c[1] = px[1]; c[2] = px[2];
    } else {
      const float sy = fmaxf(((yo + 0.5f) * Hin) / Ho - 0.5f, 0.f);
      const float sx = fmaxf(((xo + 0.5f) * Win) / Wo - 0.5f, 0.f);
      int y0 = (int)sy, x0 = (int)sx;
      y0 = min(y0, Hin - 1); x0 = min(x0, Win - 1);
      const int y1 = min(y0 + 1, Hin - 1), x1 = min(x0 + 1, Win - 1);
      const float fy = sy - y0, fx = sx - x0;
      const uint8_t* base = in + (long)b * Hin * Win * 3;
      const uint8_t* p00 = base + ((long)y0 * Win + x0) * 3;
      const uint8_t* p01 = base + ((long)y0 * Win + x1) * 3;
      const uint8_t* p10 = base + ((long)y1 * Win + x0) * 3;
      const uint8_t* p11 = base + ((long)y1 * Win + x1) * 3;
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        const float top = p00[k] + (p01[k] - (float)p00[k]) * fx;
        const float bot = p10[k] + (p11[k] - (float)p10[k]) * fx;
        c[k] = top + (bot - top) * fy;
      }
    }
    if (bgr) { const float t = c[0]; c[0] = c[2]; c[2] = t; }
  }
  normalize3(c, m0, m1, m2, is0, is1, is2, v0, v1, v2);
}

// 2-D grid (x: pixels of one padded image, y: image): no 64-bit division of a flat index per
// pixel (~100 VALU instructions each); the row is an exact float-reciprocal quotient with a
// one-step integer fix-up.  Output bit-identical to the flat version (same pre_pixel).
__global__ __launch_bounds__(256) void preprocess_kernel(const uint8_t* __restrict__ in, bf16_t* __restrict__ out,
                                  int B, int Hin, int Win, int Ho, int Wo, int Hp, int Wp,
                                  int pad_t, int pad_l, int Hc, int Wc, int off_t, int off_l,
                                  float fill, float m0, float m1, float m2,
                                  float is0, float is1, float is2, int bgr) {
  const int b = blockIdx.y;
  const int HW = Hp * Wp;
  const float inv_wp = 1.f / (float)Wp;
  const uint8_t* img = in + (long)b * Hin * Win * 3;
  bf16_t* ob = out + (long)b * HW * 4;
  for (int rem = blockIdx.x * blockDim.x + threadIdx.x; rem < HW; rem += gridDim.x * blockDim.x) {
    int yp = (int)(((float)rem + 0.5f) * inv_wp);
    if (yp * Wp > rem) --yp;
    else if ((yp + 1) * Wp <= rem) ++yp;
    const int xp = rem - yp * Wp;
    const int yc = yp - pad_t, xc = xp - pad_l;
    uint2 o = {0u, 0u};
    if (yc >= 0 && yc < Hc && xc >= 0 && xc < Wc) {
      float v0, v1, v2;
      pre_pixel(img, 0, Hin, Win, Ho, Wo, off_t, off_l, yc, xc, fill, m0, m1, m2, is0, is1, is2, bgr, v0, v1, v2);
      o.x = pack2(v0, v1);
      o.y = pack2(v2, 0.f);
    }
    *reinterpret_cast<uint2*>(ob + (long)rem * 4) = o;
  }
}

// No-resize, no-letterbox fast path (the ResNet bench: 224x224 frames into the 230x230 stem
// buffer): one wave per padded row, each lane converts 4 pixels from three dword loads (12
// bytes), so a wave keeps 768 B of frame reads in flight per load instead of 192 B of byte
// loads -- the flat kernel is read-latency bound at ~3.8 TB/s.  Same normalize3 math, so the
// output is bit-identical to preprocess_kernel.  Needs W % 4 == 0 and a 4-byte-aligned frame
// base (checked by the launcher).
__global__ __launch_bounds__(256) void preprocess_rows_kernel(
    const uint8_t* __restrict__ in, bf16_t* __restrict__ out, int H, int W, int Hp, int Wp,
    int pad_t, int pad_l, float m0, float m1, float m2, float is0, float is1, float is2, int bgr) {
  const int lane = threadIdx.x & 63;
  const int yp = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int b = blockIdx.y;
  if (yp >= Hp) return;
  bf16_t* orow = out + ((long)b * Hp + yp) * Wp * 4;
  const int yc = yp - pad_t;
  if (yc < 0 || yc >= H) {
    for (int x = lane; x < Wp; x += 64) *reinterpret_cast<uint2*>(orow + x * 4) = uint2{0u, 0u};
    return;
  }
  for (int x = lane; x < pad_l; x += 64) *reinterpret_cast<uint2*>(orow + x * 4) = uint2{0u, 0u};
  for (int x = pad_l + W + lane; x < Wp; x += 64) *reinterpret_cast<uint2*>(orow + x * 4) = uint2{0u, 0u};
  const uint32_t* irow = reinterpret_cast<const uint32_t*>(in + ((long)b * H + yc) * W * 3);
  bf16_t* oint = orow + pad_l * 4;
  for (int q = lane; q < (W >> 2); q += 64) {
    const uint32_t w0 = irow[3 * q], w1 = irow[3 * q + 1], w2 = irow[3 * q + 2];
    const uint32_t wd[3] = {w0, w1, w2};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float c[3];
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        const int byte = 3 * j + k;
        c[k] = (float)((wd[byte >> 2] >> (8 * (byte & 3))) & 0xFFu);
      }
      if (bgr) { const float t = c[0]; c[0] = c[2]; c[2] = t; }
      float v0, v1, v2;
      normalize3(c, m0, m1, m2, is0, is1, is2, v0, v1, v2);
      *reinterpret_cast<uint2*>(oint + (4 * q + j) * 4) = uint2{pack2(v0, v1), pack2(v2, 0.f)};
    }
  }
}

// ---------------------------------------------------------------------------------------------
// Fused pre-processing + first conv (YOLOv8's 3x3/2 stem; k <= 4, any stride / pad): uint8
// frames -> letterbox / normalise (pre_pixel, rounded to bf16 exactly like preprocess_kernel)
// straight into an LDS tile [IH][IW][4 ch] -> implicit GEMM on v_mfma_f32_16x16x32_bf16 with
// K = taps x 4 channels (<= 64, zero padded) -> bias + SiLU/ReLU -> bf16 NHWC.  The unfused
// path paid a bf16 canvas round trip through HBM and a 27 -> 64 padded K over a pixel-run
// layout; a VALU direct conv was LDS-bound on the weight reads.  Operand roles: A = weights
// (lane row = output channel), B = pixel patches (lane column = pixel), so each lane ends with
// 4 consecutive channels of one pixel: 8-byte stores, a wave writes 16 whole pixels.
// Workgroup = 8 x 32 output pixels; wave w owns rows 2w, 2w+1 (4 tiles of 16 pixels).
constexpr int kStemTH = 8, kStemTW = 32;
__global__ __launch_bounds__(256) void stem_direct_kernel(
    const uint8_t* __restrict__ in, bf16_t* __restrict__ out, const bf16_t* __restrict__ w,
    const float* __restrict__ bias, int Hin, int Win, int Ho, int Wo, int Hc, int Wc, int off_t, int off_l,
    float fill, float m0, float m1, float m2, float is0, float is1, float is2, int bgr, int H1, int W1,
    int Cout, int ldo, int k, int stride, int pad, int act) {
  extern __shared__ __attribute__((aligned(16))) uint32_t stile[];   // [IH][IW] x (2 dwords = 4 bf16)
  const int IH = (kStemTH - 1) * stride + k, IW = (kStemTW - 1) * stride + k;
  const int tid = threadIdx.x, b = blockIdx.z, lane = tid & 63, wave = tid >> 6;
  const int oy0 = blockIdx.y * kStemTH, ox0 = blockIdx.x * kStemTW;
  // the kernel is VALU-issue bound (PMC: ~820 VALU instructions per wave against 8 MFMAs), so
  // the fill avoids the integer division by IW (exact float reciprocal: i < 2^16) and, at scale
  // 1 (no resize, the camera-size case), pre_pixel's 64-bit per-pixel address arithmetic
  const float inv_iw = 1.f / (float)IW;
  const bool noresize = Hin == Ho && Win == Wo;
  const uint8_t* img = in + (long)b * Hin * Win * 3;
  for (int i = tid; i < IH * IW; i += 256) {
    const int ty = (int)(((float)i + 0.5f) * inv_iw), tx = i - ty * IW;
    const int yc = oy0 * stride - pad + ty, xc = ox0 * stride - pad + tx;
    uint2 o = {0u, 0u};                         // outside the canvas: the conv's zero padding
    if (yc >= 0 && yc < Hc && xc >= 0 && xc < Wc) {
      float v0, v1, v2;
      if (noresize) {
        const int yo = yc - off_t, xo = xc - off_l;
        float c[3] = {fill, fill, fill};
        if ((unsigned)yo < (unsigned)Ho && (unsigned)xo < (unsigned)Wo) {
          const uint8_t* px = img + (yo * Win + xo) * 3;
          c[0] = px[0]; c[1] = px[1]; c[2] = px[2];
          if (bgr) { const float t = c[0]; c[0] = c[2]; c[2] = t; }
        }
        normalize3(c, m0, m1, m2, is0, is1, is2, v0, v1, v2);
      } else {
        pre_pixel(in, b, Hin, Win, Ho, Wo, off_t, off_l, yc, xc, fill, m0, m1, m2, is0, is1, is2, bgr, v0, v1, v2);
      }
      o.x = pack2(v0, v1);
      o.y = pack2(v2, 0.f);
    }
    *reinterpret_cast<uint2*>(stile + 2 * i) = o;
  }
  __syncthreads();
  const int fr = lane & 15, fq = lane >> 4;
  const int taps = k * k;
  // this lane's two taps per 32-K half: k-piece pc = fq + 4 kk covers taps 2 pc, 2 pc + 1
  int toff[2][2];
#pragma unroll
  for (int kk = 0; kk < 2; ++kk)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int t = 2 * (fq + 4 * kk) + h;
      toff[kk][h] = t < taps ? (t / k) * IW + (t % k) : -1;
    }
  for (int n0 = 0; n0 < Cout; n0 += 16) {
    bf16x8 wa[2];
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
      wa[kk] = *reinterpret_cast<const bf16x8*>(w + (long)(n0 + fr) * 64 + 8 * (fq + 4 * kk));
    float cb[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) cb[e] = bias ? bias[n0 + 4 * fq + e] : 0.f;
#pragma unroll
    for (int pt = 0; pt < 4; ++pt) {
      const int ly = 2 * wave + (pt >> 1), lx = 16 * (pt & 1) + fr;
      const int base = (ly * stride) * IW + lx * stride;
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        uint2 p0 = {0u, 0u}, p1 = {0u, 0u};
        if (toff[kk][0] >= 0) p0 = *reinterpret_cast<const uint2*>(stile + 2 * (base + toff[kk][0]));
        if (toff[kk][1] >= 0) p1 = *reinterpret_cast<const uint2*>(stile + 2 * (base + toff[kk][1]));
        const u32x4 pv = {p0.x, p0.y, p1.x, p1.y};
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa[kk], __builtin_bit_cast(bf16x8, pv), acc, 0, 0, 0);
      }
      const int oy = oy0 + ly, ox = ox0 + lx;
      if (oy < H1 && ox < W1) {
        float v[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float a = acc[e] + cb[e];
          if (act == 1) a = fmaxf(a, 0.f);
          else if (act == 2) a = silu(a);
          v[e] = a;
        }
        *reinterpret_cast<uint2*>(out + (((long)b * H1 + oy) * W1 + ox) * ldo + n0 + 4 * fq) =
            make_uint2(pack2(v[0], v[1]), pack2(v[2], v[3]));
      }
    }
  }
}

// ---------------------------------------------------------------------------------------------
// The same stem for the camera-size case (no resize, mean 0, one std for the three channels —
// YOLO's /255 — 3x3/2 pad 1, 16 output channels, 4-pixel aligned image columns): VALU work per
// wave cut ~4x against stem_direct_kernel, which is VALU-issue bound (PMC: ~820 VALU per wave):
//   * the tile holds RAW pixel values (0..255, exact in bf16) and 1/(255 std) is applied to the
//     fp32 accumulator in the epilogue FMA that adds the bias — no per-pixel normalisation;
//   * it is filled 4 pixels per thread (three dword loads, v_cvt_f32_ubyte*, cvt_pk) into a
//     tile whose rows start 3 pixels early, so a group of 4 lands on 2 aligned ds_write_b128 —
//     no per-pixel index division, bounds test or byte load;
//   * letterbox bars / conv padding are decided per group (aligned groups never straddle).
// tile: TH x 32 outputs.  TH = 16 is the default: 65.3-67.5 us against 71.8-72.4 (TH 8) and
// 68.6-72.1 (TH 32) at B=64 480x640 on MI355X (same box, interleaved) — half the workgroups, half
// the per-tile weight / bias loads and 3 % input-row halo instead of 6 %
template <int ACT, bool BGR, bool WIDE, int TH = 8, int TW = 32>
__global__ __launch_bounds__(256) void stem_fast_kernel(
    const uint8_t* __restrict__ in, bf16_t* __restrict__ out, const bf16_t* __restrict__ w,
    const float* __restrict__ bias, int Hin, int Win, int Hc, int Wc, int off_t, int off_l, float fill_raw,
    float inv_std, int H1, int W1, int ldo) {
  static_assert(TH == 8 || TH == 16 || TH == 32, "8, 16 or 32 output rows per tile");
  static_assert(!WIDE || (TH == 8 && TW == 32), "the 16-B store path pairs the two half-rows of an 8 x 32 tile");
  static_assert(TW == 32 || TW == 64, "32 or 64 output columns per tile");
  constexpr int kSfTW = TW;
  constexpr int kSfG = TW / 2 + 1;               // groups of 4 pixels per input row (17 / 33)
  constexpr int kSfIW = 4 * kSfG;                // tile columns (tile col = input x - (2 ox0 - 1) + 3)
  constexpr int kSfIH = 2 * TH + 1;              // input rows (17 / 33)
  constexpr int RPW = TH / 4;                    // output rows per wave
  __shared__ __attribute__((aligned(16))) uint32_t stile[kSfIH * kSfIW * 2];   // [kSfIH][68] x 4 bf16
  const int tid = threadIdx.x, b = blockIdx.z, lane = tid & 63, wave = tid >> 6;
  const int oy0 = blockIdx.y * TH, ox0 = blockIdx.x * kSfTW;
  const int g0 = (2 * ox0 - 4) >> 2;            // first group: canvas x 2 ox0 - 4 .. 2 ox0 - 1
  const uint8_t* img = in + (long)b * Hin * Win * 3;
  const uint32_t f2 = pack2(fill_raw, fill_raw), fb = f2 & 0xffffu;
  for (int task = tid; task < kSfIH * kSfG; task += 256) {
    const int ty = task / kSfG, gi = task - ty * kSfG;
    const int yc = 2 * oy0 - 1 + ty, xc = 4 * (g0 + gi);
    u32x4 lo = {0u, 0u, 0u, 0u}, hi = {0u, 0u, 0u, 0u};    // outside the canvas: zero padding
    if (yc >= 0 && yc < Hc && xc >= 0 && xc < Wc) {
      const int yo = yc - off_t, xo = xc - off_l;
      if ((unsigned)yo < (unsigned)Hin && (unsigned)xo < (unsigned)Win) {
        const uint32_t* src = reinterpret_cast<const uint32_t*>(img + ((long)yo * Win + xo) * 3);
        const uint32_t w0 = src[0], w1 = src[1], w2 = src[2];
        // bytes: p0 = w0[0..2], p1 = w0[3] w1[0..1], p2 = w1[2..3] w2[0], p3 = w2[1..3]
        float c[12];
        const uint32_t wd[3] = {w0, w1, w2};
#pragma unroll
        for (int j = 0; j < 12; ++j) c[j] = (float)((wd[j >> 2] >> (8 * (j & 3))) & 0xFFu);
        if constexpr (BGR) {
#pragma unroll
          for (int q = 0; q < 4; ++q) { const float t = c[3 * q]; c[3 * q] = c[3 * q + 2]; c[3 * q + 2] = t; }
        }
        lo = u32x4{pack2(c[0], c[1]), pack2(c[2], 0.f), pack2(c[3], c[4]), pack2(c[5], 0.f)};
        hi = u32x4{pack2(c[6], c[7]), pack2(c[8], 0.f), pack2(c[9], c[10]), pack2(c[11], 0.f)};
      } else {                                   // letterbox bar (raw fill value)
        lo = u32x4{f2, fb, f2, fb};
        hi = lo;
      }
    }
    uint32_t* dst = stile + 2 * (ty * kSfIW + 4 * gi);
    *reinterpret_cast<u32x4*>(dst) = lo;
    *reinterpret_cast<u32x4*>(dst + 4) = hi;
  }
  __syncthreads();
  const int fr = lane & 15, fq = lane >> 4;
  // this lane's two taps per 32-K half (k-piece pc = fq + 4 kk covers taps 2 pc, 2 pc + 1);
  // tile offset of tap (dy, dx) for output (ly, lx): (2 ly + dy) row, 2 lx + dx + 2 col (the
  // output's first input column 2 ox0 - 1 sits at tile col 3)
  int toff[2][2];
#pragma unroll
  for (int kk = 0; kk < 2; ++kk)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int t = 2 * (fq + 4 * kk) + h;
      toff[kk][h] = t < 9 ? (t / 3) * kSfIW + (t % 3) + 3 : -1;
    }
  bf16x8 wa[2];
#pragma unroll
  for (int kk = 0; kk < 2; ++kk) wa[kk] = *reinterpret_cast<const bf16x8*>(w + (long)fr * 64 + 8 * (fq + 4 * kk));
  float cb[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) cb[e] = bias ? bias[4 * fq + e] : 0.f;
  // this lane's output pixel (2 wave, fr) of the tile, 32-bit element offsets from the image
  const bf16_t* obase = out + (size_t)b * H1 * W1 * ldo;
  const int orow = oy0 + RPW * wave, ocol = ox0 + fr;
  const uint32_t o0 = (uint32_t)((orow * W1 + ocol) * ldo + 4 * fq);
  const int lbase = 2 * RPW * wave * kSfIW + 2 * fr;        // tile pixel of output (RPW wave, fr)
  if constexpr (!WIDE) {
#pragma unroll
    for (int pt = 0; pt < (TW / 16) * RPW; ++pt) {
      const int dy = pt / (TW / 16), dx = 16 * (pt % (TW / 16));
      const int base = lbase + 2 * dy * kSfIW + 2 * dx;
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        uint2 p0 = {0u, 0u}, p1 = {0u, 0u};
        if (toff[kk][0] >= 0) p0 = *reinterpret_cast<const uint2*>(stile + 2 * (base + toff[kk][0]));
        if (toff[kk][1] >= 0) p1 = *reinterpret_cast<const uint2*>(stile + 2 * (base + toff[kk][1]));
        const u32x4 pv = {p0.x, p0.y, p1.x, p1.y};
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa[kk], __builtin_bit_cast(bf16x8, pv), acc, 0, 0, 0);
      }
      if (orow + dy < H1 && ocol + dx < W1) {
        float v[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float a = fmaf(acc[e], inv_std, cb[e]);
          if constexpr (ACT == 1) a = fmaxf(a, 0.f);
          else if constexpr (ACT == 2) a = silu(a);
          v[e] = a;
        }
        *reinterpret_cast<uint2*>(const_cast<bf16_t*>(obase) + o0 + (uint32_t)((dy * W1 + dx) * ldo)) =
            make_uint2(pack2(v[0], v[1]), pack2(v[2], v[3]));
      }
    }
    return;
  }
  // the two 16-pixel halves (dx = 0, 16) of one output row form a pair: after the epilogue a
  // v_permlane16_swap per packed dword gives 16-lane row 0 channels 0-7 of the left half, row 1
  // channels 0-7 of the right half, rows 2 / 3 channels 8-15 of each — one 16-B store per lane
  // per pair instead of two 8-B stores (the kernel's tail is store-issue bound)
  const int half = fq & 1;                                   // 0: left half, 1: right half
  const uint32_t o_sw = (uint32_t)(half * 16 * ldo + 8 * (fq >> 1)) - 4 * fq;   // vs o0's 4 fq
#pragma unroll
  for (int dy = 0; dy < 2; ++dy) {
    uint32_t u[2][2];
#pragma unroll
    for (int hx = 0; hx < 2; ++hx) {
      const int base = lbase + 2 * dy * kSfIW + 2 * (16 * hx);
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        uint2 p0 = {0u, 0u}, p1 = {0u, 0u};
        if (toff[kk][0] >= 0) p0 = *reinterpret_cast<const uint2*>(stile + 2 * (base + toff[kk][0]));
        if (toff[kk][1] >= 0) p1 = *reinterpret_cast<const uint2*>(stile + 2 * (base + toff[kk][1]));
        const u32x4 pv = {p0.x, p0.y, p1.x, p1.y};
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa[kk], __builtin_bit_cast(bf16x8, pv), acc, 0, 0, 0);
      }
      float v[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float a = fmaf(acc[e], inv_std, cb[e]);
        if constexpr (ACT == 1) a = fmaxf(a, 0.f);
        else if constexpr (ACT == 2) a = silu(a);
        v[e] = a;
      }
      u[hx][0] = pack2(v[0], v[1]);
      u[hx][1] = pack2(v[2], v[3]);
    }
    u32x4 o;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const auto sw = __builtin_amdgcn_permlane16_swap(u[0][j], u[1][j], false, false);
      o[j] = sw[0];
      o[2 + j] = sw[1];
    }
    if (orow + dy < H1 && ocol + 16 * half < W1)
      *reinterpret_cast<u32x4*>(const_cast<bf16_t*>(obase) + o0 + o_sw + (uint32_t)(dy * W1 * ldo)) = o;
  }
}

// ---------------------------------------------------------------------------------------------
// Max pool (k x k, stride s, pad p) NHWC bf16, C % 8 == 0: one thread per 8 channels of one
// output pixel (16-byte loads/stores).  Padding never wins (-inf).  ``ldx`` / ``ldy`` are the
// pixel pitches, so input and output may be channel slices of concat buffers (YOLO SPPF).
// YOLOv8 SPPF's three chained k x k / stride-1 max pools in one kernel: slice 0 of the concat
// buffer [B, H, W, ld] (channels [0, c)) -> slices 1, 2, 3.  One block per (image, 8 channels)
// stages the H x W map in LDS and runs each pool as a row max then a column max (clipped
// windows, so separable); max is exact, so the three slices are bit-identical to three
// maxpool_kernel launches, without two round trips through HBM and two launches.
__global__ __launch_bounds__(256) void sppf_pool_kernel(bf16_t* __restrict__ x, int H, int W, int ld,
                                                        int c, int k) {
  extern __shared__ __attribute__((aligned(16))) u32x4 tile[];   // [2][H*W]: map, row max
  const int HW = H * W, r = k / 2;
  const int c8 = blockIdx.x, b = blockIdx.y;
  u32x4* cur = tile;
  u32x4* rmax = tile + HW;
  bf16_t* img = x + (long)b * HW * ld + c8 * 8;
  for (int i = threadIdx.x; i < HW; i += 256) cur[i] = *reinterpret_cast<const u32x4*>(img + (long)i * ld);
  __syncthreads();
  const auto vmax = [](u32x4 a, u32x4 v) {
    u32x4 o;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float lo = fmaxf(__uint_as_float(a[e] << 16), __uint_as_float(v[e] << 16));
      const float hi = fmaxf(__uint_as_float(a[e] & 0xffff0000u), __uint_as_float(v[e] & 0xffff0000u));
      o[e] = (__float_as_uint(lo) >> 16) | (__float_as_uint(hi) & 0xffff0000u);
    }
    return o;
  };
  for (int it = 1; it <= 3; ++it) {
    for (int i = threadIdx.x; i < HW; i += 256) {
      const int h = i / W, w = i - h * W;
      u32x4 m = cur[i];
      for (int d = max(-r, -w); d <= min(r, W - 1 - w); ++d) m = vmax(m, cur[h * W + w + d]);
      rmax[i] = m;
    }
    __syncthreads();
    for (int i = threadIdx.x; i < HW; i += 256) {
      const int h = i / W, w = i - h * W;
      u32x4 m = rmax[i];
      for (int d = max(-r, -h); d <= min(r, H - 1 - h); ++d) m = vmax(m, rmax[(h + d) * W + w]);
      cur[i] = m;
      *reinterpret_cast<u32x4*>(img + (long)i * ld + it * c) = m;
    }
    __syncthreads();
  }
}

__global__ void maxpool_kernel(const bf16_t* __restrict__ x, bf16_t* __restrict__ y, int B,
                               int H, int W, int C, int Ho, int Wo, int k, int s, int p,
                               int ldx, int ldy) {
  const int C8 = C >> 3;
  const long total = (long)B * Ho * Wo * C8;
  for (long idx = blockIdx.x * (long)blockDim.x + threadIdx.x; idx < total;
       idx += (long)gridDim.x * blockDim.x) {
    const int c8 = idx % C8;
    long t = idx / C8;
    const int wo = t % Wo; t /= Wo;
    const int ho = t % Ho;
    const int b = t / Ho;
    float m[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) m[e] = -INFINITY;
    for (int dy = 0; dy < k; ++dy) {
      const int ih = ho * s - p + dy;
      if ((unsigned)ih >= (unsigned)H) continue;
      for (int dx = 0; dx < k; ++dx) {
        const int iw = wo * s - p + dx;
        if ((unsigned)iw >= (unsigned)W) continue;
        const u32x4 v = *reinterpret_cast<const u32x4*>(
            x + (((long)b * H + ih) * W + iw) * ldx + c8 * 8);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          m[2 * e] = fmaxf(m[2 * e], __uint_as_float(v[e] << 16));
          m[2 * e + 1] = fmaxf(m[2 * e + 1], __uint_as_float(v[e] & 0xffff0000u));
        }
      }
    }
    u32x4 o;
#pragma unroll
    for (int e = 0; e < 4; ++e) o[e] = pack2(m[2 * e], m[2 * e + 1]);
    *reinterpret_cast<u32x4*>(y + (((long)b * Ho + ho) * Wo + wo) * ldy + c8 * 8) = o;
  }
}

// ---------------------------------------------------------------------------------------------
// Global average pool NHWC bf16 [B, HW, C] -> bf16 [B, C]; one thread per 8 channels.
__global__ void avgpool_kernel(const bf16_t* __restrict__ x, bf16_t* __restrict__ y, int B,
                               int HW, int C) {
  const int C8 = C >> 3;
  const long total = (long)B * C8;
  const float inv = 1.f / HW;
  for (long idx = blockIdx.x * (long)blockDim.x + threadIdx.x; idx < total;
       idx += (long)gridDim.x * blockDim.x) {
    const int c8 = idx % C8;
    const int b = idx / C8;
    float a[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    const bf16_t* src = x + (long)b * HW * C + c8 * 8;
    // 7 rows' loads in flight per step (one wave per SIMD at ResNet's 256 x 2048 / 8 threads:
    // a load -> add chain per row was latency-bound); same summation order as row by row
    int i = 0;
    for (; i + 7 <= HW; i += 7) {
      u32x4 v[7];
#pragma unroll
      for (int u = 0; u < 7; ++u) v[u] = *reinterpret_cast<const u32x4*>(src + (long)(i + u) * C);
#pragma unroll
      for (int u = 0; u < 7; ++u)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          a[2 * e] += __uint_as_float(v[u][e] << 16);
          a[2 * e + 1] += __uint_as_float(v[u][e] & 0xffff0000u);
        }
    }
    for (; i < HW; ++i) {
      const u32x4 v = *reinterpret_cast<const u32x4*>(src + (long)i * C);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        a[2 * e] += __uint_as_float(v[e] << 16);
        a[2 * e + 1] += __uint_as_float(v[e] & 0xffff0000u);
      }
    }
    u32x4 o;
#pragma unroll
    for (int e = 0; e < 4; ++e) o[e] = pack2(a[2 * e] * inv, a[2 * e + 1] * inv);
    *reinterpret_cast<u32x4*>(y + idx * 8) = o;
  }
}

// ---------------------------------------------------------------------------------------------
// Row softmax + top-k (k <= 8) over bf16 logits [B, N]: one wave per row.  Each lane keeps
// its strided slice in registers (N <= 64 * 32), the wave reduces max / sum-exp with
// shuffles, then k rounds of wave-wide argmax extract the top-k (ties -> lowest index).
template <int PER_LANE>
__global__ void softmax_topk_kernel(const bf16_t* __restrict__ logits, float* __restrict__ prob,
                                    int* __restrict__ index, int B, int N, int k) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (row >= B) return;
  const bf16_t* src = logits + (long)row * N;
  float v[PER_LANE];
  float mx = -INFINITY;
#pragma unroll
  for (int i = 0; i < PER_LANE; ++i) {
    const int c = lane + 64 * i;
    v[i] = c < N ? bf2f(src[c]) : -INFINITY;
    mx = fmaxf(mx, v[i]);
  }
  mx = wave_max(mx);
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < PER_LANE; ++i) {
    const int c = lane + 64 * i;
    s += c < N ? __expf(v[i] - mx) : 0.f;
  }
  s = wave_sum(s);
  const float inv = 1.f / s;
  // Each round's arg-max is one unsigned wave max over 32-bit keys: the logit's bf16 bits mapped
  // to an order-preserving code (high half; -0 folded onto +0) and 0xFFFF - column (low half), so
  // ties go to the lower column exactly as the (value, index) compare did.  Logits come from bf16,
  // so the key holds the value exactly; N <= 2048 fits the low half.  A taken column's key becomes
  // the key of -INF at that column, i.e. what setting its value to -INF gave.
  unsigned key[PER_LANE];
#pragma unroll
  for (int i = 0; i < PER_LANE; ++i) {
    unsigned b = __float_as_uint(v[i]) >> 16;
    if (b == 0x8000u) b = 0;
    const unsigned ord = (b & 0x8000u) ? (~b & 0xFFFFu) : (b | 0x8000u);
    key[i] = (ord << 16) | (0xFFFFu - (unsigned)(lane + 64 * i));
  }
  const auto umax = [](float x, float y) {
    return __uint_as_float(max(__float_as_uint(x), __float_as_uint(y)));
  };
  for (int t = 0; t < k; ++t) {
    unsigned best = 0;
#pragma unroll
    for (int i = 0; i < PER_LANE; ++i) best = max(best, key[i]);
    best = __float_as_uint(wave_reduce(__uint_as_float(best), umax));
    const int bi = 0xFFFF - (int)(best & 0xFFFFu);
    const unsigned ord = best >> 16;
    const unsigned b = (ord & 0x8000u) ? (ord & 0x7FFFu) : (~ord & 0xFFFFu);
    if (lane == 0) {
      prob[(long)row * k + t] = __expf(__uint_as_float(b << 16) - mx) * inv;
      index[(long)row * k + t] = bi;
    }
#pragma unroll
    for (int i = 0; i < PER_LANE; ++i)
      if (lane + 64 * i == bi) key[i] = (0x007Fu << 16) | (0xFFFFu - (unsigned)bi);
  }
}


// ---------------------------------------------------------------------------------------------
// uint8 RGB bilinear resize [B, Hin, Win, 3] -> [B, Ho, Wo, 3] (half-pixel centres, like
// cv2.INTER_LINEAR; ImageResize on the GPU path).  One thread per output pixel.
__global__ void resize_u8_kernel(const uint8_t* __restrict__ in, uint8_t* __restrict__ out, int B,
                                 int Hin, int Win, int Ho, int Wo) {
  const long total = (long)B * Ho * Wo;
  const float sy_scale = (float)Hin / Ho, sx_scale = (float)Win / Wo;
  for (long idx = blockIdx.x * (long)blockDim.x + threadIdx.x; idx < total;
       idx += (long)gridDim.x * blockDim.x) {
    const int b = idx / ((long)Ho * Wo);
    const int rem = idx - (long)b * Ho * Wo;
    const int yo = rem / Wo, xo = rem - (rem / Wo) * Wo;
    const float sy = fmaxf((yo + 0.5f) * sy_scale - 0.5f, 0.f);
    const float sx = fmaxf((xo + 0.5f) * sx_scale - 0.5f, 0.f);
    const int y0 = min((int)sy, Hin - 1), x0 = min((int)sx, Win - 1);
    const int y1 = min(y0 + 1, Hin - 1), x1 = min(x0 + 1, Win - 1);
    const float fy = sy - y0, fx = sx - x0;
    const uint8_t* base = in + (long)b * Hin * Win * 3;
    const uint8_t* p00 = base + ((long)y0 * Win + x0) * 3;
    const uint8_t* p01 = base + ((long)y0 * Win + x1) * 3;
    const uint8_t* p10 = base + ((long)y1 * Win + x0) * 3;
    const uint8_t* p11 = base + ((long)y1 * Win + x1) * 3;
    uint8_t* o = out + idx * 3;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      const float top = p00[k] + (p01[k] - (float)p00[k]) * fx;
      const float bot = p10[k] + (p11[k] - (float)p10[k]) * fx;
      o[k] = (uint8_t)fminf(fmaxf(rintf(top + (bot - top) * fy), 0.f), 255.f);
    }
  }
}

// ---------------------------------------------------------------------------------------------
// Inference BatchNorm as a standalone op (normally folded into the preceding conv):
// y = act(x * scale[c] + shift[c]) on NHWC bf16, 8 channels per thread, pixel pitches ldx/ldy.
__global__ void batchnorm_kernel(const bf16_t* __restrict__ x, bf16_t* __restrict__ y,
                                 const float* __restrict__ scale, const float* __restrict__ shift,
                                 long P, int C, int ldx, int ldy, int act) {
  const int C8 = C >> 3;
  const long total = P * C8;
  for (long idx = blockIdx.x * (long)blockDim.x + threadIdx.x; idx < total;
       idx += (long)gridDim.x * blockDim.x) {
    const int c8 = idx % C8;
    const long pix = idx / C8;
    const u32x4 v = *reinterpret_cast<const u32x4*>(x + pix * ldx + c8 * 8);
    float f[8];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      f[2 * e] = __uint_as_float(v[e] << 16);
      f[2 * e + 1] = __uint_as_float(v[e] & 0xffff0000u);
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      float t = f[e] * scale[c8 * 8 + e] + shift[c8 * 8 + e];
      if (act == 1) t = fmaxf(t, 0.f);
      else if (act == 2) t = silu(t);
      f[e] = t;
    }
    u32x4 o;
#pragma unroll
    for (int e = 0; e < 4; ++e) o[e] = pack2(f[2 * e], f[2 * e + 1]);
    *reinterpret_cast<u32x4*>(y + pix * ldy + c8 * 8) = o;
  }
}

}  // namespace aiko

extern "C" int aiko_resize_u8(const void* in, void* out, int B, int Hin, int Win, int Ho, int Wo,
                              hipStream_t stream) {
  const long total = (long)B * Ho * Wo;
  long g = (total + 255) / 256;
  if (g > 4096) g = 4096;
  aiko::resize_u8_kernel<<<(int)g, 256, 0, stream>>>(static_cast<const uint8_t*>(in),
                                                     static_cast<uint8_t*>(out), B, Hin, Win, Ho, Wo);
  return (int)hipGetLastError();
}

extern "C" int aiko_batchnorm(const void* x, void* y, const float* scale, const float* shift, long P,
                              int C, int ldx, int ldy, int act, hipStream_t stream) {
  const long total = P * (C / 8);
  long g = (total + 255) / 256;
  if (g > 4096) g = 4096;
  aiko::batchnorm_kernel<<<(int)g, 256, 0, stream>>>(static_cast<const aiko::bf16_t*>(x),
                                                     static_cast<aiko::bf16_t*>(y), scale, shift, P,
                                                     C, ldx, ldy, act);
  return (int)hipGetLastError();
}

namespace aiko {
}  // namespace aiko

static inline int grid_for(long total, int block) {
  long g = (total + block - 1) / block;
  if (g > 256 * 16) g = 256 * 16;
  if (g < 1) g = 1;
  return (int)g;
}

extern "C" int aiko_preprocess(const void* in, void* out, int B, int Hin, int Win, int Ho,
                               int Wo, int Hp, int Wp, int pad_t, int pad_l, int Hc, int Wc,
                               int off_t, int off_l, float fill, const float* mean,
                               const float* std, int bgr, hipStream_t stream) {
  if (B <= 0 || B > 65535 || Hp <= 0 || Wp <= 0) return -1;
  if (Hin == Ho && Win == Wo && Hc == Ho && Wc == Wo && off_t == 0 && off_l == 0 && Win % 4 == 0 &&
      reinterpret_cast<uintptr_t>(in) % 4 == 0 && pad_t >= 0 && pad_l >= 0 &&
      pad_t + Hc <= Hp && pad_l + Wc <= Wp) {
    hipLaunchKernelGGL(aiko::preprocess_rows_kernel, dim3((unsigned)((Hp + 3) / 4), (unsigned)B),
                       dim3(256), 0, stream, static_cast<const uint8_t*>(in),
                       static_cast<aiko::bf16_t*>(out), Hin, Win, Hp, Wp, pad_t, pad_l, mean[0],
                       mean[1], mean[2], 1.f / std[0], 1.f / std[1], 1.f / std[2], bgr);
    return (int)hipGetLastError();
  }
  const long per_img = (long)Hp * Wp;
  long gx = (per_img + 255) / 256;
  if (gx > 1024) gx = 1024;
  hipLaunchKernelGGL(aiko::preprocess_kernel, dim3((unsigned)gx, (unsigned)B), dim3(256), 0, stream,
                     static_cast<const uint8_t*>(in), static_cast<aiko::bf16_t*>(out), B, Hin,
                     Win, Ho, Wo, Hp, Wp, pad_t, pad_l, Hc, Wc, off_t, off_l, fill, mean[0],
                     mean[1], mean[2], 1.f / std[0], 1.f / std[1], 1.f / std[2], bgr);
  return (int)hipGetLastError();
}

extern "C" int aiko_stem_direct(const void* in, void* out, const void* w, const float* bias, int B, int Hin,
                                int Win, int Ho, int Wo, int Hc, int Wc, int off_t, int off_l, float fill,
                                const float* mean, const float* std, int bgr, int H1, int W1, int Cout, int ldo,
                                int k, int stride, int pad, int act, hipStream_t stream) {
  if (Cout % 16 || ldo % 4 || k < 1 || k > 4 || stride < 1 || B <= 0) return -1;
  static const bool fast_ok = [] { const char* e = getenv("AIKO_STEM_FAST"); return !(e && *e == '0'); }();
  if (fast_ok && k == 3 && stride == 2 && pad == 1 && Cout == 16 && Ho == Hin && Wo == Win && Win % 4 == 0 &&
      ldo % 8 == 0 && reinterpret_cast<uintptr_t>(out) % 16 == 0 &&
      off_l % 4 == 0 && Wc % 4 == 0 && mean[0] == 0.f && mean[1] == 0.f && mean[2] == 0.f &&
      std[0] == std[1] && std[1] == std[2] && std[0] > 0.f) {
    const char* th_env = getenv("AIKO_STEM_FAST_TH");         // 8, 16 or 32 output rows per tile
    const int th_req = th_env ? atoi(th_env) : 16;
    const int th = th_req == 8 || th_req == 32 ? th_req : 16;
    const char* tw_env = getenv("AIKO_STEM_FAST_TW");         // 32 or 64 output columns per tile
    const int tw = tw_env && atoi(tw_env) == 64 ? 64 : 32;
    // 16-B stores through v_permlane16_swap pairs: measured no faster on MI355X (69.2-69.8 us
    // narrow vs 70.4-74.2 us wide at B=64, same box), so opt-in
    const char* wide_env = getenv("AIKO_STEM_FAST_WIDE");    // read per call (tests flip it)
    const bool wide = wide_env && *wide_env == '1';
    dim3 grid((W1 + tw - 1) / tw, (H1 + th - 1) / th, B);
    auto go = [&](auto act_tag, auto bgr_tag) {
      constexpr int A = decltype(act_tag)::value;
      constexpr bool G = decltype(bgr_tag)::value;
      auto kern = tw == 64 ? (th == 8 ? aiko::stem_fast_kernel<A, G, false, 8, 64> : aiko::stem_fast_kernel<A, G, false, 16, 64>)
                : th == 32 ? aiko::stem_fast_kernel<A, G, false, 32>
                : th == 16 ? aiko::stem_fast_kernel<A, G, false, 16>
                           : (wide ? aiko::stem_fast_kernel<A, G, true, 8> : aiko::stem_fast_kernel<A, G, false, 8>);
      kern<<<grid, 256, 0, stream>>>(
          static_cast<const uint8_t*>(in), static_cast<aiko::bf16_t*>(out), static_cast<const aiko::bf16_t*>(w),
          bias, Hin, Win, Hc, Wc, off_t, off_l, fill, 1.f / (255.f * std[0]), H1, W1, ldo);
    };
    using F = std::false_type;
    using T = std::true_type;
    if (act == 2) bgr ? go(std::integral_constant<int, 2>{}, T{}) : go(std::integral_constant<int, 2>{}, F{});
    else if (act == 1) bgr ? go(std::integral_constant<int, 1>{}, T{}) : go(std::integral_constant<int, 1>{}, F{});
    else bgr ? go(std::integral_constant<int, 0>{}, T{}) : go(std::integral_constant<int, 0>{}, F{});
    return (int)hipGetLastError();
  }
  const int IH = (aiko::kStemTH - 1) * stride + k, IW = (aiko::kStemTW - 1) * stride + k;
  const size_t lds = (size_t)IH * IW * 8;
  if (lds > 64 * 1024) return -1;
  dim3 grid((W1 + aiko::kStemTW - 1) / aiko::kStemTW, (H1 + aiko::kStemTH - 1) / aiko::kStemTH, B);
  hipLaunchKernelGGL(aiko::stem_direct_kernel, grid, dim3(256), lds, stream, static_cast<const uint8_t*>(in),
                     static_cast<aiko::bf16_t*>(out), static_cast<const aiko::bf16_t*>(w), bias, Hin, Win, Ho, Wo,
                     Hc, Wc, off_t, off_l, fill, mean[0], mean[1], mean[2], 1.f / std[0], 1.f / std[1],
                     1.f / std[2], bgr, H1, W1, Cout, ldo, k, stride, pad, act);
  return (int)hipGetLastError();
}

extern "C" int aiko_maxpool(const void* x, void* y, int B, int H, int W, int C, int Ho, int Wo,
                            int k, int s, int p, int ldx, int ldy, hipStream_t stream) {
  const long total = (long)B * Ho * Wo * (C / 8);
  hipLaunchKernelGGL(aiko::maxpool_kernel, dim3(grid_for(total, 256)), dim3(256), 0, stream,
                     static_cast<const aiko::bf16_t*>(x), static_cast<aiko::bf16_t*>(y), B, H, W,
                     C, Ho, Wo, k, s, p, ldx, ldy);
  return (int)hipGetLastError();
}

namespace aiko {
// Mean over the rows of [B, T, C] bf16 -> [B, C] fp32 (Whisper feature pooling, long T): one
// NT-thread block per (batch, CL x 8 channels); NT/CL row phases x CL lanes of 8 channels, each
// lane keeping 4 row loads in flight (guarded, so the tail is batched too), then an LDS reduction
// of the phases in a fixed order.  CL = 32 (512 B of each row per block) when B x C/256 blocks fill
// the chip; otherwise CL = 8 (one 128 B line per row) with NT = 1024 — Whisper-small's
// [14, 1500, 768] is only 168 blocks, so the bytes in flight per block set the pace (256 threads:
// 58.9 us for 32 MB in the round-5 trace, ~0.55 TB/s).
template <int CL, int NT>
__global__ __launch_bounds__(NT) void mean_rows_f32_kernel(const bf16_t* __restrict__ x,
                                                           float* __restrict__ y, int T, int C,
                                                           long ldb) {
  constexpr int PH = NT / CL;
  __shared__ float red[PH][CL][9];
  const int cl = threadIdx.x % CL, ph = threadIdx.x / CL;
  const int C8 = C >> 3;
  const int c8 = blockIdx.x * CL + cl;
  const int b = blockIdx.y;
  float a[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (c8 < C8) {
    const bf16_t* src = x + (long)b * ldb + c8 * 8;      // ldb: batch pitch (rows may be a T-prefix)
    for (int i = ph; i < T; i += 4 * PH) {
      u32x4 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u)
        v[u] = i + PH * u < T ? *reinterpret_cast<const u32x4*>(src + (long)(i + PH * u) * C) : u32x4{0u, 0u, 0u, 0u};
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          a[2 * e] += __uint_as_float(v[u][e] << 16);
          a[2 * e + 1] += __uint_as_float(v[u][e] & 0xffff0000u);
        }
    }
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) red[ph][cl][e] = a[e];
  __syncthreads();
  if (ph == 0 && c8 < C8) {
    const float inv = 1.f / T;
    float o[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      float t = 0.f;
#pragma unroll 8
      for (int q = 0; q < PH; ++q) t += red[q][cl][e];
      o[e] = t * inv;
    }
    float* dst = y + (long)b * C + c8 * 8;
    *reinterpret_cast<f32x4*>(dst) = f32x4{o[0], o[1], o[2], o[3]};
    *reinterpret_cast<f32x4*>(dst + 4) = f32x4{o[4], o[5], o[6], o[7]};
  }
}

// Zero rows b*rows and b*rows + rows - 1 of a [B*rows, C] bf16 buffer (the per-clip zero border
// rows of the Whisper conv stem; the conv over the concatenated clips writes across them)
__global__ __launch_bounds__(256) void zero_border_rows_kernel(bf16_t* __restrict__ x, int B, int rows, int C) {
  const int C8 = C >> 3;
  const long total = (long)B * 2 * C8;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int c8 = (int)(i % C8);
    const long br = i / C8;
    const int b = (int)(br >> 1), last = (int)(br & 1);
    const long row = (long)b * rows + (last ? rows - 1 : 0);
    *reinterpret_cast<u32x4*>(x + row * C + c8 * 8) = u32x4{0u, 0u, 0u, 0u};
  }
}
}  // namespace aiko

extern "C" int aiko_mean_rows_f32(const void* x, float* y, int B, int T, int C, long ldb, hipStream_t stream) {
  if (C % 8 || T < 1 || ldb < (long)T * C) return -1;
  const aiko::bf16_t* xp = static_cast<const aiko::bf16_t*>(x);
  const int C8 = C / 8;
  if ((long)B * ((C8 + 31) / 32) < 256) {
    aiko::mean_rows_f32_kernel<8, 1024><<<dim3((C8 + 7) / 8, B), 1024, 0, stream>>>(xp, y, T, C, ldb);
  } else {
    aiko::mean_rows_f32_kernel<32, 256><<<dim3((C8 + 31) / 32, B), 256, 0, stream>>>(xp, y, T, C, ldb);
  }
  return (int)hipGetLastError();
}

extern "C" int aiko_avgpool(const void* x, void* y, int B, int HW, int C, hipStream_t stream) {
  const long total = (long)B * (C / 8);
  hipLaunchKernelGGL(aiko::avgpool_kernel, dim3(grid_for(total, 256)), dim3(256), 0, stream,
                     static_cast<const aiko::bf16_t*>(x), static_cast<aiko::bf16_t*>(y), B, HW, C);
  return (int)hipGetLastError();
}

extern "C" int aiko_softmax_topk(const void* logits, float* prob, int* index, int B, int N, int k,
                                 hipStream_t stream) {
  const int rows_per_block = 4;
  dim3 grid((B + rows_per_block - 1) / rows_per_block), block(64 * rows_per_block);
  const aiko::bf16_t* l = static_cast<const aiko::bf16_t*>(logits);
  if (N <= 64 * 4) {
    aiko::softmax_topk_kernel<4><<<grid, block, 0, stream>>>(l, prob, index, B, N, k);
  } else if (N <= 64 * 16) {
    aiko::softmax_topk_kernel<16><<<grid, block, 0, stream>>>(l, prob, index, B, N, k);
  } else if (N <= 64 * 32) {
    aiko::softmax_topk_kernel<32><<<grid, block, 0, stream>>>(l, prob, index, B, N, k);
  } else {
    return -1;
  }
  return (int)hipGetLastError();
}

extern "C" int aiko_sppf_pool(void* x, int B, int H, int W, int ld, int c, int k, hipStream_t stream) {
  if (B < 1 || B > 65535 || c % 8 || ld % 8 || 4 * c > ld || k < 1 || k % 2 == 0 || (long)H * W > 2048)
    return -1;
  const size_t lds = (size_t)2 * H * W * sizeof(aiko::u32x4);
  aiko::sppf_pool_kernel<<<dim3(c / 8, B), 256, lds, stream>>>(static_cast<aiko::bf16_t*>(x), H, W, ld, c, k);
  return (int)hipGetLastError();
}

extern "C" int aiko_zero_border_rows(void* x, int B, int rows, int C, hipStream_t stream) {
  if (C % 8 || rows < 2 || B < 1) return -1;
  const long total = (long)B * 2 * (C / 8);
  long g = (total + 255) / 256;
  if (g > 4096) g = 4096;
  aiko::zero_border_rows_kernel<<<(int)g, 256, 0, stream>>>(static_cast<aiko::bf16_t*>(x), B, rows, C);
  return (int)hipGetLastError();
}
