// Direct convolution for narrow layers: 3x3 / pad 1 (stride 1 or 2) and 1x1 (stride 1), Cc (input
// channels) and Cout in {16, 32} — YOLOv8's 160x160 stage (the stride-2 16 -> 32 conv, the C2f
// bottlenecks and the C2f 1x1 convs).
//
// The implicit-GEMM kernels spend these layers on address arithmetic: with K = 144 / 288 a tile
// runs only 3-5 K blocks, so the per-row gather setup, per-piece tap decoding and the LDS-staged
// epilogue dominate (PMC: 18-28 VALU instructions per MFMA, 9 % MFMA busy, 1.3-1.7 TB/s,
// profiles/pmc_yolov8n_r2.md).  Here, as in the fused stem (vision_ops.hip stem_direct_kernel):
//   * a workgroup owns an 8 x 32 output tile; its input halo (IH x IW pixels x Cc channels, bf16)
//     is copied into LDS once, pixel-major with the channels contiguous — all of a thread's
//     16-byte loads issued before the first LDS store — and every tap reads it from there;
//   * v_mfma_f32_16x16x32_bf16 with the WEIGHTS as the A operand (lane row = output channel, held
//     in registers for the whole tile — in LDS for Cc 32) and pixels as B (lane column = pixel): a 32-wide K chunk
//     is two taps x 16 channels (Cc 16) or one tap x 32 channels (Cc 32), so a B fragment is one
//     16-byte LDS read at a per-lane tap offset computed once;
//   * each lane ends with 4 consecutive output channels of one pixel: bias, residual (before or
//     after the activation), activation and an 8-byte store straight from the accumulators — no
//     LDS round trip.  Output and residual may be channel slices (pixel pitches ldy / ldr).
#include "conv_common.h"

namespace aiko {

namespace {

struct NarrowParams {
  const bf16_t* x;       // [B, H, W, C] (pixel pitch C, channels 0..Cc-1 used)
  const bf16_t* w;       // [Cout, K]  K = 9 * Cc rounded up to 64, k = tap * Cc + c, zero padded
  const float* bias;     // [Cout] or null
  const bf16_t* res;     // residual (pitch ldr) or null
  bf16_t* y;             // [B, Ho, Wo, >= Cout] (pitch ldy)
  int H, W, C, Ho, Wo, K, act, ldy, ldr, tiles_h, tiles_w;
};

constexpr int kNTW = 32;   // output tile cols; rows TH = 8 (4 waves x 4 blocks of 16 pixels) or 16

template <int CC, int COUT, int ST, int FR = 3, int TH = 8, bool WREG = false>
__global__ __launch_bounds__(256) void conv_narrow_kernel(NarrowParams p) {
  constexpr int kNTH = TH;
  constexpr int RPW = TH / 4;                   // output rows per wave
  constexpr int TAPS = FR * FR, PAD = FR / 2;   // 3x3 / pad 1 or 1x1 / pad 0
  constexpr int IH = (kNTH - 1) * ST + FR, IW = (kNTW - 1) * ST + FR;
  constexpr int CH = CC / 8;                    // 16-byte chunks per pixel
  constexpr int NCHUNK = IH * IW * CH;
  constexpr int PER = (NCHUNK + 255) / 256;
  constexpr int KT = TAPS * CC;                 // real K
  constexpr int NKC = (KT + 31) / 32;           // 32-wide K chunks
  constexpr int NT = COUT / 16;                 // 16-channel output tiles
  // Cc 32: the 9-chunk weight set would hold 72 VGPRs per lane for the whole tile; it is staged
  // in LDS instead and read per K chunk (16-B reads, 16 lanes share a row).  Measured on the
  // YOLOv8-n Cc-32 layers: on par with the igemm kernel (28-32 us), either may win per layer.
  // WREG keeps them in registers anyway (80 VGPRs at Cout 32): the per-MFMA A read from LDS
  // (1.5 LDS reads per MFMA with the B fragment) is what bounds the LDS-staged form
  constexpr bool WLDS = CC == 32 && !WREG;
  constexpr int WELEMS = WLDS ? COUT * NKC * 32 : 8;
  __shared__ __attribute__((aligned(16))) bf16_t tile[IH * IW * CC];
  __shared__ __attribute__((aligned(16))) bf16_t wlds[WELEMS];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int per_img = p.tiles_h * p.tiles_w;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int img = bid / per_img;
  const int t = bid - img * per_img;
  const int ty = t / p.tiles_w, tx = t - ty * p.tiles_w;
  const int oy0 = ty * kNTH, ox0 = tx * kNTW;
  const int iy0 = oy0 * ST - PAD, ix0 = ox0 * ST - PAD;
  const bf16_t* xi = p.x + (long)img * p.H * p.W * p.C;

  // ---- 1. input halo -> LDS (zeros outside the image: the conv's padding) ----
  {
    u32x4 v[PER];
#pragma unroll
    for (int u = 0; u < PER; ++u) {
      const int i = u * 256 + tid;
      v[u] = u32x4{0u, 0u, 0u, 0u};
      if (i < NCHUNK) {
        const int pix = i / CH, ch = i - pix * CH;
        const int iy = pix / IW, ix = pix - iy * IW;
        const int gy = iy0 + iy, gx = ix0 + ix;
        if ((unsigned)gy < (unsigned)p.H && (unsigned)gx < (unsigned)p.W)
          v[u] = *reinterpret_cast<const u32x4*>(xi + (gy * p.W + gx) * p.C + ch * 8);
      }
    }
#pragma unroll
    for (int u = 0; u < PER; ++u) {
      const int i = u * 256 + tid;
      if (i < NCHUNK) *reinterpret_cast<u32x4*>(tile + i * 8) = v[u];
    }
  }

  // ---- 2. weights (A operand): registers (Cc 16) or LDS (Cc 32) while the halo lands ----
  const int fr = lane & 15, fq = lane >> 4;
  bf16x8 wa[NT][WLDS ? 1 : NKC];
  if constexpr (WLDS) {
    // [n][NKC * 32] row-major copy of the used K range: (COUT * NKC * 4) 16-byte pieces
    constexpr int WP = COUT * NKC * 4;
    for (int i = tid; i < WP; i += 256) {
      const int n = i / (NKC * 4), q = i - n * (NKC * 4);
      *reinterpret_cast<u32x4*>(wlds + n * (NKC * 32) + q * 8) =
          *reinterpret_cast<const u32x4*>(p.w + (long)n * p.K + q * 8);
    }
  } else {
#pragma unroll
    for (int nt = 0; nt < NT; ++nt)
#pragma unroll
      for (int kc = 0; kc < (WLDS ? 1 : NKC); ++kc)
        wa[nt][kc] = *reinterpret_cast<const bf16x8*>(p.w + (long)(nt * 16 + fr) * p.K + kc * 32 + fq * 8);
  }
  // this lane's B-fragment offset (elements, relative to the pixel) for every K chunk; -1 = the
  // zero padding past the last tap
  int toff[NKC];
#pragma unroll
  for (int kc = 0; kc < NKC; ++kc) {
    const int k0 = kc * 32 + fq * 8;
    const int tap = k0 / CC, c0 = k0 - tap * CC;
    toff[kc] = tap < TAPS ? ((tap / FR) * IW + (tap % FR)) * CC + c0 : -1;
  }
  float cb[NT][4];
#pragma unroll
  for (int nt = 0; nt < NT; ++nt)
#pragma unroll
    for (int e = 0; e < 4; ++e) cb[nt][e] = p.bias ? p.bias[nt * 16 + fq * 4 + e] : 0.f;
  __syncthreads();

  // ---- 3. MFMA per 16-pixel block + fused epilogue ----
  const bool post = (p.act & 16) != 0;
  const int act = p.act & 15;
#pragma unroll
  for (int pt = 0; pt < 2 * RPW; ++pt) {
    const int ly = RPW * wave + (pt >> 1), lx = 16 * (pt & 1) + fr;
    const int base = ((ly * ST) * IW + lx * ST) * CC;
    f32x4 acc[NT];
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) acc[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kc = 0; kc < NKC; ++kc) {
      bf16x8 b;
      if (toff[kc] >= 0) {
        b = *reinterpret_cast<const bf16x8*>(tile + base + toff[kc]);
      } else {
        b = __builtin_bit_cast(bf16x8, u32x4{0u, 0u, 0u, 0u});
      }
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) {
        bf16x8 a;
        if constexpr (WLDS) {
          a = *reinterpret_cast<const bf16x8*>(wlds + (nt * 16 + fr) * (NKC * 32) + kc * 32 + fq * 8);
        } else {
          a = wa[nt][kc];
        }
        acc[nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc[nt], 0, 0, 0);
      }
    }
    const int oy = oy0 + ly, ox = ox0 + lx;
    if (oy >= p.Ho || ox >= p.Wo) continue;
    const long m = ((long)img * p.Ho + oy) * p.Wo + ox;
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
      const int n = nt * 16 + fq * 4;
      float r[4] = {0.f, 0.f, 0.f, 0.f};
      if (p.res) {
        const uint2 rv = *reinterpret_cast<const uint2*>(p.res + m * p.ldr + n);
        r[0] = __uint_as_float(rv.x << 16);
        r[1] = __uint_as_float(rv.x & 0xffff0000u);
        r[2] = __uint_as_float(rv.y << 16);
        r[3] = __uint_as_float(rv.y & 0xffff0000u);
      }
      float v[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float a = acc[nt][e] + cb[nt][e];
        if (!post) a += r[e];
        if (act == 1) a = fmaxf(a, 0.f);
        else if (act == 2) a = silu(a);
        else if (act == 3) a = gelu_erf(a);
        if (post) a += r[e];
        v[e] = a;
      }
      *reinterpret_cast<uint2*>(p.y + m * p.ldy + n) = make_uint2(pack2(v[0], v[1]), pack2(v[2], v[3]));
    }
  }
}

}  // namespace

}  // namespace aiko

// Same arguments as aiko_conv_igemm (bm / bn / second source unused).  Supported: R = S = 3 with
// pad 1 or R = S = 1 with pad 0, stride 1 / 2, Cc and Cout in {16, 32}, K = R S Cc rounded up to
// 64; returns -1 otherwise.
extern "C" int aiko_conv_narrow(const void* x, const void* w, const float* bias, const void* res,
                                void* y, int H, int W, int C, int Cc, int R, int S, int stride,
                                int pad, int Ho, int Wo, int M, int Cout, int K, int act, int ldy,
                                int ldr, int th, int wreg, hipStream_t stream) {
  using namespace aiko;
  const bool k3 = R == 3 && S == 3 && pad == 1, k1 = R == 1 && S == 1 && pad == 0;
  if (th != 8 && th != 16) return -1;
  if ((!k3 && !k1) || (stride != 1 && stride != 2) || (Cc != 16 && Cc != 32) ||
      (Cout != 16 && Cout != 32) || K < R * S * Cc || K % 64 || C % 8 || ldy % 4 || ldr % 4 ||
      Ho <= 0 || Wo <= 0 || M % (Ho * Wo))
    return -1;
  NarrowParams p;
  p.x = static_cast<const bf16_t*>(x);
  p.w = static_cast<const bf16_t*>(w);
  p.bias = bias;
  p.res = static_cast<const bf16_t*>(res);
  p.y = static_cast<bf16_t*>(y);
  p.H = H; p.W = W; p.C = C; p.Ho = Ho; p.Wo = Wo; p.K = K; p.act = act; p.ldy = ldy; p.ldr = ldr;
  p.tiles_h = (Ho + th - 1) / th;
  p.tiles_w = (Wo + kNTW - 1) / kNTW;
  const long grid = (long)(M / (Ho * Wo)) * p.tiles_h * p.tiles_w;
  if (grid <= 0 || grid > 0x7fffffffL) return -1;
  const dim3 g((unsigned)grid), b(256);
#define AIKO_NARROW(FR, CC, CO, ST)                                                                      \
  if (R == FR && Cc == CC && Cout == CO && stride == ST) {                                                \
    if (wreg && CC == 32) {                                                                               \
      if (th == 16) conv_narrow_kernel<CC, CO, ST, FR, 16, true><<<g, b, 0, stream>>>(p);                 \
      else conv_narrow_kernel<CC, CO, ST, FR, 8, true><<<g, b, 0, stream>>>(p);                           \
    } else if (th == 16) conv_narrow_kernel<CC, CO, ST, FR, 16><<<g, b, 0, stream>>>(p);                  \
    else conv_narrow_kernel<CC, CO, ST, FR, 8><<<g, b, 0, stream>>>(p);                                   \
    return (int)hipGetLastError();                                                                      \
  }
  AIKO_NARROW(3, 16, 16, 1) AIKO_NARROW(3, 16, 32, 1) AIKO_NARROW(3, 32, 16, 1) AIKO_NARROW(3, 32, 32, 1)
  AIKO_NARROW(3, 16, 16, 2) AIKO_NARROW(3, 16, 32, 2) AIKO_NARROW(3, 32, 16, 2) AIKO_NARROW(3, 32, 32, 2)
  AIKO_NARROW(1, 16, 16, 1) AIKO_NARROW(1, 16, 32, 1) AIKO_NARROW(1, 32, 16, 1) AIKO_NARROW(1, 32, 32, 1)
#undef AIKO_NARROW
  return -1;
}
