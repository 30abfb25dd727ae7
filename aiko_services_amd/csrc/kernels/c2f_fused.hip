// Fused YOLOv8 C2f block (one bottleneck, n = 1) as a row stream, for the wide, narrow-channel
// layers where the unfused chain is bound by HBM round trips (YOLOv8-n l2 at 160 x 160: cv1 1x1
// 32 -> 32, bottleneck 3x3 16 -> 16 twice + shortcut, cv2 1x1 48 -> 32 — four launches moving
// ~730 MB at B = 64, against 210 MB for x in and y out):
//
//   [a | s] = silu(cv1(x));  t = silu(conv_a(s));  c = silu(conv_b(t)) (+ s);  y = silu(cv2([a, s, c]))
//
// (Ultralytics C2f / Bottleneck, /root/reference/src/aiko_services/examples/yolo/yolo.py runs the
// packaged model).  One workgroup streams a band of RB output rows of one image,
// full width W, through LDS row rings; one step per row, ONE barrier per step, every phase of a
// step reading only rows finished in earlier steps:
//
//   step v:  cv1(x row v+2) -> A / S rings          (x fragments loaded from HBM a step ahead)
//            conv_a(S rows v-1..v+1) -> T row v
//            conv_b(T rows v-3..v-1) + S row v-2 -> c (registers)
//            cv2(A, S rows v-2 | c) -> y row v-2    (c enters as a 16x16x16 MFMA operand straight
//                                                     from the conv_b accumulators: same layout)
//   rings: A, S 5 rows (S with a zero pixel each side), T 4 rows; rows outside the image are zero.
//
// Every product is transposed (weights on the MFMA A side, 16 output channels x 32 K, resident
// in registers for the whole launch): each lane's accumulator holds 4 consecutive channels of
// one pixel, so results go to the LDS row images (and y to HBM) as 8-byte pieces with bias and
// SiLU applied in registers.  The 3x3 convs take their K = 9 taps x 16 channels in chunks of two
// taps (lane groups 0-1: tap 2k, 2-3: tap 2k+1; the tenth tap has zero weights and re-reads tap
// 8, so the products stay finite).  Wave w owns pixel tiles PT w .. of 16 pixels.
#include <hip/hip_runtime.h>

#include "common.h"

namespace aiko {

namespace c2f {
typedef __attribute__((ext_vector_type(4))) short v4s;
typedef __attribute__((ext_vector_type(2))) unsigned u32x2;

__device__ __forceinline__ f32x4 silu4(f32x4 v) {
  return f32x4{silu(v[0]), silu(v[1]), silu(v[2]), silu(v[3])};
}
__device__ __forceinline__ u32x2 pack4(f32x4 v) { return u32x2{pack2(v[0], v[1]), pack2(v[2], v[3])}; }
__device__ __forceinline__ f32x4 unpack4(u32x2 u) {
  return f32x4{__uint_as_float(u[0] << 16), __uint_as_float(u[0] & 0xffff0000u), __uint_as_float(u[1] << 16),
               __uint_as_float(u[1] & 0xffff0000u)};
}
}  // namespace c2f

struct C2fParams {
  const bf16_t* x;       // [B][H][W][ldx] (CI channels used)
  const bf16_t* w1;      // cv1 [2C][k1]        (1x1, K = CI)
  const float* b1;
  const bf16_t* wa;      // bottleneck conv a [C][ka] (3x3, K = 9 C in (r, s, c) order, zero-padded)
  const float* ba;
  const bf16_t* wb;      // bottleneck conv b
  const float* bb;
  const bf16_t* w2;      // cv2 [CO][k2]         (1x1, K = 3C: a | s | c)
  const float* b2;
  bf16_t* y;             // [B][H][W][ldy] (CO channels written)
  int B, H, ldx, ldy, k1, ka, kb, k2, rb;
  // optional (c2f_fused_wl_kernel): input channels [0, cu) come from xu [B][H/2][W/2][ldxu] at
  // (h / 2, w / 2) — the PAN neck's nearest 2x upsample read in place, never materialised
  const bf16_t* xu;
  int ldxu, cu;
};

// W: row width (pixels), CI / C / CO: channels (C = 16: two taps per 32-wide K chunk), SC: the
// bottleneck's shortcut.  Block = W / 32 waves (two 16-pixel tiles each).
template <int W, int CI, int C, int CO, bool SC>
__global__ __launch_bounds__(W * 2, 1) void c2f_fused_kernel(C2fParams p) {
  using namespace c2f;
  static_assert(C == 16 && CI % 32 == 0 && CO % 16 == 0 && W % 32 == 0, "instantiated shapes");
  constexpr int NWAVE = W / 32, PT = 2;               // waves, pixel tiles per wave
  constexpr int KS1 = CI / 32;                         // cv1 K steps
  constexpr int N1 = 2 * C / 16;                       // cv1 output-channel tiles (a: < C / 16)
  constexpr int KC3 = (9 * C + 31) / 32;               // 3x3 K chunks (5)
  constexpr int N2 = CO / 16;
  constexpr int SW = W + 2;                            // S / T row images: one zero pixel each side
  constexpr int SROW = SW * C * 2, TROW = SW * C * 2, AROW = W * C * 2;   // bytes
  constexpr int NS = 5, NA = 5, NT = 4;
  __shared__ __attribute__((aligned(16))) unsigned char smem[NS * SROW + NA * AROW + NT * TROW];
  unsigned char* const sring = smem;
  unsigned char* const aring = sring + NS * SROW;
  unsigned char* const tring = aring + NA * AROW;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int fr = lane & 15, fq = lane >> 4;
  const int nb = p.H / p.rb;
  const int img = blockIdx.x / nb, r0 = (blockIdx.x % nb) * p.rb, r1 = r0 + p.rb;
  const int px0 = wave * 32;                           // this wave's first pixel

  // ---- weights (A operands) and biases, resident ----
  bf16x8 w1f[N1][KS1], waf[KC3], wbf[KC3], w2f[N2];
  v4s w2c[N2];
#pragma unroll
  for (int n = 0; n < N1; ++n)
#pragma unroll
    for (int k = 0; k < KS1; ++k)
      w1f[n][k] = *reinterpret_cast<const bf16x8*>(p.w1 + (long)(16 * n + fr) * p.k1 + 32 * k + 8 * fq);
#pragma unroll
  for (int k = 0; k < KC3; ++k) {
    waf[k] = *reinterpret_cast<const bf16x8*>(p.wa + (long)fr * p.ka + 32 * k + 8 * fq);
    wbf[k] = *reinterpret_cast<const bf16x8*>(p.wb + (long)fr * p.kb + 32 * k + 8 * fq);
  }
#pragma unroll
  for (int n = 0; n < N2; ++n) {
    w2f[n] = *reinterpret_cast<const bf16x8*>(p.w2 + (long)(16 * n + fr) * p.k2 + 8 * fq);
    w2c[n] = *reinterpret_cast<const v4s*>(p.w2 + (long)(16 * n + fr) * p.k2 + 2 * C + 4 * fq);
  }
  f32x4 b1v[N1], bav, bbv, b2v[N2];
#pragma unroll
  for (int n = 0; n < N1; ++n) b1v[n] = *reinterpret_cast<const f32x4*>(p.b1 + 16 * n + 4 * fq);
  bav = *reinterpret_cast<const f32x4*>(p.ba + 4 * fq);
  bbv = *reinterpret_cast<const f32x4*>(p.bb + 4 * fq);
#pragma unroll
  for (int n = 0; n < N2; ++n) b2v[n] = *reinterpret_cast<const f32x4*>(p.b2 + 16 * n + 4 * fq);

  // zero the S / T border pixels of every ring slot (never written by the row phases)
  for (int i = tid; i < (NS + NT) * 2 * (C / 8); i += NWAVE * 64) {
    const int slot = i / (2 * (C / 8)), rem = i % (2 * (C / 8));
    const int side = rem / (C / 8), piece = rem % (C / 8);
    unsigned char* base = slot < NS ? sring + slot * SROW : tring + (slot - NS) * TROW;
    *reinterpret_cast<u32x4*>(base + (side ? (W + 1) : 0) * C * 2 + piece * 16) = u32x4{0u, 0u, 0u, 0u};
  }

  // 3x3 B-fragment geometry of this lane for chunk k: tap q = 2k + (fq >> 1) (tap 9 -> tap 8 with
  // zero weights), channels 8 (fq & 1) .. +7; byte offset inside a row image (border included)
  // and the tap's row (0..2 = dy + 1)
  int toff[KC3], trow[KC3];
#pragma unroll
  for (int k = 0; k < KC3; ++k) {
    int q = 2 * k + (fq >> 1);
    if (q > 8) q = 8;
    const int dy = q / 3, dx = q % 3 - 1;
    trow[k] = dy;
    toff[k] = ((fr + 1 + dx) * C + 8 * (fq & 1)) * 2;
  }

  // ---- x fragments of one row (B operand of cv1): pixel px0 + 16 t + fr, channels 32 k + 8 fq
  bf16x8 xf[PT][KS1];
  auto load_x = [&](int row) __attribute__((always_inline)) {
    const bool ok = row >= 0 && row < p.H;
    const bf16_t* src = p.x + (((long)img * p.H + (ok ? row : 0)) * W + px0 + fr) * p.ldx + 8 * fq;
#pragma unroll
    for (int t = 0; t < PT; ++t)
#pragma unroll
      for (int k = 0; k < KS1; ++k)
        xf[t][k] = *reinterpret_cast<const bf16x8*>(src + (long)16 * t * p.ldx + 32 * k);
  };

  // cv1 of row `row` (x fragments in xf) -> A / S ring slots of that row (zeros outside the image)
  auto cv1 = [&](int row) __attribute__((always_inline)) {
    const bool ok = row >= 0 && row < p.H;
    const int slot = (row + 2 * NS) % NS;
#pragma unroll
    for (int t = 0; t < PT; ++t) {
      const int px = px0 + 16 * t + fr;
#pragma unroll
      for (int n = 0; n < N1; ++n) {
        f32x4 acc = b1v[n];
#pragma unroll
        for (int k = 0; k < KS1; ++k) acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w1f[n][k], xf[t][k], acc, 0, 0, 0);
        const u32x2 v = ok ? pack4(silu4(acc)) : u32x2{0u, 0u};
        if (n < C / 16)        // a: channels 16 n + 4 fq
          *reinterpret_cast<u32x2*>(aring + slot * AROW + (px * C + 16 * n + 4 * fq) * 2) = v;
        else                   // s
          *reinterpret_cast<u32x2*>(sring + slot * SROW + ((px + 1) * C + 16 * (n - C / 16) + 4 * fq) * 2) = v;
      }
    }
  };

  // 3x3 conv of the row centred on `row` from ring `ring` (slot stride `rstride`, NSL slots):
  // returns the accumulators of pixel tile t (bias added, before the activation)
  auto conv3 = [&](const unsigned char* ring, int nsl, int rstride, int row, const bf16x8 (&wf)[KC3], f32x4 bias,
                   int t) __attribute__((always_inline)) {
    const unsigned char* rows[3];
#pragma unroll
    for (int d = 0; d < 3; ++d) rows[d] = ring + ((row - 1 + d + 4 * nsl) % nsl) * rstride + (px0 + 16 * t) * C * 2;
    f32x4 acc = bias;
#pragma unroll
    for (int k = 0; k < KC3; ++k) {
      const unsigned char* base = trow[k] == 0 ? rows[0] : (trow[k] == 1 ? rows[1] : rows[2]);
      const bf16x8 b = *reinterpret_cast<const bf16x8*>(base + toff[k]);
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[k], b, acc, 0, 0, 0);
    }
    return acc;
  };

  // ---- prologue: cv1 of rows r0-2 .. r0, x fragments of row r0+1 in flight
  load_x(r0 - 2);
  cv1(r0 - 2);
  load_x(r0 - 1);
  cv1(r0 - 1);
  load_x(r0);
  cv1(r0);
  load_x(r0 + 1);

  for (int v = r0 - 1; v <= r1 + 1; ++v) {
    // rows of earlier steps complete (LDS only: the x loads and y stores stay in flight)
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    // cv1(v + 2): its x fragments were loaded last step; then the next row's go out
    if (v + 2 <= r1 + 1) {
      cv1(v + 2);
      if (v + 3 <= r1 + 1) load_x(v + 3);
    }
    // conv_a(v) -> T row v
    if (v <= r1) {
      const bool ok = v >= 0 && v < p.H;
      const int slot = (v + 2 * NT) % NT;
#pragma unroll
      for (int t = 0; t < PT; ++t) {
        const f32x4 acc = conv3(sring, NS, SROW, v, waf, bav, t);
        const u32x2 o = ok ? pack4(silu4(acc)) : u32x2{0u, 0u};
        *reinterpret_cast<u32x2*>(tring + slot * TROW + ((px0 + 16 * t + fr + 1) * C + 4 * fq) * 2) = o;
      }
    }
    // conv_b(v - 2) (+ shortcut) and cv2 -> y row v - 2
    const int w = v - 2;
    if (w >= r0 && w < r1) {
      const int aslot = (w + 2 * NA) % NA, sslot = (w + 2 * NS) % NS;
#pragma unroll
      for (int t = 0; t < PT; ++t) {
        const int px = px0 + 16 * t + fr;
        f32x4 c = silu4(conv3(tring, NT, TROW, w, wbf, bbv, t));
        if constexpr (SC) {
          const u32x2 s = *reinterpret_cast<const u32x2*>(sring + sslot * SROW + ((px + 1) * C + 4 * fq) * 2);
          const f32x4 sv = unpack4(s);
          c = f32x4{c[0] + sv[0], c[1] + sv[1], c[2] + sv[2], c[3] + sv[3]};
        }
        const u32x2 cb = pack4(c);
        const v4s cop = __builtin_bit_cast(v4s, cb);
        // [a | s] chunk: lane groups 0-1 read a, 2-3 read s (channels 8 (fq & 1) .. +7)
        const bf16x8 as = fq < 2 ? *reinterpret_cast<const bf16x8*>(aring + aslot * AROW + (px * C + 8 * fq) * 2)
                                 : *reinterpret_cast<const bf16x8*>(sring + sslot * SROW + ((px + 1) * C + 8 * (fq - 2)) * 2);
        bf16_t* yrow = p.y + (((long)img * p.H + w) * W + px) * p.ldy;
#pragma unroll
        for (int n = 0; n < N2; ++n) {
          // two independent products summed on the VALU: chaining the 16x16x16 MFMA's SrcC on
          // the 16x16x32 one's result read its first two accumulator VGPRs stale on gfx950
          // (measured: output channels 4k, 4k+1 wrong, 4k+2, 4k+3 right)
          const f32x4 acc1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w2f[n], as, b2v[n], 0, 0, 0);
          const f32x4 acc2 = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(w2c[n], cop, f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
          const f32x4 acc = {acc1[0] + acc2[0], acc1[1] + acc2[1], acc1[2] + acc2[2], acc1[3] + acc2[3]};
          *reinterpret_cast<u32x2*>(yrow + 16 * n + 4 * fq) = pack4(silu4(acc));
        }
      }
    }
  }
}

// The same row stream for wider channel counts (YOLOv8-n l15 at 80 x 80: cv1 1x1 192 -> 64,
// bottleneck 3x3 32 -> 32 twice, no shortcut, cv2 1x1 96 -> 64): the weights (~77 KB) live in
// LDS (rows padded by 16 bytes: the 16 rows of a fragment read start on different banks), each
// 3x3 K chunk is one tap (32 channels), one 16-pixel tile per wave (W / 16 waves), and cv2 takes
// the C / 16 tiles of c through independent 16x16x16 products summed on the VALU.
template <int W, int CI, int C, int CO, bool SC>
__global__ __launch_bounds__(W * 4, 1) void c2f_fused_wl_kernel(C2fParams p) {
  using namespace c2f;
  static_assert(C == 32 && CI % 32 == 0 && CO % 16 == 0 && W % 16 == 0, "instantiated shapes");
  constexpr int NWAVE = W / 16;
  constexpr int KS1 = CI / 32, N1 = 2 * C / 16, KC3 = 9, N3 = C / 16, N2 = CO / 16, KS2 = 2 * C / 32;
  constexpr int P1 = CI * 2 + 16, P3 = 9 * C * 2 + 16, P2 = 3 * C * 2 + 16;   // weight row pitches (bytes)
  constexpr int W1B = 2 * C * P1, W3B = C * P3, W2B = CO * P2;
  constexpr int SW = W + 2;
  constexpr int SROW = SW * C * 2, TROW = SW * C * 2, AROW = W * C * 2;
  constexpr int NS = 5, NA = 5, NT = 4;
  __shared__ __attribute__((aligned(16))) unsigned char smem[W1B + 2 * W3B + W2B + NS * SROW + NA * AROW + NT * TROW];
  unsigned char* const lw1 = smem;
  unsigned char* const lwa = lw1 + W1B;
  unsigned char* const lwb = lwa + W3B;
  unsigned char* const lw2 = lwb + W3B;
  unsigned char* const sring = lw2 + W2B;
  unsigned char* const aring = sring + NS * SROW;
  unsigned char* const tring = aring + NA * AROW;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int fr = lane & 15, fq = lane >> 4;
  const int nb = p.H / p.rb;
  const int img = blockIdx.x / nb, r0 = (blockIdx.x % nb) * p.rb, r1 = r0 + p.rb;
  const int px0 = wave * 16;

  // ---- weights -> LDS (16-B pieces), biases -> registers
  auto stage = [&](unsigned char* dst, const bf16_t* src, int rows, int kused, int kpitch, int dpitch) {
    const int per = kused / 8;
    for (int i = tid; i < rows * per; i += NWAVE * 64) {
      const int r = i / per, c = i - r * per;
      *reinterpret_cast<u32x4*>(dst + r * dpitch + c * 16) =
          *reinterpret_cast<const u32x4*>(src + (long)r * kpitch + c * 8);
    }
  };
  stage(lw1, p.w1, 2 * C, CI, p.k1, P1);
  stage(lwa, p.wa, C, 9 * C, p.ka, P3);
  stage(lwb, p.wb, C, 9 * C, p.kb, P3);
  stage(lw2, p.w2, CO, 3 * C, p.k2, P2);
  f32x4 b1v[N1], bav[N3], bbv[N3], b2v[N2];
#pragma unroll
  for (int n = 0; n < N1; ++n) b1v[n] = *reinterpret_cast<const f32x4*>(p.b1 + 16 * n + 4 * fq);
#pragma unroll
  for (int n = 0; n < N3; ++n) {
    bav[n] = *reinterpret_cast<const f32x4*>(p.ba + 16 * n + 4 * fq);
    bbv[n] = *reinterpret_cast<const f32x4*>(p.bb + 16 * n + 4 * fq);
  }
#pragma unroll
  for (int n = 0; n < N2; ++n) b2v[n] = *reinterpret_cast<const f32x4*>(p.b2 + 16 * n + 4 * fq);
  for (int i = tid; i < (NS + NT) * 2 * (C / 8); i += NWAVE * 64) {
    const int slot = i / (2 * (C / 8)), rem = i % (2 * (C / 8));
    const int side = rem / (C / 8), piece = rem % (C / 8);
    unsigned char* base = slot < NS ? sring + slot * SROW : tring + (slot - NS) * TROW;
    *reinterpret_cast<u32x4*>(base + (side ? (W + 1) : 0) * C * 2 + piece * 16) = u32x4{0u, 0u, 0u, 0u};
  }
  auto wfrag = [&](const unsigned char* lw, int pitch, int n, int koff) __attribute__((always_inline)) {
    return *reinterpret_cast<const bf16x8*>(lw + (16 * n + fr) * pitch + (koff + 8 * fq) * 2);
  };

  bf16x8 xf[KS1];
  auto load_x = [&](int row) __attribute__((always_inline)) {
    const bool ok = row >= 0 && row < p.H;
    const int r = ok ? row : 0;
    const bf16_t* src = p.x + (((long)img * p.H + r) * W + px0 + fr) * p.ldx + 8 * fq;
    const bf16_t* srcu = p.xu ? p.xu + (((long)img * (p.H / 2) + (r >> 1)) * (W / 2) + ((px0 + fr) >> 1)) * p.ldxu + 8 * fq
                              : src;
#pragma unroll
    for (int k = 0; k < KS1; ++k)
      xf[k] = *reinterpret_cast<const bf16x8*>((32 * k < p.cu ? srcu : src) + 32 * k);
  };
  auto cv1 = [&](int row) __attribute__((always_inline)) {
    const bool ok = row >= 0 && row < p.H;
    const int slot = (row + 2 * NS) % NS;
    const int px = px0 + fr;
#pragma unroll
    for (int n = 0; n < N1; ++n) {
      f32x4 acc = b1v[n];
#pragma unroll
      for (int k = 0; k < KS1; ++k) acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wfrag(lw1, P1, n, 32 * k), xf[k], acc, 0, 0, 0);
      const u32x2 v = ok ? pack4(silu4(acc)) : u32x2{0u, 0u};
      if (n < C / 16)
        *reinterpret_cast<u32x2*>(aring + slot * AROW + (px * C + 16 * n + 4 * fq) * 2) = v;
      else
        *reinterpret_cast<u32x2*>(sring + slot * SROW + ((px + 1) * C + 16 * (n - C / 16) + 4 * fq) * 2) = v;
    }
  };
  // 3x3: chunk k = tap k (dy = k / 3, dx = k % 3 - 1), channels 8 fq .. +7 of that tap's pixel
  auto conv3 = [&](const unsigned char* ring, int nsl, int rstride, int row, const unsigned char* lw,
                   const f32x4 (&bias)[N3], f32x4 (&acc)[N3]) __attribute__((always_inline)) {
    const unsigned char* rows[3];
#pragma unroll
    for (int d = 0; d < 3; ++d) rows[d] = ring + ((row - 1 + d + 4 * nsl) % nsl) * rstride + (px0 + fr + 1) * C * 2 + 16 * fq;
#pragma unroll
    for (int n = 0; n < N3; ++n) acc[n] = bias[n];
#pragma unroll
    for (int k = 0; k < KC3; ++k) {
      const bf16x8 b = *reinterpret_cast<const bf16x8*>(rows[k / 3] + (k % 3 - 1) * C * 2);
#pragma unroll
      for (int n = 0; n < N3; ++n) acc[n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wfrag(lw, P3, n, 32 * k), b, acc[n], 0, 0, 0);
    }
  };

  load_x(r0 - 2);
  cv1(r0 - 2);
  load_x(r0 - 1);
  cv1(r0 - 1);
  load_x(r0);
  cv1(r0);
  load_x(r0 + 1);

  for (int v = r0 - 1; v <= r1 + 1; ++v) {
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    if (v + 2 <= r1 + 1) {
      cv1(v + 2);
      if (v + 3 <= r1 + 1) load_x(v + 3);
    }
    if (v <= r1) {
      const bool ok = v >= 0 && v < p.H;
      const int slot = (v + 2 * NT) % NT;
      f32x4 acc[N3];
      conv3(sring, NS, SROW, v, lwa, bav, acc);
#pragma unroll
      for (int n = 0; n < N3; ++n) {
        const u32x2 o = ok ? pack4(silu4(acc[n])) : u32x2{0u, 0u};
        *reinterpret_cast<u32x2*>(tring + slot * TROW + ((px0 + fr + 1) * C + 16 * n + 4 * fq) * 2) = o;
      }
    }
    const int w = v - 2;
    if (w >= r0 && w < r1) {
      const int aslot = (w + 2 * NA) % NA, sslot = (w + 2 * NS) % NS;
      const int px = px0 + fr;
      f32x4 c[N3];
      conv3(tring, NT, TROW, w, lwb, bbv, c);
      v4s cop[N3];
#pragma unroll
      for (int n = 0; n < N3; ++n) {
        c[n] = silu4(c[n]);
        if constexpr (SC) {
          const f32x4 sv = unpack4(*reinterpret_cast<const u32x2*>(sring + sslot * SROW + ((px + 1) * C + 16 * n + 4 * fq) * 2));
          c[n] = f32x4{c[n][0] + sv[0], c[n][1] + sv[1], c[n][2] + sv[2], c[n][3] + sv[3]};
        }
        cop[n] = __builtin_bit_cast(v4s, pack4(c[n]));
      }
      // [a | s] chunks: channel g = 32 k + 8 fq of the concatenation (a below C, s from C)
      bf16x8 asf[KS2];
#pragma unroll
      for (int k = 0; k < KS2; ++k) {
        const int g = 32 * k + 8 * fq;
        asf[k] = g < C ? *reinterpret_cast<const bf16x8*>(aring + aslot * AROW + (px * C + g) * 2)
                       : *reinterpret_cast<const bf16x8*>(sring + sslot * SROW + ((px + 1) * C + g - C) * 2);
      }
      bf16_t* yrow = p.y + (((long)img * p.H + w) * W + px) * p.ldy;
#pragma unroll
      for (int n = 0; n < N2; ++n) {
        f32x4 acc = b2v[n];
#pragma unroll
        for (int k = 0; k < KS2; ++k) acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wfrag(lw2, P2, n, 32 * k), asf[k], acc, 0, 0, 0);
#pragma unroll
        for (int j = 0; j < N3; ++j) {      // independent products (see c2f_fused_kernel)
          const v4s wc = *reinterpret_cast<const v4s*>(lw2 + (16 * n + fr) * P2 + (2 * C + 16 * j + 4 * fq) * 2);
          const f32x4 pj = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(wc, cop[j], f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
          acc = f32x4{acc[0] + pj[0], acc[1] + pj[1], acc[2] + pj[2], acc[3] + pj[3]};
        }
        *reinterpret_cast<u32x2*>(yrow + 16 * n + 4 * fq) = pack4(silu4(acc));
      }
    }
  }
}

// One C2f bottleneck alone (3x3 C -> C, SiLU, 3x3 C -> C, SiLU, + shortcut) as the same row
// stream, for blocks with n = 2 whose whole C2f does not fit in LDS (YOLOv8-n l4 at 80 x 80:
// s and c are channel slices of the C2f's concat buffer): s rows are copied into the S ring a
// step ahead (one 16-B piece per thread, loaded the step before), conv_a fills the T ring, and
// conv_b + shortcut goes straight to HBM — the intermediate t never leaves LDS.
template <int W, int C, bool SC>
__global__ __launch_bounds__(W * 4, 1) void c2f_bneck_kernel(C2fParams p) {
  using namespace c2f;
  static_assert(C == 32 && W % 16 == 0 && (W * C * 2 / 16) % (W * 4) == 0, "instantiated shapes");
  constexpr int NWAVE = W / 16, NTH = W * 4;
  constexpr int KC3 = 9, N3 = C / 16;
  constexpr int P3 = 9 * C * 2 + 16, W3B = C * P3;
  constexpr int SW = W + 2, SROW = SW * C * 2, TROW = SW * C * 2;
  constexpr int NS = 5, NT = 4;
  constexpr int PPR = W * C * 2 / 16, PPT = PPR / NTH;   // 16-B pieces per row / per thread
  __shared__ __attribute__((aligned(16))) unsigned char smem[2 * W3B + NS * SROW + NT * TROW];
  unsigned char* const lwa = smem;
  unsigned char* const lwb = lwa + W3B;
  unsigned char* const sring = lwb + W3B;
  unsigned char* const tring = sring + NS * SROW;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int fr = lane & 15, fq = lane >> 4;
  const int nb = p.H / p.rb;
  const int img = blockIdx.x / nb, r0 = (blockIdx.x % nb) * p.rb, r1 = r0 + p.rb;
  const int px0 = wave * 16;

  for (int i = tid; i < C * (9 * C / 8); i += NTH) {
    const int r = i / (9 * C / 8), c = i - r * (9 * C / 8);
    *reinterpret_cast<u32x4*>(lwa + r * P3 + c * 16) = *reinterpret_cast<const u32x4*>(p.wa + (long)r * p.ka + c * 8);
    *reinterpret_cast<u32x4*>(lwb + r * P3 + c * 16) = *reinterpret_cast<const u32x4*>(p.wb + (long)r * p.kb + c * 8);
  }
  f32x4 bav[N3], bbv[N3];
#pragma unroll
  for (int n = 0; n < N3; ++n) {
    bav[n] = *reinterpret_cast<const f32x4*>(p.ba + 16 * n + 4 * fq);
    bbv[n] = *reinterpret_cast<const f32x4*>(p.bb + 16 * n + 4 * fq);
  }
  for (int i = tid; i < (NS + NT) * 2 * (C / 8); i += NTH) {
    const int slot = i / (2 * (C / 8)), rem = i % (2 * (C / 8));
    const int side = rem / (C / 8), piece = rem % (C / 8);
    unsigned char* base = slot < NS ? sring + slot * SROW : tring + (slot - NS) * TROW;
    *reinterpret_cast<u32x4*>(base + (side ? (W + 1) : 0) * C * 2 + piece * 16) = u32x4{0u, 0u, 0u, 0u};
  }

  // s row pieces of this thread: piece j = tid + NTH i -> pixel j / (C / 8), chunk j % (C / 8)
  u32x4 sreg[PPT];
  auto load_s = [&](int row) __attribute__((always_inline)) {
    const bool ok = row >= 0 && row < p.H;
#pragma unroll
    for (int i = 0; i < PPT; ++i) {
      const int j = tid + NTH * i, px = j / (C / 8), ch = j % (C / 8);
      sreg[i] = ok ? *reinterpret_cast<const u32x4*>(p.x + (((long)img * p.H + row) * W + px) * p.ldx + 8 * ch)
                   : u32x4{0u, 0u, 0u, 0u};
    }
  };
  auto put_s = [&](int row) __attribute__((always_inline)) {
    const int slot = (row + 2 * NS) % NS;
#pragma unroll
    for (int i = 0; i < PPT; ++i) {
      const int j = tid + NTH * i, px = j / (C / 8), ch = j % (C / 8);
      *reinterpret_cast<u32x4*>(sring + slot * SROW + ((px + 1) * C + 8 * ch) * 2) = sreg[i];
    }
  };
  auto conv3 = [&](const unsigned char* ring, int nsl, int rstride, int row, const unsigned char* lw,
                   const f32x4 (&bias)[N3], f32x4 (&acc)[N3]) __attribute__((always_inline)) {
    const unsigned char* rows[3];
#pragma unroll
    for (int d = 0; d < 3; ++d) rows[d] = ring + ((row - 1 + d + 4 * nsl) % nsl) * rstride + (px0 + fr + 1) * C * 2 + 16 * fq;
#pragma unroll
    for (int n = 0; n < N3; ++n) acc[n] = bias[n];
#pragma unroll
    for (int k = 0; k < KC3; ++k) {
      const bf16x8 b = *reinterpret_cast<const bf16x8*>(rows[k / 3] + (k % 3 - 1) * C * 2);
#pragma unroll
      for (int n = 0; n < N3; ++n) {
        const bf16x8 wf = *reinterpret_cast<const bf16x8*>(lw + (16 * n + fr) * P3 + (32 * k + 8 * fq) * 2);
        acc[n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf, b, acc[n], 0, 0, 0);
      }
    }
  };

  // prologue: s rows r0-2 .. r0 in the ring, row r0+1 in registers
  load_s(r0 - 2);
  put_s(r0 - 2);
  load_s(r0 - 1);
  put_s(r0 - 1);
  load_s(r0);
  put_s(r0);
  load_s(r0 + 1);

  for (int v = r0 - 1; v <= r1 + 1; ++v) {
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    if (v + 2 <= r1 + 1) {                           // s row v + 2 -> ring, row v + 3 -> registers
      put_s(v + 2);
      if (v + 3 <= r1 + 1) load_s(v + 3);
    }
    if (v <= r1) {                                   // conv_a(v) -> T row v
      const bool ok = v >= 0 && v < p.H;
      const int slot = (v + 2 * NT) % NT;
      f32x4 acc[N3];
      conv3(sring, NS, SROW, v, lwa, bav, acc);
#pragma unroll
      for (int n = 0; n < N3; ++n) {
        const u32x2 o = ok ? pack4(silu4(acc[n])) : u32x2{0u, 0u};
        *reinterpret_cast<u32x2*>(tring + slot * TROW + ((px0 + fr + 1) * C + 16 * n + 4 * fq) * 2) = o;
      }
    }
    const int w = v - 2;
    if (w >= r0 && w < r1) {                         // conv_b(w) (+ s) -> y row w
      const int sslot = (w + 2 * NS) % NS;
      const int px = px0 + fr;
      f32x4 c[N3];
      conv3(tring, NT, TROW, w, lwb, bbv, c);
      bf16_t* yrow = p.y + (((long)img * p.H + w) * W + px) * p.ldy;
#pragma unroll
      for (int n = 0; n < N3; ++n) {
        c[n] = silu4(c[n]);
        if constexpr (SC) {
          const f32x4 sv = unpack4(*reinterpret_cast<const u32x2*>(sring + sslot * SROW + ((px + 1) * C + 16 * n + 4 * fq) * 2));
          c[n] = f32x4{c[n][0] + sv[0], c[n][1] + sv[1], c[n][2] + sv[2], c[n][3] + sv[3]};
        }
        *reinterpret_cast<u32x2*>(yrow + 16 * n + 4 * fq) = pack4(c[n]);
      }
    }
  }
}

}  // namespace aiko

// x [B, H, W, ldx] -> y [B, H, W, ldy] through the fused C2f (n = 1); weights as the ConvSpecs
// hold them ([Cout][K] bf16, K padded).  Returns -1 for shapes without an instantiation.
extern "C" int aiko_c2f_fused(const void* x, int ldx, const void* w1, const float* b1, int k1, const void* wa,
                              const float* ba, int ka, const void* wb, const float* bb, int kb, const void* w2,
                              const float* b2, int k2, void* y, int ldy, int B, int H, int W, int CI, int C, int CO,
                              int shortcut, int rb, const void* xu, int ldxu, int cu, hipStream_t stream) {
  using namespace aiko;
  if (rb <= 0 || H % rb || B <= 0) return -1;
  C2fParams p{};
  p.xu = static_cast<const bf16_t*>(xu);
  p.ldxu = ldxu;
  p.cu = xu ? cu : 0;
  p.x = static_cast<const bf16_t*>(x);
  p.w1 = static_cast<const bf16_t*>(w1); p.b1 = b1;
  p.wa = static_cast<const bf16_t*>(wa); p.ba = ba;
  p.wb = static_cast<const bf16_t*>(wb); p.bb = bb;
  p.w2 = static_cast<const bf16_t*>(w2); p.b2 = b2;
  p.y = static_cast<bf16_t*>(y);
  p.B = B; p.H = H; p.ldx = ldx; p.ldy = ldy; p.k1 = k1; p.ka = ka; p.kb = kb; p.k2 = k2; p.rb = rb;
  const dim3 grid((unsigned)(B * (H / rb)));
  if (W == 160 && CI == 32 && C == 16 && CO == 32 && shortcut) {
    if (xu) return -1;                             // (in-place upsample: the wide-channel kernel only)
    c2f_fused_kernel<160, 32, 16, 32, true><<<grid, dim3(320), 0, stream>>>(p);
  } else if (W == 80 && CI == 192 && C == 32 && CO == 64 && !shortcut) {
    c2f_fused_wl_kernel<80, 192, 32, 64, false><<<grid, dim3(320), 0, stream>>>(p);
  } else {
    return -1;
  }
  return (int)hipGetLastError();
}

// One C2f bottleneck (3x3 C -> C twice, SiLU, optional shortcut) over channel-slice views:
// x = s [B, H, W, pitch ldx], y = c [B, H, W, pitch ldy] (c2f_bneck_kernel).
extern "C" int aiko_c2f_bneck(const void* x, int ldx, const void* wa, const float* ba, int ka, const void* wb,
                              const float* bb, int kb, void* y, int ldy, int B, int H, int W, int C, int shortcut,
                              int rb, hipStream_t stream) {
  using namespace aiko;
  if (rb <= 0 || H % rb || B <= 0) return -1;
  C2fParams p{};
  p.x = static_cast<const bf16_t*>(x);
  p.wa = static_cast<const bf16_t*>(wa); p.ba = ba;
  p.wb = static_cast<const bf16_t*>(wb); p.bb = bb;
  p.y = static_cast<bf16_t*>(y);
  p.B = B; p.H = H; p.ldx = ldx; p.ldy = ldy; p.ka = ka; p.kb = kb; p.rb = rb;
  const dim3 grid((unsigned)(B * (H / rb)));
  if (W == 80 && C == 32 && shortcut) {
    c2f_bneck_kernel<80, 32, true><<<grid, dim3(320), 0, stream>>>(p);
  } else {
    return -1;
  }
  return (int)hipGetLastError();
}

