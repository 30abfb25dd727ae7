// Shared parameter block of the implicit-GEMM convolution kernels (register-staged and
// global_load_lds variants).
#pragma once
#include "common.h"

namespace aiko {

struct ConvParams {
  const bf16_t* x;
  const bf16_t* w;      // [Cout][K]
  const float* bias;    // [Cout] or nullptr
  const bf16_t* res;    // [M][ldr] or nullptr
  bf16_t* y;            // [M][ldy]
  int H, W, C;          // input spatial dims and pixel pitch in elements
  int Cc;               // contiguous channel run per tap (multiple of 8)
  int R, S, stride, pad;
  int Ho, Wo, M, Cout, K;
  int act;              // bits 0-3: 0 none, 1 relu, 2 silu, 3 gelu(erf); bit 4: residual added AFTER the
                        // activation (YOLO/CSP bottleneck x + silu(conv)) instead of before
  int ldy, ldr;
  // optional second A source (K columns [K1, K)): a 1x1 / stride-s2 conv over x2, used to
  // fuse a ResNet projection shortcut into the block's last conv (K-concatenation)
  const bf16_t* x2;
  int K1, H2, W2, C2, stride2;
  // magic numbers for n / (Ho*Wo), n / Wo, n / Cc, n / S without a VALU division loop (fdiv)
  uint32_t mHoWo, mWo, mCc, mS;
  int lHoWo, lWo, lCc, lS;
};

// n / d for 0 <= n < 2^31 as (umulhi(n, m) + n) >> l with l = ceil(log2 d),
// m = floor(2^32 (2^l - d) / d) + 1 (Hacker's Delight 10-9): 3 VALU instead of ~30.
__host__ inline void fastdiv_init(int d, uint32_t* m, int* l) {
  int k = 0;
  while ((1LL << k) < d) ++k;
  *l = k;
  *m = (uint32_t)(((1ULL << 32) * ((1ULL << k) - (unsigned long long)d)) / (unsigned long long)d + 1ULL);
}

__device__ __forceinline__ int fdiv(int n, uint32_t m, int l) {
  return (int)((__umulhi((uint32_t)n, m) + (uint32_t)n) >> l);
}

__host__ inline void conv_params_finalize(ConvParams& p) {
  fastdiv_init(p.Ho * p.Wo, &p.mHoWo, &p.lHoWo);
  fastdiv_init(p.Wo, &p.mWo, &p.lWo);
  fastdiv_init(p.Cc, &p.mCc, &p.lCc);
  fastdiv_init(p.S, &p.mS, &p.lS);
}

}  // namespace aiko
