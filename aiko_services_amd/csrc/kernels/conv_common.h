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
};

}  // namespace aiko
