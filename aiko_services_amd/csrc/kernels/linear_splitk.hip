// Split-K linear layer for short-M, long-K GEMMs (the ResNet-50 classifier: B=256 x 2048 ->
// 1000).  Tiled over M x N alone that GEMM is 64 workgroups of 64 x 64 on a 256-CU chip, each
// walking K = 2048 serially (45 us in the bench trace, 22 us isolated).  Here the K range is cut
// into S slices: S x ceil(M/32) x ceil(N/32) one-wave workgroups (1,024 for the classifier),
// each a 32 x 32 tile over K / S, fragments loaded straight from global memory (the operands
// are L2-resident: 1 MB of activations, 4 MB of weights), fp32 partials to a workspace; a
// second kernel sums the S partials in a fixed order (deterministic, no atomics), adds the bias
// and writes bf16.
//
// MFMA v_mfma_f32_16x16x32_bf16 with the WEIGHTS as the A operand (rows = output channels n)
// and the activations as B (columns = rows m of x): lane (fr, fq) ends with output channels
// 4 fq .. 4 fq + 3 of row fr — one 16-B fp32 store per accumulator tile.
#include "common.h"

namespace aiko {

namespace {

struct SplitKParams {
  const bf16_t* x;      // [M][ldx]
  const bf16_t* w;      // [N][ldw]
  const float* bias;    // [N] or nullptr
  float* part;          // [S][M][N]
  bf16_t* y;            // [M][ldy]
  int M, N, ldx, ldw, ldy, ks, S;
};

__global__ __launch_bounds__(64) void linear_splitk_partial_kernel(SplitKParams p) {
  const int lane = threadIdx.x;
  const int fr = lane & 15, fq = lane >> 4;
  const int tn = (p.N + 31) / 32, tm = (p.M + 31) / 32;
  int bid = blockIdx.x;
  const int nt = bid % tn;
  bid /= tn;
  const int mt = bid % tm;
  const int s = bid / tm;
  const int k0 = s * p.ks;
  // fragment rows (clamped into range; results for rows past M / N are never stored)
  const bf16_t* wr[2];
  const bf16_t* xr[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int n = min(nt * 32 + j * 16 + fr, p.N - 1);
    wr[j] = p.w + (size_t)n * p.ldw + k0 + 8 * fq;
    const int m = min(mt * 32 + j * 16 + fr, p.M - 1);
    xr[j] = p.x + (size_t)m * p.ldx + k0 + 8 * fq;
  }
  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int steps = p.ks / 32;
#pragma unroll 4
  for (int st = 0; st < steps; ++st) {
    bf16x8 a[2], b[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      a[j] = *reinterpret_cast<const bf16x8*>(wr[j] + st * 32);
      b[j] = *reinterpret_cast<const bf16x8*>(xr[j] + st * 32);
    }
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
  }
  // acc[i][j]: channels nt*32 + i*16 + 4 fq .. +3 of row mt*32 + j*16 + fr
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int n = nt * 32 + i * 16 + 4 * fq;
      const int m = mt * 32 + j * 16 + fr;
      if (m < p.M && n < p.N)
        *reinterpret_cast<f32x4*>(p.part + ((size_t)s * p.M + m) * p.N + n) = acc[i][j];
    }
}

__global__ __launch_bounds__(256) void linear_splitk_reduce_kernel(SplitKParams p) {
  const int per_row = p.N / 4;
  const int idx = blockIdx.x * 256 + threadIdx.x;
  if (idx >= p.M * per_row) return;
  const int m = idx / per_row, n = (idx - m * per_row) * 4;
  f32x4 v = p.bias ? *reinterpret_cast<const f32x4*>(p.bias + n) : f32x4{0.f, 0.f, 0.f, 0.f};
  for (int s = 0; s < p.S; ++s) v += *reinterpret_cast<const f32x4*>(p.part + ((size_t)s * p.M + m) * p.N + n);
  *reinterpret_cast<uint2*>(p.y + (size_t)m * p.ldy + n) = make_uint2(pack2(v[0], v[1]), pack2(v[2], v[3]));
}

}  // namespace

}  // namespace aiko

// y[m, n] = sum_k x[m, k] w[n, k] + bias[n] (bf16 in / out, fp32 accumulation) with K cut into S
// slices.  Host preconditions (binding): K % (32 S) == 0, N % 4 == 0, 16-B aligned rows (ldx, ldw,
// ldy multiples of 8), part holds S * M * N floats.
extern "C" int aiko_linear_splitk(const void* x, const void* w, const float* bias, float* part, void* y, int M,
                                  int N, int K, int ldx, int ldw, int ldy, int S, hipStream_t stream) {
  using namespace aiko;
  if (S < 1 || K % (32 * S) || N % 4 || M < 1 || N < 1) return -1;
  SplitKParams p;
  p.x = static_cast<const bf16_t*>(x);
  p.w = static_cast<const bf16_t*>(w);
  p.bias = bias;
  p.part = part;
  p.y = static_cast<bf16_t*>(y);
  p.M = M; p.N = N; p.ldx = ldx; p.ldw = ldw; p.ldy = ldy; p.ks = K / S; p.S = S;
  const long tiles = (long)S * ((M + 31) / 32) * ((N + 31) / 32);
  linear_splitk_partial_kernel<<<dim3((unsigned)tiles), dim3(64), 0, stream>>>(p);
  const long quads = (long)M * (N / 4);
  linear_splitk_reduce_kernel<<<dim3((unsigned)((quads + 255) / 256)), dim3(256), 0, stream>>>(p);
  return (int)hipGetLastError();
}
