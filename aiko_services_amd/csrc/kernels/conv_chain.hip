// Chained 1x1 convolutions for ResNet bottleneck boundaries (gfx950, wave64, MFMA bf16):
//
//   Y = relu(A . W1^T + b1 + R)      block b's expansion conv3 (K1 = 64 -> N1 = 256, identity
//                                    residual R) — Y is written (it is block b+1's residual)
//   Z = relu(Y . W2^T + b2)          block b+1's reduction conv1 (K2 = 256 -> N2 = 64 / 128)
//
// Unchained, the 256-channel Y (411 MB at B=256, 56x56) is written by one kernel and read back
// in full by the next; here Z is computed from the Y tile while it is still in LDS, so the
// chain moves A + R + Y + Z once (stage 1: 1028 MB instead of 1439 MB).  Both GEMMs are
// bandwidth-bound by a wide margin, so the kernel is organised around keeping HBM busy:
// a persistent grid (512 threads = 8 waves per workgroup; 2 workgroups per CU for stage 1,
// 1 for stage 2's 64 KB Y tile) walks 64-pixel tiles;
// the next tile's A and R rows are loaded into registers while the current tile computes and
// land in LDS behind the barrier that ends it.  Per tile:
//   1. GEMM1 on v_mfma_f32_16x16x32_bf16: wave w owns Y columns w N1/8 .. (w+1) N1/8 (64 rows,
//      all of K1), A fragments from the XOR-swizzled LDS A tile, W1 fragments held in registers
//      for the whole kernel;
//   2. epilogue in place: the R tile already sits in LDS where Y goes; each lane adds bias and
//      residual, applies ReLU and overwrites its R element with Y (bf16) — the tile becomes the
//      A operand of GEMM2 and the source of coalesced 16-byte Y stores;
//   3. GEMM2: N2 = 64: wave w owns Z columns 16 (w & 3) .. over K half w >> 2 (partials meet in
//      LDS); N2 >= 128: wave w owns column tiles w, w + 8, ... over all of K; W2 fragments
//      streamed from L2 four k-steps at a time;
//   4. Z epilogue (bias, ReLU) straight from the accumulators.
#include <hip/hip_runtime.h>

#include "common.h"

namespace aiko {

namespace chain {
constexpr int BM = 64, NT = 512;
}  // namespace chain

// swizzled 16-byte chunk offsets (bytes) for rows of `rb` bytes
__device__ __forceinline__ int sw_off(int row, int chunk, int rb, int mask) {
  return row * rb + ((chunk ^ (row & mask)) << 4);
}

// K1 -> N1 expansion (+ residual), then N1 -> N2 reduction; stage 1: (64, 256, 64 | 128),
// stage 2: (128, 512, 128 | 256).
// DUAL: the expansion is a block's first conv3 with its 1x1 projection shortcut fused by
// K-concatenation (A = [t2 | x], K1 = 64 + 64, no residual term), as in ops.conv.fuse_shortcut.
template <int K1, int N1, int N2, bool DUAL = false>
__global__ __launch_bounds__(512, (N1 <= 256 ? 2 : 1)) void conv_chain_kernel(
    const bf16_t* __restrict__ A, const bf16_t* __restrict__ A2, const bf16_t* __restrict__ W1,
    const float* __restrict__ b1,
    const bf16_t* __restrict__ R, bf16_t* __restrict__ Y, const bf16_t* __restrict__ W2,
    const float* __restrict__ b2, bf16_t* __restrict__ Z, int M) {
  using namespace chain;
  constexpr int K2 = N1;
  constexpr int A_BYTES = BM * K1 * 2, Y_BYTES = BM * N1 * 2;
  constexpr int ARB = K1 * 2, YRB = N1 * 2;              // row bytes
  constexpr int ACH = ARB / 16, YCH = YRB / 16;          // 16-byte chunks per row
  constexpr int AMASK = ACH >= 16 ? 15 : ACH - 1, YMASK = 15;
  constexpr int CT2 = N2 / 16;                            // GEMM2 column tiles
  constexpr int KH = CT2 < 8 ? 8 / CT2 : 1;               // K split over wave groups
  constexpr int J2 = CT2 >= 8 ? CT2 / 8 : 1;              // column tiles per wave
  constexpr int RED_BYTES = KH > 1 ? BM * N2 * 4 : 0;
  constexpr int J1 = N1 / 8 / 16, KS1 = K1 / 32;
  constexpr int APT = BM * ACH / NT, RPT = BM * YCH / NT; // chunks per thread
  static_assert(APT >= 1 && RPT >= 1 && KH <= 2, "tile shape");
  __shared__ __attribute__((aligned(16))) unsigned char smem[A_BYTES + Y_BYTES + RED_BYTES];
  unsigned char* As = smem;
  unsigned char* Ys = smem + A_BYTES;
  float* Red = reinterpret_cast<float*>(smem + A_BYTES + Y_BYTES);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int fr = lane & 15, fq = lane >> 4;
  const int ntiles = M / BM;

  // W1 fragments for this wave's N1/8 columns: kept in registers for the whole kernel when they
  // are few (stage 1: 16 VGPRs); stage 2's 64 would spill, so they are re-read from L2 per tile
  constexpr bool W1_RESIDENT = J1 * KS1 <= 8;
  bf16x8 w1f[J1][KS1];
  auto load_w1 = [&]() {
#pragma unroll
    for (int j = 0; j < J1; ++j)
#pragma unroll
      for (int ks = 0; ks < KS1; ++ks)
        w1f[j][ks] = *reinterpret_cast<const bf16x8*>(W1 + (long)(N1 / 8 * wave + 16 * j + fr) * K1 + 32 * ks + 8 * fq);
  };
  if constexpr (W1_RESIDENT) load_w1();
  (void)load_w1;
  float bias1[J1];
#pragma unroll
  for (int j = 0; j < J1; ++j) bias1[j] = b1[N1 / 8 * wave + 16 * j + fr];

  u32x4 ra[APT], rr[RPT];
  auto load_tile = [&](int tile) {
    const long m0 = (long)tile * BM;
#pragma unroll
    for (int i = 0; i < APT; ++i) {
      const int c = tid + NT * i;
      if constexpr (DUAL) {                    // chunks 0..7 from t2, 8..15 from the block input
        const int ch = c % ACH;
        ra[i] = ch < ACH / 2 ? *reinterpret_cast<const u32x4*>(A + (m0 + c / ACH) * (K1 / 2) + ch * 8)
                             : *reinterpret_cast<const u32x4*>(A2 + (m0 + c / ACH) * (K1 / 2) + (ch - ACH / 2) * 8);
      } else {
        ra[i] = *reinterpret_cast<const u32x4*>(A + (m0 + c / ACH) * K1 + (c % ACH) * 8);
      }
    }
#pragma unroll
    for (int i = 0; i < RPT; ++i) {
      const int c = tid + NT * i;
      if constexpr (!DUAL) rr[i] = *reinterpret_cast<const u32x4*>(R + (m0 + c / YCH) * N1 + (c % YCH) * 8);
    }
  };
  auto store_tile_lds = [&]() {
#pragma unroll
    for (int i = 0; i < APT; ++i) {
      const int c = tid + NT * i;
      *reinterpret_cast<u32x4*>(As + sw_off(c / ACH, c % ACH, ARB, AMASK)) = ra[i];
    }
#pragma unroll
    for (int i = 0; i < RPT; ++i) {
      const int c = tid + NT * i;
      if constexpr (!DUAL) *reinterpret_cast<u32x4*>(Ys + sw_off(c / YCH, c % YCH, YRB, YMASK)) = rr[i];
    }
  };

  int tile = blockIdx.x;
  if (tile < ntiles) {
    load_tile(tile);
    store_tile_lds();
  }
  __syncthreads();
  for (; tile < ntiles; tile += gridDim.x) {
    const long m0 = (long)tile * BM;
    const int next = tile + gridDim.x;
    if (next < ntiles) load_tile(next);        // in flight during this tile's compute
    // ---- 1. GEMM1: rows 16 i + (4 fq + e), cols N1/8 wave + 16 j + fr
    {
      f32x4 acc[4][J1];
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < J1; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
      if constexpr (W1_RESIDENT) {
#pragma unroll
        for (int ks = 0; ks < KS1; ++ks)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const bf16x8 af = *reinterpret_cast<const bf16x8*>(As + sw_off(16 * i + fr, 4 * ks + fq, ARB, AMASK));
#pragma unroll
            for (int j = 0; j < J1; ++j)
              acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, w1f[j][ks], acc[i][j], 0, 0, 0);
          }
      } else {
        // one k-step of weight fragments live at a time (L2-resident weights), bounded registers
#pragma unroll 1
        for (int ks = 0; ks < KS1; ++ks) {
          bf16x8 wk[J1];
#pragma unroll
          for (int j = 0; j < J1; ++j)
            wk[j] = *reinterpret_cast<const bf16x8*>(W1 + (long)(N1 / 8 * wave + 16 * j + fr) * K1 + 32 * ks + 8 * fq);
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const bf16x8 af = *reinterpret_cast<const bf16x8*>(As + sw_off(16 * i + fr, 4 * ks + fq, ARB, AMASK));
#pragma unroll
            for (int j = 0; j < J1; ++j)
              acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, wk[j], acc[i][j], 0, 0, 0);
          }
        }
      }
      // ---- 2. Y = relu(acc + b1 + R) in place of R
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < J1; ++j) {
          const int col = N1 / 8 * wave + 16 * j + fr;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int row = 16 * i + 4 * fq + e;
            bf16_t* p = reinterpret_cast<bf16_t*>(Ys + sw_off(row, col >> 3, YRB, YMASK)) + (col & 7);
            *p = f2bf(fmaxf(acc[i][j][e] + bias1[j] + (DUAL ? 0.f : bf2f(*p)), 0.f));
          }
        }
    }
    __syncthreads();
    // Y tile -> global, 16-byte chunks
#pragma unroll
    for (int i = 0; i < RPT; ++i) {
      const int c = tid + NT * i;
      *reinterpret_cast<u32x4*>(Y + (m0 + c / YCH) * N1 + (c % YCH) * 8) =
          *reinterpret_cast<const u32x4*>(Ys + sw_off(c / YCH, c % YCH, YRB, YMASK));
    }
    // ---- 3. GEMM2: wave -> column tiles ct0 + 8 j (J2 of them) over K part kh (of KH)
    const int ct0 = KH > 1 ? (wave % CT2) : wave;
    const int kh = KH > 1 ? (wave / CT2) : 0;
    constexpr int KS2 = K2 / 32 / KH;
    f32x4 acc2[J2][4];
#pragma unroll
    for (int j = 0; j < J2; ++j)
#pragma unroll
      for (int i = 0; i < 4; ++i) acc2[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};
    auto gemm2_step = [&](int k4) {        // 4 k-steps of W2 fragments in flight
      bf16x8 w2f[J2][4];
#pragma unroll
      for (int j = 0; j < J2; ++j)
#pragma unroll
        for (int u = 0; u < 4; ++u)
          w2f[j][u] = *reinterpret_cast<const bf16x8*>(W2 + (long)(16 * (ct0 + 8 * j) + fr) * K2 +
                                                        32 * (kh * KS2 + k4 + u) + 8 * fq);
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int kc = 4 * (kh * KS2 + k4 + u) + fq;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const bf16x8 af = *reinterpret_cast<const bf16x8*>(Ys + sw_off(16 * i + fr, kc, YRB, YMASK));
#pragma unroll
          for (int j = 0; j < J2; ++j)
            acc2[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, w2f[j][u], acc2[j][i], 0, 0, 0);
        }
      }
    };
    if constexpr (N1 <= 256) {                   // stage 1: fully unrolled (no spills at 2 waves/SIMD)
#pragma unroll
      for (int k4 = 0; k4 < KS2; k4 += 4) gemm2_step(k4);
    } else {                                     // stage 2: bounded live registers
#pragma unroll 1
      for (int k4 = 0; k4 < KS2; k4 += 4) gemm2_step(k4);
    }
    if constexpr (KH > 1) {
      if (kh == 1) {
#pragma unroll
        for (int i = 0; i < 4; ++i) *reinterpret_cast<f32x4*>(Red + ((ct0 * 4 + i) * 64 + lane) * 4) = acc2[0][i];
      }
    }
    __syncthreads();                             // Y / A reads done; partials visible
    if (KH == 1 || kh == 0) {
      if constexpr (KH > 1) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const f32x4 o = *reinterpret_cast<const f32x4*>(Red + ((ct0 * 4 + i) * 64 + lane) * 4);
#pragma unroll
          for (int e = 0; e < 4; ++e) acc2[0][i][e] += o[e];
        }
      }
#pragma unroll
      for (int j = 0; j < J2; ++j) {
        const int n = 16 * (ct0 + 8 * j) + fr;
        const float bb = b2[n];
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int e = 0; e < 4; ++e)
            Z[(m0 + 16 * i + 4 * fq + e) * N2 + n] = f2bf(fmaxf(acc2[j][i][e] + bb, 0.f));
      }
    }
    // ---- next tile's rows into LDS (this tile's reads all finished at the barrier above)
    if (next < ntiles) store_tile_lds();
    __syncthreads();
  }
}

}  // namespace aiko

extern "C" int aiko_conv_chain2(const void* A, const void* W1, const float* b1, const void* R, void* Y,
                                const void* W2, const float* b2, void* Z, int M, int K1, int N1, int N2,
                                int grid, hipStream_t stream);

extern "C" int aiko_conv_chain(const void* A, const void* W1, const float* b1, const void* R, void* Y,
                               const void* W2, const float* b2, void* Z, const void* A2, int M, int K1, int N1, int N2,
                               int grid, hipStream_t stream) {
  using namespace aiko;
  if (M <= 0 || M % chain::BM) return -1;
  const int ntiles = M / chain::BM;
  const int per_cu = N1 <= 256 ? 2 : 1;
  if (grid <= 0) grid = 256 * per_cu;
  if (grid > ntiles) grid = ntiles;
  auto a = static_cast<const bf16_t*>(A);
  auto w1 = static_cast<const bf16_t*>(W1);
  auto r = static_cast<const bf16_t*>(R);
  auto y = static_cast<bf16_t*>(Y);
  auto w2 = static_cast<const bf16_t*>(W2);
  auto z = static_cast<bf16_t*>(Z);
#define AIKO_CHAIN(k1, n1, n2)                                                                           \
  if (!A2 && K1 == k1 && N1 == n1 && N2 == n2) {                                                               \
    hipLaunchKernelGGL((conv_chain_kernel<k1, n1, n2>), dim3(grid), dim3(chain::NT), 0, stream, a, nullptr, w1, b1, r, y, \
                       w2, b2, z, M);                                                                   \
    return (int)hipGetLastError();                                                                      \
  }
  AIKO_CHAIN(64, 256, 64)
  AIKO_CHAIN(64, 256, 128)
  // stage 2 -> 128: weights-in-registers kernel (conv_chain2.hip)
  if (!A2 && K1 == 128 && N1 == 512 && N2 == 128)
    return aiko_conv_chain2(A, W1, b1, R, Y, W2, b2, Z, M, K1, N1, N2, grid, stream);
  if (A2 && K1 == 128 && N1 == 256 && N2 == 64) {
    hipLaunchKernelGGL((conv_chain_kernel<128, 256, 64, true>), dim3(grid), dim3(chain::NT), 0, stream, a,
                       static_cast<const bf16_t*>(A2), w1, b1, r, y, w2, b2, z, M);
    return (int)hipGetLastError();
  }
#undef AIKO_CHAIN
  return -1;
}
