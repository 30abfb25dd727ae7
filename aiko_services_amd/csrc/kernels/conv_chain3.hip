// Chained 1x1 convolutions at a ResNet stage-3 bottleneck boundary (gfx950, wave64, MFMA bf16):
//
//   Y = relu(A . W1^T + b1 + R)     block b's expansion conv3 (K1 = 256 -> N1 = 1024, identity R)
//   Z = relu(Y . W2^T + b2)         block b+1's reduction conv1 (K2 = 1024 -> N2 = 256)
//
// Unchained, the 1024-channel Y is written by one kernel and read back whole by the next (at
// B = 320: 128 MB read again, ~33 us of a 101 us pair).  The stage-2 chain keeps both weight
// matrices in registers and a whole 64-pixel Y tile in LDS; at stage 3 neither fits (W1 + W2
// are 1 MB, a 64 x 1024 Y tile is 128 KB).  Instead this kernel walks Y in CHUNKS of 128
// channels: per 64-pixel tile and chunk c
//   1. GEMM1 (transposed, weights on the MFMA A side): Y^T[128 c + 16 w + 4 fq + e][16 i + fr] for
//      wave w's 16 channels over the whole K1 = 256, X fragments from the LDS A tile;
//   2. epilogue: + b1 + R (the residual chunk, staged in LDS), ReLU, 8-byte stores of Y to HBM and
//      in place of R in LDS;
//   3. GEMM2 partial: Z^T[32 w + 16 j + 4 fq + e][16 i + fr] += W2[:, chunk] . Ychunk^T — the Z
//      accumulators (64 pixels x 256 channels = 32 VGPRs per lane) live across all 8 chunks;
//   4. after chunk 7: Z = relu(acc + b2), 8-byte stores.
// Weight fragments for a chunk (W1: 8, W2: 8 per lane) come from L2 (1 MB per tile, L2-resident)
// at the top of the chunk, BEFORE the chunk's HBM prefetches are issued, so that the compiler's
// in-order vmcnt waits for them never retire the younger prefetches: the residual chunk two
// steps ahead (and the next tile's A rows, a quarter per step from chunk 2 on) travel in
// registers and land in LDS only after the NEXT step's middle barrier.  The kernel is HBM-bound (A + R + Y + Z = 320 KB per
// tile, vs 448 KB unchained), so the point of the schedule is that those loads are always in
// flight.
//
// Measured (MI355X, M = 62720, scripts/r5_chain3.py / r5_chain3_exp.sh): bit-exact against the two
// unchained convs, but 179-185 us against 101 us for the unchained pair the model runs (68 us
// expansion on conv_pw_rb + 33 us reduction), so it is OPT-IN (AIKO_CHAIN3=1) and off by default.
// Diagnostic builds (template EXP) place the time: without the per-chunk weight loads 103 us,
// without the residual / A prefetches 175 us, without both 84 us, and with the Y stores also
// removed 74 us.  The weights are the problem: every wave re-reads 17 KB of fragments from L2 per
// 64-pixel chunk step (1 MB per tile, 26 us of L2->CU bandwidth per CU at this M), and since
// vmcnt retires in order, waiting for them each step also retires every older HBM prefetch, so
// the lookahead never exceeds ~1 step; a 64 x 1024 Y tile or a resident W1 + W2 (1 MB) does not
// fit a CU.  The stage-2 chain (conv_chain2.hip) works because its 256 KB of weights DO fit the
// register file.
#include <hip/hip_runtime.h>

#include <type_traits>

#include "common.h"

namespace aiko {

namespace chain3 {
constexpr int BM = 64, NT = 512, K1 = 256, N1 = 1024, N2 = 256, CH = 128, NCH = N1 / CH;
constexpr int AROW = K1 * 2, RROW = CH * 2;              // LDS row bytes (A tile, R/Y chunk)
constexpr int A_BYTES = BM * AROW, R_BYTES = BM * RROW;  // 32 KB, 16 KB
constexpr int APT = A_BYTES / 16 / NT, RPT = R_BYTES / 16 / NT;   // 16-B chunks per thread: 4, 2

// 16-byte chunk `c` of LDS row `row`, XOR-swizzled over 16 positions (conflict-free b128 reads of
// 16 rows at one logical chunk)
__device__ __forceinline__ int sw(int row, int c, int rowbytes) { return row * rowbytes + ((c ^ (row & 15)) << 4); }
}  // namespace chain3

// EXP: diagnostic builds only (see the measurements above): 1 = no R / A prefetch loads, 2 = no
// per-step weight loads (fragments from the first load), 4 = no Y stores to HBM
template <int EXP = 0>
__global__ __launch_bounds__(512, 1) void conv_chain3_kernel(
    const bf16_t* __restrict__ A, const bf16_t* __restrict__ W1, const float* __restrict__ b1,
    const bf16_t* __restrict__ R, bf16_t* __restrict__ Y, const bf16_t* __restrict__ W2,
    const float* __restrict__ b2, bf16_t* __restrict__ Z, int M) {
  using namespace chain3;
  constexpr int MI = BM / 16, KS1 = K1 / 32, KS2 = CH / 32, NJ2 = N2 / 8 / 16;
  __shared__ __attribute__((aligned(16))) unsigned char smem[2 * A_BYTES + 2 * R_BYTES];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int fr = lane & 15, fq = lane >> 4;
  const int ntiles = M / BM;

  const bf16x8 wconst = *reinterpret_cast<const bf16x8*>(W1 + (long)(16 * wave + fr) * K1 + 8 * fq);
  float bias2[NJ2][4];
#pragma unroll
  for (int j = 0; j < NJ2; ++j) {
    const f32x4 u = *reinterpret_cast<const f32x4*>(b2 + 32 * wave + 16 * j + 4 * fq);
    bias2[j][0] = u[0]; bias2[j][1] = u[1]; bias2[j][2] = u[2]; bias2[j][3] = u[3];
  }

  // prefetch registers: the next tile's A rows one quarter (16 B per thread) per step, residual
  // chunks two steps deep
  u32x4 pa[2], pr[2][RPT];
  auto load_a = [&](int tile, int u, u32x4& dst) {
    const int q = tid + NT * u;
    dst = *reinterpret_cast<const u32x4*>(A + ((long)tile * BM + (q >> 5)) * K1 + (q & 31) * 8);
  };
  auto store_a = [&](int buf, int u, const u32x4& src) {
    const int q = tid + NT * u;
    *reinterpret_cast<u32x4*>(smem + buf * A_BYTES + sw(q >> 5, q & 31, AROW)) = src;
  };
  auto load_r = [&](int tile, int c, u32x4 (&dst)[RPT]) {
#pragma unroll
    for (int u = 0; u < RPT; ++u) {
      const int q = tid + NT * u;
      dst[u] = *reinterpret_cast<const u32x4*>(R + ((long)tile * BM + (q >> 4)) * N1 + CH * c + (q & 15) * 8);
    }
  };
  auto store_r = [&](int slot, const u32x4 (&src)[RPT]) {
#pragma unroll
    for (int u = 0; u < RPT; ++u) {
      const int q = tid + NT * u;
      *reinterpret_cast<u32x4*>(smem + 2 * A_BYTES + slot * R_BYTES + sw(q >> 4, q & 15, RROW)) = src[u];
    }
  };

  int tile = blockIdx.x;
  if (tile >= ntiles) return;
  // prologue: A tile 0 and R chunk 0 in LDS, R chunk 1 in flight
  {
    u32x4 a0[APT];
#pragma unroll
    for (int u = 0; u < APT; ++u) load_a(tile, u, a0[u]);
    load_r(tile, 0, pr[0]);
#pragma unroll
    for (int u = 0; u < APT; ++u) store_a(0, u, a0[u]);
  }
  store_r(0, pr[0]);
  load_r(tile, 1, pr[1]);
  __syncthreads();

  int abuf = 0;
  for (; tile < ntiles; tile += gridDim.x, abuf ^= 1) {
    const long m0 = (long)tile * BM;
    const int next = tile + gridDim.x;
    const unsigned char* As = smem + abuf * A_BYTES;
    f32x4 acc2[NJ2][MI];
#pragma unroll
    for (int j = 0; j < NJ2; ++j)
#pragma unroll
      for (int i = 0; i < MI; ++i) acc2[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};

    // one chunk step; P = c & 1 as a compile-time constant (prefetch register set, LDS slot)
    auto step = [&](const int c, auto P) __attribute__((always_inline)) {
      constexpr int p = decltype(P)::value;
      unsigned char* Rs = smem + 2 * A_BYTES + p * R_BYTES;
      // ---- weight fragments and bias for this chunk (L2), then the HBM prefetches
      const int n1 = CH * c + 16 * wave;          // this wave's first GEMM1 channel
      bf16x8 w1f[KS1], w2f[NJ2][KS2];
#pragma unroll
      for (int ks = 0; ks < KS1; ++ks)
        w1f[ks] = (EXP & 2) ? wconst : *reinterpret_cast<const bf16x8*>(W1 + (long)(n1 + fr) * K1 + 32 * ks + 8 * fq);
#pragma unroll
      for (int j = 0; j < NJ2; ++j)
#pragma unroll
        for (int ks = 0; ks < KS2; ++ks)
          w2f[j][ks] = (EXP & 2) ? wconst : *reinterpret_cast<const bf16x8*>(W2 + (long)(32 * wave + 16 * j + fr) * N1 + CH * c + 32 * ks + 8 * fq);
      const f32x4 bb1 = *reinterpret_cast<const f32x4*>(b1 + n1 + 4 * fq);
      // The prefetches are issued AFTER the weight loads (scheduling fences on both sides, and
      // branch-free: clamped addresses, the last tile re-reads its own rows) so the compiler's
      // waits for the weights never retire them.
      __builtin_amdgcn_sched_barrier(0);
      // residual chunk two steps ahead (this tile's c + 2, or the next tile's first two)
      const int tn = next < ntiles ? next : tile;
      if (!(EXP & 1)) load_r(c + 2 < NCH ? tile : tn, c + 2 < NCH ? c + 2 : c + 2 - NCH, pr[p]);
      // next tile's A quarter c - 2 on steps 2 .. 5 (stored one step later)
      if (!(EXP & 1)) load_a(tn, min(max(c - 2, 0), APT - 1), pa[p]);
      __builtin_amdgcn_sched_barrier(0);

      // ---- GEMM1: Y^T[n1 + 4 fq + e][16 i + fr]
      f32x4 acc1[MI];
#pragma unroll
      for (int i = 0; i < MI; ++i) acc1[i] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < KS1; ++ks) {
        bf16x8 xf[MI];
#pragma unroll
        for (int i = 0; i < MI; ++i)
          xf[i] = *reinterpret_cast<const bf16x8*>(As + sw(16 * i + fr, 4 * ks + fq, AROW));
#pragma unroll
        for (int i = 0; i < MI; ++i) acc1[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w1f[ks], xf[i], acc1[i], 0, 0, 0);
      }
      // ---- epilogue 1: Y = relu(acc + b1 + R), in place of R in LDS and to HBM (8 B per pixel)
      const int cl = 16 * wave + 4 * fq;          // channel within the chunk
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        const int row = 16 * i + fr;
        uint2* slot = reinterpret_cast<uint2*>(Rs + sw(row, cl >> 3, RROW) + (cl & 7) * 2);
        const uint2 r = *slot;
        uint2 o;
        o.x = pack2(fmaxf(acc1[i][0] + bb1[0] + __uint_as_float(r.x << 16), 0.f),
                    fmaxf(acc1[i][1] + bb1[1] + __uint_as_float(r.x & 0xffff0000u), 0.f));
        o.y = pack2(fmaxf(acc1[i][2] + bb1[2] + __uint_as_float(r.y << 16), 0.f),
                    fmaxf(acc1[i][3] + bb1[3] + __uint_as_float(r.y & 0xffff0000u), 0.f));
        *slot = o;
        if (!(EXP & 4)) *reinterpret_cast<uint2*>(Y + (m0 + row) * N1 + CH * c + cl) = o;
      }
      __syncthreads();   // Y chunk complete in LDS; every wave is past chunk c-1's GEMM2
      // residual chunk c + 1 into the other slot (read by no one since chunk c-1's GEMM2)
      if (c + 1 < NCH) store_r(p ^ 1, pr[p ^ 1]);
      else if (next < ntiles) store_r(0, pr[0]);
      // the other A buffer was last read by the previous tile: free for the whole tile
      if (c >= 3 && c < 3 + APT && next < ntiles) store_a(abuf ^ 1, c - 3, pa[p ^ 1]);

      // ---- GEMM2 partial over this chunk's 128 channels
#pragma unroll
      for (int ks = 0; ks < KS2; ++ks) {
        bf16x8 yf[MI];
#pragma unroll
        for (int i = 0; i < MI; ++i)
          yf[i] = *reinterpret_cast<const bf16x8*>(Rs + sw(16 * i + fr, 4 * ks + fq, RROW));
#pragma unroll
        for (int j = 0; j < NJ2; ++j)
#pragma unroll
          for (int i = 0; i < MI; ++i)
            acc2[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w2f[j][ks], yf[i], acc2[j][i], 0, 0, 0);
      }
      __syncthreads();   // chunk c + 1 residual (and the next A tile) visible; slot c & 1 free
    };
#pragma unroll 1
    for (int c = 0; c < NCH; c += 2) {
      step(c, std::integral_constant<int, 0>{});
      step(c + 1, std::integral_constant<int, 1>{});
    }
    // ---- epilogue 2: Z = relu(acc2 + b2), 4 channels (8 B) per lane and pixel
#pragma unroll
    for (int j = 0; j < NJ2; ++j)
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        uint2 o;
        o.x = pack2(fmaxf(acc2[j][i][0] + bias2[j][0], 0.f), fmaxf(acc2[j][i][1] + bias2[j][1], 0.f));
        o.y = pack2(fmaxf(acc2[j][i][2] + bias2[j][2], 0.f), fmaxf(acc2[j][i][3] + bias2[j][3], 0.f));
        *reinterpret_cast<uint2*>(Z + (m0 + 16 * i + fr) * N2 + 32 * wave + 16 * j + 4 * fq) = o;
      }
  }
}

}  // namespace aiko

// Y = relu(A W1^T + b1 + R) [M, 1024], Z = relu(Y W2^T + b2) [M, 256]; A [M, 256]; M % 64 == 0.
extern "C" int aiko_conv_chain3(const void* A, const void* W1, const float* b1, const void* R, void* Y,
                                const void* W2, const float* b2, void* Z, int M, int K1, int N1, int N2,
                                int grid, hipStream_t stream) {
  using namespace aiko;
  if (M <= 0 || M % chain3::BM || K1 != chain3::K1 || N1 != chain3::N1 || N2 != chain3::N2) return -1;
  const int ntiles = M / chain3::BM;
  if (grid <= 0) grid = 256;
  if (grid > ntiles) grid = ntiles;
  hipLaunchKernelGGL(conv_chain3_kernel<0>, dim3(grid), dim3(chain3::NT), 0, stream, static_cast<const bf16_t*>(A),
                     static_cast<const bf16_t*>(W1), b1, static_cast<const bf16_t*>(R), static_cast<bf16_t*>(Y),
                     static_cast<const bf16_t*>(W2), b2, static_cast<bf16_t*>(Z), M);
  return (int)hipGetLastError();
}
