// Implicit-GEMM convolution, persistent buffer-LDS-DMA variant (variant 4).
//
// Why: the ResNet 1x1 / short-K layers (K = 64..512, N up to 2048, M = B*H*W up to 800k) ran at
// 2-4 TB/s and 400-550 TFLOP/s in every tile shape and occupancy of conv_buf.hip — as fast as
// hipBLASLt on the same GEMMs, and far from both roofs.  Per workgroup a tile is only 2-8 K
// blocks, so each tile starts with an empty ring (one full HBM/L2 latency exposed) and drains
// it at the end (nothing in flight during the last blocks and the epilogue): the bytes in
// flight per CU, not the matrix pipe or HBM, set the pace.
//
// Here a workgroup owns a contiguous run of output tiles and streams K blocks through ONE
// ring across tile boundaries: while tile i finishes its last blocks and runs its epilogue,
// tile i+1's first blocks are already being DMA'd.  Consequences:
//   * the issue side has its own cursor (tile, tap, channel offset, per-piece offsets) that runs
//     D = NS-1 blocks ahead of the compute side and recomputes piece geometry when it enters a
//     new tile; the compute side only needs the tile's (m0, n0) for the epilogue;
//   * the epilogue cannot alias the ring (it is full of the next tile's data): the fp32 tile is
//     staged through a separate LDS region in row passes (EPI rows at a time);
//   * the residual of a tile is prefetched into registers by ordinary loads when its first K
//     block is consumed, so it lands during the tile's K loop;
//   * every wait is a counted `s_waitcnt vmcnt(N)`: N = the DMA ops issued after the awaited
//     block, or 0 at the end of the stream; the epilogue's ordinary loads/stores only ever make
//     a wait stricter (vmcnt retires in order), never wrong.
// Slot addresses are runtime (scalar) here — the tile loop does not unroll by ring depth.
//
// Measured (MI355X, B=256 ResNet layers, scripts/layer_bench.py): the 64x128 / 3-slot / 2 WG/CU
// configuration matches the best non-persistent tile (b4.conv3 117 vs 119 us, b8.conv3 76 vs
// 70 us); the 1 WG/CU deep-ring configurations are 1.3-2x slower.  Removing the per-tile ring
// bubble did not move these layers: with 64x128 tiles the LDS traffic per K block (DMA writes
// + fragment reads of both operands, ~144 KB per CU-step at 2 WG/CU) exceeds the matrix pipe's
// time, so the LDS, not the memory latency, is the co-limit.  Kept as a tuner candidate.
#include "conv_common.h"

namespace aiko {

namespace {

constexpr uint32_t kPOOB = 0x80000000u;
constexpr uint32_t kPRecords = 0x7ffffff0u;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t p_rsrc(const void* base) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)kPRecords, 0x00020000);
}

__device__ __forceinline__ void p_dma16(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff, void* lds) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(
      r, reinterpret_cast<__attribute__((address_space(3))) void*>(reinterpret_cast<uintptr_t>(lds)), 16,
      voff, soff, 0, 0);
}

template <int N>
__device__ __forceinline__ void p_vm_barrier() {
  asm volatile("s_waitcnt vmcnt(%0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::"n"(N) : "memory");
}

}  // namespace

// BM x BN tile, 4 waves (2 x 2), NS ring slots of (BM + BN) x 64 bf16, EPI rows per epilogue
// pass, OCC workgroups per CU.
template <int BM, int BN, int NS, int EPI, int OCC, int CPAD = 4>
__global__ __launch_bounds__(256, OCC) void conv_persist_kernel(ConvParams p, int tiles, int per_wg) {
  constexpr int NW = 4, NT = 256;
  constexpr int WGM = 2, WGN = 2;
  constexpr int BK = 64;
  constexpr int D = NS - 1;
  constexpr int WM = BM / WGM, WN = BN / WGN;
  constexpr int MI = WM / 16, NI = WN / 16;
  constexpr int RPI = 8 * NW;                  // tile rows filled per DMA instruction (32)
  constexpr int APT = BM / RPI, BPT = BN / RPI;
  constexpr int PER = APT + BPT;               // DMA instructions per K block per thread
  constexpr int STAGE_ELEMS = (BM + BN) * BK;
  constexpr int RING_BYTES = NS * STAGE_ELEMS * 2;
  constexpr int LDC = BN + CPAD;
  constexpr int EPI_BYTES = EPI * LDC * 4;
  static_assert((RING_BYTES + EPI_BYTES) * OCC <= 160 * 1024, "LDS budget");
  static_assert(BM % EPI == 0 && EPI % 16 == 0, "epilogue passes of whole 16-row blocks");
  constexpr int CPR = BN / 8, CHUNKS = BM * CPR, CPT = CHUNKS / NT, E_ROWS = NT / CPR;
  static_assert(CHUNKS % NT == 0 && EPI % E_ROWS == 0, "whole chunks per thread and pass");
  constexpr int PASSES = BM / EPI, CPP = CPT / PASSES;     // chunks per thread per pass

  __shared__ __attribute__((aligned(16))) unsigned char smem[RING_BYTES + EPI_BYTES];
  bf16_t* ring = reinterpret_cast<bf16_t*>(smem);
  float* Cs = reinterpret_cast<float*>(smem + RING_BYTES);

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave / WGN, wc = wave % WGN;
  const int ntn = (p.Cout + BN - 1) / BN;
  const int t_begin = blockIdx.x * per_wg;
  const int t_end = min(tiles, t_begin + per_wg);
  if (t_begin >= t_end) return;
  const int ntiles = t_end - t_begin;

  const int lrow = wave * 8 + (lane >> 3);
  const int lp = (lane & 7) ^ (lane >> 3);
  const int HoWo = p.Ho * p.Wo;
  const int RS = p.R * p.S;
  const __amdgpu_buffer_rsrc_t rx = p_rsrc(p.x);
  const __amdgpu_buffer_rsrc_t rw = p_rsrc(p.w);
  const __amdgpu_buffer_rsrc_t rx2 = p_rsrc(p.x2 ? p.x2 : p.x);
  const int K1 = p.x2 ? p.K1 : p.K;
  const int nkb = p.K / BK;
  const int total = ntiles * nkb;               // K blocks this workgroup streams

  // ---- issue side: cursor + piece geometry of the tile being fetched ----
  int iss_tile = -1, iss_kb = 0, iss_tap = 0, iss_c = 0, cur_tap = -1;   // issue cursor
  int a_base[APT];
  uint32_t a_mask[APT], a2_off[APT], a_off[APT], b_off[BPT];

  auto enter_tile = [&](int t) {                // piece geometry of tile t (workgroup-local index)
    const int tg = t_begin + t;
    const int m0 = (tg / ntn) * BM, n0 = (tg % ntn) * BN;
#pragma unroll
    for (int i = 0; i < APT; ++i) {
      const int m = m0 + lrow + RPI * i;
      a_mask[i] = 0u;
      a_base[i] = 0;
      a2_off[i] = kPOOB;
      a_off[i] = kPOOB;
      if (m < p.M) {
        const int img = fdiv(m, p.mHoWo, p.lHoWo);
        const int rem = m - img * HoWo;
        const int oh = fdiv(rem, p.mWo, p.lWo);
        const int ow = rem - oh * p.Wo;
        const int ih0 = oh * p.stride - p.pad, iw0 = ow * p.stride - p.pad;
        a_base[i] = (((img * p.H + ih0) * p.W + iw0) * p.C + lp * 8) * 2;
        for (int t2 = 0; t2 < RS; ++t2) {
          const int r = t2 / p.S, s = t2 - r * p.S;
          if ((unsigned)(ih0 + r) < (unsigned)p.H && (unsigned)(iw0 + s) < (unsigned)p.W) a_mask[i] |= 1u << t2;
        }
        a2_off[i] = (uint32_t)((((img * p.H2 + oh * p.stride2) * p.W2 + ow * p.stride2) * p.C2 + lp * 8) * 2);
      }
    }
#pragma unroll
    for (int i = 0; i < BPT; ++i) {
      const int n = n0 + lrow + RPI * i;
      b_off[i] = n < p.Cout ? (uint32_t)(((long)n * p.K + lp * 8) * 2) : kPOOB;
    }
    iss_tap = 0;
    iss_c = 0;
    cur_tap = -1;
  };

  int iss_slot = 0;
  auto issue = [&]() {                          // DMA the next K block of the stream
    bf16_t* As = ring + iss_slot * STAGE_ELEMS;
    bf16_t* Bs = As + BM * BK;
    if (iss_kb == 0) {
      ++iss_tile;
      enter_tile(iss_tile);
    }
    const int k0 = iss_kb * BK;
    if (++iss_kb == nkb) iss_kb = 0;
    if (++iss_slot == NS) iss_slot = 0;
    if (k0 >= K1) {
      const uint32_t soff = (uint32_t)((k0 - K1) * 2);
#pragma unroll
      for (int i = 0; i < APT; ++i) p_dma16(rx2, a2_off[i], soff, As + (i * RPI + wave * 8) * BK);
    } else {
      if (iss_tap != cur_tap) {
        cur_tap = iss_tap;
        const int r = iss_tap / p.S, s = iss_tap - r * p.S;
        const int tap_off = ((r * p.W + s) * p.C) * 2;
#pragma unroll
        for (int i = 0; i < APT; ++i)
          a_off[i] = (a_mask[i] >> iss_tap) & 1u ? (uint32_t)(a_base[i] + tap_off) : kPOOB;
      }
      const uint32_t soff = (uint32_t)(iss_c * 2);
#pragma unroll
      for (int i = 0; i < APT; ++i) p_dma16(rx, a_off[i], soff, As + (i * RPI + wave * 8) * BK);
      iss_c += BK;
      if (iss_c >= p.Cc) {
        iss_c = 0;
        ++iss_tap;
      }
    }
    const uint32_t sb = (uint32_t)(k0 * 2);
#pragma unroll
    for (int i = 0; i < BPT; ++i) p_dma16(rw, b_off[i], sb, Bs + (i * RPI + wave * 8) * BK);
  };

  // ---- compute side ----
  f32x4 acc[MI][NI];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int fr = lane & 15, fq = lane >> 4;
  int a_rd[MI], b_rd[NI];
#pragma unroll
  for (int i = 0; i < MI; ++i) a_rd[i] = (wr * WM + i * 16 + fr) * BK;
#pragma unroll
  for (int j = 0; j < NI; ++j) b_rd[j] = BM * BK + (wc * WN + j * 16 + fr) * BK;
  const int sw = fr & 7;

  // epilogue geometry (thread -> 8-channel chunks of rows e_row0 + E_ROWS * i)
  const int e_cc = tid % CPR, e_row0 = tid / CPR;
  u32x4 e_res[CPT];
  float e_bias[8];

  auto prefetch_epilogue = [&](int t) {         // bias + residual of tile t into registers
    const int tg = t_begin + t;
    const int m0 = (tg / ntn) * BM, e_n = (tg % ntn) * BN + e_cc * 8;
#pragma unroll
    for (int e = 0; e < 8; ++e) e_bias[e] = 0.f;
    if (p.bias && e_n < p.Cout) {
      const f32x4 b0 = *reinterpret_cast<const f32x4*>(p.bias + e_n);
      const f32x4 b1 = *reinterpret_cast<const f32x4*>(p.bias + e_n + 4);
      e_bias[0] = b0[0]; e_bias[1] = b0[1]; e_bias[2] = b0[2]; e_bias[3] = b0[3];
      e_bias[4] = b1[0]; e_bias[5] = b1[1]; e_bias[6] = b1[2]; e_bias[7] = b1[3];
    }
    if (p.res) {
#pragma unroll
      for (int i = 0; i < CPT; ++i) {
        const int m = m0 + e_row0 + E_ROWS * i;
        const bool ok = m < p.M && e_n < p.Cout;
        e_res[i] = *reinterpret_cast<const u32x4*>(p.res + (ok ? (size_t)m * p.ldr + e_n : 0));
      }
    }
  };

  auto epilogue = [&](int t) {
    const int tg = t_begin + t;
    const int m0 = (tg / ntn) * BM, e_n = (tg % ntn) * BN + e_cc * 8;
    const bool post = (p.act & 16) != 0;
    const int act = p.act & 15;
#pragma unroll
    for (int ps = 0; ps < PASSES; ++ps) {
      // rows [ps * EPI, (ps + 1) * EPI): the waves holding them stage their accumulators
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        const int row_blk = wr * WM + i * 16;
        if (row_blk >= ps * EPI && row_blk < (ps + 1) * EPI) {
#pragma unroll
          for (int j = 0; j < NI; ++j) {
            const int col = wc * WN + j * 16 + fr;
#pragma unroll
            for (int e = 0; e < 4; ++e) Cs[(row_blk - ps * EPI + fq * 4 + e) * LDC + col] = acc[i][j][e];
          }
        }
      }
      __syncthreads();
#pragma unroll
      for (int ci = 0; ci < CPP; ++ci) {
        const int i = ps * CPP + ci;
        const int row = e_row0 + E_ROWS * i;
        const int m = m0 + row;
        if (m >= p.M || e_n >= p.Cout) continue;
        const float* src = Cs + (row - ps * EPI) * LDC + e_cc * 8;
        const f32x4 v0 = *reinterpret_cast<const f32x4*>(src);
        const f32x4 v1 = *reinterpret_cast<const f32x4*>(src + 4);
        float v[8] = {v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] += e_bias[e];
        if (p.res && !post) {
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            v[2 * e] += __uint_as_float(e_res[i][e] << 16);
            v[2 * e + 1] += __uint_as_float(e_res[i][e] & 0xffff0000u);
          }
        }
        if (act == 1) {
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] = fmaxf(v[e], 0.f);
        } else if (act == 2) {
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] = silu(v[e]);
        } else if (act == 3) {
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] = gelu_erf(v[e]);
        }
        if (p.res && post) {
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            v[2 * e] += __uint_as_float(e_res[i][e] << 16);
            v[2 * e + 1] += __uint_as_float(e_res[i][e] & 0xffff0000u);
          }
        }
        u32x4 o;
#pragma unroll
        for (int e = 0; e < 4; ++e) o[e] = pack2(v[2 * e], v[2 * e + 1]);
        *reinterpret_cast<u32x4*>(p.y + (size_t)m * p.ldy + e_n) = o;
      }
      __syncthreads();
    }
  };

  // ---- the stream ----
  for (int v = 0; v < D && v < total; ++v) issue();
  int slot = 0, kb = 0, t = 0;
  for (int v = 0; v < total; ++v) {
    // block v landed: D-1 younger blocks may stay in flight (all of them near the end)
    if (v + D - 1 < total && D >= 2) {
      p_vm_barrier<(D - 1) * PER>();
    } else {
      p_vm_barrier<0>();
    }
    if (kb == 0) prefetch_epilogue(t);          // lands during this tile's K loop
    if (v + D < total) issue();                 // refill the slot freed by block v-1
    const bf16_t* St = ring + slot * STAGE_ELEMS;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8 af[MI], bfr[NI];
      const int pc = ((fq + 4 * kk) ^ sw) << 3;
#pragma unroll
      for (int i = 0; i < MI; ++i) af[i] = *reinterpret_cast<const bf16x8*>(St + a_rd[i] + pc);
#pragma unroll
      for (int j = 0; j < NI; ++j) bfr[j] = *reinterpret_cast<const bf16x8*>(St + b_rd[j] + pc);
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NI; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    if (kb == nkb - 1) {
      epilogue(t);
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NI; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
      kb = 0;
      ++t;
    } else {
      ++kb;
    }
    if (++slot == NS) slot = 0;
  }
}

}  // namespace aiko

static int cu_count() {
  static int n = 0;
  if (n == 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
      n = 256;
  }
  return n;
}

// Same arguments as aiko_conv_buf (host preconditions identical: Cc and K-K1 multiples of 64,
// R*S <= 32, operands < 2 GiB).  cfg selects the tile / ring / occupancy configuration.
extern "C" int aiko_conv_persist(const void* x, const void* w, const float* bias, const void* res,
                                 void* y, int H, int W, int C, int Cc, int R, int S, int stride,
                                 int pad, int Ho, int Wo, int M, int Cout, int K, int act, int ldy,
                                 int ldr, int bm, int bn, const void* x2, int K1, int H2, int W2,
                                 int C2, int stride2, hipStream_t stream) {
  using namespace aiko;
  if (Cc % 64 || R * S > 32 || (x2 && (K - K1) % 64) || K % 64) return -1;
  ConvParams p;
  p.x = static_cast<const bf16_t*>(x);
  p.w = static_cast<const bf16_t*>(w);
  p.bias = bias;
  p.res = static_cast<const bf16_t*>(res);
  p.y = static_cast<bf16_t*>(y);
  p.H = H; p.W = W; p.C = C; p.Cc = Cc; p.R = R; p.S = S;
  p.stride = stride; p.pad = pad; p.Ho = Ho; p.Wo = Wo; p.M = M; p.Cout = Cout; p.K = K;
  p.act = act; p.ldy = ldy; p.ldr = ldr;
  p.x2 = static_cast<const bf16_t*>(x2);
  p.K1 = x2 ? K1 : K; p.H2 = H2; p.W2 = W2; p.C2 = C2; p.stride2 = stride2;
  conv_params_finalize(p);
  const int tiles = ((M + bm - 1) / bm) * ((Cout + bn - 1) / bn);
  int occ;
  if (bm == 64 && bn == 128) occ = 2;
  else if (bm == 128 && bn == 128) occ = 1;
  else if (bm == 64 && bn == 64) occ = 2;
  else return -1;
  const int slots = cu_count() * occ;
  const int per_wg = (tiles + slots - 1) / slots;
  const int grid = (tiles + per_wg - 1) / per_wg;
  if (bm == 64 && bn == 128)
    conv_persist_kernel<64, 128, 3, 16, 2, 0><<<grid, 256, 0, stream>>>(p, tiles, per_wg);
  else if (bm == 128 && bn == 128)
    conv_persist_kernel<128, 128, 4, 32, 1><<<grid, 256, 0, stream>>>(p, tiles, per_wg);
  else
    conv_persist_kernel<64, 64, 4, 32, 2><<<grid, 256, 0, stream>>>(p, tiles, per_wg);
  return (int)hipGetLastError();
}
