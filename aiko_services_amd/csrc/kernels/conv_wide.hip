// Implicit-GEMM convolution, 8-wave wide tiles with a register-direct epilogue (tuner variant 8).
//
// conv_buf.hip computes C = X . W^T (pixels on the MFMA A side) and leaves each lane four
// consecutive PIXELS of one channel, so its epilogue has to bounce the whole fp32 tile through
// LDS (128 ds_write_b32 per lane for a 64 x 64 wave tile, a barrier, then the read-back) before
// it can store rows.  For the short-K layers (1x1 convs with K = 128..512: 2-8 K blocks per
// tile) that bounce is a third to a half of the tile's time, and it pins the LDS footprint.
//
// Here the product is transposed, C^T = W . X^T: the MFMA A operand is the weight tile
// (channels), B the activation tile (pixels), so v_mfma_f32_16x16x32_bf16 leaves lane l four
// consecutive CHANNELS (4 (l >> 4) .. +3) of pixel (l & 15).  One v_permlane16_swap per fp32
// pair of adjacent 16-channel blocks turns that into eight consecutive channels per lane
// (row 0: channels 0-7, row 1: 16-23, row 2: 8-15, row 3: 24-31 of the 32-channel pair), so
// bias (2 x float4), residual (one 16-B load) and the output (one 16-B store) move straight
// between registers and memory — no LDS epilogue, no barrier, and a residual prefetched
// before the K loop sits in 4 VGPRs per block pair.
//
// Staging is conv_buf's (buffer_load_dwordx4 ... lds with a scalar tap cursor, out-of-range
// offsets as zero padding, XOR-swizzled 128-B rows, counted vmcnt + raw s_barrier, NS-slot
// ring), at 512 threads and one workgroup per CU, so the tile can be 256 wide on either side.
#include <cstdlib>
#include <type_traits>

#include "conv_common.h"

namespace aiko {

namespace {

constexpr uint32_t kWideOOB = 0x80000000u;        // offsets >= num_records read as zero
constexpr uint32_t kWideRecords = 0x7ffffff0u;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t wide_rsrc(const void* base) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)kWideRecords, 0x00020000);
}

__device__ __forceinline__ void wide_dma16(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff, void* lds) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(
      r, reinterpret_cast<__attribute__((address_space(3))) void*>(reinterpret_cast<uintptr_t>(lds)), 16,
      voff, soff, 0, 0);
}

template <int N>
__device__ __forceinline__ void wide_vm_barrier() {
  asm volatile("s_waitcnt vmcnt(%0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::"n"(N) : "memory");
}

}  // namespace

// BM pixels x BN channels per workgroup, WGM x WGN waves (4 or 8), NS ring slots of one
// 64-deep K block each, OCC workgroups per CU.  RES_PF: prefetch the residual into registers
// before the K loop.  The 4-wave / multi-workgroup shapes are for the short-K, bandwidth-bound
// layers: there a second resident workgroup's loads and stores cover one tile's prologue and
// epilogue, which a lone 8-wave workgroup leaves exposed.
// BK = 32 (tuner variant 11): half-depth K blocks in a 4-slot ring, so a 256 x 256 tile keeps
// three blocks in flight across every barrier (the 64-deep ring fits only two slots there and
// retires each block with one block of MFMA work to cover its DMA); 64-B rows swizzled by
// (row >> 1) & 3.
// NR (tuner variant 18, "exact N"): the tile computes only NR <= BN channels — BN is the
// DMA's row count (whole DMA pieces), NR the channels the MFMAs and epilogue cover and the
// channel step between tiles — so a layer with N = 80 or 144 (the YOLO heads) runs on a
// 80- / 144-channel tile instead of wasting 3/8 or 1/4 of a 128 / 192-channel tile's MFMA work.
// An odd number of 16-channel blocks per wave ends in an unpaired block: its lane holds 4
// consecutive channels and stores them as 8 bytes.
template <int BM, int BN, int WGM, int WGN, int NS, bool RES_PF, int OCC, int BK = 64, int NR = 0>
__global__ __launch_bounds__(64 * WGM * WGN, OCC) void conv_wide_kernel(ConvParams p) {
  constexpr int NW = WGM * WGN;
  static_assert(NW == 4 || NW == 8, "4 or 8 waves");
  static_assert(BK == 64 || BK == 32, "64- or 32-deep K blocks");
  constexpr int PPR = BK / 8;                    // 16-B pieces per tile row
  constexpr int D = NS - 1;                      // K blocks in flight ahead of the one computed
  constexpr int BNR = NR ? NR : BN;              // channels computed per tile
  static_assert(BNR <= BN && BNR % (16 * WGN) == 0, "exact-N tile");
  constexpr int WM = BM / WGM, WN = BNR / WGN;   // pixels / channels per wave
  constexpr int MI = WM / 16, NI = WN / 16;
  static_assert((NR != 0 || NI % 2 == 0) && MI >= 1, "wave tile: whole 16-pixel blocks, channel blocks in pairs");
  constexpr bool TAIL = NI % 2 != 0;             // an unpaired last channel block
  constexpr int RPW = 64 / PPR;                  // tile rows per wave DMA instruction
  constexpr int RPI = RPW * NW;                  // tile rows filled per DMA instruction
  static_assert(BM % RPI == 0 && BN % RPI == 0, "tile rows in whole DMA pieces");
  constexpr int APT = BM / RPI, BPT = BN / RPI;
  constexpr int PER = APT + BPT;                 // DMA instructions per K block per thread
  constexpr int STAGE_ELEMS = (BM + BN) * BK;
  static_assert(NS * STAGE_ELEMS * 2 * OCC <= 160 * 1024, "LDS budget");
  __shared__ __attribute__((aligned(16))) bf16_t ring[NS * STAGE_ELEMS];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave / WGN, wc = wave % WGN;
  const int ntn = (p.Cout + BNR - 1) / BNR;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int tile_n = bid % ntn, tile_m = bid / ntn;
  const int m0 = tile_m * BM, n0 = tile_n * BNR;

  const int lrow = wave * RPW + lane / PPR;
  // source-side swizzle: physical piece (lane % PPR) of the row holds logical piece lp
  const int lp = BK == 64 ? ((lane & 7) ^ (lane >> 3)) : ((lane & 3) ^ ((lrow >> 1) & 3));
  const int HoWo = p.Ho * p.Wo;
  const __amdgpu_buffer_rsrc_t rx = wide_rsrc(p.x);
  const __amdgpu_buffer_rsrc_t rw = wide_rsrc(p.w);
  const __amdgpu_buffer_rsrc_t rx2 = wide_rsrc(p.x2 ? p.x2 : p.x);

  // per-piece activation geometry (as conv_buf): tap-(0,0) byte offset + valid filter rows/cols
  int a_base[APT];
  uint32_t a_mask[APT], a2_off[APT];
#pragma unroll
  for (int i = 0; i < APT; ++i) {
    const int m = m0 + lrow + RPI * i;
    a_mask[i] = 0u;
    a_base[i] = 0;
    a2_off[i] = kWideOOB;
    if (m < p.M) {
      const int img = fdiv(m, p.mHoWo, p.lHoWo);
      const int rem = m - img * HoWo;
      const int oh = fdiv(rem, p.mWo, p.lWo);
      const int ow = rem - oh * p.Wo;
      const int ih0 = oh * p.stride - p.pad, iw0 = ow * p.stride - p.pad;
      a_base[i] = (((img * p.H + ih0) * p.W + iw0) * p.C + lp * 8) * 2;
      const int r_lo = max(0, -ih0), r_hi = min(p.R, p.H - ih0);
      const int s_lo = max(0, -iw0), s_hi = min(p.S, p.W - iw0);
      const uint32_t mr = r_hi > r_lo ? ((1u << r_hi) - 1u) & ~((1u << r_lo) - 1u) : 0u;
      const uint32_t ms = s_hi > s_lo ? ((1u << s_hi) - 1u) & ~((1u << s_lo) - 1u) : 0u;
      a_mask[i] = mr | (ms << 16);
      a2_off[i] = (uint32_t)((((img * p.H2 + oh * p.stride2) * p.W2 + ow * p.stride2) * p.C2 + lp * 8) * 2);
    }
  }
  uint32_t b_off[BPT];
#pragma unroll
  for (int i = 0; i < BPT; ++i) {
    const int n = n0 + lrow + RPI * i;
    b_off[i] = n < p.Cout ? (uint32_t)(((long)n * p.K + lp * 8) * 2) : kWideOOB;
  }

  // ---- epilogue geometry: lane (fr, fq) owns pixel fr of each 16-pixel block and, after the
  // swap, 8 consecutive channels at coff of each 32-channel block pair
  const int fr = lane & 15, fq = lane >> 4;
  const int coff = ((fq & 1) << 4) | ((fq >> 1) << 3);
  constexpr int NP = NI / 2;
  float e_bias[NP][8];
#pragma unroll
  for (int q = 0; q < NP; ++q) {
    const int n = n0 + wc * WN + q * 32 + coff;
#pragma unroll
    for (int e = 0; e < 8; ++e) e_bias[q][e] = 0.f;
    if (p.bias && n < p.Cout) {
      const f32x4 b0 = *reinterpret_cast<const f32x4*>(p.bias + n);
      const f32x4 b1 = *reinterpret_cast<const f32x4*>(p.bias + n + 4);
      e_bias[q][0] = b0[0]; e_bias[q][1] = b0[1]; e_bias[q][2] = b0[2]; e_bias[q][3] = b0[3];
      e_bias[q][4] = b1[0]; e_bias[q][5] = b1[1]; e_bias[q][6] = b1[2]; e_bias[q][7] = b1[3];
    }
  }
  // the unpaired block (TAIL): lane holds channels 4 fq .. 4 fq + 3 of pixel fr
  float e_btail[4] = {0.f, 0.f, 0.f, 0.f};
  const int ntail = n0 + wc * WN + (NI - 1) * 16 + 4 * fq;
  if constexpr (TAIL) {
    if (p.bias && ntail < p.Cout) {
      const f32x4 b0 = *reinterpret_cast<const f32x4*>(p.bias + ntail);
      e_btail[0] = b0[0]; e_btail[1] = b0[1]; e_btail[2] = b0[2]; e_btail[3] = b0[3];
    }
  }
  u32x4 e_res[RES_PF ? MI : 1][RES_PF && NP > 0 ? NP : 1];
  uint2 e_rtail[RES_PF && TAIL ? MI : 1];
  if constexpr (RES_PF) {
    if (p.res) {
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        const int m = m0 + wr * WM + i * 16 + fr;
#pragma unroll
        for (int q = 0; q < NP; ++q) {
          const int n = n0 + wc * WN + q * 32 + coff;
          const bool ok = m < p.M && n < p.Cout;
          e_res[i][q] = *reinterpret_cast<const u32x4*>(p.res + (ok ? (size_t)m * p.ldr + n : 0));
        }
        if constexpr (TAIL) {
          const bool ok = m < p.M && ntail < p.Cout;
          e_rtail[i] = *reinterpret_cast<const uint2*>(p.res + (ok ? (size_t)m * p.ldr + ntail : 0));
        }
      }
    }
  }
  // the bias / residual loads stay in flight under the first K blocks: the loop's counted
  // vmcnt(N) waits retire them together with block 0 (they are older), and nothing reads them
  // before the epilogue

  // scalar K-block cursor for the DMA issue
  const int K1 = p.x2 ? p.K1 : p.K;
  int cur_tap = -1;
  uint32_t a_off[APT];
#pragma unroll
  for (int i = 0; i < APT; ++i) a_off[i] = kWideOOB;
  int iss_tap = 0, iss_c = 0, iss_r = 0, iss_s = 0;

  auto issue = [&](int kb, auto slot_tag) {
    constexpr int SLOT = decltype(slot_tag)::value;
    bf16_t* Xs = ring + SLOT * STAGE_ELEMS;
    bf16_t* Ws = Xs + BM * BK;
    const int k0 = kb * BK;
    const uint32_t sb = (uint32_t)(k0 * 2);
#pragma unroll
    for (int i = 0; i < BPT; ++i) wide_dma16(rw, b_off[i], sb, Ws + (i * RPI + wave * RPW) * BK);
    if (k0 >= K1) {
      const uint32_t soff = (uint32_t)((k0 - K1) * 2);
#pragma unroll
      for (int i = 0; i < APT; ++i) wide_dma16(rx2, a2_off[i], soff, Xs + (i * RPI + wave * RPW) * BK);
    } else {
      if (iss_tap != cur_tap) {
        cur_tap = iss_tap;
        const int tap_off = ((iss_r * p.W + iss_s) * p.C) * 2;
        const uint32_t bit = (1u << iss_r) | (1u << (iss_s + 16));
#pragma unroll
        for (int i = 0; i < APT; ++i)
          a_off[i] = (a_mask[i] & bit) == bit ? (uint32_t)(a_base[i] + tap_off) : kWideOOB;
      }
      const uint32_t soff = (uint32_t)(iss_c * 2);
#pragma unroll
      for (int i = 0; i < APT; ++i) wide_dma16(rx, a_off[i], soff, Xs + (i * RPI + wave * RPW) * BK);
      iss_c += BK;
      if (iss_c >= p.Cc) {
        iss_c = 0;
        ++iss_tap;
        if (++iss_s == p.S) {
          iss_s = 0;
          ++iss_r;
        }
      }
    }
  };

  f32x4 acc[NI][MI];
#pragma unroll
  for (int j = 0; j < NI; ++j)
#pragma unroll
    for (int i = 0; i < MI; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};

  // fragment row offsets (elements): weight rows (A operand) and pixel rows (B operand)
  const int sw = BK == 64 ? (fr & 7) : ((fr >> 1) & 3);
  int w_rd[NI], x_rd[MI];
#pragma unroll
  for (int j = 0; j < NI; ++j) w_rd[j] = BM * BK + (wc * WN + j * 16 + fr) * BK;
#pragma unroll
  for (int i = 0; i < MI; ++i) x_rd[i] = (wr * WM + i * 16 + fr) * BK;

  auto compute = [&](auto slot_tag) {
    constexpr int SLOT = decltype(slot_tag)::value;
    const bf16_t* St = ring + SLOT * STAGE_ELEMS;
#pragma unroll
    for (int kk = 0; kk < BK / 32; ++kk) {
      const int pc = ((fq + 4 * kk) ^ sw) << 3;
      bf16x8 wf[NI], xf[MI];
#pragma unroll
      for (int j = 0; j < NI; ++j) wf[j] = *reinterpret_cast<const bf16x8*>(St + w_rd[j] + pc);
#pragma unroll
      for (int i = 0; i < MI; ++i) xf[i] = *reinterpret_cast<const bf16x8*>(St + x_rd[i] + pc);
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NI; ++j)
          acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[j], xf[i], acc[j][i], 0, 0, 0);
    }
  };

  const int nkb = p.K / BK;
  auto step = [&](int kb, auto slot_tag) {
    constexpr int SLOT = decltype(slot_tag)::value;
    constexpr int PREV = SLOT == 0 ? NS - 1 : SLOT - 1;
    // block kb must have landed; D - 1 younger blocks may stay in flight
    if constexpr (D >= 3) {
      if (kb + 2 < nkb) wide_vm_barrier<PER * 2>();
      else if (kb + 1 < nkb) wide_vm_barrier<PER>();
      else wide_vm_barrier<0>();
    } else if constexpr (D == 2) {
      if (kb + 1 < nkb) wide_vm_barrier<PER>();
      else wide_vm_barrier<0>();
    } else {
      wide_vm_barrier<0>();
    }
    if (kb + D < nkb) issue(kb + D, std::integral_constant<int, PREV>{});
    compute(slot_tag);
  };

  using S0 = std::integral_constant<int, 0>;
  using S1 = std::integral_constant<int, 1>;
  using S2 = std::integral_constant<int, 2>;
  using S3 = std::integral_constant<int, 3>;
  issue(0, S0{});
  if constexpr (NS == 4) {
    if (1 < nkb) issue(1, S1{});
    if (2 < nkb) issue(2, S2{});
    int kb = 0;
    for (; kb + 4 <= nkb; kb += 4) {
      step(kb, S0{});
      step(kb + 1, S1{});
      step(kb + 2, S2{});
      step(kb + 3, S3{});
    }
    if (kb < nkb) step(kb, S0{});
    if (kb + 1 < nkb) step(kb + 1, S1{});
    if (kb + 2 < nkb) step(kb + 2, S2{});
  } else if constexpr (NS == 3) {
    if (1 < nkb) issue(1, S1{});
    int kb = 0;
    for (; kb + 3 <= nkb; kb += 3) {
      step(kb, S0{});
      step(kb + 1, S1{});
      step(kb + 2, S2{});
    }
    if (kb < nkb) step(kb, S0{});
    if (kb + 1 < nkb) step(kb + 1, S1{});
  } else {
    static_assert(NS == 2, "2- or 3-slot ring");
    int kb = 0;
    for (; kb + 2 <= nkb; kb += 2) {
      step(kb, S0{});
      step(kb + 1, S1{});
    }
    if (kb < nkb) step(kb, S0{});
  }

  // ---- register-direct epilogue ----
  const bool post = (p.act & 16) != 0;
  const int act = p.act & 15;
#pragma unroll
  for (int i = 0; i < MI; ++i) {
    const int m = m0 + wr * WM + i * 16 + fr;
#pragma unroll
    for (int q = 0; q < NP; ++q) {
      f32x4 lo = acc[2 * q][i], hi = acc[2 * q + 1][i];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const auto s = __builtin_amdgcn_permlane16_swap(__float_as_uint(lo[e]), __float_as_uint(hi[e]), false, false);
        lo[e] = __uint_as_float(s[0]);
        hi[e] = __uint_as_float(s[1]);
      }
      const int n = n0 + wc * WN + q * 32 + coff;
      if (m >= p.M || n >= p.Cout) continue;
      u32x4 r = {0u, 0u, 0u, 0u};
      if (p.res) {
        if constexpr (RES_PF) r = e_res[i][q];
        else r = *reinterpret_cast<const u32x4*>(p.res + (size_t)m * p.ldr + n);
      }
      float v[8] = {lo[0] + e_bias[q][0], lo[1] + e_bias[q][1], lo[2] + e_bias[q][2], lo[3] + e_bias[q][3],
                    hi[0] + e_bias[q][4], hi[1] + e_bias[q][5], hi[2] + e_bias[q][6], hi[3] + e_bias[q][7]};
      if (p.res && !post) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          v[2 * e] += __uint_as_float(r[e] << 16);
          v[2 * e + 1] += __uint_as_float(r[e] & 0xffff0000u);
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
          v[2 * e] += __uint_as_float(r[e] << 16);
          v[2 * e + 1] += __uint_as_float(r[e] & 0xffff0000u);
        }
      }
      u32x4 o;
#pragma unroll
      for (int e = 0; e < 4; ++e) o[e] = pack2(v[2 * e], v[2 * e + 1]);
      *reinterpret_cast<u32x4*>(p.y + (size_t)m * p.ldy + n) = o;
    }
    if constexpr (TAIL) {                        // 4 consecutive channels, 8-byte store
      if (m >= p.M || ntail >= p.Cout) continue;
      const f32x4 a = acc[NI - 1][i];
      uint2 r = {0u, 0u};
      if (p.res) {
        if constexpr (RES_PF) r = e_rtail[i];
        else r = *reinterpret_cast<const uint2*>(p.res + (size_t)m * p.ldr + ntail);
      }
      float v[4] = {a[0] + e_btail[0], a[1] + e_btail[1], a[2] + e_btail[2], a[3] + e_btail[3]};
      const float rv[4] = {__uint_as_float(r.x << 16), __uint_as_float(r.x & 0xffff0000u),
                           __uint_as_float(r.y << 16), __uint_as_float(r.y & 0xffff0000u)};
      if (p.res && !post) {
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] += rv[e];
      }
      if (act == 1) {
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = fmaxf(v[e], 0.f);
      } else if (act == 2) {
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = silu(v[e]);
      } else if (act == 3) {
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = gelu_erf(v[e]);
      }
      if (p.res && post) {
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] += rv[e];
      }
      *reinterpret_cast<uint2*>(p.y + (size_t)m * p.ldy + ntail) = uint2{pack2(v[0], v[1]), pack2(v[2], v[3])};
    }
  }
}


// ---------------------------------------------------------------------------------------------
// Persistent form (tuner variant 20) for the short-K, residual-free layers (ResNet reductions,
// projections: K = 384..1536, 6-24 K blocks per tile): one workgroup per CU walks tiles lid,
// lid + G, ... with ONE ring of 64-deep K blocks running across tile boundaries, so the next
// tile's first block is in flight while the current tile finishes its last block and stores its
// epilogue — the per-tile ring fill that the one-shot grid pays with every new workgroup is
// hidden (gemm_fp8_pers2_kernel's walk, applied to the implicit-GEMM conv).  The epilogue stores
// are buffer stores that are ALWAYS issued (rows / channels past the tensor get an out-of-range
// offset), so the wait for a tile's first block — whose younger VMEM ops are exactly the previous
// tile's NST stores (plus the blocks issued after it) — is an exact counted vmcnt, never a
// drain.  Biases are read from LDS (staged once), so no VGPR-destination global load is ever
// waited on while DMAs are in flight.
// RES: a residual added in the epilogue — each tile's residual chunks are buffer-loaded into
// registers D + 1 steps before its epilogue (after that step's wait, before its DMA issue), so
// they have D + 1 blocks of compute to land.
template <int BM, int BN, int WGM, int WGN, int NS, bool RES = false>
__global__ __launch_bounds__(64 * WGM * WGN, 1) void conv_wide_pers_kernel(ConvParams p) {
  constexpr int BK = 64, PPR = 8;
  constexpr int NW = WGM * WGN;
  static_assert(NW == 8, "8 waves");
  static_assert(NS == 2 || NS == 3, "2- or 3-slot ring");
  constexpr int D = NS - 1;
  constexpr int WM = BM / WGM, WN = BN / WGN;
  constexpr int MI = WM / 16, NI = WN / 16, NP = NI / 2;
  static_assert(NI % 2 == 0, "channel blocks in pairs");
  constexpr int RPW = 64 / PPR, RPI = RPW * NW;
  static_assert(BM % RPI == 0 && BN % RPI == 0, "tile rows in whole DMA pieces");
  constexpr int APT = BM / RPI, BPT = BN / RPI, PER = APT + BPT;
  constexpr int NST = MI * NP;                   // epilogue stores per thread and tile
  constexpr int STAGE_ELEMS = (BM + BN) * BK;
  constexpr int BIAS_FLOATS = 2048;              // Cout <= 2048 (host check)
  static_assert(NS * STAGE_ELEMS * 2 + BIAS_FLOATS * 4 <= 160 * 1024, "LDS budget");
  __shared__ __attribute__((aligned(16))) bf16_t ring[NS * STAGE_ELEMS + BIAS_FLOATS * 2];
  float* const sbias = reinterpret_cast<float*>(ring + NS * STAGE_ELEMS);

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave / WGN, wc = wave % WGN;
  const int ntn = (p.Cout + BN - 1) / BN;
  const int ntiles = ((p.M + BM - 1) / BM) * ntn;
  const int G = gridDim.x;
  const int lid = xcd_remap(blockIdx.x, G);
  if (lid >= ntiles) return;
  const int nkb = p.K / BK;
  const int nblocks = ((ntiles - lid + G - 1) / G) * nkb;   // this workgroup's K blocks, all tiles

  // biases into LDS once (before any DMA: these plain loads are waited for here, nothing else
  // is in flight yet)
  for (int c = tid; c < BIAS_FLOATS; c += 64 * NW) sbias[c] = (p.bias && c < p.Cout) ? p.bias[c] : 0.f;
  __syncthreads();

  const int lrow = wave * RPW + lane / PPR;
  const int lp = (lane & 7) ^ (lane >> 3);
  const int HoWo = p.Ho * p.Wo;
  const __amdgpu_buffer_rsrc_t rx = wide_rsrc(p.x);
  const __amdgpu_buffer_rsrc_t rw = wide_rsrc(p.w);
  const __amdgpu_buffer_rsrc_t rx2 = wide_rsrc(p.x2 ? p.x2 : p.x);
  const __amdgpu_buffer_rsrc_t ry = wide_rsrc(p.y);
  const __amdgpu_buffer_rsrc_t rr = wide_rsrc(p.res ? p.res : p.y);

  // ---- issue side: the tile whose blocks are being DMA'd (runs up to D blocks ahead) ----
  int it = lid, ikb = 0;
  int a_base[APT];
  uint32_t a_mask[APT], a2_off[APT], b_off[BPT], a_off[APT];
  int cur_tap = -1, iss_tap = 0, iss_c = 0, iss_r = 0, iss_s = 0;
  const int K1 = p.x2 ? p.K1 : p.K;
  auto setup_issue = [&](int t) __attribute__((always_inline)) {
    const int m0 = (t / ntn) * BM, n0 = (t % ntn) * BN;
#pragma unroll
    for (int i = 0; i < APT; ++i) {
      const int m = m0 + lrow + RPI * i;
      a_mask[i] = 0u;
      a_base[i] = 0;
      a2_off[i] = kWideOOB;
      a_off[i] = kWideOOB;
      if (m < p.M) {
        const int img = fdiv(m, p.mHoWo, p.lHoWo);
        const int rem = m - img * HoWo;
        const int oh = fdiv(rem, p.mWo, p.lWo);
        const int ow = rem - oh * p.Wo;
        const int ih0 = oh * p.stride - p.pad, iw0 = ow * p.stride - p.pad;
        a_base[i] = (((img * p.H + ih0) * p.W + iw0) * p.C + lp * 8) * 2;
        const int r_lo = max(0, -ih0), r_hi = min(p.R, p.H - ih0);
        const int s_lo = max(0, -iw0), s_hi = min(p.S, p.W - iw0);
        const uint32_t mr = r_hi > r_lo ? ((1u << r_hi) - 1u) & ~((1u << r_lo) - 1u) : 0u;
        const uint32_t ms = s_hi > s_lo ? ((1u << s_hi) - 1u) & ~((1u << s_lo) - 1u) : 0u;
        a_mask[i] = mr | (ms << 16);
        a2_off[i] = (uint32_t)((((img * p.H2 + oh * p.stride2) * p.W2 + ow * p.stride2) * p.C2 + lp * 8) * 2);
      }
    }
#pragma unroll
    for (int i = 0; i < BPT; ++i) {
      const int n = n0 + lrow + RPI * i;
      b_off[i] = n < p.Cout ? (uint32_t)(((long)n * p.K + lp * 8) * 2) : kWideOOB;
    }
    cur_tap = -1;
    iss_tap = iss_c = iss_r = iss_s = 0;
  };
  // DMA of block ikb of tile it into ring slot SLOT, then advance (to the next tile after its last)
  auto issue_next = [&](auto slot_tag) __attribute__((always_inline)) {
    constexpr int SLOT = decltype(slot_tag)::value;
    if (it >= ntiles) return;
    bf16_t* Xs = ring + SLOT * STAGE_ELEMS;
    bf16_t* Ws = Xs + BM * BK;
    const int k0 = ikb * BK;
    const uint32_t sb = (uint32_t)(k0 * 2);
#pragma unroll
    for (int i = 0; i < BPT; ++i) wide_dma16(rw, b_off[i], sb, Ws + (i * RPI + wave * RPW) * BK);
    if (k0 >= K1) {
      const uint32_t soff = (uint32_t)((k0 - K1) * 2);
#pragma unroll
      for (int i = 0; i < APT; ++i) wide_dma16(rx2, a2_off[i], soff, Xs + (i * RPI + wave * RPW) * BK);
    } else {
      if (iss_tap != cur_tap) {
        cur_tap = iss_tap;
        const int tap_off = ((iss_r * p.W + iss_s) * p.C) * 2;
        const uint32_t bit = (1u << iss_r) | (1u << (iss_s + 16));
#pragma unroll
        for (int i = 0; i < APT; ++i)
          a_off[i] = (a_mask[i] & bit) == bit ? (uint32_t)(a_base[i] + tap_off) : kWideOOB;
      }
      const uint32_t soff = (uint32_t)(iss_c * 2);
#pragma unroll
      for (int i = 0; i < APT; ++i) wide_dma16(rx, a_off[i], soff, Xs + (i * RPI + wave * RPW) * BK);
      iss_c += BK;
      if (iss_c >= p.Cc) {
        iss_c = 0;
        ++iss_tap;
        if (++iss_s == p.S) {
          iss_s = 0;
          ++iss_r;
        }
      }
    }
    if (++ikb == nkb) {
      ikb = 0;
      it += G;
      if (it < ntiles) setup_issue(it);
    }
  };

  // ---- compute side ----
  const int fr = lane & 15, fq = lane >> 4;
  const int coff = ((fq & 1) << 4) | ((fq >> 1) << 3);
  const int sw = fr & 7;
  int w_rd[NI], x_rd[MI];
#pragma unroll
  for (int j = 0; j < NI; ++j) w_rd[j] = BM * BK + (wc * WN + j * 16 + fr) * BK;
#pragma unroll
  for (int i = 0; i < MI; ++i) x_rd[i] = (wr * WM + i * 16 + fr) * BK;
  f32x4 acc[NI][MI];
#pragma unroll
  for (int j = 0; j < NI; ++j)
#pragma unroll
    for (int i = 0; i < MI; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto compute = [&](auto slot_tag) __attribute__((always_inline)) {
    constexpr int SLOT = decltype(slot_tag)::value;
    const bf16_t* St = ring + SLOT * STAGE_ELEMS;
#pragma unroll
    for (int kk = 0; kk < BK / 32; ++kk) {
      const int pc = ((fq + 4 * kk) ^ sw) << 3;
      bf16x8 wf[NI], xf[MI];
#pragma unroll
      for (int j = 0; j < NI; ++j) wf[j] = *reinterpret_cast<const bf16x8*>(St + w_rd[j] + pc);
#pragma unroll
      for (int i = 0; i < MI; ++i) xf[i] = *reinterpret_cast<const bf16x8*>(St + x_rd[i] + pc);
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NI; ++j)
          acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[j], xf[i], acc[j][i], 0, 0, 0);
    }
  };
  const int act = p.act & 15;
  const bool post = (p.act & 16) != 0;
  u32x4 e_res[RES ? MI : 1][RES ? NP : 1];
  auto load_res = [&](int t) __attribute__((always_inline)) {                  // tile t's residual chunks -> registers
    const int m0 = (t / ntn) * BM, n0 = (t % ntn) * BN;
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int q = 0; q < NP; ++q) {
        const int m = m0 + wr * WM + i * 16 + fr, n = n0 + wc * WN + q * 32 + coff;
        const uint32_t off = (m < p.M && n < p.Cout) ? (uint32_t)(((size_t)m * p.ldr + n) * 2) : kWideOOB;
        e_res[i][q] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rr, off, 0, 0));
      }
  };
  // epilogue of tile t: NST buffer stores per thread, always issued (out-of-range offset masks)
  auto epilogue = [&](int t) __attribute__((always_inline)) {
    const int m0 = (t / ntn) * BM, n0 = (t % ntn) * BN;
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      const int m = m0 + wr * WM + i * 16 + fr;
#pragma unroll
      for (int q = 0; q < NP; ++q) {
        f32x4 lo = acc[2 * q][i], hi = acc[2 * q + 1][i];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const auto s2 = __builtin_amdgcn_permlane16_swap(__float_as_uint(lo[e]), __float_as_uint(hi[e]), false, false);
          lo[e] = __uint_as_float(s2[0]);
          hi[e] = __uint_as_float(s2[1]);
        }
        const int n = n0 + wc * WN + q * 32 + coff;
        const bool ok = m < p.M && n < p.Cout;
        const f32x4 b0 = *reinterpret_cast<const f32x4*>(sbias + (ok ? n : 0));
        const f32x4 b1 = *reinterpret_cast<const f32x4*>(sbias + (ok ? n : 0) + 4);
        float v[8] = {lo[0] + b0[0], lo[1] + b0[1], lo[2] + b0[2], lo[3] + b0[3],
                      hi[0] + b1[0], hi[1] + b1[1], hi[2] + b1[2], hi[3] + b1[3]};
        if constexpr (RES) {
          if (!post) {
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              v[2 * e] += __uint_as_float(e_res[i][q][e] << 16);
              v[2 * e + 1] += __uint_as_float(e_res[i][q][e] & 0xffff0000u);
            }
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
        if constexpr (RES) {
          if (post) {
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              v[2 * e] += __uint_as_float(e_res[i][q][e] << 16);
              v[2 * e + 1] += __uint_as_float(e_res[i][q][e] & 0xffff0000u);
            }
          }
        }
        u32x4 o;
#pragma unroll
        for (int e = 0; e < 4; ++e) o[e] = pack2(v[2 * e], v[2 * e + 1]);
        const uint32_t off = ok ? (uint32_t)(((size_t)m * p.ldy + n) * 2) : kWideOOB;
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, o), ry, off, 0, 0);
      }
    }
#pragma unroll
    for (int j = 0; j < NI; ++j)
#pragma unroll
      for (int i = 0; i < MI; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};
  };

  setup_issue(it);
  using S0 = std::integral_constant<int, 0>;
  using S1 = std::integral_constant<int, 1>;
  using S2 = std::integral_constant<int, 2>;
  issue_next(S0{});
  if constexpr (NS == 3) issue_next(S1{});
  int ct = lid, ckb = 0;
  bool epi_prev = false;                        // the previous step ended a tile (NST stores)
  bool epi_prev2 = false;                       // ... the step before it (NS == 3)
  // step for global block g: wait for it, publish, issue block g + D, compute, maybe epilogue
  auto step = [&](int g, auto slot_tag) __attribute__((always_inline)) {
    constexpr int SLOT = decltype(slot_tag)::value;
    constexpr int PREV = SLOT == 0 ? NS - 1 : SLOT - 1;
    // younger VMEM ops than block g: the D - 1 blocks issued after it (if any) and the stores
    // of an epilogue that ran after its issue; counting fewer is only stricter
    if constexpr (D == 1) {
      if (epi_prev) wide_vm_barrier<NST>();
      else wide_vm_barrier<0>();
    } else {
      const bool more = g + 1 < nblocks;        // block g + 1 was issued (at step g - 1)
      const bool epi = epi_prev || epi_prev2;
      if (more && epi) wide_vm_barrier<PER + NST>();
      else if (more) wide_vm_barrier<PER>();
      else if (epi) wide_vm_barrier<NST>();
      else wide_vm_barrier<0>();
    }
    if constexpr (RES) {
      // (nkb >= D + 1, host check) the residual of tile ct, D + 1 blocks before its epilogue
      if (ckb == nkb - 1 - D) load_res(ct);
    }
    issue_next(std::integral_constant<int, PREV>{});
    compute(slot_tag);
    epi_prev2 = epi_prev;
    epi_prev = false;
    if (++ckb == nkb) {
      epilogue(ct);
      ct += G;
      ckb = 0;
      epi_prev = true;
    }
  };
  int g = 0;
  if constexpr (NS == 2) {
    for (; g + 2 <= nblocks; g += 2) {
      step(g, S0{});
      step(g + 1, S1{});
    }
    if (g < nblocks) step(g, S0{});
  } else {
    for (; g + 3 <= nblocks; g += 3) {
      step(g, S0{});
      step(g + 1, S1{});
      step(g + 2, S2{});
    }
    if (g < nblocks) step(g, S0{});
    if (g + 1 < nblocks) step(g + 1, S1{});
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}
}  // namespace aiko

// Same arguments as aiko_conv_buf (no occupancy / MFMA-shape options).  Host preconditions
// (checked by the binding): Cc and, with a second source, K - K1 are multiples of 64; R*S <= 32;
// Cout % 8 == 0; every operand fits 2^31 bytes.
extern "C" int aiko_conv_wide(const void* x, const void* w, const float* bias, const void* res,
                              void* y, int H, int W, int C, int Cc, int R, int S, int stride,
                              int pad, int Ho, int Wo, int M, int Cout, int K, int act, int ldy,
                              int ldr, int bm, int bn, const void* x2, int K1, int H2, int W2,
                              int C2, int stride2, int occ, hipStream_t stream) {
  using namespace aiko;
  if (Cc % 64 || R * S > 32 || R > 16 || S > 16 || (x2 && (K - K1) % 64) || Cout % 8) return -1;
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
  dim3 grid(((M + bm - 1) / bm) * ((Cout + bn - 1) / bn));
  if (occ == 18) {                    // exact-N tiles: bn = the channels computed per tile
    if (Cout % 16) return -1;
    if (bm == 256 && bn == 80)        // 8 waves of 32 pixels x 80 channels (5 blocks), 128-row weight DMA
      conv_wide_kernel<256, 128, 8, 1, 2, true, 1, 64, 80><<<grid, 512, 0, stream>>>(p);
    else if (bm == 128 && bn == 80)   // 8 waves of 16 x 80, 2 workgroups per CU
      conv_wide_kernel<128, 128, 8, 1, 2, true, 2, 64, 80><<<grid, 512, 0, stream>>>(p);
    else if (bm == 256 && bn == 144)  // 8 waves of 32 x 144 (9 blocks), 192-row weight DMA
      conv_wide_kernel<256, 192, 8, 1, 2, true, 1, 64, 144><<<grid, 512, 0, stream>>>(p);
    else if (bm == 128 && bn == 144)  // 8 waves of 16 x 144, 2 workgroups per CU (64 + 64 KB ring)
      conv_wide_kernel<128, 192, 8, 1, 2, true, 1, 64, 144><<<grid, 512, 0, stream>>>(p);
    else
      return -1;
  } else if (occ == 20) {             // persistent walk (host checks: K >= 3 blocks with a residual)
    if (Cout > 2048 || (res != nullptr && K < 192)) return -1;
    int dev = 0, cus = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) cus = 256;
    const char* cap = getenv("AIKO_CONV_PERS_GRID");   // tests: force several tiles per workgroup
    if (cap && atoi(cap) > 0) cus = atoi(cap);
    const int ntiles = (int)grid.x;
    dim3 pg(ntiles < cus ? ntiles : cus);
    const bool r = res != nullptr;
    if (bm == 256 && bn == 256 && !r)
      conv_wide_pers_kernel<256, 256, 2, 4, 2><<<pg, 512, 0, stream>>>(p);
    else if (bm == 256 && bn == 128 && !r)
      conv_wide_pers_kernel<256, 128, 4, 2, 3><<<pg, 512, 0, stream>>>(p);
    else if (bm == 128 && bn == 256 && !r)
      conv_wide_pers_kernel<128, 256, 2, 4, 3><<<pg, 512, 0, stream>>>(p);
    else if (bm == 256 && bn == 128)
      conv_wide_pers_kernel<256, 128, 4, 2, 3, true><<<pg, 512, 0, stream>>>(p);
    else if (bm == 128 && bn == 256)
      conv_wide_pers_kernel<128, 256, 2, 4, 3, true><<<pg, 512, 0, stream>>>(p);
    else
      return -1;
  } else if (occ == 19) {             // 4 waves of 64 x 64 (half the fragment reads per MFMA of
                                      // the 8-wave 128 x 128 form), 2-slot ring, 2 workgroups per CU
    if (bm == 128 && bn == 128)
      conv_wide_kernel<128, 128, 2, 2, 2, true, 2><<<grid, 256, 0, stream>>>(p);
    else if (bm == 128 && bn == 256)  // 4 waves of 64 x 128, 1 workgroup per CU (3-slot ring)
      conv_wide_kernel<128, 256, 2, 2, 3, true, 1><<<grid, 256, 0, stream>>>(p);
    else
      return -1;
  } else if (occ <= 1) {                     // 8 waves, one workgroup per CU
    if (bm == 256 && bn == 256)
      conv_wide_kernel<256, 256, 2, 4, 2, false, 1><<<grid, 512, 0, stream>>>(p);
    else if (bm == 256 && bn == 128)
      conv_wide_kernel<256, 128, 4, 2, 3, true, 1><<<grid, 512, 0, stream>>>(p);
    else if (bm == 128 && bn == 256)
      conv_wide_kernel<128, 256, 2, 4, 3, true, 1><<<grid, 512, 0, stream>>>(p);
    else if (bm == 256 && bn == 64)
      conv_wide_kernel<256, 64, 4, 2, 3, true, 1><<<grid, 512, 0, stream>>>(p);
    else if (bm == 128 && bn == 128)
      conv_wide_kernel<128, 128, 2, 4, 3, true, 1><<<grid, 512, 0, stream>>>(p);
    else
      return -1;
  } else if (occ == 11) {             // 8 waves, 32-deep K blocks in a 4-slot ring
    if (bm == 256 && bn == 256)
      conv_wide_kernel<256, 256, 2, 4, 4, false, 1, 32><<<grid, 512, 0, stream>>>(p);
    else if (bm == 256 && bn == 128)
      conv_wide_kernel<256, 128, 4, 2, 4, true, 1, 32><<<grid, 512, 0, stream>>>(p);
    else if (bm == 128 && bn == 256)
      conv_wide_kernel<128, 256, 2, 4, 4, true, 1, 32><<<grid, 512, 0, stream>>>(p);
    else
      return -1;
  } else {                            // several workgroups per CU
    if (bm == 128 && bn == 128)       // 8 waves, 2-slot ring (64 KB), 2 per CU
      conv_wide_kernel<128, 128, 2, 4, 2, true, 2><<<grid, 512, 0, stream>>>(p);
    else if (bm == 256 && bn == 64)   // 8 waves, 2-slot ring (80 KB), 2 per CU
      conv_wide_kernel<256, 64, 4, 2, 2, true, 2><<<grid, 512, 0, stream>>>(p);
    else if (bm == 128 && bn == 64)   // 4 waves of 64 x 32, 3-slot ring (72 KB), 2 per CU
      conv_wide_kernel<128, 64, 2, 2, 3, true, 2><<<grid, 256, 0, stream>>>(p);
    else if (bm == 64 && bn == 128)   // 4 waves of 32 x 64, 3-slot ring (72 KB), 2 per CU
      conv_wide_kernel<64, 128, 2, 2, 3, true, 2><<<grid, 256, 0, stream>>>(p);
    else if (bm == 64 && bn == 64)    // 4 waves of 32 x 32, 3-slot ring (48 KB), 3 per CU
      conv_wide_kernel<64, 64, 2, 2, 3, true, 3><<<grid, 256, 0, stream>>>(p);
    else
      return -1;
  }
  return (int)hipGetLastError();
}
