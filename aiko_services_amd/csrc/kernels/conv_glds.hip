// Implicit-GEMM convolution, global_load_lds variant (gfx950 LDS-DMA staging).
//
// Same math, tiles, epilogue and LDS image as conv_igemm.hip, but operands go HBM -> LDS with
// `global_load_lds_dwordx4` (no VGPR staging, no ds_write pass) through a 3-slot ring: stage
// kb+2 is issued right after the barrier that retires stage kb, so two K-blocks stay in flight
// across the barrier.  Synchronisation follows the LDS-DMA rules:
//   * RAW: each wave retires its own DMAs for stage kb with a COUNTED `s_waitcnt vmcnt(PER)`
//     (PER = DMA instructions per stage), then a raw `s_barrier`; only then is the slot read;
//   * WAR: a slot is re-issued one iteration after its last ds_read, behind a barrier that
//     every wave reaches after `s_waitcnt lgkmcnt(0)` (its reads of that slot have landed);
//   * never `__syncthreads()` inside the loop: its fence would drain vmcnt to 0 (the in-flight
//     stage), one LDS array only (a second __shared__ object makes hipcc drain before reads).
// The DMA destination is lane-linear (wave base + lane * 16 B), so the XOR swizzle moves to
// the SOURCE: lane l of a row group fetches logical 16-B piece (l & 7) ^ (row & 7) into
// physical slot l & 7 — exactly the image the fragment reads of the register-staged kernel
// expect.  Conv zero padding (and rows / channels past the edge) are fetched from a zeroed
// 16-B global page instead of being predicated away.
#include "conv_common.h"

namespace aiko {

// B-tile rows staged per K block: BN rounded up to the 32-row DMA granule (exact-N tiles)
template <int BN>
constexpr int glds_bn_pad() {
  return (BN + 31) / 32 * 32;
}
// ring slots: 3 (two stages in flight) where 2 workgroups still fit the 160 KB LDS, else 2
template <int BM, int BN>
constexpr int glds_slots() {
  return (BM + glds_bn_pad<BN>()) * 64 * 2 * 3 <= 80 * 1024 ? 3 : 2;
}
template <int BM, int BN>
constexpr int glds_occupancy() {
  return (BM == 64 && BN == 64) ? 3 : 2;
}

__device__ __forceinline__ void glds16(const void* g, bf16_t* lds_wave_base) {
  __builtin_amdgcn_global_load_lds(g, reinterpret_cast<__attribute__((address_space(3))) void*>(
                                          reinterpret_cast<uintptr_t>(lds_wave_base)),
                                   16, 0, 0);
}

template <int N>
__device__ __forceinline__ void wait_vm_barrier() {
  asm volatile("s_waitcnt vmcnt(%0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::"n"(N) : "memory");
}

// TAIL: a following 1x1 conv fused into the epilogue (YOLOv8 detect head: 3x3 80 -> 80 + SiLU,
// then the 1x1 80 -> 80 class logits; 3x3 64 -> 64, then the 1x1 64 -> 64 box distribution).
// The activated 3x3 tile is packed to bf16 in LDS (K columns BN..K2 zeroed) and never written to
// HBM; the 1x1's weights ([N2][ldw2], K zero-padded
// to a multiple of 64 as every conv spec is) come straight from L2 as B fragments.
struct GldsTail {
  const bf16_t* w2;
  const float* b2;
  bf16_t* y2;
  int ldy2, ldw2, act2;   // act2: 0 none, 2 SiLU on the 1x1's output
  // dmode 1 / 2: YOLOv8 decode in the epilogue instead of storing the 1x1's output (the detect
  // head's box / class branch): 1 = DFL expectation of the 4 x 16 box bins -> xyxy boxes,
  // 2 = max / argmax over the first nc class logits -> sigmoid score + class.  Values are rounded
  // to bf16 first, as the stored head output would be (ops.detect.yolo_decode semantics).
  int dmode, nc, HW, Wl, lstride, astart, A;
  float4* boxes;
  float* scores;
  int* cls;
};

// reductions over lanes l, l^16, l^32, l^48 (gfx950 v_permlane16/32_swap with both operands = v
// return the two halves of the exchange: combining the pair reduces over the xor partner)
__device__ __forceinline__ float tail_sum4(float v) {
  const auto a = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = __uint_as_float(a[0]) + __uint_as_float(a[1]);
  const auto b = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(b[0]) + __uint_as_float(b[1]);
}
__device__ __forceinline__ float tail_max4(float v) {
  const auto a = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = fmaxf(__uint_as_float(a[0]), __uint_as_float(a[1]));
  const auto b = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(b[0]), __uint_as_float(b[1]));
}
__device__ __forceinline__ int tail_min4(int v) {
  const auto a = __builtin_amdgcn_permlane32_swap((unsigned)v, (unsigned)v, false, false);
  v = min((int)a[0], (int)a[1]);
  const auto b = __builtin_amdgcn_permlane16_swap((unsigned)v, (unsigned)v, false, false);
  return min((int)b[0], (int)b[1]);
}
__device__ __forceinline__ float tail_bf16(float x) { return __uint_as_float((pack2(x, 0.f) & 0xffffu) << 16); }

// WGM x WGN waves (2 x 2; exact-N tiles such as BN = 80: 4 x 1, each wave all BN columns)
template <int BM, int BN, int WGM = 2, int WGN = 2, bool TAIL = false>
__global__ __launch_bounds__(256, (glds_occupancy<BM, BN>())) void conv_glds_kernel(ConvParams p,
                                                                                 const bf16_t* zero,
                                                                                 GldsTail tl) {
  static_assert(WGM * WGN == 4, "four waves");
  constexpr int BK = 64;
  constexpr int NS = glds_slots<BM, BN>();     // LDS ring slots
  constexpr int D = NS - 1;                    // stages in flight
  constexpr int WM = BM / WGM, WN = BN / WGN;
  constexpr int MI = WM / 16, NI = WN / 16;
  static_assert(WM % 16 == 0 && WN % 16 == 0, "whole 16 x 16 fragments per wave");
  constexpr int BNP = glds_bn_pad<BN>();       // staged B rows (rows past BN read the zero page)
  constexpr int APT = BM / 32, BPT = BNP / 32; // DMA instructions per thread per stage
  constexpr int PER = APT + BPT;
  constexpr int STAGE_ELEMS = (BM + BNP) * BK;
  constexpr int CPAD = 4;
  constexpr int EPI_BYTES = BM * (BN + CPAD) * 4;
  constexpr int RING_BYTES = NS * STAGE_ELEMS * 2;
  static_assert(!TAIL || BN == 64 || BN == 80 || BN == 128, "tail: 64-, 80- or 128-channel tiles");
  constexpr int K2 = (BN + 31) / 32 * 32;      // tail: the 1x1's K (zero-padded to the MFMA depth)
  constexpr int TP = K2 + 8;                   // tail: bf16 row pitch of the activated tile
  constexpr int TAIL_BYTES = TAIL ? BM * TP * 2 : 0;
  constexpr int LDS_NEED = EPI_BYTES + TAIL_BYTES;
  constexpr int LDS_BYTES = LDS_NEED > RING_BYTES ? LDS_NEED : RING_BYTES;
  __shared__ __attribute__((aligned(16))) unsigned char smem[LDS_BYTES];
  bf16_t* ring = reinterpret_cast<bf16_t*>(smem);

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wr = wave / WGN, wc = wave % WGN;
  const int ntn = (p.Cout + BN - 1) / BN;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int tile_n = bid % ntn, tile_m = bid / ntn;
  const int m0 = tile_m * BM, n0 = tile_n * BN;

  // DMA lane mapping: instruction i of wave w covers rows i*32 + w*8 .. +7, lane l -> row
  // (l >> 3) of that group, physical slot (l & 7), logical piece lp = (l & 7) ^ (l >> 3)
  const int lrow = wave * 8 + (lane >> 3);
  const int lp = (lane & 7) ^ (lane >> 3);
  const int HoWo = p.Ho * p.Wo;
  int a_base[APT], a_ih[APT], a_iw[APT], a2_base[APT];
#pragma unroll
  for (int i = 0; i < APT; ++i) {
    const int m = m0 + lrow + 32 * i;
    if (m < p.M) {
      const int img = fdiv(m, p.mHoWo, p.lHoWo);
      const int rem = m - img * HoWo;
      const int oh = fdiv(rem, p.mWo, p.lWo);
      const int ow = rem - oh * p.Wo;
      a_ih[i] = oh * p.stride - p.pad;
      a_iw[i] = ow * p.stride - p.pad;
      a_base[i] = ((img * p.H + a_ih[i]) * p.W + a_iw[i]) * p.C;
      a2_base[i] = ((img * p.H2 + oh * p.stride2) * p.W2 + ow * p.stride2) * p.C2;
    } else {
      a_ih[i] = -(1 << 28);
      a_iw[i] = 0;
      a_base[i] = 0;
      a2_base[i] = -1;
    }
  }
  const bf16_t* b_src[BPT];
#pragma unroll
  for (int i = 0; i < BPT; ++i) {
    const int n = n0 + lrow + 32 * i;
    b_src[i] = n < p.Cout && lrow + 32 * i < BN ? p.w + (long)n * p.K + lp * 8 : nullptr;
  }

  // epilogue operands, prefetched before the K loop (ordinary loads, older than every DMA).
  // Chunk c = tid + 256 i of the tile's BM x BN / 8 eight-column chunks: row c / CPR, column
  // chunk c % CPR — for power-of-two CPR every i has the same column chunk (bias loaded once)
  constexpr int CPR = BN / 8, CHUNKS = BM * CPR, CPT = CHUNKS / 256;
  static_assert(CHUNKS % 256 == 0, "tile must give every thread whole chunks");
  constexpr bool FIXED_CC = 256 % CPR == 0;
  auto e_cc_of = [&](int i) { return (tid + 256 * i) % CPR; };
  auto e_row_of = [&](int i) { return (tid + 256 * i) / CPR; };
  // (otherwise the bias is read per chunk in the epilogue: no registers held over the K loop)
  auto load_bias = [&](int i, float (&b)[8]) {
    const int en = n0 + e_cc_of(i) * 8;
#pragma unroll
    for (int e = 0; e < 8; ++e) b[e] = 0.f;
    if (p.bias && en < p.Cout) {
      const f32x4 b0 = *reinterpret_cast<const f32x4*>(p.bias + en);
      const f32x4 b1 = *reinterpret_cast<const f32x4*>(p.bias + en + 4);
      b[0] = b0[0]; b[1] = b0[1]; b[2] = b0[2]; b[3] = b0[3];
      b[4] = b1[0]; b[5] = b1[1]; b[6] = b1[2]; b[7] = b1[3];
    }
  };
  float e_bias[8];
  if constexpr (FIXED_CC) load_bias(0, e_bias);
  u32x4 e_res[CPT];
  if (p.res) {
#pragma unroll
    for (int i = 0; i < CPT; ++i) {
      const int m = m0 + e_row_of(i), en = n0 + e_cc_of(i) * 8;
      const bool ok = m < p.M && en < p.Cout;
      e_res[i] = *reinterpret_cast<const u32x4*>(p.res + (ok ? (size_t)m * p.ldr + en : 0));
    }
  }

  // tail: the 1x1's weight fragments (A operand: 16 output channels x 32 K) and bias, loaded
  // before the first DMA so they land under the K loop (the first counted wait retires them)
  constexpr int NI2 = BN / 16, KS2 = K2 / 32;
  constexpr bool W2_PRE = TAIL && KS2 * NI2 <= 16;
  bf16x8 w2f[W2_PRE ? KS2 : 1][W2_PRE ? NI2 : 1];
  f32x4 b2v[TAIL ? NI2 : 1];
  if constexpr (TAIL) {
    const int fr0 = lane & 15, fq0 = lane >> 4;
    if constexpr (W2_PRE) {
#pragma unroll
      for (int ks = 0; ks < KS2; ++ks)
#pragma unroll
        for (int j = 0; j < NI2; ++j)
          w2f[ks][j] = *reinterpret_cast<const bf16x8*>(tl.w2 + (size_t)(16 * j + fr0) * tl.ldw2 + 32 * ks + 8 * fq0);
    }
#pragma unroll
    for (int j = 0; j < NI2; ++j) b2v[j] = *reinterpret_cast<const f32x4*>(tl.b2 + 16 * j + 4 * fq0);
  }

  const bf16_t* zp = zero;
  auto issue = [&](int kb, int slot) {
    bf16_t* As = ring + slot * STAGE_ELEMS;
    bf16_t* Bs = As + BM * BK;
    if (p.x2 && kb * BK >= p.K1) {
      const int c2 = kb * BK - p.K1 + lp * 8;
#pragma unroll
      for (int i = 0; i < APT; ++i) {
        const bf16_t* g = a2_base[i] >= 0 ? p.x2 + (a2_base[i] + c2) : zp;
        glds16(g, As + (i * 32 + wave * 8) * BK);
      }
    } else {
      const int koff = kb * BK + lp * 8;
      const int tap = fdiv(koff, p.mCc, p.lCc);
      const int c = koff - tap * p.Cc;
      const int r = fdiv(tap, p.mS, p.lS);
      const int s = tap - r * p.S;
      const int tap_off = (r * p.W + s) * p.C + c;
#pragma unroll
      for (int i = 0; i < APT; ++i) {
        const int ih = a_ih[i] + r, iw = a_iw[i] + s;
        const bool ok = (unsigned)ih < (unsigned)p.H && (unsigned)iw < (unsigned)p.W;
        const bf16_t* g = ok ? p.x + (a_base[i] + tap_off) : zp;
        glds16(g, As + (i * 32 + wave * 8) * BK);
      }
    }
#pragma unroll
    for (int i = 0; i < BPT; ++i) {
      const bf16_t* g = b_src[i] ? b_src[i] + kb * BK : zp;
      glds16(g, Bs + (i * 32 + wave * 8) * BK);
    }
  };

  f32x4 acc[MI][NI];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nkb = p.K / BK;
#pragma unroll
  for (int j = 0; j < D; ++j)
    if (j < nkb) issue(j, j);
  const int fr = lane & 15, fq = lane >> 4;

  int slot = 0;
  for (int kb = 0; kb < nkb; ++kb) {
    // retire stage kb (this wave's DMAs), keep the younger ones in flight, then barrier
    if (D == 2 && kb + 1 < nkb) {
      wait_vm_barrier<PER>();
    } else {
      wait_vm_barrier<0>();
    }
    if (kb + D < nkb) issue(kb + D, slot == 0 ? NS - 1 : slot - 1);   // the slot of stage kb-1
    const bf16_t* As = ring + slot * STAGE_ELEMS;
    const bf16_t* Bs = As + BM * BK;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8 af[MI], bfr[NI];
      const int pc = fq + 4 * kk;
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        const int row = wr * WM + i * 16 + fr;
        af[i] = *reinterpret_cast<const bf16x8*>(As + row * BK + ((pc ^ (row & 7)) << 3));
      }
#pragma unroll
      for (int j = 0; j < NI; ++j) {
        const int row = wc * WN + j * 16 + fr;
        bfr[j] = *reinterpret_cast<const bf16x8*>(Bs + row * BK + ((pc ^ (row & 7)) << 3));
      }
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NI; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    slot = slot == NS - 1 ? 0 : slot + 1;
  }
  wait_vm_barrier<0>();                // every wave's last fragment reads done before Cs reuse

  // ---- epilogue (as conv_igemm) ----
  float* Cs = reinterpret_cast<float*>(smem);
  constexpr int LDC = BN + CPAD;
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j) {
      const int col = wc * WN + j * 16 + fr;
#pragma unroll
      for (int e = 0; e < 4; ++e) Cs[(wr * WM + i * 16 + fq * 4 + e) * LDC + col] = acc[i][j][e];
    }
  __syncthreads();
  const bool post = (p.act & 16) != 0;
  const int act = p.act & 15;
#pragma unroll
  for (int i = 0; i < CPT; ++i) {
    const int row = e_row_of(i), cc = e_cc_of(i);
    const int m = m0 + row, e_n = n0 + cc * 8;
    if (m >= p.M || e_n >= p.Cout) continue;
    const f32x4 v0 = *reinterpret_cast<const f32x4*>(Cs + row * LDC + cc * 8);
    const f32x4 v1 = *reinterpret_cast<const f32x4*>(Cs + row * LDC + cc * 8 + 4);
    float v[8] = {v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
    if constexpr (!FIXED_CC) load_bias(i, e_bias);
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
    if constexpr (TAIL)
      *reinterpret_cast<u32x4*>(smem + EPI_BYTES + (row * TP + cc * 8) * 2) = o;
    else
      *reinterpret_cast<u32x4*>(p.y + (size_t)m * p.ldy + e_n) = o;
  }
  if constexpr (TAIL) {
    bf16_t* Ts = reinterpret_cast<bf16_t*>(smem + EPI_BYTES);
    // K columns BN..K2 of every row are zero (16-B chunks); rows past M stay whatever the
    // skipped chunks left — their outputs are never stored
    constexpr int ZC = (K2 - BN) / 8;
    if constexpr (ZC > 0)
      for (int c = tid; c < BM * ZC; c += 256)
        *reinterpret_cast<u32x4*>(Ts + (c / ZC) * TP + BN + (c % ZC) * 8) = u32x4{0u, 0u, 0u, 0u};
    __syncthreads();                   // activated tile complete; every Cs read done
    // 1x1, transposed (weights on the A side): out^T[16 j + 4 fq + e][(BM / 4) w + 16 i + fr]
    // over K2 (32-deep steps), each wave a quarter of the pixels and all BN channels — every lane
    // ends with 4 consecutive channels of one pixel: bias, activation and an 8-byte store
    // straight from the accumulators
    constexpr int MI2 = BM / 4 / 16;
    f32x4 acc2[MI2][NI2];
#pragma unroll
    for (int i = 0; i < MI2; ++i)
#pragma unroll
      for (int j = 0; j < NI2; ++j) acc2[i][j] = b2v[j];
#pragma unroll
    for (int ks = 0; ks < KS2; ++ks) {
      bf16x8 tf[MI2], wf[NI2];
#pragma unroll
      for (int i = 0; i < MI2; ++i)
        tf[i] = *reinterpret_cast<const bf16x8*>(Ts + (wave * (BM / 4) + 16 * i + fr) * TP + 32 * ks + 8 * fq);
#pragma unroll
      for (int j = 0; j < NI2; ++j) {
        if constexpr (W2_PRE)
          wf[j] = w2f[ks][j];
        else
          wf[j] = *reinterpret_cast<const bf16x8*>(tl.w2 + (size_t)(16 * j + fr) * tl.ldw2 + 32 * ks + 8 * fq);
      }
#pragma unroll
      for (int i = 0; i < MI2; ++i)
#pragma unroll
        for (int j = 0; j < NI2; ++j)
          acc2[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[j], tf[i], acc2[i][j], 0, 0, 0);
    }
    if (tl.dmode == 1) {                 // box branch: DFL -> xyxy (4 sides x 16 bins = NI2 x 16)
#pragma unroll
      for (int i = 0; i < MI2; ++i) {
        const int m = m0 + wave * (BM / 4) + 16 * i + fr;
        float dist[NI2];
#pragma unroll
        for (int j = 0; j < NI2; ++j) {
          float v[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = tail_bf16(acc2[i][j][e]);
          const float mx = tail_max4(fmaxf(fmaxf(v[0], v[1]), fmaxf(v[2], v[3])));
          float se = 0.f, sk = 0.f;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float ex = __expf(v[e] - mx);
            se += ex;
            sk += ex * (float)(4 * fq + e);
          }
          dist[j] = tail_sum4(sk) / tail_sum4(se);
        }
        if (m < p.M && fq == 0) {
          const int b = m / tl.HW, r = m - b * tl.HW, h = r / tl.Wl, w = r - h * tl.Wl;
          const float sc = (float)tl.lstride, ax = w + 0.5f, ay = h + 0.5f;
          tl.boxes[(long)b * tl.A + tl.astart + r] =
              make_float4((ax - dist[0]) * sc, (ay - dist[1]) * sc, (ax + dist[2]) * sc, (ay + dist[3]) * sc);
        }
      }
      return;
    }
    if (tl.dmode == 2) {                 // class branch: max / argmax (lowest index on ties)
#pragma unroll
      for (int i = 0; i < MI2; ++i) {
        const int m = m0 + wave * (BM / 4) + 16 * i + fr;
        float best = -INFINITY;
        int bi = 0x7fffffff;
#pragma unroll
        for (int j = 0; j < NI2; ++j)
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int c = 16 * j + 4 * fq + e;
            const float v = tail_bf16(acc2[i][j][e]);
            if (c < tl.nc && v > best) { best = v; bi = c; }
          }
        const float g = tail_max4(best);
        int cand = tail_min4(best == g ? bi : 0x7fffffff);
        if (cand == 0x7fffffff) cand = 0;
        if (m < p.M && fq == 0) {
          const int b = m / tl.HW, r = m - b * tl.HW;
          const long idx = (long)b * tl.A + tl.astart + r;
          tl.scores[idx] = 1.f / (1.f + __expf(-g));
          tl.cls[idx] = cand;
        }
      }
      return;
    }
#pragma unroll
    for (int i = 0; i < MI2; ++i) {
      const int m = m0 + wave * (BM / 4) + 16 * i + fr;
      if (m >= p.M) continue;
#pragma unroll
      for (int j = 0; j < NI2; ++j) {
        f32x4 v = acc2[i][j];
        if (tl.act2 == 2) v = f32x4{silu(v[0]), silu(v[1]), silu(v[2]), silu(v[3])};
        uint2 o;
        o.x = pack2(v[0], v[1]);
        o.y = pack2(v[2], v[3]);
        *reinterpret_cast<uint2*>(tl.y2 + (size_t)m * tl.ldy2 + 16 * j + 4 * fq) = o;
      }
    }
  }
}

}  // namespace aiko

// Same arguments as aiko_conv_igemm plus the zero page (>= 16 B of zeros in device memory).
extern "C" int aiko_conv_glds(const void* x, const void* w, const float* bias, const void* res,
                              void* y, int H, int W, int C, int Cc, int R, int S, int stride,
                              int pad, int Ho, int Wo, int M, int Cout, int K, int act, int ldy,
                              int ldr, int bm, int bn, const void* x2, int K1, int H2, int W2,
                              int C2, int stride2, const void* zero, hipStream_t stream) {
  using namespace aiko;
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
  const bf16_t* z = static_cast<const bf16_t*>(zero);
  dim3 grid(((M + bm - 1) / bm) * ((Cout + bn - 1) / bn)), block(256);
  if (bm == 128 && bn == 128) {
    conv_glds_kernel<128, 128><<<grid, block, 0, stream>>>(p, z, GldsTail{});
  } else if (bm == 128 && bn == 64) {
    conv_glds_kernel<128, 64><<<grid, block, 0, stream>>>(p, z, GldsTail{});
  } else if (bm == 64 && bn == 64) {
    conv_glds_kernel<64, 64><<<grid, block, 0, stream>>>(p, z, GldsTail{});
  } else if (bm == 64 && bn == 128) {
    conv_glds_kernel<64, 128><<<grid, block, 0, stream>>>(p, z, GldsTail{});
  } else if (bm == 128 && bn == 80) {              // exact-N tiles (YOLO's 80-class head convs)
    conv_glds_kernel<128, 80, 4, 1><<<grid, block, 0, stream>>>(p, z, GldsTail{});
  } else if (bm == 256 && bn == 80) {
    conv_glds_kernel<256, 80, 4, 1><<<grid, block, 0, stream>>>(p, z, GldsTail{});
  } else {
    return -1;
  }
  return (int)hipGetLastError();
}

// R x S conv with an exact N-channel tile (N = 80: 128 x 80, 4 x 1 waves; N = 64: 128 x 64, 2 x 2;
// N = 128: 64 x 128, 2 x 2)
// and a fused trailing 1x1 N -> N (+ bias, no activation) in the epilogue:
// y2 [M][ldy2] = act2((act(conv(x) + bias)) . w2[:, :N]^T + b2).  Geometry as aiko_conv_glds (no residual,
// no second source).
extern "C" int aiko_conv_glds_tail(const void* x, const void* w, const float* bias, int H, int W, int C, int Cc,
                                   int R, int S, int stride, int pad, int Ho, int Wo, int M, int K, int N, int act,
                                   const void* w2, const float* b2, void* y2, int ldy2, int ldw2, int act2, const void* zero,
                                   const int* dec, void* boxes, float* scores, int* cls, hipStream_t stream) {
  using namespace aiko;
  ConvParams p;
  p.x = static_cast<const bf16_t*>(x);
  p.w = static_cast<const bf16_t*>(w);
  p.bias = bias;
  p.res = nullptr;
  p.y = nullptr;
  p.H = H; p.W = W; p.C = C; p.Cc = Cc; p.R = R; p.S = S;
  p.stride = stride; p.pad = pad; p.Ho = Ho; p.Wo = Wo; p.M = M; p.Cout = N; p.K = K;
  p.act = act; p.ldy = N; p.ldr = 0;
  p.x2 = nullptr;
  p.K1 = K; p.H2 = 1; p.W2 = 1; p.C2 = 8; p.stride2 = 1;
  conv_params_finalize(p);
  GldsTail tl{};
  tl.w2 = static_cast<const bf16_t*>(w2);
  tl.b2 = b2;
  tl.y2 = static_cast<bf16_t*>(y2);
  tl.ldy2 = ldy2; tl.ldw2 = ldw2; tl.act2 = act2;
  if (dec) {
    tl.dmode = dec[0]; tl.nc = dec[1]; tl.HW = Ho * Wo; tl.Wl = Wo; tl.lstride = dec[2]; tl.astart = dec[3];
    tl.A = dec[4];
    tl.boxes = static_cast<float4*>(boxes); tl.scores = scores; tl.cls = cls;
  }
  dim3 grid((M + 127) / 128), block(256);
  if (N == 80)
    conv_glds_kernel<128, 80, 4, 1, true><<<grid, block, 0, stream>>>(p, static_cast<const bf16_t*>(zero), tl);
  else if (N == 64)
    conv_glds_kernel<128, 64, 2, 2, true><<<grid, block, 0, stream>>>(p, static_cast<const bf16_t*>(zero), tl);
  else if (N == 128)   // 64 x 128 tiles (the 128-row form would hold 102 KB of LDS: one workgroup per CU)
    conv_glds_kernel<64, 128, 2, 2, true><<<dim3((M + 63) / 64), block, 0, stream>>>(p, static_cast<const bf16_t*>(zero), tl);
  else
    return -1;
  return (int)hipGetLastError();
}
