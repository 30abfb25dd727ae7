// Implicit-GEMM convolution, buffer-LDS-DMA variant (gfx950 `buffer_load_dwordx4 ... lds`).
//
// Same tile, LDS image, MFMA loop and epilogue as conv_glds.hip, but every operand piece is
// fetched through a buffer resource: the per-lane byte offset (VGPR) is fixed for a whole conv
// tap and the K-block position inside the tap is the scalar `soffset`, so the steady-state
// k-loop issues its DMAs without any vector address arithmetic.  PMC on the global_load_lds
// kernel showed ~5 VALU instructions per MFMA (per-lane tap division, bounds tests and 64-bit
// address math on every piece, every K block) — the VALU issue, not the matrix pipe, set the
// pace of the compute-bound layers.  Here:
//   * a K block (64 channels) never straddles a tap (host requires Cc % 64 == 0), so the tap
//     (r, s) and channel offset are scalars, advanced incrementally (no divisions);
//   * per-lane offsets are recomputed only when the tap changes (a wave-uniform branch): the
//     piece's row is valid for tap t iff bit t of a mask precomputed in the prologue is set;
//     invalid rows (conv padding, rows past M, weight rows past Cout) get an offset beyond the
//     buffer's num_records, which the hardware returns as zeros — no zero page, no selects;
//   * the K loop is unrolled by the ring depth so every LDS slot address is an immediate.
// Synchronisation is conv_glds.hip's: counted `s_waitcnt vmcnt(N)` + raw `s_barrier`, one LDS
// array, never __syncthreads() inside the loop.
#include <type_traits>

#include "conv_common.h"

namespace aiko {

namespace {

constexpr uint32_t kBufOOB = 0x80000000u;        // offsets >= num_records read as zero
constexpr uint32_t kBufRecords = 0x7ffffff0u;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)kBufRecords, 0x00020000);
}

__device__ __forceinline__ void buf16(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff, void* lds) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(
      r, reinterpret_cast<__attribute__((address_space(3))) void*>(reinterpret_cast<uintptr_t>(lds)), 16,
      voff, soff, 0, 0);
}

template <int N>
__device__ __forceinline__ void vm_barrier() {
  asm volatile("s_waitcnt vmcnt(%0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::"n"(N) : "memory");
}

}  // namespace

// WGM x WGN waves per workgroup; ring slots as many as fit the workgroup's LDS share (up to 3).
// OCC > 0 forces that many workgroups per CU (high-occupancy variant 3: short-K GEMMs are
// bound by one memory latency per tile, so more tiles in flight per CU beat a deeper ring).
template <int BM, int BN, int NW, int OCC>
constexpr int buf_wgs_per_cu() {
  return OCC ? OCC : (NW == 8 ? 1 : ((BM == 64 && BN == 64) ? 3 : 2));
}
template <int BM, int BN, int NW, int OCC>
constexpr int buf_slots() {
  return (BM + BN) * 64 * 2 * 3 <= (160 * 1024) / buf_wgs_per_cu<BM, BN, NW, OCC>() ? 3 : 2;
}

// MF: MFMA shape — 16 (v_mfma_f32_16x16x32_bf16) or 32 (v_mfma_f32_32x32x16_bf16).  The
// 32x32x16 form does the same FLOPs in half the instructions, each holding the SIMD's vector
// issue for 8 of its 32 cycles instead of 8 of 16: three times the free issue slots per MFMA for
// the LDS-DMA pieces (60-185 issue cycles each beside MFMAs, MI355X_MICROARCH.md) and the
// fragment reads — the issue budget, not the matrix pipe, bounds the long-K (3x3) convs.
template <int BM, int BN, int WGM, int WGN, int OCC = 0, int MF = 16>
__global__ __launch_bounds__(64 * WGM * WGN, (buf_wgs_per_cu<BM, BN, WGM * WGN, OCC>())) void conv_buf_kernel(
    ConvParams p) {
  constexpr int NW = WGM * WGN, NT = 64 * NW;
  constexpr int BK = 64;
  constexpr int NS = buf_slots<BM, BN, NW, OCC>();
  constexpr int D = NS - 1;
  constexpr int WM = BM / WGM, WN = BN / WGN;
  constexpr int MI = WM / 16, NI = WN / 16;
  constexpr int RPI = 8 * NW;                  // tile rows filled per DMA instruction
  constexpr int APT = BM / RPI, BPT = BN / RPI;
  constexpr int PER = APT + BPT;
  constexpr int STAGE_ELEMS = (BM + BN) * BK;
  constexpr int CPAD = 4;
  constexpr int EPI_BYTES = BM * (BN + CPAD) * 4;
  constexpr int RING_BYTES = NS * STAGE_ELEMS * 2;
  constexpr int LDS_BYTES = EPI_BYTES > RING_BYTES ? EPI_BYTES : RING_BYTES;
  static_assert(LDS_BYTES * buf_wgs_per_cu<BM, BN, NW, OCC>() <= 160 * 1024, "LDS budget");
  __shared__ __attribute__((aligned(16))) unsigned char smem[LDS_BYTES];
  bf16_t* ring = reinterpret_cast<bf16_t*>(smem);

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);   // scalar: DMA LDS bases in SGPRs
  const int wr = wave / WGN, wc = wave % WGN;
  const int ntn = (p.Cout + BN - 1) / BN;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int tile_n = bid % ntn, tile_m = bid / ntn;
  const int m0 = tile_m * BM, n0 = tile_n * BN;

  const int lrow = wave * 8 + (lane >> 3);
  const int lp = (lane & 7) ^ (lane >> 3);
  const int HoWo = p.Ho * p.Wo;
  const int RS = p.R * p.S;
  const __amdgpu_buffer_rsrc_t rx = make_rsrc(p.x);
  const __amdgpu_buffer_rsrc_t rw = make_rsrc(p.w);
  const __amdgpu_buffer_rsrc_t rx2 = make_rsrc(p.x2 ? p.x2 : p.x);

  // per-piece geometry: byte offset of the tap-(0,0) pixel and the valid filter rows / columns
  // (bit r of the low half, bit s of the high half: tap (r, s) reads inside the image iff both
  // bits are set — two clamps per piece instead of a test per tap)
  int a_base[APT];
  uint32_t a_mask[APT], a2_off[APT];
#pragma unroll
  for (int i = 0; i < APT; ++i) {
    const int m = m0 + lrow + RPI * i;
    a_mask[i] = 0u;
    a_base[i] = 0;
    a2_off[i] = kBufOOB;
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
    b_off[i] = n < p.Cout ? (uint32_t)(((long)n * p.K + lp * 8) * 2) : kBufOOB;
  }

  // epilogue operands, prefetched before the K loop
  constexpr int CPR = BN / 8, CHUNKS = BM * CPR, CPT = CHUNKS / NT, E_ROWS = NT / CPR;
  static_assert(CHUNKS % NT == 0, "tile must give every thread whole chunks");
  const int e_cc = tid % CPR, e_row0 = tid / CPR;
  const int e_n = n0 + e_cc * 8;
  float e_bias[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) e_bias[e] = 0.f;
  if (p.bias && e_n < p.Cout) {
    const f32x4 b0 = *reinterpret_cast<const f32x4*>(p.bias + e_n);
    const f32x4 b1 = *reinterpret_cast<const f32x4*>(p.bias + e_n + 4);
    e_bias[0] = b0[0]; e_bias[1] = b0[1]; e_bias[2] = b0[2]; e_bias[3] = b0[3];
    e_bias[4] = b1[0]; e_bias[5] = b1[1]; e_bias[6] = b1[2]; e_bias[7] = b1[3];
  }
  u32x4 e_res[CPT];
  if (p.res) {
#pragma unroll
    for (int i = 0; i < CPT; ++i) {
      const int m = m0 + e_row0 + E_ROWS * i;
      const bool ok = m < p.M && e_n < p.Cout;
      e_res[i] = *reinterpret_cast<const u32x4*>(p.res + (ok ? (size_t)m * p.ldr + e_n : 0));
    }
  }
  // every ordinary load above is retired before the first DMA, so the compiler's own vmcnt
  // bookkeeping never has to count DMAs inside the loop
#pragma unroll
  for (int i = 0; i < CPT; ++i) asm volatile("" : "+v"(e_res[i]));
  asm volatile("" : "+v"(e_bias[0]), "+v"(e_bias[7]));

  // scalar K-block cursor for the DMA issue: tap index and channel offset inside the tap
  const int K1 = p.x2 ? p.K1 : p.K;
  int cur_tap = -1;                       // tap whose offsets a_off holds
  uint32_t a_off[APT];
#pragma unroll
  for (int i = 0; i < APT; ++i) a_off[i] = kBufOOB;
  int iss_tap = 0, iss_c = 0;             // position of the next K block to issue
  int iss_r = 0, iss_s = 0;               // its filter row / column

  auto issue = [&](int kb, auto slot_tag) {
    constexpr int SLOT = decltype(slot_tag)::value;
    bf16_t* As = ring + SLOT * STAGE_ELEMS;
    bf16_t* Bs = As + BM * BK;
    const int k0 = kb * BK;
    if (k0 >= K1) {
      const uint32_t soff = (uint32_t)((k0 - K1) * 2);
#pragma unroll
      for (int i = 0; i < APT; ++i) buf16(rx2, a2_off[i], soff, As + (i * RPI + wave * 8) * BK);
    } else {
      if (iss_tap != cur_tap) {           // wave-uniform: new tap -> new per-lane offsets
        cur_tap = iss_tap;
        const int r = iss_r, s = iss_s;
        const int tap_off = ((r * p.W + s) * p.C) * 2;
        const uint32_t bit = (1u << r) | (1u << (s + 16));
#pragma unroll
        for (int i = 0; i < APT; ++i)
          a_off[i] = (a_mask[i] & bit) == bit ? (uint32_t)(a_base[i] + tap_off) : kBufOOB;
      }
      const uint32_t soff = (uint32_t)(iss_c * 2);
#pragma unroll
      for (int i = 0; i < APT; ++i) buf16(rx, a_off[i], soff, As + (i * RPI + wave * 8) * BK);
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
    const uint32_t sb = (uint32_t)(k0 * 2);
#pragma unroll
    for (int i = 0; i < BPT; ++i) buf16(rw, b_off[i], sb, Bs + (i * RPI + wave * 8) * BK);
  };

  static_assert(MF == 16 || (WM % 32 == 0 && WN % 32 == 0), "32x32 MFMA needs 32-multiple wave tiles");
  constexpr int MI2 = MF == 32 ? WM / 32 : 1, NI2 = MF == 32 ? WN / 32 : 1;
  f32x4 acc[MF == 16 ? MI : 1][MF == 16 ? NI : 1];
  f32x16 acc2[MI2][NI2];
  if constexpr (MF == 16) {
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NI; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  } else {
#pragma unroll
    for (int i = 0; i < MI2; ++i)
#pragma unroll
      for (int j = 0; j < NI2; ++j)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc2[i][j][e] = 0.f;
  }

  const int fr = lane & 15, fq = lane >> 4;
  const int r32 = lane & 31, h32 = lane >> 5;
  int a_rd[MF == 16 ? MI : MI2], b_rd[MF == 16 ? NI : NI2];   // per-lane fragment offsets (elements)
  if constexpr (MF == 16) {
#pragma unroll
    for (int i = 0; i < MI; ++i) a_rd[i] = (wr * WM + i * 16 + fr) * BK;
#pragma unroll
    for (int j = 0; j < NI; ++j) b_rd[j] = BM * BK + (wc * WN + j * 16 + fr) * BK;
  } else {
#pragma unroll
    for (int i = 0; i < MI2; ++i) a_rd[i] = (wr * WM + i * 32 + r32) * BK;
#pragma unroll
    for (int j = 0; j < NI2; ++j) b_rd[j] = BM * BK + (wc * WN + j * 32 + r32) * BK;
  }
  const int sw = (MF == 16 ? fr : r32) & 7;   // row & 7 of every fragment row (8-aligned bases)

  auto compute = [&](auto slot_tag) {
    constexpr int SLOT = decltype(slot_tag)::value;
    const bf16_t* St = ring + SLOT * STAGE_ELEMS;
    if constexpr (MF == 16) {
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
    } else {
      // k-step ks covers K 16 ks .. 16 ks + 15: lane half h32 holds chunk 2 ks + h32 of its row
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        bf16x8 af[MI2], bfr[NI2];
        const int pc = ((2 * ks + h32) ^ sw) << 3;
#pragma unroll
        for (int i = 0; i < MI2; ++i) af[i] = *reinterpret_cast<const bf16x8*>(St + a_rd[i] + pc);
#pragma unroll
        for (int j = 0; j < NI2; ++j) bfr[j] = *reinterpret_cast<const bf16x8*>(St + b_rd[j] + pc);
#pragma unroll
        for (int i = 0; i < MI2; ++i)
#pragma unroll
          for (int j = 0; j < NI2; ++j)
            acc2[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[i], bfr[j], acc2[i][j], 0, 0, 0);
      }
    }
  };

  const int nkb = p.K / BK;
  // one pipeline step: retire K block kb, refill the slot freed by kb-1 with kb+D, compute kb
  auto step = [&](int kb, auto slot_tag) {
    constexpr int SLOT = decltype(slot_tag)::value;
    constexpr int PREV = SLOT == 0 ? NS - 1 : SLOT - 1;
    if (D == 2 && kb + 1 < nkb) {
      vm_barrier<PER>();
    } else {
      vm_barrier<0>();
    }
    if (kb + D < nkb) issue(kb + D, std::integral_constant<int, PREV>{});
    compute(slot_tag);
  };

  using S0 = std::integral_constant<int, 0>;
  using S1 = std::integral_constant<int, 1>;
  using S2 = std::integral_constant<int, 2>;
  issue(0, S0{});
  if (D == 2) {
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
    int kb = 0;
    for (; kb + 2 <= nkb; kb += 2) {
      step(kb, S0{});
      step(kb + 1, S1{});
    }
    if (kb < nkb) step(kb, S0{});
  }
  vm_barrier<0>();

  // ---- epilogue (as conv_glds) ----
  float* Cs = reinterpret_cast<float*>(smem);
  constexpr int LDC = BN + CPAD;
  if constexpr (MF == 16) {
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NI; ++j) {
        const int col = wc * WN + j * 16 + fr;
#pragma unroll
        for (int e = 0; e < 4; ++e) Cs[(wr * WM + i * 16 + fq * 4 + e) * LDC + col] = acc[i][j][e];
      }
  } else {
    // 32x32 C/D: col = lane & 31, row = (reg & 3) + 8 (reg >> 2) + 4 (lane >> 5)
#pragma unroll
    for (int i = 0; i < MI2; ++i)
#pragma unroll
      for (int j = 0; j < NI2; ++j) {
        const int col = wc * WN + j * 32 + r32;
#pragma unroll
        for (int e = 0; e < 16; ++e)
          Cs[(wr * WM + i * 32 + (e & 3) + 8 * (e >> 2) + 4 * h32) * LDC + col] = acc2[i][j][e];
      }
  }
  __syncthreads();
  const bool post = (p.act & 16) != 0;
  const int act = p.act & 15;
#pragma unroll
  for (int i = 0; i < CPT; ++i) {
    const int row = e_row0 + E_ROWS * i;
    const int m = m0 + row;
    if (m >= p.M || e_n >= p.Cout) continue;
    const f32x4 v0 = *reinterpret_cast<const f32x4*>(Cs + row * LDC + e_cc * 8);
    const f32x4 v1 = *reinterpret_cast<const f32x4*>(Cs + row * LDC + e_cc * 8 + 4);
    // packed fp32 pairs (v_pk_add_f32) for the bias and residual adds
    f32x2 v2[4] = {f32x2{v0[0], v0[1]} + f32x2{e_bias[0], e_bias[1]},
                   f32x2{v0[2], v0[3]} + f32x2{e_bias[2], e_bias[3]},
                   f32x2{v1[0], v1[1]} + f32x2{e_bias[4], e_bias[5]},
                   f32x2{v1[2], v1[3]} + f32x2{e_bias[6], e_bias[7]}};
    if (p.res && !post) {
#pragma unroll
      for (int e = 0; e < 4; ++e)
        v2[e] += f32x2{__uint_as_float(e_res[i][e] << 16), __uint_as_float(e_res[i][e] & 0xffff0000u)};
    }
    float v[8] = {v2[0][0], v2[0][1], v2[1][0], v2[1][1], v2[2][0], v2[2][1], v2[3][0], v2[3][1]};
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
}

}  // namespace aiko

// Same arguments as aiko_conv_igemm.  Host preconditions (checked by the binding): Cc and, with
// a second source, C2 are multiples of 64; R*S <= 32; every operand fits 2^31 bytes.
extern "C" int aiko_conv_buf(const void* x, const void* w, const float* bias, const void* res,
                             void* y, int H, int W, int C, int Cc, int R, int S, int stride,
                             int pad, int Ho, int Wo, int M, int Cout, int K, int act, int ldy,
                             int ldr, int bm, int bn, const void* x2, int K1, int H2, int W2,
                             int C2, int stride2, int occ, int mf32, hipStream_t stream) {
  using namespace aiko;
  if (Cc % 64 || R * S > 32 || R > 16 || S > 16 || (x2 && (K - K1) % 64)) return -1;
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
  dim3 grid(((M + bm - 1) / bm) * ((Cout + bn - 1) / bn)), block(256);
  if (occ) {                               // variant 3: high occupancy, 2-slot rings
    if (bm == 64 && bn == 64 && occ == 5)
      conv_buf_kernel<64, 64, 2, 2, 5><<<grid, block, 0, stream>>>(p);
    else if (bm == 64 && bn == 128 && occ == 3)
      conv_buf_kernel<64, 128, 2, 2, 3><<<grid, block, 0, stream>>>(p);
    else if (bm == 128 && bn == 64 && occ == 3)
      conv_buf_kernel<128, 64, 2, 2, 3><<<grid, block, 0, stream>>>(p);
    else if (bm == 64 && bn == 64 && occ == 4)
      conv_buf_kernel<64, 64, 2, 2, 4><<<grid, block, 0, stream>>>(p);
    // variant 6: 4 waves of 128 x 64 / 64 x 128 (one workgroup per CU, 3-slot ring in 144 KB):
    // half the LDS fragment bytes per MFMA of the 8-wave 64 x 64 layout — the wide 3x3 tiles are
    // bound by LDS read bandwidth, not by the matrix pipe
    else if (bm == 256 && bn == 128 && occ == 1)
      conv_buf_kernel<256, 128, 2, 2, 1><<<grid, block, 0, stream>>>(p);
    else if (bm == 128 && bn == 256 && occ == 1)
      conv_buf_kernel<128, 256, 2, 2, 1><<<grid, block, 0, stream>>>(p);
    else
      return -1;
  } else if (mf32) {                       // variant 5: 32x32x16 MFMA
    if (bm == 128 && bn == 128)
      conv_buf_kernel<128, 128, 2, 2, 0, 32><<<grid, block, 0, stream>>>(p);
    else if (bm == 128 && bn == 64)
      conv_buf_kernel<128, 64, 2, 2, 0, 32><<<grid, block, 0, stream>>>(p);
    else if (bm == 64 && bn == 128)
      conv_buf_kernel<64, 128, 2, 2, 0, 32><<<grid, block, 0, stream>>>(p);
    else if (bm == 256 && bn == 128)
      conv_buf_kernel<256, 128, 4, 2, 0, 32><<<grid, 512, 0, stream>>>(p);
    else if (bm == 128 && bn == 256)
      conv_buf_kernel<128, 256, 2, 4, 0, 32><<<grid, 512, 0, stream>>>(p);
    else
      return -1;
  } else if (bm == 128 && bn == 128) {
    conv_buf_kernel<128, 128, 2, 2><<<grid, block, 0, stream>>>(p);
  } else if (bm == 128 && bn == 64) {
    conv_buf_kernel<128, 64, 2, 2><<<grid, block, 0, stream>>>(p);
  } else if (bm == 64 && bn == 64) {
    conv_buf_kernel<64, 64, 2, 2><<<grid, block, 0, stream>>>(p);
  } else if (bm == 64 && bn == 128) {
    conv_buf_kernel<64, 128, 2, 2><<<grid, block, 0, stream>>>(p);
  } else if (bm == 256 && bn == 128) {     // 8 waves, one workgroup per CU, 3-slot ring
    conv_buf_kernel<256, 128, 4, 2><<<grid, 512, 0, stream>>>(p);
  } else if (bm == 128 && bn == 256) {
    conv_buf_kernel<128, 256, 2, 4><<<grid, 512, 0, stream>>>(p);
  } else if (bm == 256 && bn == 64) {      // narrow Cout (ResNet stage 1): 8 waves of 64 x 32
    conv_buf_kernel<256, 64, 4, 2><<<grid, 512, 0, stream>>>(p);
  } else {
    return -1;
  }
  return (int)hipGetLastError();
}
