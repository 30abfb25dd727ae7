// Pointwise (1x1 / stride 1) convolution as a persistent, bandwidth-shaped GEMM (tuner variant 12).
//
//   y[m, n] = act(x[m, :] . w[n, :] + bias[n] (+ res[m, n]))      (residual before or after act)
//
// For the ResNet expansion convs with a residual (stage 3: M = B*196, K = 256, N = 1024; stage 4:
// K = 512, N = 2048) every tiled kernel of conv_buf / conv_wide ran at 400-700 TFLOP/s and
// 3.1-3.6 TB/s counting the residual: a tile is only 4-8 K blocks, so each workgroup pays one
// L2/HBM round trip to fill its ring, a second for the residual, and drains everything during its
// epilogue — the bytes in flight per CU, not HBM or the matrix pipe, set the pace.  Here:
//   * one 512-thread workgroup per CU walks a column of output tiles: its channel block n0 is
//     fixed (bias in registers, weights L2-resident), its 128-pixel row blocks step by the grid's
//     group count; the ntn workgroups of one row block are adjacent logical ids, i.e. on the same
//     XCD (xcd_remap), so each activation row block is fetched from HBM once into that XCD's L2;
//   * ONE 4-slot ring of 64-deep K blocks streams across tile boundaries (K % 256 == 0, so block
//     kb always uses slot kb % 4 and every slot address is an immediate): while a tile finishes
//     its last blocks and runs its epilogue, the next tile's first three blocks are in flight;
//   * the residual tile is DMA'd (buffer_load ... lds) into its own 32 KB LDS region at the
//     tile's second K step, source-swizzled so the epilogue's 16-byte reads are conflict-free —
//     no ordinary global loads are ever waited on while DMAs are in flight;
//   * the product is transposed (weights on the MFMA A side) and one v_permlane16_swap per fp32
//     pair gives each lane 8 consecutive channels of one pixel: bias, residual, activation and a
//     16-byte store straight from registers (conv_wide.hip's epilogue), no LDS bounce;
//   * every wait is a counted `s_waitcnt vmcnt(N)`, N = the DMA ops issued after the awaited
//     one (loads retire in order, so the epilogue's stores can only make a wait stricter), and a
//     raw s_barrier — never __syncthreads() with DMAs in flight.  The last tile waits vmcnt(0).
// LDS: 4 x 32 KB ring + 32 KB residual = 160 KB, one workgroup per CU.
//
// Measured (MI355X, ResNet-50 at B=320, scripts/pw_check.sh, tuner medians): stage-3 expansion
// M=62720 N=1024 K=256 + residual 77.9 us vs 80 us for the best tiled kernel (picked); stage-4
// N=2048 K=512 53.8 vs 45.3 us, stage-3 reductions N=256 K=1024 42.4 vs 34 us (not picked).  So
// the per-tile ring fill / residual round trip was not what held those layers at 3.6 TB/s: with
// three 32 KB blocks in flight per CU across tile boundaries the kernel still spends ~5 us per
// 128 x 128 tile (17 % MFMA, ~37 % LDS, 3.8 TB/s HBM).  Kept as a tuner candidate.
#include "conv_common.h"

namespace aiko {

namespace {

constexpr uint32_t kPwOOB = 0x80000000u;          // offsets >= num_records read as zero
constexpr uint32_t kPwRecords = 0x7ffffff0u;
constexpr int kPwBM = 128, kPwBN = 128, kPwBK = 64, kPwNS = 4;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t pw_rsrc(const void* base) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)kPwRecords, 0x00020000);
}

__device__ __forceinline__ void pw_dma16(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff, void* lds) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(
      r, reinterpret_cast<__attribute__((address_space(3))) void*>(reinterpret_cast<uintptr_t>(lds)), 16,
      voff, soff, 0, 0);
}

template <int N>
__device__ __forceinline__ void pw_vm_barrier() {
  asm volatile("s_waitcnt vmcnt(%0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::"n"(N) : "memory");
}

struct PwParams {
  const bf16_t* x;      // [M][ldx], K channels used (the first KA of them with a second source)
  const bf16_t* w;      // [N][K]
  const float* bias;    // [N] or nullptr
  const bf16_t* res;    // [M][ldr] or nullptr
  bf16_t* y;            // [M][ldy]
  int M, N, K, ldx, ldy, ldr, act;
  int ntn, mtiles, groups;
  // optional second source (K columns [KA, K)): a 1x1 / stride-s2 conv over x2 [B][H2][W2][ldx2]
  // sampled at output pixel (n, ho, wo) -> (n, s2 ho, s2 wo): the ResNet projection shortcut
  const bf16_t* x2;
  int ldx2, hw, wo, h2, w2, s2;
  uint32_t mhw, mwo;
  int lhw, lwo;
};

template <bool RES>
__global__ __launch_bounds__(512, 1) void conv_pw_kernel(PwParams p) {
  constexpr int BM = kPwBM, BN = kPwBN, BK = kPwBK, NS = kPwNS;
  constexpr int WGN = 4, WM = 64, WN = 32, MI = WM / 16, NI = WN / 16;
  constexpr int RPW = 8, RPI = 64;                // tile rows per wave / per workgroup DMA instruction
  constexpr int APT = BM / RPI, BPT = BN / RPI, P = APT + BPT;
  constexpr int NR = RES ? BM / 32 : 0;           // residual DMA instructions per thread
  constexpr int STAGE = (BM + BN) * BK;           // elements per ring slot
  constexpr int RES_ELEMS = BM * BN;
  __shared__ __attribute__((aligned(16))) bf16_t lds[NS * STAGE + RES_ELEMS];
  bf16_t* const resb = lds + NS * STAGE;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave / WGN, wc = wave % WGN;
  const int lid = xcd_remap(blockIdx.x, gridDim.x);
  const int tile_n = lid % p.ntn, group = lid / p.ntn;
  if (group >= p.groups) return;                   // (host sizes the grid to ntn * groups)
  const int n0 = tile_n * BN;
  const int ntiles = group < p.mtiles ? (p.mtiles - 1 - group) / p.groups + 1 : 0;
  if (ntiles == 0) return;
  const int nkb = p.K / BK;                        // multiple of NS (host)

  const __amdgpu_buffer_rsrc_t rx = pw_rsrc(p.x);
  const __amdgpu_buffer_rsrc_t rw = pw_rsrc(p.w);
  const __amdgpu_buffer_rsrc_t rr = pw_rsrc(RES ? p.res : p.x);

  const int lrow = wave * RPW + (lane >> 3);
  const int lp = (lane & 7) ^ (lane >> 3);        // source-side swizzle of the 128-B rows
  uint32_t b_off[BPT];
#pragma unroll
  for (int i = 0; i < BPT; ++i) b_off[i] = (uint32_t)(((n0 + lrow + RPI * i) * p.K + lp * 8) * 2);
  // residual DMA: 16 pieces (256 B) per tile row, 4 rows per wave instruction; the piece a lane
  // writes at LDS position lane & 15 of row rrow is logical piece (lane & 15) ^ (rrow & 15)
  const int rrow0 = wave * 4 + (lane >> 4);
  const int rpiece = (lane & 15) ^ (rrow0 & 15);   // (rrow0 + 32 r) & 15 == rrow0 & 15

  // ---- bias for the fixed channel block, consumed before any DMA is in flight ----
  const int fr = lane & 15, fq = lane >> 4;
  const int coff = ((fq & 1) << 4) | ((fq >> 1) << 3);
  const int nl = wc * WN + coff;                   // tile-local first channel of this lane's 8
  float e_bias[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) e_bias[e] = 0.f;
  if (p.bias) {
    const f32x4 b0 = *reinterpret_cast<const f32x4*>(p.bias + n0 + nl);
    const f32x4 b1 = *reinterpret_cast<const f32x4*>(p.bias + n0 + nl + 4);
    e_bias[0] = b0[0]; e_bias[1] = b0[1]; e_bias[2] = b0[2]; e_bias[3] = b0[3];
    e_bias[4] = b1[0]; e_bias[5] = b1[1]; e_bias[6] = b1[2]; e_bias[7] = b1[3];
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) asm volatile("" ::"v"(e_bias[e]));   // retire the loads here

  auto issue = [&](int f, auto slot_tag) {         // flat K block f = tile * nkb + kb
    constexpr int SLOT = decltype(slot_tag)::value;
    const int t = f / nkb, kb = f - t * nkb;
    if (t >= ntiles) return;
    const int m0 = (group + t * p.groups) * BM;
    bf16_t* Xs = lds + SLOT * STAGE;
    bf16_t* Ws = Xs + BM * BK;
    const uint32_t sb = (uint32_t)(kb * BK * 2);
#pragma unroll
    for (int i = 0; i < BPT; ++i) pw_dma16(rw, b_off[i], sb, Ws + (i * RPI + wave * RPW) * BK);
#pragma unroll
    for (int i = 0; i < APT; ++i) {
      const int m = m0 + lrow + RPI * i;
      const uint32_t off = m < p.M ? (uint32_t)((m * p.ldx + lp * 8) * 2) : kPwOOB;
      pw_dma16(rx, off, sb, Xs + (i * RPI + wave * RPW) * BK);
    }
  };
  auto issue_res = [&](int t) {
    const int m0 = (group + t * p.groups) * BM;
#pragma unroll
    for (int r = 0; r < NR; ++r) {
      const int m = m0 + rrow0 + 32 * r;
      const uint32_t off = m < p.M ? (uint32_t)((m * p.ldr + n0 + rpiece * 8) * 2) : kPwOOB;
      pw_dma16(rr, off, 0u, resb + (r * 32 + wave * 4) * BN);
    }
  };

  const int sw = fr & 7;
  int w_rd[NI], x_rd[MI];
#pragma unroll
  for (int j = 0; j < NI; ++j) w_rd[j] = BM * BK + (wc * WN + j * 16 + fr) * BK;
#pragma unroll
  for (int i = 0; i < MI; ++i) x_rd[i] = (wr * WM + i * 16 + fr) * BK;

  f32x4 acc[NI][MI];
  auto compute = [&](auto slot_tag) {
    constexpr int SLOT = decltype(slot_tag)::value;
    const bf16_t* St = lds + SLOT * STAGE;
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

  using S0 = std::integral_constant<int, 0>;
  using S1 = std::integral_constant<int, 1>;
  using S2 = std::integral_constant<int, 2>;
  using S3 = std::integral_constant<int, 3>;
  issue(0, S0{});
  issue(1, S1{});
  issue(2, S2{});

  const bool post = (p.act & 16) != 0;
  const int act = p.act & 15;
  for (int t = 0; t < ntiles; ++t) {
    const bool last = t + 1 == ntiles;
    const int m0 = (group + t * p.groups) * BM;
#pragma unroll
    for (int j = 0; j < NI; ++j)
#pragma unroll
      for (int i = 0; i < MI; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int kq = 0; kq < nkb; kq += NS) {
      const int f = t * nkb + kq;
      // block f + s: younger DMA ops = the next two blocks (+ this tile's residual, issued at
      // step 1 before block f + 4, while it is outstanding behind blocks (t, 2) and (t, 3))
      if (last && kq + NS >= nkb) pw_vm_barrier<0>(); else pw_vm_barrier<2 * P>();
      issue(f + 3, S3{});
      compute(S0{});
      if (last && kq + NS >= nkb) pw_vm_barrier<0>(); else pw_vm_barrier<2 * P>();
      if (RES && kq == 0) issue_res(t);
      issue(f + 4, S0{});
      compute(S1{});
      if (last && kq + NS >= nkb) pw_vm_barrier<0>();
      else if (RES && kq == 0) pw_vm_barrier<2 * P + NR>();
      else pw_vm_barrier<2 * P>();
      issue(f + 5, S1{});
      compute(S2{});
      if (last && kq + NS >= nkb) pw_vm_barrier<0>();
      else if (RES && kq == 0) pw_vm_barrier<2 * P + NR>();
      else pw_vm_barrier<2 * P>();
      issue(f + 6, S2{});
      compute(S3{});
    }
    // residual landed (younger: the nkb - 1 blocks issued since) and visible to every wave
    if (RES) {
      if (last) pw_vm_barrier<0>();
      else if (nkb == 4) pw_vm_barrier<3 * P>();
      else pw_vm_barrier<0>();
    }

    // ---- register-direct epilogue ----
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      const int ml = wr * WM + i * 16 + fr;
      const int m = m0 + ml;
      f32x4 lo = acc[0][i], hi = acc[1][i];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const auto s = __builtin_amdgcn_permlane16_swap(__float_as_uint(lo[e]), __float_as_uint(hi[e]), false, false);
        lo[e] = __uint_as_float(s[0]);
        hi[e] = __uint_as_float(s[1]);
      }
      u32x4 r = {0u, 0u, 0u, 0u};
      if constexpr (RES) r = *reinterpret_cast<const u32x4*>(resb + ml * BN + (((nl >> 3) ^ fr) << 3));
      if (m >= p.M) continue;
      float v[8] = {lo[0] + e_bias[0], lo[1] + e_bias[1], lo[2] + e_bias[2], lo[3] + e_bias[3],
                    hi[0] + e_bias[4], hi[1] + e_bias[5], hi[2] + e_bias[6], hi[3] + e_bias[7]};
      if (RES && !post) {
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
      if (RES && post) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          v[2 * e] += __uint_as_float(r[e] << 16);
          v[2 * e + 1] += __uint_as_float(r[e] & 0xffff0000u);
        }
      }
      u32x4 o;
#pragma unroll
      for (int e = 0; e < 4; ++e) o[e] = pack2(v[2 * e], v[2 * e + 1]);
      *reinterpret_cast<u32x4*>(p.y + (size_t)m * p.ldy + n0 + nl) = o;
    }
  }
}

// ---- resident-weight variant (tuner variant 13): K == 128, 256 or 512 ----
//
// conv_pw_kernel keeps three 32 KB blocks in flight per CU: ~1 us of MFMA work to cover a ~2 us
// L2 / HBM round trip, so every K step stalls.  With the workgroup's channel block fixed, its
// weight block (64 KB) is loaded into LDS once; the ring then carries only activation blocks of a
// 64-pixel tile (8 KB each) beside the weights and two residual tiles.  Slots cycle every two
// tiles when a tile has fewer K blocks than the ring has slots (block kb of tile t uses slot
// NKB (t & 1) + kb), so the tile loop is unrolled by two and every slot address is an immediate.
//   KW = 128 (stage-2 expansions 128 -> 512): a 256 x 128 weight block, 8 waves of 64 x 32, a
//            4-slot ring (three blocks = 1.5 tiles in flight), two 32 KB residual tiles: 160 KB;
//   KW = 256 (stage-3 expansions, 256 -> 128 reductions): 128 x 256 weights, 4 x 2 waves of
//            32 x 32, an 8-slot ring (seven blocks in flight), two 16 KB residual tiles: 160 KB;
//   KW = 512 (stage-4 expansions, 512 -> 256/128 reductions): 64 x 512 weights, 4 x 2 waves of
//            16 x 32, one tile per ring cycle, two 8 KB residual tiles: 144 KB.
// The residual is the largest operand of an expansion (2x-4x the activation bytes) and used only
// by the epilogue, so it is DMA'd ONE TILE AHEAD into the other residual buffer: tile t + 1's
// residual is issued at tile t's first K step and has a whole tile (~2-4 us at the HBM pace) to
// land, where issuing it at its own tile's first step left ~0.5-2 us — an exposed round trip
// per tile.  Stores go through buffer_store with an out-of-range offset for the ragged rows (never
// skipped), so the number of vector-memory ops a wave issues per tile is fixed and every
// `s_waitcnt vmcnt(N)` below is the EXACT count of ops younger than the awaited one (computed at
// compile time from the issue order by pw_young_*), for the first tiles and the steady state;
// the tiles the lookahead runs past the end of the walk wait for everything.
// Measured (MI355X, B=320, scripts/pw_check.sh): with the residual issued at its own tile the
// stage-3 expansion M=62720 N=1024 K=256 + residual ran 65.6 us (500 TF, 4.4 TB/s with the
// residual) against 77.9 us for conv_pw_kernel and 80 us for the best tiled kernel.  Round 4, one
// box: the stage-2 expansion M=250880 N=512 K=128 + residual 105.5 us one tile ahead vs 110.9 us at
// its own tile (PF = 0, tuner variant 14) and 133 us for the best tiled kernel — 5.6 TB/s counting
// the residual; K = 256 71.4 vs 71.8 us, K = 512 81.1 vs 79.8 us (no difference there).

// Issue order per wave (virtual steps s < 0 are the prologue): step s of tile t = s / NKB issues
// [res(t + 1): NR ops if s % NKB == 0] [x block s + LA: 1 op]; after a tile's last step its
// epilogue issues MI stores.  res(0) sits at virtual step -NKB (or before everything if NKB > LA).
// With PF == 0 (A/B form, tuner variant 14) step s issues res(t) itself and there is no virtual one.
__host__ __device__ constexpr bool pw_res_at(int s, int NKB, int LA, int PF = 1) {
  return s >= 0 ? s % NKB == 0 : (PF == 0 ? false : NKB <= LA ? s == -NKB : s == -LA);
}
__host__ __device__ constexpr int pw_res_id(int s, int NKB, int PF = 1) { return s >= 0 ? s / NKB + PF : 0; }

// ops issued after x block f and before step f's wait
__host__ __device__ constexpr int pw_young_blk(int f, int NKB, int LA, int NR, int MI, int PF = 1) {
  int cnt = 0;
  bool on = false;
  for (int s = -LA; s < f; ++s) {
    if (NR && pw_res_at(s, NKB, LA, PF) && on) cnt += NR;
    if (on) cnt += 1;
    if (s + LA == f) on = true;
    if (s >= 0 && s % NKB == NKB - 1 && on) cnt += MI;
  }
  return cnt;
}

// ops issued after res(t) and before tile t's epilogue wait (i.e. after its last step's issue)
__host__ __device__ constexpr int pw_young_res(int t, int NKB, int LA, int NR, int MI, int PF = 1) {
  int cnt = 0;
  bool on = false;
  const int last = NKB * t + NKB - 1;
  for (int s = -LA; s <= last; ++s) {
    if (pw_res_at(s, NKB, LA, PF)) {
      if (on) cnt += NR;
      if (pw_res_id(s, NKB, PF) == t) on = true;
    }
    if (on) cnt += 1;
    if (s >= 0 && s % NKB == NKB - 1 && s != last && on) cnt += MI;
  }
  return cnt;
}

template <bool RES, int KW, int PF = 1, int KA = KW>
__global__ __launch_bounds__(512, 1) void conv_pw_rb_kernel(PwParams p) {
  static_assert(KW == 128 || KW == 256 || KW == 384 || KW == 512, "K = 128, 256, 384 or 512");
  static_assert(PF == 0 || PF == 1, "residual issued at its own tile (0) or one tile ahead (1)");
  static_assert(KA == KW || (KW == 384 && KA == 128 && !RES), "second source: 128 + 256 columns, no residual");
  constexpr int BN = KW == 128 ? 256 : KW == 512 ? 64 : 128;
  constexpr int BM = 64, BK = 64, NKB = KW / BK, NKA = KA / BK;
  constexpr int NS = KW == 128 ? 4 : KW == 384 ? 6 : 8;
  constexpr int WGN = KW == 128 ? 8 : KW == 512 ? 2 : 4;
  constexpr int WM = BM / (8 / WGN), WN = BN / WGN, MI = WM / 16, NI = WN / 16;
  static_assert(NI == 2, "the epilogue pairs two 16-channel fragments");
  constexpr int RPC = BN / 8;                     // 16-B pieces per residual row (32 / 16 / 8)
  constexpr int RMASK = RPC < 16 ? RPC - 1 : 15;  // residual swizzle: piece ^ (row & RMASK)
  constexpr int NR = RES ? BM * RPC / 512 : 0;    // residual DMA instructions per thread (4 / 2 / 1)
  constexpr int LA = NS - 1;                      // blocks in flight
  constexpr int TAIL = (LA + NKB - 1) / NKB;      // tiles the lookahead reaches ahead (2 / 2 / 1)
  constexpr int SLOT = BM * BK;                   // elements per ring slot (8 KB)
  constexpr int W_ELEMS = BN * KW;                // resident weights (64 KB)
  constexpr int R_ELEMS = RES ? BM * BN : 0;      // one residual tile
  __shared__ __attribute__((aligned(16))) bf16_t lds[W_ELEMS + NS * SLOT + 2 * R_ELEMS];
  bf16_t* const wres = lds;
  bf16_t* const ring = lds + W_ELEMS;
  bf16_t* const resb = ring + NS * SLOT;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave / WGN, wc = wave % WGN;
  const int lid = xcd_remap(blockIdx.x, gridDim.x);
  const int tile_n = lid % p.ntn, group = lid / p.ntn;
  if (group >= p.groups) return;
  const int n0 = tile_n * BN;
  const int ntiles = group < p.mtiles ? (p.mtiles - 1 - group) / p.groups + 1 : 0;
  if (ntiles == 0) return;

  const __amdgpu_buffer_rsrc_t rx = pw_rsrc(p.x);
  const __amdgpu_buffer_rsrc_t rw = pw_rsrc(p.w);
  const __amdgpu_buffer_rsrc_t rr = pw_rsrc(RES ? p.res : p.x);
  const __amdgpu_buffer_rsrc_t ry = pw_rsrc(p.y);
  const __amdgpu_buffer_rsrc_t rx2 = pw_rsrc(KA < KW ? p.x2 : p.x);

  const int fr = lane & 15, fq = lane >> 4;
  const int coff = ((fq & 1) << 4) | ((fq >> 1) << 3);
  const int nl = wc * WN + coff;
  float e_bias[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) e_bias[e] = 0.f;
  if (p.bias) {
    const f32x4 b0 = *reinterpret_cast<const f32x4*>(p.bias + n0 + nl);
    const f32x4 b1 = *reinterpret_cast<const f32x4*>(p.bias + n0 + nl + 4);
    e_bias[0] = b0[0]; e_bias[1] = b0[1]; e_bias[2] = b0[2]; e_bias[3] = b0[3];
    e_bias[4] = b1[0]; e_bias[5] = b1[1]; e_bias[6] = b1[2]; e_bias[7] = b1[3];
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) asm volatile("" ::"v"(e_bias[e]));

  // resident weights: KW / 8 16-B pieces per row, 64 consecutive pieces per wave instruction; LDS
  // position pos of row n holds logical piece (pos & ~7) | ((pos & 7) ^ (n & 7))
  constexpr int WI = BN * KW / 8 / 512;           // weight DMA instructions per thread (8 / 8 / 12 / 8)
#pragma unroll
  for (int i = 0; i < WI; ++i) {
    const int idx = (i * 8 + wave) * 64 + lane;
    const int row = idx / (KW / 8);
    const int pos = idx % (KW / 8);
    const int lpc = (pos & ~7) | ((pos & 7) ^ (row & 7));
    pw_dma16(rw, (uint32_t)(((n0 + row) * KW + lpc * 8) * 2), 0u, wres + (i * 8 + wave) * 64 * 8);
  }

  const int lrow = wave * 8 + (lane >> 3);         // activation DMA: 8 rows per wave, 64 per block
  const int lp = (lane & 7) ^ (lane >> 3);
  constexpr int RRW = 64 / RPC;                   // residual rows per wave instruction (2 / 4 / 8)
  const int rrow0 = wave * RRW + lane / RPC;      // (rrow0 + 8 RRW r) & RMASK == rrow0 & RMASK
  const int rpiece = (lane % RPC) ^ (rrow0 & RMASK);

  auto issue = [&](int f, auto slot_tag) {
    constexpr int S = decltype(slot_tag)::value;
    const int t = f / NKB, kb = f % NKB;
    if (t >= ntiles) return;
    const int m = (group + t * p.groups) * BM + lrow;
    if (KA == KW || kb < NKA) {
      const uint32_t off = m < p.M ? (uint32_t)((m * p.ldx + lp * 8) * 2) : kPwOOB;
      pw_dma16(rx, off, (uint32_t)(kb * BK * 2), ring + S * SLOT + wave * 8 * BK);
    } else {                                       // the strided second source
      const int n = fdiv(m, p.mhw, p.lhw);
      const int r = m - n * p.hw;
      const int ho = fdiv(r, p.mwo, p.lwo);
      const int row2 = (n * p.h2 + ho * p.s2) * p.w2 + (r - ho * p.wo) * p.s2;
      const uint32_t off = m < p.M ? (uint32_t)((row2 * p.ldx2 + lp * 8) * 2) : kPwOOB;
      pw_dma16(rx2, off, (uint32_t)((kb - NKA) * BK * 2), ring + S * SLOT + wave * 8 * BK);
    }
  };
  auto issue_res = [&](int t, auto buf_tag) {      // residual of tile t into buffer B
    constexpr int B = decltype(buf_tag)::value;
    if (t >= ntiles) return;
    const int m0 = (group + t * p.groups) * BM;
#pragma unroll
    for (int r = 0; r < NR; ++r) {
      const int m = m0 + rrow0 + 8 * RRW * r;
      const uint32_t off = m < p.M ? (uint32_t)((m * p.ldr + n0 + rpiece * 8) * 2) : kPwOOB;
      pw_dma16(rr, off, 0u, resb + B * R_ELEMS + (r * 8 * RRW + wave * RRW) * BN);
    }
  };

  const int sw = fr & 7;
  int w_rd[NI], x_rd[MI];
#pragma unroll
  for (int j = 0; j < NI; ++j) w_rd[j] = (wc * WN + j * 16 + fr) * KW;
#pragma unroll
  for (int i = 0; i < MI; ++i) x_rd[i] = (wr * WM + i * 16 + fr) * BK;

  f32x4 acc[NI][MI];
  auto compute = [&](auto slot_tag, auto kb_tag) {
    constexpr int S = decltype(slot_tag)::value, KB = decltype(kb_tag)::value;
    const bf16_t* Xs = ring + S * SLOT;
#pragma unroll
    for (int kk = 0; kk < BK / 32; ++kk) {
      const int pc = ((fq + 4 * kk) ^ sw) << 3;
      bf16x8 wf[NI], xf[MI];
#pragma unroll
      for (int j = 0; j < NI; ++j) wf[j] = *reinterpret_cast<const bf16x8*>(wres + w_rd[j] + KB * 64 + pc);
#pragma unroll
      for (int i = 0; i < MI; ++i) xf[i] = *reinterpret_cast<const bf16x8*>(Xs + x_rd[i] + pc);
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NI; ++j)
          acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[j], xf[i], acc[j][i], 0, 0, 0);
    }
  };

  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  // prologue = virtual steps -LA .. -1: x blocks 0 .. LA - 1 (block b in slot b), res(0) at its
  // virtual step
  auto pro = [&](auto b_tag) {
    constexpr int B = decltype(b_tag)::value;
    if constexpr (B < LA) {
      if constexpr (RES && pw_res_at(B - LA, NKB, LA, PF)) issue_res(0, I0{});
      issue(B, b_tag);
    }
  };
  pro(I0{}); pro(I1{}); pro(std::integral_constant<int, 2>{}); pro(std::integral_constant<int, 3>{});
  pro(std::integral_constant<int, 4>{}); pro(std::integral_constant<int, 5>{});
  pro(std::integral_constant<int, 6>{});

  const bool post = (p.act & 16) != 0;
  const int act = p.act & 15;
  // one K step of tile t (H = t & 1): wait for its block, issue the lookahead (and at KB == 0 the
  // next tile's residual), run the MFMAs
  auto step = [&](int t, bool tail, auto h_tag, auto kb_tag) {
    constexpr int H = decltype(h_tag)::value, KB = decltype(kb_tag)::value;
    constexpr int SL = (NKB < NS ? NKB * H : 0) + KB;
    constexpr int Y0 = pw_young_blk(KB, NKB, LA, NR, MI, PF);
    constexpr int Y1 = pw_young_blk(NKB + KB, NKB, LA, NR, MI, PF);
    constexpr int YS = pw_young_blk(NKB * TAIL + KB, NKB, LA, NR, MI, PF);
    if (tail) pw_vm_barrier<0>();
    else if (t == 0) pw_vm_barrier<Y0>();
    else if (TAIL > 1 && t == 1) pw_vm_barrier<Y1>();
    else pw_vm_barrier<YS>();
    if constexpr (RES && KB == 0) issue_res(t + PF, std::integral_constant<int, H ^ PF>{});
    issue(NKB * t + KB + LA, std::integral_constant<int, (SL + LA) % NS>{});
    compute(std::integral_constant<int, SL>{}, kb_tag);
  };
  auto tile = [&](int t, auto half_tag) {
    constexpr int H = decltype(half_tag)::value;
    const bool tail = t + TAIL >= ntiles;
#pragma unroll
    for (int j = 0; j < NI; ++j)
#pragma unroll
      for (int i = 0; i < MI; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};
    step(t, tail, half_tag, I0{});
    step(t, tail, half_tag, I1{});
    if constexpr (NKB >= 4) {
      step(t, tail, half_tag, std::integral_constant<int, 2>{});
      step(t, tail, half_tag, std::integral_constant<int, 3>{});
    }
    if constexpr (NKB >= 6) {
      step(t, tail, half_tag, std::integral_constant<int, 4>{});
      step(t, tail, half_tag, std::integral_constant<int, 5>{});
    }
    if constexpr (NKB == 8) {
      step(t, tail, half_tag, std::integral_constant<int, 6>{});
      step(t, tail, half_tag, std::integral_constant<int, 7>{});
    }
    if constexpr (RES) {                           // this tile's residual landed, every wave
      constexpr int R0 = pw_young_res(0, NKB, LA, NR, MI, PF);
      constexpr int RS = pw_young_res(1, NKB, LA, NR, MI, PF);
      if (tail) pw_vm_barrier<0>();
      else if (t == 0) pw_vm_barrier<R0>();
      else pw_vm_barrier<RS>();
    }
    const bf16_t* const rt = resb + H * R_ELEMS;
    const int m0 = (group + t * p.groups) * BM;
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      const int ml = wr * WM + i * 16 + fr;
      const int m = m0 + ml;
      f32x4 lo = acc[0][i], hi = acc[1][i];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const auto s = __builtin_amdgcn_permlane16_swap(__float_as_uint(lo[e]), __float_as_uint(hi[e]), false, false);
        lo[e] = __uint_as_float(s[0]);
        hi[e] = __uint_as_float(s[1]);
      }
      u32x4 r = {0u, 0u, 0u, 0u};
      if constexpr (RES) r = *reinterpret_cast<const u32x4*>(rt + ml * BN + (((nl >> 3) ^ (ml & RMASK)) << 3));
      float v[8] = {lo[0] + e_bias[0], lo[1] + e_bias[1], lo[2] + e_bias[2], lo[3] + e_bias[3],
                    hi[0] + e_bias[4], hi[1] + e_bias[5], hi[2] + e_bias[6], hi[3] + e_bias[7]};
      if (RES && !post) {
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
      if (RES && post) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          v[2 * e] += __uint_as_float(r[e] << 16);
          v[2 * e + 1] += __uint_as_float(r[e] & 0xffff0000u);
        }
      }
      u32x4 o;
#pragma unroll
      for (int e = 0; e < 4; ++e) o[e] = pack2(v[2 * e], v[2 * e + 1]);
      // always issued (ragged rows at an out-of-range offset): the vmcnt counts above include it
      const uint32_t off = m < p.M ? (uint32_t)(((size_t)m * p.ldy + n0 + nl) * 2) : kPwOOB;
      __builtin_amdgcn_raw_buffer_store_b128(o, ry, off, 0, 0);
    }
  };
  for (int t = 0; t < ntiles; t += 2) {
    tile(t, I0{});
    if (t + 1 < ntiles) tile(t + 1, I1{});
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

}  // namespace

}  // namespace aiko

// 1x1 / stride-1 conv over x [M][ldx] (first K channels): K % 256 == 0 (mode 0) or K in {128, 256,
// 512} (mode 1), N a multiple of the channel block, ldx / ldy / ldr multiples of 8, 16-byte aligned
// operands, every operand < 2^31 bytes (host checks).
// ``cus``: compute units to size the persistent grid for; ``mode`` 1: resident-weight kernel, 2: the
// same with each tile's residual issued at its own first K step (A/B form).
extern "C" int aiko_conv_pw(const void* x, const void* w, const float* bias, const void* res, void* y, int M,
                            int N, int K, int ldx, int ldy, int ldr, int act, int cus, int mode,
                            hipStream_t stream) {
  using namespace aiko;
  const bool rb = mode == 1 || mode == 2;
  const int bn = rb ? (K == 128 ? 256 : K == 256 ? 128 : 64) : kPwBN;
  if (N % bn || M <= 0 || ldx % 8 || ldy % 8 || (res && ldr % 8) || ldx < K) return -1;
  if (rb ? (K != 128 && K != 256 && K != 512) : K % (kPwBK * kPwNS) != 0) return -1;
  PwParams p;
  p.x = static_cast<const bf16_t*>(x);
  p.w = static_cast<const bf16_t*>(w);
  p.bias = bias;
  p.res = static_cast<const bf16_t*>(res);
  p.y = static_cast<bf16_t*>(y);
  p.M = M; p.N = N; p.K = K; p.ldx = ldx; p.ldy = ldy; p.ldr = ldr; p.act = act;
  p.ntn = N / bn;
  const int bm = rb ? 64 : kPwBM;
  p.mtiles = (M + bm - 1) / bm;
  int groups = (cus > 0 ? cus : 256) / p.ntn;
  if (groups < 1) groups = 1;
  if (groups > p.mtiles) groups = p.mtiles;
  p.groups = groups;
  const dim3 grid((unsigned)(groups * p.ntn));
  if (mode == 1 || mode == 2) {                     // 2: residual at its own tile (A/B form)
    auto go = [&](auto kw_tag) {
      constexpr int KWv = decltype(kw_tag)::value;
      if (res && mode == 2)
        conv_pw_rb_kernel<true, KWv, 0><<<grid, 512, 0, stream>>>(p);
      else if (res)
        conv_pw_rb_kernel<true, KWv, 1><<<grid, 512, 0, stream>>>(p);
      else
        conv_pw_rb_kernel<false, KWv, 1><<<grid, 512, 0, stream>>>(p);
    };
    if (K == 128) go(std::integral_constant<int, 128>{});
    else if (K == 256) go(std::integral_constant<int, 256>{});
    else go(std::integral_constant<int, 512>{});
  } else if (res) {
    conv_pw_kernel<true><<<grid, 512, 0, stream>>>(p);
  } else {
    conv_pw_kernel<false><<<grid, 512, 0, stream>>>(p);
  }
  return (int)hipGetLastError();
}

// Fused ResNet projection (stage-2 entry): y = act(x[:, :128] . w[:, :128] + x2(strided)[:, :256] .
// w[:, 128:] + bias) over the resident-weight kernel with a 128 x 384 weight block (96 KB) and a
// 6-slot ring (one tile per cycle): x [M][ldx] is the block's 3x3 output at (Ho, Wo), x2
// [B][H2][W2][ldx2] the block input sampled at stride s2.  N % 128 == 0, no residual.
extern "C" int aiko_conv_pw_dual(const void* x, const void* x2, const void* w, const float* bias, void* y, int M,
                                 int N, int ldx, int ldx2, int ldy, int act, int Ho, int Wo, int H2, int W2, int s2,
                                 int cus, hipStream_t stream) {
  using namespace aiko;
  if (N % 128 || M <= 0 || M % (Ho * Wo) || ldx % 8 || ldx2 % 8 || ldy % 8 || ldx < 128 || ldx2 < 256) return -1;
  PwParams p{};
  p.x = static_cast<const bf16_t*>(x);
  p.x2 = static_cast<const bf16_t*>(x2);
  p.w = static_cast<const bf16_t*>(w);
  p.bias = bias;
  p.res = nullptr;
  p.y = static_cast<bf16_t*>(y);
  p.M = M; p.N = N; p.K = 384; p.ldx = ldx; p.ldy = ldy; p.ldr = 0; p.act = act;
  p.ldx2 = ldx2; p.hw = Ho * Wo; p.wo = Wo; p.h2 = H2; p.w2 = W2; p.s2 = s2;
  fastdiv_init(Ho * Wo, &p.mhw, &p.lhw);
  fastdiv_init(Wo, &p.mwo, &p.lwo);
  p.ntn = N / 128;
  p.mtiles = (M + 63) / 64;
  int groups = (cus > 0 ? cus : 256) / p.ntn;
  if (groups < 1) groups = 1;
  if (groups > p.mtiles) groups = p.mtiles;
  p.groups = groups;
  conv_pw_rb_kernel<false, 384, 1, 128><<<dim3((unsigned)(groups * p.ntn)), 512, 0, stream>>>(p);
  return (int)hipGetLastError();
}
