// Flash-attention forward (non-causal, head dim 64) for CDNA4 (gfx950), bf16 in / fp32 softmax.
//
// Built for the Whisper encoder (1500 tokens x 12 heads x 64): one workgroup of NW waves per
// (32*NW-query block, head, sequence); each wave owns 32 queries and streams the sequence's
// keys in 64-key tiles through a 4-slot LDS ring filled by LDS-DMA (global_load_lds, three
// tiles in flight behind a counted vmcnt + raw barrier).  K and V are both stored row-major
// ([key][dh]; the DMA destination is lane-linear, so the swizzles are applied to the source
// rows): K with a 16-B XOR swizzle for ds_read_b128, V with a 32-B chunk swizzle
// (chunk ^ ((key >> 1) & 3)) read by the gfx950 hardware-transpose ds_read_b64_tr_b16
// (conflict-free per 32-lane half), which hands every lane a 4-key column of V.  The
// products are computed
// TRANSPOSED — S^T = K Q^T and O^T = V^T P^T with v_mfma_f32_16x16x32_bf16 — so that:
//   * each lane's accumulator column is one query: the online-softmax rescale of O^T is a
//     per-lane scalar, and row statistics need only 2 cross-lane shuffles (xor 16, 32);
//   * the bf16 probabilities P^T are consumed as the B operand straight from the S^T
//     accumulator registers (no LDS round trip): element j of lane group g of k-step s is key
//     32s + 16(j>>2) + 4g + (j&3), and the V^T fragment is two transposed reads of rows
//     32s + 4g .. +3 and 32s + 16 + 4g .. +3 — that same key order.
// Measured and dropped (round 2): software-pipelining S^T of tile it+1 under the softmax of
// tile it (FA3-style, one extra S block = +32 VGPRs): 201-224 VGPRs -> 2 waves / SIMD, 216-240
// us against 186 us for this kernel at 124 VGPRs / 4 waves; forcing 3 waves spills.  Occupancy
// (other waves' MFMAs under this wave's softmax) beats intra-wave overlap here.
// Q stays in registers for the whole key loop.  Sequences are rows b*Tpad .. b*Tpad+T-1 of
// q/k/v (any row pitch: q, k, v may be column slices of one fused QKV buffer).
#include <cstdlib>
#include <type_traits>

#include "common.h"

namespace aiko {

struct AttnParams {
  const bf16_t* q;
  const bf16_t* k;
  const bf16_t* v;
  bf16_t* o;
  int ldq, ldk, ldv, ldo;
  int T, Tpad, H;
  float scale_log2;     // softmax scale * log2(e)
  // split-KV tail (split_s > 0; SM = 1 kernels): 1-D grid, per XCD `split_full` whole items
  // then `split_r` items cut into split_s key ranges; see aiko_attn_fwd
  int nqb, split_s, split_full, split_r, split_fence;
  int prio;             // 1: waves NW/2 .. NW-1 run at s_setprio 1 (static young-half priority)
  float* part;          // [pieces][QB][64] fp32 partial O, then [pieces][QB] (m, l) pairs
  int* cnt;             // [8 * split_r] arrival counters, zero between launches
  // MX-fp8 output instead of bf16 o (the out-projection's A operand): e4m3 [rows][ldoq] and
  // E8M0 scales [H*64/128][osr][4], one per 32 consecutive columns — each head's 64 columns
  // are two whole blocks, so a workgroup quantises its own output (no per-row pass later)
  uint8_t* oq;
  uint8_t* osc;
  int ldoq, osr;
};

constexpr int kKB = 64, kDH = 64;
constexpr float kRescale = 8.f;   // lazy-rescale threshold (log2 units): P <= 2^8, safe in bf16/fp32

__device__ __forceinline__ bf16x8 as_bf16x8(u32x4 u) { return __builtin_bit_cast(bf16x8, u); }

// max over lanes l, l^16, l^32, l^48 on the VALU: gfx950's v_permlane32_swap / v_permlane16_swap
// with both operands = v return the two halves (rows) of the exchange, so max(result pair) is
// the xor-32 (xor-16) reduction — no ds_bpermute LDS round trip (~100+ cycles each) on the
// softmax's critical path
__device__ __forceinline__ float max_xor16_32(float v) {
  const auto a = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = fmaxf(__uint_as_float(a[0]), __uint_as_float(a[1]));
  const auto b = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(b[0]), __uint_as_float(b[1]));
}

typedef __attribute__((ext_vector_type(4))) short v4i16;

// target builtins behind __device__ helpers (the host pass of a __global__ template must not
// see them directly, or the kernel's host stub is silently dropped)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t attn_rsrc(const void* base, int bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, bytes, 0x00020000);
}

__device__ __forceinline__ void attn_setprio1() { __builtin_amdgcn_s_setprio(1); }

__device__ __forceinline__ void attn_dma16(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff, void* lds) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(
      r, reinterpret_cast<__attribute__((address_space(3))) void*>(reinterpret_cast<uintptr_t>(lds)), 16, voff,
      soff, 0, 0);
}

// byte offset of 16-bit column `col` (multiple of 4) of key row `row` in the V image
__device__ __forceinline__ int v_off(int row, int col) {
  return row * (kDH * 2) + (((col >> 4) ^ ((row >> 1) & 3)) << 5) + ((col & 15) << 1);
}

// REG = 1: register staging (guide T14, "issue early / write late"): tile it+2's K/V pieces are
// loaded into VGPRs while tile it computes and written to the LDS slot of tile it+1 right
// after the barrier that retires tile it-1 — two LDS slots, plain loads + ds_write_b128
// (a handful of issue cycles) instead of one LDS-DMA per piece (60-185 issue cycles each beside
// MFMAs, MI355X_MICROARCH.md).  REG = 0: the LDS-DMA ring (4 slots, counted vmcnt).
// SM = 1: softmax with the per-score VALU work cut to v_exp + cvt (the kernel is VALU-issue
// bound beside its MFMAs, 6.2 VALU per MFMA in round 2):
//   * Q is pre-scaled by scale*log2(e) once (bf16), so scores come out of the MFMA in log2 units;
//   * the S accumulators start at -m_run (the running max): S' = Q K^T - m needs no subtraction
//     and feeds v_exp_f32 directly; the tile max (v_max3 tree + 2 permlane swaps) only decides
//     the lazy rescale (grow by > kRescale) — the rare rescale path shifts this tile's scores;
//   * the row sums come out of the MFMA pipe: one extra 16x16x32 MFMA per P fragment with an
//     all-ones A operand (rowsum(P) in every row of the result, no fp32 add chain and no
//     end-of-kernel reduction), summing the same bf16 P that enters O.
// Removed after measurement (round 5, kept in profiles/attn_pmc_r5.md): inline-asm V^T reads with
// an explicit lgkmcnt (the builtin's vmcnt(0) drain turned out off the critical path: K/V tiles
// are L2 hits) and s_setprio over the MFMA clusters (no effect) — former variants 16-20.
template <int NW, int VPRE, int REG = 0, int SM = 0>
__global__ __launch_bounds__(64 * NW, 16 / NW) void attn_fwd_kernel(AttnParams p) {
  constexpr int NT = 64 * NW;
  constexpr int QB = 32 * NW;
  constexpr int TILE = kKB * kDH;                // elements
  constexpr int PIECES = TILE / 8;               // 16-B pieces per tile (512)
  constexpr int PPT = PIECES / NT;               // DMA pieces per thread per operand
  constexpr int NS = REG ? 2 : 4;                // LDS ring slots (DMA: tiles it+1 .. it+3 in flight)
  constexpr int PER = 2 * PPT;                   // DMA instructions per thread per tile
  __shared__ __attribute__((aligned(16))) bf16_t smem[NS * 2 * TILE];   // one array: [slot][K|V]

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int fr = lane & 15, g = lane >> 4;
  const int ntiles = (p.T + kKB - 1) / kKB;
  // XCD-aware mapping: the query blocks of one (sequence, head) share its K/V stream, so they
  // are placed on one XCD (one L2) instead of round-robin over all eight
  const int nqb = p.nqb;
  int lin, piece = -1, su = 0, tb = 0, te = ntiles;
  if (p.split_s == 0) {
    lin = xcd_remap(blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z),
                    gridDim.x * gridDim.y * gridDim.z);
  } else {
    // split-KV tail: workgroup b runs on XCD b % 8 as that XCD's (b / 8)-th dispatch; each XCD
    // owns a contiguous range of items, the last split_r of them cut into split_s key ranges
    // that fill the final round's slots instead of leaving them idle
    const int xcd = blockIdx.x & 7, idx = blockIdx.x >> 3;
    const int n = p.split_full + p.split_r;
    if (idx < p.split_full) {
      lin = xcd * n + idx;
    } else {
      const int j = idx - p.split_full;
      lin = xcd * n + p.split_full + j / p.split_s;
      piece = j % p.split_s;
      su = xcd * p.split_r + j / p.split_s;
      tb = piece * ntiles / p.split_s;
      te = (piece + 1) * ntiles / p.split_s;
    }
  }
  const int qblk = lin % nqb, h = (lin / nqb) % p.H, b = lin / (nqb * p.H);
  // static priority for the second-dispatched half of the workgroup (MI355X_MICROARCH.md, two
  // waves per SIMD, item 4): it loses every VALU arbitration by age otherwise
  if (p.prio && wave >= NW / 2) attn_setprio1();
  const long seq0 = (long)b * p.Tpad;
  const int q0 = qblk * QB + wave * 32;
  const int hc = h * kDH;

  // Q^T fragments (B operand): lane holds Q[q][ks*32 + 8g .. +7] for q = q0 + qt*16 + fr
  bf16x8 qf[2][2];
#pragma unroll
  for (int qt = 0; qt < 2; ++qt) {
    const int q = q0 + qt * 16 + fr;
    const int qc = q < p.T ? q : p.T - 1;     // rows past T: clamped, never written
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const u32x4 raw = *reinterpret_cast<const u32x4*>(p.q + (seq0 + qc) * p.ldq + hc + ks * 32 + 8 * g);
      if constexpr (SM >= 1) {
        u32x4 w;
#pragma unroll
        for (int e = 0; e < 4; ++e)
          w[e] = pack2(__uint_as_float(raw[e] << 16) * p.scale_log2, __uint_as_float(raw[e] & 0xffff0000u) * p.scale_log2);
        qf[qt][ks] = as_bf16x8(w);
      } else {
        qf[qt][ks] = as_bf16x8(raw);
      }
    }
  }
  // consume Q here, before the first (asm, compiler-invisible) DMA: the compiler's own vmcnt
  // for these loads would otherwise land inside the key loop and count the DMAs too
#pragma unroll
  for (int qt = 0; qt < 2; ++qt)
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) asm volatile("" : "+v"(qf[qt][ks]));

  // K / V tiles by LDS-DMA (lane-linear destination, swizzle on the SOURCE): instruction i of
  // wave w fills rows (NT/8)*i + 8w .. +7; lane l -> row (l >> 3), physical 16-B slot (l & 7).
  // buffer_load ... lds against a per-sequence descriptor: the per-lane 32-bit offsets are
  // tile-invariant and the tile's key offset rides in the scalar soffset, so issuing a tile
  // costs no VALU (the 64-bit address math was ~35 VALU per tile); keys past T fall outside
  // num_records and read as zeros (masked in the last tile, and p = 0 x V = 0).
  const int drow = wave * 8 + (lane >> 3);
  const int ps = lane & 7;
  const int k_lp = ps ^ (lane >> 3);                                   // K: piece ^ (row & 7)
  const __amdgpu_buffer_rsrc_t rk = attn_rsrc(p.k + seq0 * p.ldk, p.T * p.ldk * 2);
  const __amdgpu_buffer_rsrc_t rv = attn_rsrc(p.v + seq0 * p.ldv, p.T * p.ldv * 2);
  uint32_t k_off[PPT], v_off_b[PPT];
#pragma unroll
  for (int i = 0; i < PPT; ++i) {
    const int row = drow + (NT / 8) * i;
    const int v_lp = ((((ps >> 1) ^ ((row >> 1) & 3))) << 1) | (ps & 1);
    k_off[i] = (uint32_t)(row * p.ldk + hc + k_lp * 8) * 2u;
    v_off_b[i] = (uint32_t)(row * p.ldv + hc + v_lp * 8) * 2u;
  }
  auto issue = [&](int t0, int slot) {
    bf16_t* Ks = smem + slot * 2 * TILE;
    bf16_t* Vs = Ks + TILE;
    const uint32_t sk = (uint32_t)(t0 * p.ldk) * 2u, sv = (uint32_t)(t0 * p.ldv) * 2u;
#pragma unroll
    for (int i = 0; i < PPT; ++i) {
      attn_dma16(rk, k_off[i], sk, Ks + ((NT / 8) * i + wave * 8) * kDH);
      attn_dma16(rv, v_off_b[i], sv, Vs + ((NT / 8) * i + wave * 8) * kDH);
    }
  };

  // register staging: the same source pieces and LDS image as the DMA path (lane-linear
  // destination), through VGPRs
  u32x4 kreg[PPT], vreg[PPT];
  auto load_regs = [&](int t0) {
#pragma unroll
    for (int i = 0; i < PPT; ++i) {
      const int row = drow + (NT / 8) * i;
      const int key = min(t0 + row, p.T - 1);
      const int v_lp = ((((ps >> 1) ^ ((row >> 1) & 3))) << 1) | (ps & 1);
      kreg[i] = *reinterpret_cast<const u32x4*>(p.k + (seq0 + key) * p.ldk + hc + k_lp * 8);
      vreg[i] = *reinterpret_cast<const u32x4*>(p.v + (seq0 + key) * p.ldv + hc + v_lp * 8);
    }
  };
  auto write_regs = [&](int slot) {
    bf16_t* Ks = smem + slot * 2 * TILE;
    bf16_t* Vs = Ks + TILE;
#pragma unroll
    for (int i = 0; i < PPT; ++i) {
      *reinterpret_cast<u32x4*>(Ks + ((NT / 8) * i + wave * 8) * kDH + lane * 8) = kreg[i];
      *reinterpret_cast<u32x4*>(Vs + ((NT / 8) * i + wave * 8) * kDH + lane * 8) = vreg[i];
    }
  };

  f32x4 o[4][2];
#pragma unroll
  for (int d = 0; d < 4; ++d)
#pragma unroll
    for (int qt = 0; qt < 2; ++qt) o[d][qt] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m_run[2] = {SM ? 0.f : -INFINITY, SM ? 0.f : -INFINITY}, l_run[2] = {0.f, 0.f};
  f32x4 lsum[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};   // SM = 1 row sums
  const bf16x8 ones = as_bf16x8(u32x4{0x3F803F80u, 0x3F803F80u, 0x3F803F80u, 0x3F803F80u});

  // transposed-read lane geometry: lane 4q'+p' of its 16-lane group addresses row q', cols 4p'
  const int trq = fr >> 2, trp = fr & 3;

  if constexpr (REG) {
    load_regs(tb * kKB);
    write_regs(0);
    if (tb + 1 < te) load_regs((tb + 1) * kKB);  // tile tb+1 in flight in VGPRs
  } else {
#pragma unroll
    for (int j = 0; j < NS - 1; ++j)
      if (tb + j < te) issue((tb + j) * kKB, j);
  }
  int slot = 0;
  // one key tile; MASK only for the ragged last tile (keeps the compare/select chain out of the
  // steady-state loop, where hipcc would otherwise if-convert it into every iteration)
  auto tile = [&](int it, auto mask_tag) {
    constexpr bool MASK = decltype(mask_tag)::value;
    const int t0 = it * kKB;
    if constexpr (REG) {
      // tile it is in LDS (written last iteration) and every wave is done with tile it-1, whose
      // slot now takes tile it+1 from the VGPRs; then tile it+2's loads go out under compute
      __syncthreads();
      if (it + 1 < te) {
        write_regs(slot ^ 1);
        if (it + 2 < te) load_regs(t0 + 2 * kKB);
      }
    } else {
      // retire tile it (this wave's DMAs; the younger tiles stay in flight), then barrier
      if (it + 2 < te) {
        asm volatile("s_waitcnt vmcnt(%0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::"n"(2 * PER) : "memory");
      } else if (it + 1 < te) {
        asm volatile("s_waitcnt vmcnt(%0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::"n"(PER) : "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      }
      if (it + NS - 1 < te) issue(t0 + (NS - 1) * kKB, slot == 0 ? NS - 1 : slot - 1);
    }
    const bf16_t* Kc = smem + slot * 2 * TILE;
    const bf16_t* Vc = Kc + TILE;
    // V^T fragments by hardware-transposed reads of the row-major V tile; the first VPRE
    // d-blocks are read before the softmax so their LDS latency hides under its VALU work
    const unsigned char* vb = reinterpret_cast<const unsigned char*>(Vc);
    bf16x8 vfr[4][2];
    auto read_v = [&](int d) {
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const int r0 = 32 * ks + 4 * g + trq;
        const v4i16 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (__attribute__((address_space(3))) v4i16*)(vb + v_off(r0, d * 16 + 4 * trp)));
        const v4i16 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (__attribute__((address_space(3))) v4i16*)(vb + v_off(r0 + 16, d * 16 + 4 * trp)));
        vfr[d][ks] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
      }
    };

  // S^T = K Q^T : 4 key tiles x 2 query tiles
    f32x4 s[4][2];
#pragma unroll
    for (int kt = 0; kt < 4; ++kt) {
#pragma unroll
      for (int qt = 0; qt < 2; ++qt) {
        const float init = SM ? -m_run[qt] : 0.f;
        s[kt][qt] = f32x4{init, init, init, init};
      }
      const int row = kt * 16 + fr;
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const bf16x8 kf = *reinterpret_cast<const bf16x8*>(
            &Kc[row * kDH + (((ks * 4 + g) ^ (row & 7)) << 3)]);
#pragma unroll
        for (int qt = 0; qt < 2; ++qt)
          s[kt][qt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf, qf[qt][ks], s[kt][qt], 0, 0, 0);
      }
    }

#pragma unroll
    for (int d = 0; d < VPRE; ++d) read_v(d);

    // online softmax per query column (scores kept unscaled: p = exp2(s*c - m*c), one FMA per
    // score; key masking only on the ragged last tile; the running max is only raised — and O,
    // l rescaled — when it grows by more than kRescale (log2 units): otherwise exp2 stays
    // bounded by 2^kRescale and the stale max is exact for the final normalisation)
    const float c = p.scale_log2;
    bf16x8 pf[2][2];
    // SM >= 1 softmax of query tile qt: tile max relative to m_run (v_max3 tree + 2 permlane
    // swaps), lazy rescale, v_exp straight off the accumulators, bf16 pack
    auto softmax_qt = [&](int qt) {
        if constexpr (MASK) {
#pragma unroll
          for (int kt = 0; kt < 4; ++kt)
#pragma unroll
            for (int j = 0; j < 4; ++j)
              if (t0 + kt * 16 + 4 * g + j >= p.T) s[kt][qt][j] = -INFINITY;
        }
        // tile max relative to m_run: a v_max3 tree
        float m01 = fmaxf(s[0][qt][0], fmaxf(s[0][qt][1], s[0][qt][2]));
        float m23 = fmaxf(s[0][qt][3], fmaxf(s[1][qt][0], s[1][qt][1]));
        float m45 = fmaxf(s[1][qt][2], fmaxf(s[1][qt][3], s[2][qt][0]));
        float m67 = fmaxf(s[2][qt][1], fmaxf(s[2][qt][2], s[2][qt][3]));
        float m89 = fmaxf(s[3][qt][0], fmaxf(s[3][qt][1], s[3][qt][2]));
        float mloc = fmaxf(s[3][qt][3], fmaxf(m01, m23));
        mloc = fmaxf(mloc, fmaxf(m45, m67));
        mloc = max_xor16_32(fmaxf(mloc, m89));
        if (it == tb || mloc > kRescale) {
          // first tile: m_run = the tile max; later: raise it (lazy, > kRescale) — shift this
          // tile's scores to the new max and rescale what O / l hold
          if (it != tb) {
            const float alpha = fast_exp2(-mloc);
            lsum[qt] *= alpha;
#pragma unroll
            for (int d = 0; d < 4; ++d) o[d][qt] *= alpha;
          }
          m_run[qt] += mloc;
#pragma unroll
          for (int kt = 0; kt < 4; ++kt) s[kt][qt] -= mloc;
        }
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
          u32x4 u;
          u[0] = pack2(fast_exp2(s[2 * ks][qt][0]), fast_exp2(s[2 * ks][qt][1]));
          u[1] = pack2(fast_exp2(s[2 * ks][qt][2]), fast_exp2(s[2 * ks][qt][3]));
          u[2] = pack2(fast_exp2(s[2 * ks + 1][qt][0]), fast_exp2(s[2 * ks + 1][qt][1]));
          u[3] = pack2(fast_exp2(s[2 * ks + 1][qt][2]), fast_exp2(s[2 * ks + 1][qt][3]));
          pf[qt][ks] = as_bf16x8(u);
        }
    };
    auto pv_qt = [&](int qt) {
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        read_v(d);
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
          o[d][qt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vfr[d][ks], pf[qt][ks], o[d][qt], 0, 0, 0);
      }
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
        lsum[qt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ones, pf[qt][ks], lsum[qt], 0, 0, 0);
    };
    if constexpr (SM == 2) {
      // ping-pong the two query tiles: query tile 0's PV MFMAs are issued before tile 1's
      // softmax, so the matrix pipe works on tile 0 while the VALU runs tile 1's exp / pack (V
      // fragments are re-read for tile 1: +16 LDS reads, no extra VGPRs).  Same operations per
      // accumulator in the same order as SM = 1: bit-identical output.  Measured (variant 15,
      // scripts/attn_pp_ab.sh): 141.8-142.6 us against 134.2-134.5 us for SM = 1 — the V re-reads
      // cost more than the overlap returns; kept opt-in
      softmax_qt(0);
      pv_qt(0);
      softmax_qt(1);
      pv_qt(1);
    } else if constexpr (SM == 1) {
      softmax_qt(0);
      softmax_qt(1);
    } else {
#pragma unroll
    for (int qt = 0; qt < 2; ++qt) {
      float mloc = -INFINITY;
      if constexpr (MASK) {
#pragma unroll
        for (int kt = 0; kt < 4; ++kt)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            if (t0 + kt * 16 + 4 * g + j >= p.T) s[kt][qt][j] = -INFINITY;
      }
#pragma unroll
      for (int kt = 0; kt < 4; ++kt)
#pragma unroll
        for (int j = 0; j < 4; ++j) mloc = fmaxf(mloc, s[kt][qt][j]);
      mloc = max_xor16_32(mloc);
      if (mloc * c > m_run[qt] * c + kRescale || m_run[qt] == -INFINITY) {   // wave-uniform per column group
        const float m_new = fmaxf(m_run[qt], mloc);
        const float alpha = fast_exp2((m_run[qt] - m_new) * c);
        m_run[qt] = m_new;
        l_run[qt] *= alpha;
#pragma unroll
        for (int d = 0; d < 4; ++d) o[d][qt] *= alpha;
      }
      // packed fp32 (v_pk_fma_f32 / v_pk_add_f32): two scores per VALU issue — the softmax is
      // VALU-issue bound beside the MFMAs, only v_exp_f32 has no packed form
      const f32x2 c2 = {c, c};
      const f32x2 nmc2 = {-m_run[qt] * c, -m_run[qt] * c};
      f32x2 lsum2 = {0.f, 0.f};
      f32x2 pv[4][2];
#pragma unroll
      for (int kt = 0; kt < 4; ++kt)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const f32x2 x = f32x2{s[kt][qt][2 * j], s[kt][qt][2 * j + 1]} * c2 + nmc2;
          pv[kt][j] = f32x2{fast_exp2(x[0]), fast_exp2(x[1])};
          lsum2 += pv[kt][j];
        }
      l_run[qt] += lsum2[0] + lsum2[1];
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        u32x4 u;
        u[0] = pack2(pv[2 * ks][0][0], pv[2 * ks][0][1]);
        u[1] = pack2(pv[2 * ks][1][0], pv[2 * ks][1][1]);
        u[2] = pack2(pv[2 * ks + 1][0][0], pv[2 * ks + 1][0][1]);
        u[3] = pack2(pv[2 * ks + 1][1][0], pv[2 * ks + 1][1][1]);
        pf[qt][ks] = as_bf16x8(u);
      }
    }
    }

    // O^T += V^T P^T (fragments read above / here)
    if constexpr (SM != 2) {
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      if (d >= VPRE) read_v(d);
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int qt = 0; qt < 2; ++qt)
          o[d][qt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vfr[d][ks], pf[qt][ks], o[d][qt], 0, 0, 0);
    }
    if constexpr (SM == 1) {
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int qt = 0; qt < 2; ++qt)
          lsum[qt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ones, pf[qt][ks], lsum[qt], 0, 0, 0);
    }
    }

    slot = slot == NS - 1 ? 0 : slot + 1;
  };
  const int nfull = p.T / kKB;               // tiles with every key < T
  const int tfull = te < nfull ? te : nfull;
  for (int it = tb; it < tfull; ++it) tile(it, std::false_type{});
  if (nfull < te) tile(nfull, std::true_type{});

  if constexpr (SM >= 1) {
    if (piece >= 0) {
      // a key-range piece: publish (m, l, unnormalised O) for its rows; the last of the
      // split_s pieces to arrive merges them: O = sum_i 2^(m_i - M) O_i / sum_i 2^(m_i - M) l_i
      const int pieces = 8 * p.split_r * p.split_s;
      float* po = p.part + (size_t)(su * p.split_s + piece) * QB * kDH;
      float* pml = p.part + (size_t)pieces * QB * kDH + (size_t)(su * p.split_s + piece) * QB * 2;
#pragma unroll
      for (int qt = 0; qt < 2; ++qt) {
        const int lr = wave * 32 + qt * 16 + fr;
#pragma unroll
        for (int d = 0; d < 4; ++d) *reinterpret_cast<f32x4*>(po + lr * kDH + d * 16 + 4 * g) = o[d][qt];
        if (g == 0) *reinterpret_cast<f32x2*>(pml + lr * 2) = f32x2{m_run[qt], lsum[qt][0]};
      }
      __shared__ int last;
      if (p.split_fence) {
        __threadfence();
      } else {
        // the pieces of one item run on one XCD (see the mapping above), so its L2 is the point
        // of coherence: the stores only have to be complete at L2 before the arrival count
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      __syncthreads();
      if (tid == 0) {
        const int old = atomicAdd(p.cnt + su, 1);
        last = old == p.split_s - 1;
        if (last) p.cnt[su] = 0;                 // re-armed for the next launch
      }
      __syncthreads();
      if (!last) return;
      if (p.split_fence) __threadfence();
      const float* po0 = p.part + (size_t)su * p.split_s * QB * kDH;
      const float* pml0 = p.part + (size_t)pieces * QB * kDH + (size_t)su * p.split_s * QB * 2;
#pragma unroll
      for (int qt = 0; qt < 2; ++qt) {
        const int lr = wave * 32 + qt * 16 + fr;
        float mx = -INFINITY;
        for (int i = 0; i < p.split_s; ++i) mx = fmaxf(mx, pml0[(size_t)i * QB * 2 + lr * 2]);
        float l = 0.f;
        f32x4 acc[4] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f},
                        f32x4{0.f, 0.f, 0.f, 0.f}};
        for (int i = 0; i < p.split_s; ++i) {
          const f32x2 ml = *reinterpret_cast<const f32x2*>(pml0 + (size_t)i * QB * 2 + lr * 2);
          const float w = fast_exp2(ml[0] - mx);
          l += w * ml[1];
#pragma unroll
          for (int d = 0; d < 4; ++d)
            acc[d] += w * *reinterpret_cast<const f32x4*>(po0 + (size_t)i * QB * kDH + lr * kDH + d * 16 + 4 * g);
        }
#pragma unroll
        for (int d = 0; d < 4; ++d) o[d][qt] = acc[d];
        lsum[qt] = f32x4{l, l, l, l};
      }
    }
  }

  // normalise and write O[q][dh]: lane holds dh = d*16 + 4g + j for its query
  if (p.oq) {
#pragma unroll
    for (int qt = 0; qt < 2; ++qt) {
      float l;
      if constexpr (SM >= 1) {
        l = lsum[qt][0];
      } else {
        l = l_run[qt];
        l += __shfl_xor(l, 16, 64);
        l += __shfl_xor(l, 32, 64);
      }
      const float inv = 1.f / l;
      const int q = q0 + qt * 16 + fr;
      const bool live = q < p.T;
      const long row = seq0 + q;
#pragma unroll
      for (int b = 0; b < 2; ++b) {              // MX block b: dh 32b .. 32b+31 = d 2b, 2b+1
        float v[8];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          v[e] = o[2 * b][qt][e] * inv;
          v[4 + e] = o[2 * b + 1][qt][e] * inv;
        }
        float amax = 0.f;
#pragma unroll
        for (int e = 0; e < 8; ++e) amax = fmaxf(amax, fabsf(v[e]));
        amax = max_xor16_32(amax);                 // the 4 lanes of this query (g = 0..3)
        const int ex = mx_exponent(amax);
        const float s2 = __uint_as_float((uint32_t)(127 - ex) << 23);
        unsigned w0 = 0u, w1 = 0u;
        w0 = __builtin_amdgcn_cvt_pk_fp8_f32(fminf(fmaxf(v[0] * s2, -448.f), 448.f),
                                             fminf(fmaxf(v[1] * s2, -448.f), 448.f), w0, false);
        w0 = __builtin_amdgcn_cvt_pk_fp8_f32(fminf(fmaxf(v[2] * s2, -448.f), 448.f),
                                             fminf(fmaxf(v[3] * s2, -448.f), 448.f), w0, true);
        w1 = __builtin_amdgcn_cvt_pk_fp8_f32(fminf(fmaxf(v[4] * s2, -448.f), 448.f),
                                             fminf(fmaxf(v[5] * s2, -448.f), 448.f), w1, false);
        w1 = __builtin_amdgcn_cvt_pk_fp8_f32(fminf(fmaxf(v[6] * s2, -448.f), 448.f),
                                             fminf(fmaxf(v[7] * s2, -448.f), 448.f), w1, true);
        if (live) {
          uint8_t* dq = p.oq + row * p.ldoq + hc + 32 * b;
          *reinterpret_cast<unsigned*>(dq + 4 * g) = w0;          // dh 32b + 4g .. +3
          *reinterpret_cast<unsigned*>(dq + 16 + 4 * g) = w1;     // dh 32b + 16 + 4g .. +3
          const int col = hc + 32 * b;
          if (g == 0) p.osc[((long)(col >> 7) * p.osr + row) * 4 + ((col >> 5) & 3)] = (uint8_t)(ex + 127);
        }
      }
    }
    return;
  }
#pragma unroll
  for (int qt = 0; qt < 2; ++qt) {
    float l;
    if constexpr (SM >= 1) {
      l = lsum[qt][0];                 // every row of the ones-MFMA result is the row sum
    } else {
      l = l_run[qt];
      l += __shfl_xor(l, 16, 64);
      l += __shfl_xor(l, 32, 64);
    }
    const float inv = 1.f / l;
    const int q = q0 + qt * 16 + fr;
    if (q >= p.T) continue;
    bf16_t* dst = p.o + (seq0 + q) * p.ldo + hc;
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      uint2 w;
      w.x = pack2(o[d][qt][0] * inv, o[d][qt][1] * inv);
      w.y = pack2(o[d][qt][2] * inv, o[d][qt][3] * inv);
      *reinterpret_cast<uint2*>(dst + d * 16 + 4 * g) = w;
    }
  }
}

}  // namespace aiko

// work / work_bytes: optional zero-initialised workspace (fp32 partials + arrival counters) for
// the split-KV tail: when the (query block, head, sequence) items leave a partial last round on
// each XCD (Whisper-small: 1,152 items = 2.25 rounds of 512 slots), that round's items are cut
// into key ranges so it runs at full occupancy.  Without a workspace (or for the round-2 softmax
// variants) the grid is the plain one.
extern "C" int aiko_attn_fwd(const void* q, const void* k, const void* v, void* o, int ldq, int ldk,
                             int ldv, int ldo, int B, int H, int T, int Tpad, int dh, float scale,
                             void* work, long work_bytes, void* oq, void* osc, int ldoq, int osr,
                             hipStream_t stream) {
  if (dh != aiko::kDH || T < 1 || Tpad < T) return -1;
  aiko::AttnParams p;
  p.oq = static_cast<uint8_t*>(oq);
  p.osc = static_cast<uint8_t*>(osc);
  p.ldoq = ldoq;
  p.osr = osr;
  p.q = static_cast<const aiko::bf16_t*>(q);
  p.k = static_cast<const aiko::bf16_t*>(k);
  p.v = static_cast<const aiko::bf16_t*>(v);
  p.o = static_cast<aiko::bf16_t*>(o);
  p.ldq = ldq; p.ldk = ldk; p.ldv = ldv; p.ldo = ldo;
  p.T = T; p.Tpad = Tpad; p.H = H;
  p.scale_log2 = scale * 1.4426950408889634f;
  p.split_s = p.split_full = p.split_r = 0;
  p.part = nullptr;
  p.cnt = nullptr;
  const char* variant_env = getenv("AIKO_ATTN_VARIANT");   // read per call (tests flip it)
  const int variant = variant_env ? atoi(variant_env) : 0;
  // pieces per split item; 0 = no split.  Measured on MI355X at Whisper-small shapes (median of
  // 7 x 50 launches, scripts/attn_split_ab.sh): unsplit 135.1-135.4 us, s=2 133.2-134.4, s=4
  // 147.5-148.3, s=8 134.1-135.4, and the 1-D mapping alone (s=1) 139.7-140.4 — the final-round
  // model (whole slots idle) does not hold on the hardware, so the split stays opt-in
  const char* split_env = getenv("AIKO_ATTN_SPLIT_S");   // read per call (tests flip it)
  const int force_s = split_env ? atoi(split_env) : 0;
  static const int fence = [] {
    const char* v = getenv("AIKO_ATTN_SPLIT_FENCE");
    return v ? atoi(v) : 0;
  }();
  p.split_fence = fence;
  const char* prio_env = getenv("AIKO_ATTN_PRIO");       // read per call (A/B runs flip it)
  p.prio = prio_env ? atoi(prio_env) : 0;
  static const int cus = [] {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      return 0;
    return n;
  }();
  auto launch = [&](auto nw_tag, auto vpre_tag, auto reg_tag, auto sm_tag) {
    constexpr int NW = decltype(nw_tag)::value, VPRE = decltype(vpre_tag)::value;
    constexpr int REG = decltype(reg_tag)::value, SM = decltype(sm_tag)::value;
    constexpr int QB = 32 * NW;
    p.nqb = (T + QB - 1) / QB;
    const long items = (long)p.nqb * H * B;
    const int ntiles = (T + aiko::kKB - 1) / aiko::kKB;
    if (SM >= 1 && work && force_s > 0 && cus >= 8 && items % 8 == 0) {
      const long n = items / 8;
      const int slots = (16 / NW) * (cus / 8);          // resident workgroups per XCD
      const int r = (int)(n % slots);
      if (r > 0 && 2 * r <= slots) {
        const int sp = force_s < ntiles ? force_s : ntiles;
        const long cnt_b = ((8L * r * 4 + 255) / 256) * 256;
        const long need = cnt_b + 8L * r * sp * QB * (aiko::kDH + 2) * 4;
        if (sp >= 1 && need <= work_bytes) {
          p.split_s = sp;
          p.split_r = r;
          p.split_full = (int)(n - r);
          p.cnt = static_cast<int*>(work);
          p.part = reinterpret_cast<float*>(static_cast<char*>(work) + cnt_b);
          dim3 grid((unsigned)(8 * (p.split_full + (long)r * sp))), block(64 * NW);
          aiko::attn_fwd_kernel<NW, VPRE, REG, SM><<<grid, block, 0, stream>>>(p);
          return;
        }
      }
    }
    dim3 grid(p.nqb, H, B), block(64 * NW);
    aiko::attn_fwd_kernel<NW, VPRE, REG, SM><<<grid, block, 0, stream>>>(p);
  };
  using R0 = std::integral_constant<int, 0>;
  using R1 = std::integral_constant<int, 1>;
  using I8 = std::integral_constant<int, 8>;
  using I4 = std::integral_constant<int, 4>;
  using V0 = std::integral_constant<int, 0>;
  using V2 = std::integral_constant<int, 2>;
  switch (variant) {
    case 1: launch(I8{}, V2{}, R0{}, R0{}); break;
    case 2: launch(I8{}, std::integral_constant<int, 4>{}, R0{}, R0{}); break;
    case 3: launch(I4{}, V0{}, R0{}, R0{}); break;
    case 4: launch(I4{}, V2{}, R0{}, R0{}); break;
    case 5: launch(I8{}, V0{}, R1{}, R0{}); break;
    case 6: launch(I8{}, V2{}, R1{}, R0{}); break;
    case 7: launch(I4{}, V0{}, R1{}, R0{}); break;
    case 8: launch(I4{}, V2{}, R1{}, R0{}); break;
    case 10: launch(I8{}, V0{}, R0{}, R0{}); break;        // round-2 softmax
    case 11: launch(I8{}, V2{}, R0{}, R1{}); break;
    case 12: launch(I8{}, V0{}, R1{}, R1{}); break;
    case 13: launch(I4{}, V0{}, R0{}, R1{}); break;
    case 14: launch(I4{}, V2{}, R1{}, R1{}); break;
    case 15: launch(I8{}, V0{}, R0{}, std::integral_constant<int, 2>{}); break;   // ping-pong query tiles
    default: launch(I8{}, V0{}, R0{}, R1{}); break;
  }
  return (int)hipGetLastError();
}
