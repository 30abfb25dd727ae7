// FP8 (OCP e4m3fn) GEMM for CDNA4 (gfx950) on the block-scaled MFMA
// v_mfma_scale_f32_16x16x128_f8f6f4 — twice the bf16 MFMA rate per clock.
//
//   y[m, n] = act( sa[m] * sb[n] * sum_k A[m, k] * B[n, k] + bias[n] ) (+ residual[m, n])
//
// A: activations [M][lda] fp8, one fp32 scale per row (dynamic per-token quantisation, written
// by the LayerNorm / quantise kernels); B: weights [N][K] fp8, one fp32 scale per output
// channel (quantised once at load).  The MX block scales of the instruction are set to 1.0
// (E8M0 127): per-row/per-channel scales are exact in the fp32 epilogue and keep the MX rate.
//
// Tiling mirrors the bf16 igemm: 256 threads = 4 waves (2 x 2), block tile BM x BN x 128
// (one 128-byte K block = 8 16-B pieces per row), register-staged 2-deep LDS ring, pieces
// XOR-swizzled by (row & 7) so each lane's two ds_read_b128 per fragment are conflict-free,
// XCD-aware block remap, fp32 epilogue staged through padded LDS (bias, GELU, residual add,
// 16-byte bf16 stores).  For 16x16x128 every lane holds 32 K bytes of one row (row = lane & 15):
// 16-B pieces g and g + 4 of the 128-B K block, g = lane >> 4 — a K permutation applied to both
// operands alike, so A and B still pair element for element (the MX block scales are uniform).
// With the (row & 7) XOR swizzle this makes both ds_read_b128 of a fragment bank-conflict free
// over the instruction's lane groups (consecutive pieces 2g, 2g + 1 would be 2-way).
#include <cstdlib>
#include <type_traits>

#include "common.h"

namespace aiko {

typedef __attribute__((ext_vector_type(8))) int i32x8;

struct Fp8GemmParams {
  const uint8_t* a;     // [M][lda]
  const uint8_t* b;     // [N][K]
  const float* sa;      // [M]
  const float* sb;      // [N]
  const float* bias;    // [N] or nullptr
  const bf16_t* res;    // [M][ldr] or nullptr (added after the activation)
  bf16_t* y;            // [M][ldy]
  int M, N, K, lda, ldy, ldr;
  int act;              // 0 none, 1 relu, 2 silu, 3 gelu (erf)
  // MX-fp8 activations (OCP microscaling: one E8M0 scale per 32 consecutive K values).  For
  // v_mfma_scale_f32_16x16x128_f8f6f4 the A scale of lane l applies to row l % 16 and K block
  // l / 16 of the instruction's 128 (measured: scripts/probe/mfma_scale_probe.hip — the block is
  // the low 16 bytes of lane groups 2b', 2b'+1 or the high 16 bytes, which under this kernel's
  // piece order g, g + 4 is exactly the natural K range [32 b, 32 b + 32)).  Scale bytes are
  // laid out [K/128][rows][4].
  const uint8_t* amx;   // A scales (sa unused when set), rows = mxr
  int mxr;
  uint8_t* yq;          // MX output instead of y: e4m3 [M][ldq] + scales [N/128][ysr][4]
  uint8_t* ysc;
  int ldq, ysr;
  // LayerNorm folded across a GEMM pair (persistent 256 x 256 kernel only; see the comment above
  // gemm_fp8_pers2_kernel): the producer (LN 1) also writes y's MX-fp8 copy to yq / ysc and the
  // per-row partial sum / sum of squares of every 256-column tile to st [N / 256][sts] float2;
  // the consumer (LN 2) reads stp of those partials per row, cs [N] = sum_k W'[n, k] (W' = W
  // diag(gamma), dequantised), bias = b + W beta, over ln_d columns with ln_eps
  float* st;
  const float* cs;
  int sts, stp, ln_d;
  float ln_eps;
};




// Epilogue for a WGM x WGN grid of waves, each owning (BM / WGM) x (BN / WGN) of the tile: the
// fp32 accumulators go through padded LDS so that every thread then owns whole 8-column chunks
// (16-B bf16 stores); scales, bias, activation and residual are applied on the way out.
template <int BM, int BN, int WGM = 2, int WGN = 2, bool MXO = false>
__device__ __forceinline__ void fp8_epilogue(const Fp8GemmParams& p,
                                             f32x4 (&acc)[BM / WGM / 16][BN / WGN / 16],
                                             unsigned char* smem, int m0, int n0) {
  constexpr int NT = 64 * WGM * WGN;
  constexpr int WM = BM / WGM, WN = BN / WGN, MI = WM / 16, NI = WN / 16, CPAD = 4;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave / WGN, wc = wave % WGN, fr = lane & 15, fg = lane >> 4;
  float* Cs = reinterpret_cast<float*>(smem);
  constexpr int LDC = BN + CPAD;
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j) {
      const int col = wc * WN + j * 16 + fr;
#pragma unroll
      for (int e = 0; e < 4; ++e) Cs[(wr * WM + i * 16 + fg * 4 + e) * LDC + col] = acc[i][j][e];
    }
  __syncthreads();
  constexpr int CPR = BN / 8, CHUNKS = BM * CPR, CPT = CHUNKS / NT, E_ROWS = NT / CPR;
  static_assert(CHUNKS % NT == 0, "whole chunks per thread");
  const int e_cc = tid % CPR, e_row0 = tid / CPR;
  const int e_n = n0 + e_cc * 8;
  static_assert(!MXO || BN % 128 == 0, "MX output needs whole 128-column K chunks per tile");
  if (e_n >= p.N) return;
  float cs[8], cb[8];
  {
    const f32x4 s0 = *reinterpret_cast<const f32x4*>(p.sb + e_n);
    const f32x4 s1 = *reinterpret_cast<const f32x4*>(p.sb + e_n + 4);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      cs[e] = s0[e];
      cs[e + 4] = s1[e];
    }
    if (p.bias) {
      const f32x4 b0 = *reinterpret_cast<const f32x4*>(p.bias + e_n);
      const f32x4 b1 = *reinterpret_cast<const f32x4*>(p.bias + e_n + 4);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        cb[e] = b0[e];
        cb[e + 4] = b1[e];
      }
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) cb[e] = 0.f;
    }
  }
#pragma unroll
  for (int i = 0; i < CPT; ++i) {
    const int row = e_row0 + E_ROWS * i;
    const int m = m0 + row;
    const bool live = m < p.M;
    if (!MXO && !live) continue;            // (MX output: every lane joins the block shuffles)
    const float rs = p.sa && live ? p.sa[m] : 1.f;
    const f32x4 c0 = *reinterpret_cast<const f32x4*>(Cs + row * LDC + e_cc * 8);
    const f32x4 c1 = *reinterpret_cast<const f32x4*>(Cs + row * LDC + e_cc * 8 + 4);
    float v[8];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      v[e] = c0[e] * rs * cs[e] + cb[e];
      v[e + 4] = c1[e] * rs * cs[e + 4] + cb[e + 4];
    }
    if (p.act == 1) {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = fmaxf(v[e], 0.f);
    } else if (p.act == 2) {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = silu(v[e]);
    } else if (p.act == 3) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const f32x2 g = gelu_erf2(f32x2{v[2 * e], v[2 * e + 1]});
        v[2 * e] = g[0];
        v[2 * e + 1] = g[1];
      }
    }
    if constexpr (MXO) {
      // MX block b = columns 32b .. 32b+31 of this 128-column tile row = chunks 4b .. 4b+3,
      // held by lanes that differ in bits 0-1
      float amax = 0.f;
#pragma unroll
      for (int e = 0; e < 8; ++e) amax = fmaxf(amax, fabsf(v[e]));
      amax = fmaxf(amax, dpp_f32<0xB1>(amax));     // quad_perm: lanes ^1 (DPP, no LDS trip)
      amax = fmaxf(amax, dpp_f32<0x4E>(amax));     // lanes ^2
      const int ex = mx_exponent(amax);
      const float inv = __uint_as_float((uint32_t)(127 - ex) << 23);
      unsigned w0 = 0u, w1 = 0u;
      w0 = __builtin_amdgcn_cvt_pk_fp8_f32(fminf(fmaxf(v[0] * inv, -448.f), 448.f),
                                           fminf(fmaxf(v[1] * inv, -448.f), 448.f), w0, false);
      w0 = __builtin_amdgcn_cvt_pk_fp8_f32(fminf(fmaxf(v[2] * inv, -448.f), 448.f),
                                           fminf(fmaxf(v[3] * inv, -448.f), 448.f), w0, true);
      w1 = __builtin_amdgcn_cvt_pk_fp8_f32(fminf(fmaxf(v[4] * inv, -448.f), 448.f),
                                           fminf(fmaxf(v[5] * inv, -448.f), 448.f), w1, false);
      w1 = __builtin_amdgcn_cvt_pk_fp8_f32(fminf(fmaxf(v[6] * inv, -448.f), 448.f),
                                           fminf(fmaxf(v[7] * inv, -448.f), 448.f), w1, true);
      if (live) {
        *reinterpret_cast<uint2*>(p.yq + (long)m * p.ldq + e_n) = make_uint2(w0, w1);
        if ((e_cc & 3) == 0)
          p.ysc[((long)(e_n >> 7) * p.ysr + m) * 4 + ((e_n >> 5) & 3)] = (uint8_t)(ex + 127);
      }
      continue;
    }
    if (p.res) {
      const u32x4 r = *reinterpret_cast<const u32x4*>(p.res + (long)m * p.ldr + e_n);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        v[2 * e] += __uint_as_float(r[e] << 16);
        v[2 * e + 1] += __uint_as_float(r[e] & 0xffff0000u);
      }
    }
    u32x4 o;
#pragma unroll
    for (int e = 0; e < 4; ++e) o[e] = pack2(v[2 * e], v[2 * e + 1]);
    *reinterpret_cast<u32x4*>(p.y + (long)m * p.ldy + e_n) = o;
  }
}

// One output row-chunk of 8 columns (shared by the epilogues below): scales, bias, activation,
// then MX-fp8 quantisation (every lane takes part in the DPP block reduction; ``live`` gates
// the stores) or residual add + bf16 store.
template <bool MXO>
__device__ __forceinline__ void fp8_store_chunk(const Fp8GemmParams& p, float (&v)[8], int m, int e_n, int e_cc,
                                                bool live) {
  if (p.act == 1) {
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = fmaxf(v[e], 0.f);
  } else if (p.act == 2) {
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = silu(v[e]);
  } else if (p.act == 3) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const f32x2 g = gelu_erf2(f32x2{v[2 * e], v[2 * e + 1]});
      v[2 * e] = g[0];
      v[2 * e + 1] = g[1];
    }
  }
  if constexpr (MXO) {
    float amax = 0.f;
#pragma unroll
    for (int e = 0; e < 8; ++e) amax = fmaxf(amax, fabsf(v[e]));
    amax = fmaxf(amax, dpp_f32<0xB1>(amax));
    amax = fmaxf(amax, dpp_f32<0x4E>(amax));
    const int ex = mx_exponent(amax);
    const float inv = __uint_as_float((uint32_t)(127 - ex) << 23);
    unsigned w0 = 0u, w1 = 0u;
    w0 = __builtin_amdgcn_cvt_pk_fp8_f32(fminf(fmaxf(v[0] * inv, -448.f), 448.f),
                                         fminf(fmaxf(v[1] * inv, -448.f), 448.f), w0, false);
    w0 = __builtin_amdgcn_cvt_pk_fp8_f32(fminf(fmaxf(v[2] * inv, -448.f), 448.f),
                                         fminf(fmaxf(v[3] * inv, -448.f), 448.f), w0, true);
    w1 = __builtin_amdgcn_cvt_pk_fp8_f32(fminf(fmaxf(v[4] * inv, -448.f), 448.f),
                                         fminf(fmaxf(v[5] * inv, -448.f), 448.f), w1, false);
    w1 = __builtin_amdgcn_cvt_pk_fp8_f32(fminf(fmaxf(v[6] * inv, -448.f), 448.f),
                                         fminf(fmaxf(v[7] * inv, -448.f), 448.f), w1, true);
    if (live) {
      *reinterpret_cast<uint2*>(p.yq + (long)m * p.ldq + e_n) = make_uint2(w0, w1);
      if ((e_cc & 3) == 0) p.ysc[((long)(e_n >> 7) * p.ysr + m) * 4 + ((e_n >> 5) & 3)] = (uint8_t)(ex + 127);
    }
    return;
  }
  if (!live) return;
  if (p.res) {
    const u32x4 r = *reinterpret_cast<const u32x4*>(p.res + (long)m * p.ldr + e_n);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      v[2 * e] += __uint_as_float(r[e] << 16);
      v[2 * e + 1] += __uint_as_float(r[e] & 0xffff0000u);
    }
  }
  u32x4 o;
#pragma unroll
  for (int e = 0; e < 4; ++e) o[e] = pack2(v[2 * e], v[2 * e + 1]);
  *reinterpret_cast<u32x4*>(p.y + (long)m * p.ldy + e_n) = o;
}

template <int BM, int BN>
__global__ __launch_bounds__(256, 2) void gemm_fp8_kernel(Fp8GemmParams p) {
  constexpr int BK = 128;                      // bytes == fp8 elements
  constexpr int WM = BM / 2, WN = BN / 2;
  constexpr int MI = WM / 16, NI = WN / 16;
  constexpr int APT = BM / 32, BPT = BN / 32;  // 16-B pieces per thread per K block
  constexpr int STAGE_BYTES = (BM + BN) * BK;
  constexpr int CPAD = 4;
  constexpr int EPI_BYTES = BM * (BN + CPAD) * 4;
  constexpr int RING_BYTES = 2 * STAGE_BYTES;
  constexpr int LDS_BYTES = EPI_BYTES > RING_BYTES ? EPI_BYTES : RING_BYTES;
  __shared__ __attribute__((aligned(16))) unsigned char smem[LDS_BYTES];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 1, wc = wave & 1;
  const int ntn = (p.N + BN - 1) / BN;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int m0 = (bid / ntn) * BM, n0 = (bid % ntn) * BN;

  const int piece = tid & 7, prow = tid >> 3;
  long a_off[APT];
  bool a_ok[APT];
#pragma unroll
  for (int i = 0; i < APT; ++i) {
    const int m = m0 + prow + 32 * i;
    a_ok[i] = m < p.M;
    a_off[i] = (long)(a_ok[i] ? m : 0) * p.lda + piece * 16;
  }
  long b_off[BPT];
  bool b_ok[BPT];
#pragma unroll
  for (int i = 0; i < BPT; ++i) {
    const int n = n0 + prow + 32 * i;
    b_ok[i] = n < p.N;
    b_off[i] = (long)(b_ok[i] ? n : 0) * p.K + piece * 16;
  }

  u32x4 ra[APT], rb[BPT];
  auto load_global = [&](int kb) {
    const int k0 = kb * BK;
#pragma unroll
    for (int i = 0; i < APT; ++i)
      ra[i] = a_ok[i] ? *reinterpret_cast<const u32x4*>(p.a + a_off[i] + k0) : u32x4{0u, 0u, 0u, 0u};
#pragma unroll
    for (int i = 0; i < BPT; ++i)
      rb[i] = b_ok[i] ? *reinterpret_cast<const u32x4*>(p.b + b_off[i] + k0) : u32x4{0u, 0u, 0u, 0u};
  };
  auto store_lds = [&](int slot) {
    unsigned char* As = smem + slot * STAGE_BYTES;
    unsigned char* Bs = As + BM * BK;
#pragma unroll
    for (int i = 0; i < APT; ++i) {
      const int row = prow + 32 * i;
      *reinterpret_cast<u32x4*>(As + row * BK + ((piece ^ (row & 7)) << 4)) = ra[i];
    }
#pragma unroll
    for (int i = 0; i < BPT; ++i) {
      const int row = prow + 32 * i;
      *reinterpret_cast<u32x4*>(Bs + row * BK + ((piece ^ (row & 7)) << 4)) = rb[i];
    }
  };

  f32x4 acc[MI][NI];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nkb = p.K / BK;
  load_global(0);
  store_lds(0);
  __syncthreads();
  const int fr = lane & 15, fg = lane >> 4;   // fragment row, K group (32 bytes each)

  for (int kb = 0; kb < nkb; ++kb) {
    const int cur = kb & 1;
    if (kb + 1 < nkb) load_global(kb + 1);
    const unsigned char* As = smem + cur * STAGE_BYTES;
    const unsigned char* Bs = As + BM * BK;
    i32x8 af[MI], bfr[NI];
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      const int row = wr * WM + i * 16 + fr;
      const u32x4 lo = *reinterpret_cast<const u32x4*>(As + row * BK + ((fg ^ (row & 7)) << 4));
      const u32x4 hi = *reinterpret_cast<const u32x4*>(As + row * BK + (((fg + 4) ^ (row & 7)) << 4));
      af[i] = i32x8{(int)lo[0], (int)lo[1], (int)lo[2], (int)lo[3], (int)hi[0], (int)hi[1], (int)hi[2], (int)hi[3]};
    }
#pragma unroll
    for (int j = 0; j < NI; ++j) {
      const int row = wc * WN + j * 16 + fr;
      const u32x4 lo = *reinterpret_cast<const u32x4*>(Bs + row * BK + ((fg ^ (row & 7)) << 4));
      const u32x4 hi = *reinterpret_cast<const u32x4*>(Bs + row * BK + (((fg + 4) ^ (row & 7)) << 4));
      bfr[j] = i32x8{(int)lo[0], (int)lo[1], (int)lo[2], (int)lo[3], (int)hi[0], (int)hi[1], (int)hi[2], (int)hi[3]};
    }
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NI; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(af[i], bfr[j], acc[i][j], 0, 0,
                                                                      0, 127, 0, 127);
    if (kb + 1 < nkb) store_lds(cur ^ 1);
    __syncthreads();
  }

  fp8_epilogue<BM, BN>(p, acc, smem, m0, n0);
}

// ---------------------------------------------------------------------------------------------
// LDS-DMA variant: the same tile / MFMA / epilogue with operands staged by
// global_load_lds_dwordx4 through a ring of NS slots (see conv_glds.hip for the protocol:
// counted vmcnt + raw barrier, source-side swizzle, lane-linear DMA destination).  Rows past
// M / N read a zeroed 16-B page.
template <int BM, int BN>
constexpr int fp8_glds_slots() {
  return (BM + BN) * 128 * 3 <= 80 * 1024 ? 3 : 2;
}

__device__ __forceinline__ void glds16_u8(const void* g, unsigned char* lds_wave_base) {
  __builtin_amdgcn_global_load_lds(g, reinterpret_cast<__attribute__((address_space(3))) void*>(
                                          reinterpret_cast<uintptr_t>(lds_wave_base)),
                                   16, 0, 0);
}

template <int N>
__device__ __forceinline__ void fp8_wait_vm_barrier() {
  asm volatile("s_waitcnt vmcnt(%0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::"n"(N) : "memory");
}

template <int I, int N, typename F>
__device__ __forceinline__ void fp8_static_for(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    fp8_static_for<I + 1, N>(f);
  }
}

// LDS fragment reads the compiler does not see: their completion is waited for by hand with a
// counted lgkmcnt (fp8_lgkm_tie), which names the fragments as in/out operands so no use of them
// can be scheduled above the wait.  (The compiler's own waits on these reads were lgkmcnt(0)
// every other MFMA group, draining the read-ahead.)
template <int OFF>
__device__ __forceinline__ u32x4 fp8_lds_rd128(uint32_t addr) {
  u32x4 v;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(v) : "v"(addr), "n"(OFF) : "memory");
  return v;
}
template <int N>
__device__ __forceinline__ void fp8_lgkm_tie(u32x4& a, u32x4& b) {
  asm volatile("s_waitcnt lgkmcnt(%2)" : "+v"(a), "+v"(b) : "n"(N) : "memory");
}
template <int N>
__device__ __forceinline__ void fp8_lgkm_tie(u32x4 (&l)[4], u32x4 (&h)[4], u32x4& a, u32x4& b) {
  asm volatile("s_waitcnt lgkmcnt(%10)"
               : "+v"(l[0]), "+v"(l[1]), "+v"(l[2]), "+v"(l[3]), "+v"(h[0]), "+v"(h[1]), "+v"(h[2]), "+v"(h[3]),
                 "+v"(a), "+v"(b)
               : "n"(N) : "memory");
}
__device__ __forceinline__ void fp8_pin(const f32x4 (&a)[4]) {
  asm volatile("" ::"v"(a[0]), "v"(a[1]), "v"(a[2]), "v"(a[3]));
}
__device__ __forceinline__ i32x8 fp8_frag(const u32x4& lo, const u32x4& hi) {
  return i32x8{(int)lo[0], (int)lo[1], (int)lo[2], (int)lo[3], (int)hi[0], (int)hi[1], (int)hi[2], (int)hi[3]};
}

template <int BM, int BN, bool MXA = false, bool MXO = false>
__global__ __launch_bounds__(256, 2) void gemm_fp8_glds_kernel(Fp8GemmParams p, const uint8_t* zero) {
  constexpr int BK = 128;
  constexpr int NS = fp8_glds_slots<BM, BN>();
  constexpr int D = NS - 1;
  constexpr int WM = BM / 2, WN = BN / 2;
  constexpr int MI = WM / 16, NI = WN / 16;
  constexpr int APT = BM / 32, BPT = BN / 32;
  constexpr int PER = APT + BPT + (MXA ? 1 : 0);   // + one scale-tile DMA per wave
  constexpr int TILE_BYTES = (BM + BN) * BK;
  constexpr int STAGE_BYTES = TILE_BYTES + (MXA ? BM * 4 : 0);
  constexpr int CPAD = 4;
  constexpr int EPI_BYTES = BM * (BN + CPAD) * 4;
  constexpr int RING_BYTES = NS * STAGE_BYTES;
  constexpr int LDS_BYTES = EPI_BYTES > RING_BYTES ? EPI_BYTES : RING_BYTES;
  __shared__ __attribute__((aligned(16))) unsigned char smem[LDS_BYTES];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 1, wc = wave & 1;
  const int ntn = (p.N + BN - 1) / BN;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int m0 = (bid / ntn) * BM, n0 = (bid % ntn) * BN;
  const int lrow = wave * 8 + (lane >> 3);
  const int lp = (lane & 7) ^ (lane >> 3);

  const uint8_t* a_src[APT];
#pragma unroll
  for (int i = 0; i < APT; ++i) {
    const int m = m0 + lrow + 32 * i;
    a_src[i] = m < p.M ? p.a + (long)m * p.lda + lp * 16 : nullptr;
  }
  const uint8_t* b_src[BPT];
#pragma unroll
  for (int i = 0; i < BPT; ++i) {
    const int n = n0 + lrow + 32 * i;
    b_src[i] = n < p.N ? p.b + (long)n * p.K + lp * 16 : nullptr;
  }
  // MX scale tile of a K block: rows m0 .. m0+BM-1, 4 bytes each, contiguous in the [K/128][rows][4]
  // layout; wave w fetches rows w*BM/4 .. (w+1)*BM/4 - 1 with BM/16 lanes of 16 B
  constexpr int SC_LANES = BM / 16;
  auto issue = [&](int kb, int slot) {
    unsigned char* As = smem + slot * STAGE_BYTES;
    unsigned char* Bs = As + BM * BK;
    const int k0 = kb * BK;
#pragma unroll
    for (int i = 0; i < APT; ++i) glds16_u8(a_src[i] ? a_src[i] + k0 : zero, As + (i * 32 + wave * 8) * BK);
#pragma unroll
    for (int i = 0; i < BPT; ++i) glds16_u8(b_src[i] ? b_src[i] + k0 : zero, Bs + (i * 32 + wave * 8) * BK);
    if constexpr (MXA) {
      const uint8_t* src = p.amx + ((long)kb * p.mxr + m0 + wave * (BM / 4)) * 4 + lane * 16;
      if (lane < SC_LANES) glds16_u8(src, As + TILE_BYTES + wave * BM);
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
  const int fr = lane & 15, fg = lane >> 4;
  int slot = 0;
  for (int kb = 0; kb < nkb; ++kb) {
    if (D == 2 && kb + 1 < nkb) {
      fp8_wait_vm_barrier<PER>();
    } else {
      fp8_wait_vm_barrier<0>();
    }
    if (kb + D < nkb) issue(kb + D, slot == 0 ? NS - 1 : slot - 1);
    const unsigned char* As = smem + slot * STAGE_BYTES;
    const unsigned char* Bs = As + BM * BK;
    int asc[MI];                       // E8M0 scale of this lane's A block, in byte 0
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      if constexpr (MXA) {
        const uint32_t w4 = *reinterpret_cast<const uint32_t*>(As + TILE_BYTES + (wr * WM + i * 16 + fr) * 4);
        asc[i] = (int)(w4 >> (8 * fg));
      } else {
        asc[i] = 127;
      }
    }
    i32x8 af[MI], bfr[NI];
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      const int row = wr * WM + i * 16 + fr;
      const u32x4 lo = *reinterpret_cast<const u32x4*>(As + row * BK + ((fg ^ (row & 7)) << 4));
      const u32x4 hi = *reinterpret_cast<const u32x4*>(As + row * BK + (((fg + 4) ^ (row & 7)) << 4));
      af[i] = i32x8{(int)lo[0], (int)lo[1], (int)lo[2], (int)lo[3], (int)hi[0], (int)hi[1], (int)hi[2], (int)hi[3]};
    }
#pragma unroll
    for (int j = 0; j < NI; ++j) {
      const int row = wc * WN + j * 16 + fr;
      const u32x4 lo = *reinterpret_cast<const u32x4*>(Bs + row * BK + ((fg ^ (row & 7)) << 4));
      const u32x4 hi = *reinterpret_cast<const u32x4*>(Bs + row * BK + (((fg + 4) ^ (row & 7)) << 4));
      bfr[j] = i32x8{(int)lo[0], (int)lo[1], (int)lo[2], (int)lo[3], (int)hi[0], (int)hi[1], (int)hi[2], (int)hi[3]};
    }
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NI; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(af[i], bfr[j], acc[i][j], 0, 0,
                                                                      0, asc[i], 0, 127);
    slot = slot == NS - 1 ? 0 : slot + 1;
  }
  fp8_wait_vm_barrier<0>();
  fp8_epilogue<BM, BN, 2, 2, MXO>(p, acc, smem, m0, n0);
}

// ---------------------------------------------------------------------------------------------
// 8-wave LDS-DMA variant for long-M GEMMs: 512 threads as 4 (M) x 2 (N) waves over a 256 x BN
// tile, each wave 64 x BN/2.  One workgroup per CU with a 3-slot ring (2 K blocks in flight
// across every barrier): the register-staged / 2-slot kernels above retire each K block with
// only one block of MFMA work (512 cycles per wave) to cover an L2/MALL round trip, which left
// the 16x16x128 pipe idle most of the time (PMC: ~10 % MFMA-busy per wave at K = 768).
// The MFMA block runs at raised wave priority so the co-resident wave's DMA issue and fragment
// reads slot into the MFMA shadow instead of the other way round.
template <int BN>
__global__ __launch_bounds__(512, 1) void gemm_fp8_w8_kernel(Fp8GemmParams p, const uint8_t* zero) {
  constexpr int BM = 256, BK = 128, NS = 3, D = NS - 1;
  constexpr int WGM = 4, WGN = 2;
  constexpr int WM = BM / WGM, WN = BN / WGN;
  constexpr int MI = WM / 16, NI = WN / 16;
  constexpr int APT = BM / 64, BPT = BN / 64;   // DMA instructions per thread per stage
  constexpr int PER = APT + BPT;
  constexpr int STAGE_BYTES = (BM + BN) * BK;
  constexpr int CPAD = 4;
  constexpr int EPI_BYTES = BM * (BN + CPAD) * 4;
  constexpr int RING_BYTES = NS * STAGE_BYTES;
  constexpr int LDS_BYTES = EPI_BYTES > RING_BYTES ? EPI_BYTES : RING_BYTES;
  static_assert(LDS_BYTES <= 160 * 1024, "LDS");
  __shared__ __attribute__((aligned(16))) unsigned char smem[LDS_BYTES];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave / WGN, wc = wave % WGN;
  const int ntn = (p.N + BN - 1) / BN;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int m0 = (bid / ntn) * BM, n0 = (bid % ntn) * BN;
  // DMA instruction i of wave w fills rows i*64 + w*8 .. +7 (lane l: row l >> 3, slot l & 7)
  const int lrow = wave * 8 + (lane >> 3);
  const int lp = (lane & 7) ^ (lane >> 3);

  const uint8_t* a_src[APT];
#pragma unroll
  for (int i = 0; i < APT; ++i) {
    const int m = m0 + lrow + 64 * i;
    a_src[i] = m < p.M ? p.a + (long)m * p.lda + lp * 16 : nullptr;
  }
  const uint8_t* b_src[BPT];
#pragma unroll
  for (int i = 0; i < BPT; ++i) {
    const int n = n0 + lrow + 64 * i;
    b_src[i] = n < p.N ? p.b + (long)n * p.K + lp * 16 : nullptr;
  }
  auto issue = [&](int kb, int slot) {
    unsigned char* As = smem + slot * STAGE_BYTES;
    unsigned char* Bs = As + BM * BK;
    const int k0 = kb * BK;
#pragma unroll
    for (int i = 0; i < APT; ++i) glds16_u8(a_src[i] ? a_src[i] + k0 : zero, As + (i * 64 + wave * 8) * BK);
#pragma unroll
    for (int i = 0; i < BPT; ++i) glds16_u8(b_src[i] ? b_src[i] + k0 : zero, Bs + (i * 64 + wave * 8) * BK);
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
  const int fr = lane & 15, fg = lane >> 4;
  int slot = 0;
  for (int kb = 0; kb < nkb; ++kb) {
    if (kb + 1 < nkb) {
      fp8_wait_vm_barrier<PER>();
    } else {
      fp8_wait_vm_barrier<0>();
    }
    if (kb + D < nkb) issue(kb + D, slot == 0 ? NS - 1 : slot - 1);
    const unsigned char* As = smem + slot * STAGE_BYTES;
    const unsigned char* Bs = As + BM * BK;
    i32x8 af[MI], bfr[NI];
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      const int row = wr * WM + i * 16 + fr;
      const u32x4 lo = *reinterpret_cast<const u32x4*>(As + row * BK + ((fg ^ (row & 7)) << 4));
      const u32x4 hi = *reinterpret_cast<const u32x4*>(As + row * BK + (((fg + 4) ^ (row & 7)) << 4));
      af[i] = i32x8{(int)lo[0], (int)lo[1], (int)lo[2], (int)lo[3], (int)hi[0], (int)hi[1], (int)hi[2], (int)hi[3]};
    }
#pragma unroll
    for (int j = 0; j < NI; ++j) {
      const int row = wc * WN + j * 16 + fr;
      const u32x4 lo = *reinterpret_cast<const u32x4*>(Bs + row * BK + ((fg ^ (row & 7)) << 4));
      const u32x4 hi = *reinterpret_cast<const u32x4*>(Bs + row * BK + (((fg + 4) ^ (row & 7)) << 4));
      bfr[j] = i32x8{(int)lo[0], (int)lo[1], (int)lo[2], (int)lo[3], (int)hi[0], (int)hi[1], (int)hi[2], (int)hi[3]};
    }
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NI; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(af[i], bfr[j], acc[i][j], 0, 0,
                                                                      0, 127, 0, 127);
    __builtin_amdgcn_s_setprio(0);
    slot = slot == NS - 1 ? 0 : slot + 1;
  }
  fp8_wait_vm_barrier<0>();
  fp8_epilogue<BM, BN, WGM, WGN>(p, acc, smem, m0, n0);
}

// ---------------------------------------------------------------------------------------------
// 256 x 256 tile, 8 waves as 2 (M) x 4 (N), each wave 128 x 64 (8 x 4 accumulators).  The per-
// wave register blocking is what the 16x16x128 fp8 MFMA needs: a 64 x 64 wave tile reads 2 KB
// of fragments per 32-cycle MFMA, so 8 such waves would demand the whole 256 B/clk of the CU's
// LDS; 128 x 64 reads 0.75 KB per MFMA.  Double-buffered 64 KB stages (LDS-DMA, counted vmcnt +
// raw barrier), 1024 MFMA cycles per wave per stage to cover the next stage's flight.  The fp32
// epilogue is staged through LDS in two 128-row halves.
template <bool MXA = false, bool MXO = false>
__global__ __launch_bounds__(512, 1) void gemm_fp8_big_kernel(Fp8GemmParams p, const uint8_t* zero) {
  constexpr int BM = 256, BN = 256, BK = 128, NS = 2;
  constexpr int WGN = 4;
  constexpr int WM = 128, WN = 64, MI = WM / 16, NI = WN / 16;
  constexpr int APT = BM / 64, BPT = BN / 64;   // DMA instructions per thread per stage
  constexpr int PER = APT + BPT;
  constexpr int TILE_BYTES = (BM + BN) * BK;   // 64 KB
  constexpr int STAGE_BYTES = TILE_BYTES + (MXA ? BM * 4 : 0);   // + the MX scale tile of A
  constexpr int CPAD = 4, LDC = BN + CPAD;
  constexpr int EPI_BYTES = 128 * LDC * 4;     // one 128-row half
  constexpr int RING_BYTES = NS * STAGE_BYTES;
  constexpr int LDS_BYTES = EPI_BYTES > RING_BYTES ? EPI_BYTES : RING_BYTES;
  static_assert(LDS_BYTES <= 160 * 1024, "LDS");
  __shared__ __attribute__((aligned(16))) unsigned char smem[LDS_BYTES];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave / WGN, wc = wave % WGN;
  const int ntn = (p.N + BN - 1) / BN;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int m0 = (bid / ntn) * BM, n0 = (bid % ntn) * BN;
  const int lrow = wave * 8 + (lane >> 3);
  const int lp = (lane & 7) ^ (lane >> 3);

  const uint8_t* a_src[APT];
#pragma unroll
  for (int i = 0; i < APT; ++i) {
    const int m = m0 + lrow + 64 * i;
    a_src[i] = m < p.M ? p.a + (long)m * p.lda + lp * 16 : nullptr;
  }
  const uint8_t* b_src[BPT];
#pragma unroll
  for (int i = 0; i < BPT; ++i) {
    const int n = n0 + lrow + 64 * i;
    b_src[i] = n < p.N ? p.b + (long)n * p.K + lp * 16 : nullptr;
  }
  auto issue = [&](int kb, int slot) {
    unsigned char* As = smem + slot * STAGE_BYTES;
    unsigned char* Bs = As + BM * BK;
    const int k0 = kb * BK;
#pragma unroll
    for (int i = 0; i < APT; ++i) glds16_u8(a_src[i] ? a_src[i] + k0 : zero, As + (i * 64 + wave * 8) * BK);
#pragma unroll
    for (int i = 0; i < BPT; ++i) glds16_u8(b_src[i] ? b_src[i] + k0 : zero, Bs + (i * 64 + wave * 8) * BK);
    if constexpr (MXA) {   // scale rows m0 .. m0+255 (4 B each): wave w takes 32 rows with 8 lanes
      // (the scale tensor holds M rounded up to 128 rows: a 32-row group past it reads zeros)
      const int r0 = m0 + wave * 32;
      const uint8_t* src = r0 < p.mxr ? p.amx + ((long)kb * p.mxr + r0) * 4 + lane * 16 : zero;
      if (lane < 8) glds16_u8(src, As + TILE_BYTES + wave * 128);
    }
  };

  f32x4 acc[MI][NI];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nkb = p.K / BK;
  issue(0, 0);
  const int fr = lane & 15, fg = lane >> 4;
  const int sw = fr & 7;
  const int off_lo = (fg ^ sw) << 4, off_hi = ((fg + 4) ^ sw) << 4;
  for (int kb = 0; kb < nkb; ++kb) {
    const int slot = kb & 1;
    fp8_wait_vm_barrier<0>();          // stage kb landed (this wave's DMAs) and slot kb-1 free
    if (kb + 1 < nkb) issue(kb + 1, slot ^ 1);
    const unsigned char* As = smem + slot * STAGE_BYTES + (wr * WM + fr) * BK;
    const unsigned char* Bs = smem + slot * STAGE_BYTES + BM * BK + (wc * WN + fr) * BK;
    i32x8 bfr[NI];
#pragma unroll
    for (int j = 0; j < NI; ++j) {
      const u32x4 lo = *reinterpret_cast<const u32x4*>(Bs + j * 16 * BK + off_lo);
      const u32x4 hi = *reinterpret_cast<const u32x4*>(Bs + j * 16 * BK + off_hi);
      bfr[j] = i32x8{(int)lo[0], (int)lo[1], (int)lo[2], (int)lo[3], (int)hi[0], (int)hi[1], (int)hi[2], (int)hi[3]};
    }
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      const u32x4 lo = *reinterpret_cast<const u32x4*>(As + i * 16 * BK + off_lo);
      const u32x4 hi = *reinterpret_cast<const u32x4*>(As + i * 16 * BK + off_hi);
      const i32x8 af = i32x8{(int)lo[0], (int)lo[1], (int)lo[2], (int)lo[3], (int)hi[0], (int)hi[1], (int)hi[2], (int)hi[3]};
      int asc = 127;                   // E8M0 scale of this lane's A block (byte fg of its row's word)
      if constexpr (MXA) {
        const uint32_t w4 = *reinterpret_cast<const uint32_t*>(smem + slot * STAGE_BYTES + TILE_BYTES +
                                                               (wr * WM + i * 16 + fr) * 4);
        asc = (int)(w4 >> (8 * fg));
      }
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int j = 0; j < NI; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(af, bfr[j], acc[i][j], 0, 0, 0, asc, 0, 127);
      __builtin_amdgcn_s_setprio(0);
    }
  }
  fp8_wait_vm_barrier<0>();

  // ---- epilogue: two 128-row halves through LDS ----
  float* Cs = reinterpret_cast<float*>(smem);
  constexpr int CPR = BN / 8, CHUNKS = 128 * CPR, CPT = CHUNKS / 512, E_ROWS = 512 / CPR;
  const int e_cc = tid % CPR, e_row0 = tid / CPR;
  const int e_n = n0 + e_cc * 8;
  float cs[8], cb[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) cs[e] = cb[e] = 0.f;
  if (e_n < p.N) {
    const f32x4 s0 = *reinterpret_cast<const f32x4*>(p.sb + e_n);
    const f32x4 s1 = *reinterpret_cast<const f32x4*>(p.sb + e_n + 4);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      cs[e] = s0[e];
      cs[e + 4] = s1[e];
    }
    if (p.bias) {
      const f32x4 b0 = *reinterpret_cast<const f32x4*>(p.bias + e_n);
      const f32x4 b1 = *reinterpret_cast<const f32x4*>(p.bias + e_n + 4);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        cb[e] = b0[e];
        cb[e + 4] = b1[e];
      }
    }
  }
#pragma unroll
  for (int half = 0; half < 2; ++half) {
    if (wr == half) {
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NI; ++j) {
          const int col = wc * WN + j * 16 + fr;
#pragma unroll
          for (int e = 0; e < 4; ++e) Cs[(i * 16 + fg * 4 + e) * LDC + col] = acc[i][j][e];
        }
    }
    __syncthreads();
    if (e_n < p.N) {
#pragma unroll
      for (int i = 0; i < CPT; ++i) {
        const int row = e_row0 + E_ROWS * i;
        const int m = m0 + half * 128 + row;
        const bool live = m < p.M;
        if (!MXO && !live) continue;     // (MX output: every lane joins the block reduction)
        const float rs = p.sa && live ? p.sa[m] : 1.f;
        const f32x4 c0 = *reinterpret_cast<const f32x4*>(Cs + row * LDC + e_cc * 8);
        const f32x4 c1 = *reinterpret_cast<const f32x4*>(Cs + row * LDC + e_cc * 8 + 4);
        float v[8];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          v[e] = c0[e] * rs * cs[e] + cb[e];
          v[e + 4] = c1[e] * rs * cs[e + 4] + cb[e + 4];
        }
        fp8_store_chunk<MXO>(p, v, m, e_n, e_cc, live);
      }
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------------------------
// Persistent 256 x 256 kernel (tuner variant 4) for the short-K encoder GEMMs (qkv: N = 2304,
// fc1: N = 3072, K = 768 — six K blocks per tile).  gemm_fp8_big_kernel pays, per tile, an
// unhidden first-block round trip, an fp32 epilogue staged through LDS in two halves behind
// __syncthreads, and the tile-quantisation tail of a one-shot grid; at K = 768 that is about as
// long as the six blocks of MFMA work, so the tuner picked the 2-workgroups-per-CU 128 x 128
// kernel (~1.1 PFLOP/s) instead.  Here one workgroup per CU walks tiles lid, lid + G, ... with
// ONE 2-slot ring of 64 KB K blocks running across tile boundaries (the next tile's first block
// is in flight during the current tile's last block and its epilogue), and the epilogue goes
// straight from registers: the product is transposed (weights on the MFMA A side), so lane l
// holds four consecutive output COLUMNS of row l & 15 and one v_permlane16_swap per fp32 pair
// gives it eight — per-channel scale and bias come from LDS (loaded once per workgroup for the
// whole N), then GELU, then a 16-B bf16 store or MX-fp8 quantisation (32-column blocks = the
// four lane rows of one fragment pair: two permlane swaps for the block max).  Stores are
// buffer stores with an out-of-range offset for rows past M (always issued), so the only vmcnt
// wait that is not 0 — the first block of a tile, whose younger ops are exactly the previous
// tile's NST stores — is exact.  N % 256 == 0, N <= 3072, K % 128 == 0, K >= 256, per-row A
// scales (no MX input), no residual.
template <bool MXO>
__global__ __launch_bounds__(512, 1) void gemm_fp8_pers_kernel(Fp8GemmParams p, const uint8_t* zero, int tiles_n,
                                                               int ntiles, int diag) {
  constexpr int BM = 256, BN = 256, BK = 128, WGN = 4, WM = 128, WN = 64, MI = WM / 16, NI = WN / 16;
  constexpr int APT = BM / 64, BPT = BN / 64;
  constexpr int STAGE_BYTES = (BM + BN) * BK;  // 64 KB
  constexpr int MAXN = 3072;
  constexpr int NST = MXO ? 2 * MI * (NI / 2) : MI * (NI / 2);   // store instructions per tile per wave
  __shared__ __attribute__((aligned(16))) unsigned char smem[2 * STAGE_BYTES + 2 * MAXN * 4];
  float* const s_sb = reinterpret_cast<float*>(smem + 2 * STAGE_BYTES);
  float* const s_bias = s_sb + MAXN;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave / WGN, wc = wave % WGN;
  const int G = gridDim.x;
  const int lid = xcd_remap(blockIdx.x, G);
  if (lid >= ntiles) return;
  const int my_tiles = (ntiles - 1 - lid) / G + 1;
  const int nkb = p.K / BK;
  const int lrow = wave * 8 + (lane >> 3);
  const int lp = (lane & 7) ^ (lane >> 3);
  const int fr = lane & 15, fg = lane >> 4;
  const int coff = ((fg & 1) << 4) | ((fg >> 1) << 3);

  // per-channel scales and bias for the whole N, once (retired by the first block's wait)
  for (int n = tid; n < p.N; n += 512) {
    s_sb[n] = p.sb[n];
    s_bias[n] = p.bias ? p.bias[n] : 0.f;
  }

  auto issue = [&](int f) {                          // flat K block f of this workgroup's walk
    const int k = f / nkb, kb = f - k * nkb;
    if (k >= my_tiles) return;
    if ((diag & 1) && f > 1) return;                 // timing diagnostic: MFMA + LDS on stale blocks
    const int tau = lid + k * G;
    const int m0 = (tau / tiles_n) * BM, n0 = (tau % tiles_n) * BN;
    unsigned char* As = smem + (f & 1) * STAGE_BYTES;
    unsigned char* Bs = As + BM * BK;
    const int k0 = kb * BK;
#pragma unroll
    for (int i = 0; i < APT; ++i) {
      const int m = m0 + lrow + 64 * i;
      glds16_u8(m < p.M ? p.a + (long)m * p.lda + lp * 16 + k0 : zero, As + (i * 64 + wave * 8) * BK);
    }
#pragma unroll
    for (int i = 0; i < BPT; ++i)
      glds16_u8(p.b + (long)(n0 + lrow + 64 * i) * p.K + lp * 16 + k0, Bs + (i * 64 + wave * 8) * BK);
  };

  const __amdgpu_buffer_rsrc_t ry = __builtin_amdgcn_make_buffer_rsrc(MXO ? (void*)p.yq : (void*)p.y, (short)0,
                                                                      0x7ffffff0, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsc = __builtin_amdgcn_make_buffer_rsrc(MXO ? (void*)p.ysc : (void*)p.y, (short)0,
                                                                       0x7ffffff0, 0x00020000);
  const int off_lo = (fg ^ (fr & 7)) << 4, off_hi = ((fg + 4) ^ (fr & 7)) << 4;

  issue(0);
  f32x4 acc[MI][NI];
  float rs[MI];
  for (int k = 0; k < my_tiles; ++k) {
    const int tau = lid + k * G;
    const int m0 = (tau / tiles_n) * BM, n0 = (tau % tiles_n) * BN;
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NI; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int kb = 0; kb < nkb; ++kb) {
      const int f = k * nkb + kb;
      if (diag & 4) asm volatile("s_waitcnt vmcnt(0)\n\ts_waitcnt lgkmcnt(0)" ::: "memory");   // diag: no barrier
      else if (kb == 0 && k > 0) fp8_wait_vm_barrier<NST>();   // younger: the previous tile's stores
      else fp8_wait_vm_barrier<0>();
      if (kb == 0) {                                 // row scales, older than the next block's DMA
#pragma unroll
        for (int i = 0; i < MI; ++i) {
          const int m = m0 + wr * WM + i * 16 + fr;
          rs[i] = p.sa && m < p.M ? p.sa[m] : 1.f;
        }
      }
      issue(f + 1);
      const unsigned char* As = smem + (f & 1) * STAGE_BYTES + (wr * WM + fr) * BK;
      const unsigned char* Bs = smem + (f & 1) * STAGE_BYTES + BM * BK + (wc * WN + fr) * BK;
      auto frag = [&](const unsigned char* base) {
        const u32x4 lo = *reinterpret_cast<const u32x4*>(base + off_lo);
        const u32x4 hi = *reinterpret_cast<const u32x4*>(base + off_hi);
        return i32x8{(int)lo[0], (int)lo[1], (int)lo[2], (int)lo[3], (int)hi[0], (int)hi[1], (int)hi[2], (int)hi[3]};
      };
      // software-pipelined fragment reads: A fragment i + 1 is read while the MFMAs on fragment
      // i run, so only the weight fragments and A0 are exposed after the barrier, and 2 A
      // fragments (not MI) are live.  The sched_group_barriers pin that order: left alone the
      // scheduler hoists all 24 reads above the first MFMA and waits on lgkmcnt(0).
      i32x8 bfr[NI];
#pragma unroll
      for (int j = 0; j < NI; ++j) bfr[j] = frag(Bs + j * 16 * BK);
      i32x8 acur = frag(As);
      __builtin_amdgcn_sched_group_barrier(0x100, 2 * NI + 2, 0);
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        i32x8 anxt = acur;
        if (i + 1 < MI) {
          anxt = frag(As + (i + 1) * 16 * BK);
          __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
        }
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int j = 0; j < NI; ++j)   // transposed: weights first, so lanes end with 4 consecutive columns
          acc[i][j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(bfr[j], acur, acc[i][j], 0, 0, 0, 127, 0, 127);
        __builtin_amdgcn_sched_group_barrier(0x008, NI, 0);
        __builtin_amdgcn_s_setprio(0);
        acur = anxt;
      }
    }
    // ---- register-direct epilogue (the ring is not touched: no barrier) ----
    if (diag & 8) {                                  // timing diagnostic: no epilogue at all
      if (acc[0][0][0] == 12345.f) __builtin_amdgcn_s_sleep(1);   // keeps the MFMAs live
      continue;
    }
#pragma unroll
    for (int pp = 0; pp < NI / 2; ++pp) {
      const int nb = n0 + wc * WN + pp * 32;         // first column of this fragment pair
      const int n = nb + coff;                       // this lane's 8 columns
      const f32x4 sc0 = *reinterpret_cast<const f32x4*>(s_sb + n);
      const f32x4 sc1 = *reinterpret_cast<const f32x4*>(s_sb + n + 4);
      const f32x4 bi0 = *reinterpret_cast<const f32x4*>(s_bias + n);
      const f32x4 bi1 = *reinterpret_cast<const f32x4*>(s_bias + n + 4);
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        const int m = m0 + wr * WM + i * 16 + fr;
        f32x4 lo = acc[i][2 * pp], hi = acc[i][2 * pp + 1];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const auto sw = __builtin_amdgcn_permlane16_swap(__float_as_uint(lo[e]), __float_as_uint(hi[e]), false, false);
          lo[e] = __uint_as_float(sw[0]);
          hi[e] = __uint_as_float(sw[1]);
        }
        float v[8];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          v[e] = lo[e] * rs[i] * sc0[e] + bi0[e];
          v[e + 4] = hi[e] * rs[i] * sc1[e] + bi1[e];
        }
        if (p.act == 1) {
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] = fmaxf(v[e], 0.f);
        } else if (p.act == 2) {
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] = silu(v[e]);
        } else if (p.act == 3) {
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const f32x2 g = gelu_erf2(f32x2{v[2 * e], v[2 * e + 1]});
            v[2 * e] = g[0];
            v[2 * e + 1] = g[1];
          }
        }
        const bool live = m < p.M;
        if constexpr (MXO) {
          float amax = 0.f;
#pragma unroll
          for (int e = 0; e < 8; ++e) amax = fmaxf(amax, fabsf(v[e]));
          {
            const auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(amax), __float_as_uint(amax), false, false);
            amax = fmaxf(__uint_as_float(a[0]), __uint_as_float(a[1]));
          }
          {
            const auto a = __builtin_amdgcn_permlane32_swap(__float_as_uint(amax), __float_as_uint(amax), false, false);
            amax = fmaxf(__uint_as_float(a[0]), __uint_as_float(a[1]));
          }
          const int ex = mx_exponent(amax);
          const float inv = __uint_as_float((uint32_t)(127 - ex) << 23);
          unsigned w0 = 0u, w1 = 0u;
          w0 = __builtin_amdgcn_cvt_pk_fp8_f32(fminf(fmaxf(v[0] * inv, -448.f), 448.f),
                                               fminf(fmaxf(v[1] * inv, -448.f), 448.f), w0, false);
          w0 = __builtin_amdgcn_cvt_pk_fp8_f32(fminf(fmaxf(v[2] * inv, -448.f), 448.f),
                                               fminf(fmaxf(v[3] * inv, -448.f), 448.f), w0, true);
          w1 = __builtin_amdgcn_cvt_pk_fp8_f32(fminf(fmaxf(v[4] * inv, -448.f), 448.f),
                                               fminf(fmaxf(v[5] * inv, -448.f), 448.f), w1, false);
          w1 = __builtin_amdgcn_cvt_pk_fp8_f32(fminf(fmaxf(v[6] * inv, -448.f), 448.f),
                                               fminf(fmaxf(v[7] * inv, -448.f), 448.f), w1, true);
          typedef __attribute__((ext_vector_type(2))) unsigned u32x2v;
          const uint32_t qoff = live ? (uint32_t)((long)m * p.ldq + n) : 0x80000000u;
          __builtin_amdgcn_raw_buffer_store_b64(u32x2v{w0, w1}, ry, qoff, 0, 0);
          const uint32_t soff = live && fg == 0 ? (uint32_t)(((long)(nb >> 7) * p.ysr + m) * 4 + ((nb >> 5) & 3))
                                                : 0x80000000u;
          __builtin_amdgcn_raw_buffer_store_b8((unsigned char)(ex + 127), rsc, soff, 0, 0);
        } else {
          u32x4 o;
#pragma unroll
          for (int e = 0; e < 4; ++e) o[e] = pack2(v[2 * e], v[2 * e + 1]);
          const uint32_t yoff = live ? (uint32_t)(((long)m * p.ldy + n) * 2) : 0x80000000u;
          if (!(diag & 2)) __builtin_amdgcn_raw_buffer_store_b128(o, ry, yoff, 0, 0);
        }
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// Epilogue of one 16-row fragment group of the persistent kernels' 128 x 64 wave tile: both
// 32-column fragment pairs (lane l: row l & 15, eight consecutive columns after the permlane
// swap), per-channel scale + bias from LDS, activation, bf16 or MX-fp8 store.
// AIKO_FP8_POLY_GELU=0 at build time (-DAIKO_FP8_POLY_GELU=0): the erf GELU in the MX-out epilogue
#ifndef AIKO_FP8_POLY_GELU
#define AIKO_FP8_POLY_GELU 1
#endif
constexpr bool kFp8PolyGelu = AIKO_FP8_POLY_GELU != 0;

// four fp32 -> e4m3 bytes (a in byte 0) divided by the power-of-two MX scale, in two
// v_cvt_scalef32_pk_fp8_f32 (gfx950)
__device__ __forceinline__ unsigned mx_pack4(float a, float b, float c, float d, float scale) {
  typedef __attribute__((ext_vector_type(2))) short v2s;
  v2s r = __builtin_amdgcn_cvt_scalef32_pk_fp8_f32(v2s{0, 0}, a, b, scale, false);
  r = __builtin_amdgcn_cvt_scalef32_pk_fp8_f32(r, c, d, scale, true);
  return __builtin_bit_cast(unsigned, r);
}

__device__ __forceinline__ float fp8_h2f(uint32_t bits) {
  return (float)__builtin_bit_cast(_Float16, (unsigned short)bits);
}

// LN 2 (LayerNorm-folded consumer): rs = rstd of row m, r2 = -mean * rstd, and s_bias holds
// (cs, bias) as half2 — v = rstd * (acc * sb - mean * cs) + bias.  LN 1 (producer): after the
// bf16 store, the stored values' MX-fp8 copy (yq / ysc) and their row sum / sum of squares over
// this wave's 64 columns into LDS (s_part, lane group 0).
template <bool MXO, int ACT, bool RES, int LN = 0>
__device__ __forceinline__ void fp8_pers_epi(const Fp8GemmParams& p, const f32x4 (&acc)[4], float rs, float r2, int m,
                                             int nw, int coff, int fg, const float* s_sb, const float* s_bias,
                                             __amdgpu_buffer_rsrc_t ry, __amdgpu_buffer_rsrc_t rsc,
                                             const u32x4 (&rv)[2], __amdgpu_buffer_rsrc_t rq, float* s_part) {
  [[maybe_unused]] float s1 = 0.f, s2 = 0.f;
  [[maybe_unused]] int ex2[2] = {0, 0};
#pragma unroll
  for (int pp = 0; pp < 2; ++pp) {
    const int nb = nw + pp * 32, n = nb + coff;
    const f32x4 sc0 = *reinterpret_cast<const f32x4*>(s_sb + n);
    const f32x4 sc1 = *reinterpret_cast<const f32x4*>(s_sb + n + 4);
    const f32x4 bi0 = *reinterpret_cast<const f32x4*>(s_bias + n);
    const f32x4 bi1 = *reinterpret_cast<const f32x4*>(s_bias + n + 4);
    f32x4 lo = acc[2 * pp], hi = acc[2 * pp + 1];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const auto sw = __builtin_amdgcn_permlane16_swap(__float_as_uint(lo[e]), __float_as_uint(hi[e]), false, false);
      lo[e] = __uint_as_float(sw[0]);
      hi[e] = __uint_as_float(sw[1]);
    }
    float v[8];
    if constexpr (LN == 2) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const uint32_t c0 = __float_as_uint(bi0[e]), c1 = __float_as_uint(bi1[e]);   // (cs, bias) half2
        v[e] = (lo[e] * sc0[e]) * rs + (r2 * fp8_h2f(c0 & 0xffffu) +
                                        fp8_h2f(c0 >> 16));
        v[e + 4] = (hi[e] * sc1[e]) * rs + (r2 * fp8_h2f(c1 & 0xffffu) +
                                            fp8_h2f(c1 >> 16));
      }
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        v[e] = lo[e] * rs * sc0[e] + bi0[e];
        v[e + 4] = hi[e] * rs * sc1[e] + bi1[e];
      }
    }
    if constexpr (ACT == 1) {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = fmaxf(v[e], 0.f);
    } else if constexpr (ACT == 2) {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = silu(v[e]);
    } else if constexpr (ACT == 3 && MXO && kFp8PolyGelu) {   // MX-fp8 out: transcendental-free GELU
      f32x2 g[4] = {{v[0], v[1]}, {v[2], v[3]}, {v[4], v[5]}, {v[6], v[7]}};
      gelu_poly_n<4>(g);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        v[2 * e] = g[e][0];
        v[2 * e + 1] = g[e][1];
      }
    } else if constexpr (ACT == 3) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const f32x2 g = gelu_erf2(f32x2{v[2 * e], v[2 * e + 1]});
        v[2 * e] = g[0];
        v[2 * e + 1] = g[1];
      }
    }
    if constexpr (RES) {                             // residual (8 bf16, prefetched), after the activation
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        v[2 * e] += __uint_as_float(rv[pp][e] << 16);
        v[2 * e + 1] += __uint_as_float(rv[pp][e] & 0xffff0000u);
      }
    }
    const bool live = m < p.M;
    if constexpr (MXO) {
      float amax = 0.f;
#pragma unroll
      for (int e = 0; e < 8; ++e) amax = fmaxf(amax, fabsf(v[e]));
      {
        const auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(amax), __float_as_uint(amax), false, false);
        amax = fmaxf(__uint_as_float(a[0]), __uint_as_float(a[1]));
      }
      {
        const auto a = __builtin_amdgcn_permlane32_swap(__float_as_uint(amax), __float_as_uint(amax), false, false);
        amax = fmaxf(__uint_as_float(a[0]), __uint_as_float(a[1]));
      }
      const int ex = mx_exponent(amax);
      // one v_cvt_scalef32_pk_fp8_f32 per pair (divides by the 2^ex scale; |v| / 2^ex <= 448 by
      // the exponent's choice, so no clamp): scripts/probe/cvt_scale_probe.hip
      const float sc2 = __uint_as_float((uint32_t)(ex + 127) << 23);
      const unsigned w0 = mx_pack4(v[0], v[1], v[2], v[3], sc2), w1 = mx_pack4(v[4], v[5], v[6], v[7], sc2);
      typedef __attribute__((ext_vector_type(2))) unsigned u32x2v;
      const uint32_t qoff = live ? (uint32_t)((long)m * p.ldq + n) : 0x80000000u;
      __builtin_amdgcn_raw_buffer_store_b64(u32x2v{w0, w1}, ry, qoff, 0, 0);
      const uint32_t soff = live && fg == 0 ? (uint32_t)(((long)(nb >> 7) * p.ysr + m) * 4 + ((nb >> 5) & 3))
                                            : 0x80000000u;
      __builtin_amdgcn_raw_buffer_store_b8((unsigned char)(ex + 127), rsc, soff, 0, 0);
    } else {
      u32x4 o;
#pragma unroll
      for (int e = 0; e < 4; ++e) o[e] = pack2(v[2 * e], v[2 * e + 1]);
      const uint32_t yoff = live ? (uint32_t)(((long)m * p.ldy + n) * 2) : 0x80000000u;
      __builtin_amdgcn_raw_buffer_store_b128(o, ry, yoff, 0, 0);
      if constexpr (LN == 1) {                       // the stored (bf16-rounded) values
        float w[8];
        float amax = 0.f;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          w[2 * e] = __uint_as_float(o[e] << 16);
          w[2 * e + 1] = __uint_as_float(o[e] & 0xffff0000u);
        }
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          amax = fmaxf(amax, fabsf(w[e]));
          s1 += w[e];
          s2 += w[e] * w[e];
        }
        {
          const auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(amax), __float_as_uint(amax), false, false);
          amax = fmaxf(__uint_as_float(a[0]), __uint_as_float(a[1]));
        }
        {
          const auto a = __builtin_amdgcn_permlane32_swap(__float_as_uint(amax), __float_as_uint(amax), false, false);
          amax = fmaxf(__uint_as_float(a[0]), __uint_as_float(a[1]));
        }
        const int ex = mx_exponent(amax);
        ex2[pp] = ex;
        const float inv = __uint_as_float((uint32_t)(127 - ex) << 23);
        unsigned w0 = 0u, w1 = 0u;
        w0 = __builtin_amdgcn_cvt_pk_fp8_f32(fminf(fmaxf(w[0] * inv, -448.f), 448.f),
                                             fminf(fmaxf(w[1] * inv, -448.f), 448.f), w0, false);
        w0 = __builtin_amdgcn_cvt_pk_fp8_f32(fminf(fmaxf(w[2] * inv, -448.f), 448.f),
                                             fminf(fmaxf(w[3] * inv, -448.f), 448.f), w0, true);
        w1 = __builtin_amdgcn_cvt_pk_fp8_f32(fminf(fmaxf(w[4] * inv, -448.f), 448.f),
                                             fminf(fmaxf(w[5] * inv, -448.f), 448.f), w1, false);
        w1 = __builtin_amdgcn_cvt_pk_fp8_f32(fminf(fmaxf(w[6] * inv, -448.f), 448.f),
                                             fminf(fmaxf(w[7] * inv, -448.f), 448.f), w1, true);
        typedef __attribute__((ext_vector_type(2))) unsigned u32x2v;
        const uint32_t qoff = live ? (uint32_t)((long)m * p.ldq + n) : 0x80000000u;
        __builtin_amdgcn_raw_buffer_store_b64(u32x2v{w0, w1}, rq, qoff, 0, 0);
      }
    }
  }
  if constexpr (LN == 1) {
    // both 32-column blocks' scale bytes are adjacent (nw % 64 == 0): one 2-byte store
    const bool live = m < p.M;
    const uint32_t soff = live && fg == 0 ? (uint32_t)(((long)(nw >> 7) * p.ysr + m) * 4 + ((nw >> 5) & 3))
                                          : 0x80000000u;
    __builtin_amdgcn_raw_buffer_store_b16((unsigned short)((ex2[0] + 127) | ((ex2[1] + 127) << 8)), rsc, soff, 0, 0);
    // row partials over the lane group's four 8-column pieces
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      float& u = t ? s2 : s1;
      const auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(u), __float_as_uint(u), false, false);
      u = __uint_as_float(a[0]) + __uint_as_float(a[1]);
      const auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(u), __float_as_uint(u), false, false);
      u = __uint_as_float(b[0]) + __uint_as_float(b[1]);
    }
    if (fg == 0) *reinterpret_cast<float2*>(s_part) = make_float2(s1, s2);
  }
}

// Persistent 256 x 256 fp8 GEMM, epilogue overlapped with MFMA work (tuner variant 4;
// AIKO_FP8_OVERLAP=0 selects gemm_fp8_pers_kernel above).  qkv 56.3 -> 51.5 us, fc1 (GELU + MX
// out) 75.1 -> 68.0 us, Whisper-small 14-stream bench 3,076 / 3,125 -> 3,208 / 3,226 windows/s
// (scripts/fp8_diag.sh, interleaved).  Same walk, ring and store layout, two
// changes in the schedule:
//   - the epilogue of tile k runs interleaved with the first K block of tile k + 1: fragment
//     group i is stored, then its accumulators take the next tile's group-i MFMAs (started from
//     zero), so the epilogue's VALU and store issue overlap the matrix pipe instead of leaving it
//     idle for ~20 % of the kernel (AIKO_FP8_DIAG=8 on the kernel above: 36.8 -> 29.9 us, qkv);
//   - the fragment reads are issued by hand (fp8_lds_rd128) with counted lgkmcnt waits, A
//     fragment i + LA in flight while the MFMAs on fragment i run.
// vmcnt: block (k, 1)'s DMA is issued right after the fused block's barrier, before that
// block's stores, so its wait is vmcnt(NST); every other wait is vmcnt(0).
//
// LayerNorm folded across a GEMM pair (LN template argument; Whisper's out-proj / fc2 -> qkv / fc1):
//   LN(x) W^T + b = rstd * (x - mean) (W diag g)^T + (b + W beta)
//                 = rstd * (x W'^T) - rstd * mean * cs + b',   cs[n] = sum_k W'[n, k]
// so the consumer (LN 2) multiplies the MX-fp8 copy of the raw residual stream x by the folded
// weights and applies the row's statistics in its epilogue; no normalised / quantised copy of x
// is ever materialised.  The producer (LN 1: the GEMM that writes x, with its residual add)
// quantises its own output tile to MX-fp8 (block scales are local to 32 columns) and reduces the
// row sum / sum of squares of each 256-column tile: per wave in registers, across the tile's four
// column waves in LDS, written out one K block into the next tile (after that block's barrier)
// as st[tile_n][m] — deterministic, no atomics.  The consumer reads the stp partials of its rows
// a K block ahead (lane group g loads partial g), reduces them across the lane groups and forms
// (rstd, -mean * rstd).
template <int BM, bool MXO, int ACT, bool MXA, bool RES, int LN = 0>
__global__ __launch_bounds__(512, 1) void gemm_fp8_pers2_kernel(Fp8GemmParams p, const uint8_t* zero, int tiles_n,
                                                                int ntiles, int diag) {
  constexpr int BN = 256, BK = 128, WGN = 4, WM = BM / 2, WN = 64, MI = WM / 16, NI = WN / 16;
  constexpr int APT = BM / 64, BPT = BN / 64;
  constexpr int TILE_BYTES = (BM + BN) * BK;
  constexpr int STAGE_BYTES = TILE_BYTES + (MXA ? BM * 4 : 0);   // + the MX scale tile of A
  constexpr int MAXN = LN == 1 ? 1024 : 3072;
  // store instructions per tile per wave (LN 1: bf16 + MX bytes per 32-column pair, one 2-byte
  // scale store per fragment group)
  constexpr int NST = MXO ? 2 * MI * (NI / 2) : LN == 1 ? 5 * MI : MI * (NI / 2);
  constexpr int LA = (MXO && ACT == 3) || (BM == 256 && RES) ? 1 : 2;   // A fragments read ahead (1: registers)
  // residual loads (LN 2: row-statistics partials) per tile per wave, always issued
  constexpr int NRL = RES ? 2 * MI : (LN == 2 ? MI : 0);
  static_assert(NST + NRL <= 63, "vmcnt is a 6-bit counter");
  static_assert(LN == 0 || BM == 256, "LayerNorm folding: 256 x 256 tiles");
  static_assert(LN != 1 || (RES && !MXO && ACT == 0), "LN producer: bf16 out + residual, no activation");
  constexpr int PART_BYTES = LN == 1 ? BM * 4 * 8 : 0;   // [BM rows][4 column waves] float2
  __shared__ __attribute__((aligned(16))) unsigned char smem[2 * STAGE_BYTES + 2 * MAXN * 4 + PART_BYTES];
  float* const s_sb = reinterpret_cast<float*>(smem + 2 * STAGE_BYTES);
  float* const s_bias = s_sb + MAXN;
  [[maybe_unused]] float* const s_part = s_bias + MAXN;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave / WGN, wc = wave % WGN;
  const int G = gridDim.x;
  const int lid = xcd_remap(blockIdx.x, G);
  if (lid >= ntiles) return;
  const int my_tiles = (ntiles - 1 - lid) / G + 1;
  const int nkb = p.K / BK;
  const int lrow = wave * 8 + (lane >> 3);
  const int lp = (lane & 7) ^ (lane >> 3);
  const int fr = lane & 15, fg = lane >> 4;
  const int coff = ((fg & 1) << 4) | ((fg >> 1) << 3);

  for (int n = tid; n < p.N; n += 512) {
    s_sb[n] = p.sb[n];
    if constexpr (LN == 2) {                         // (cs, bias) as half2
      const float b = p.bias ? p.bias[n] : 0.f;
      const uint32_t lo = __builtin_bit_cast(unsigned short, (_Float16)p.cs[n]);
      const uint32_t hi = __builtin_bit_cast(unsigned short, (_Float16)b);
      s_bias[n] = __uint_as_float(lo | (hi << 16));
    } else {
      s_bias[n] = p.bias ? p.bias[n] : 0.f;
    }
  }

  auto issue = [&](int f) {                          // flat K block f of this workgroup's walk
    const int k = f / nkb, kb = f - k * nkb;
    if (k >= my_tiles) return;
    if ((diag & 1) && f > 1) return;                 // timing diagnostic: MFMA + LDS on stale blocks
    const int tau = lid + k * G;
    const int m0 = (tau / tiles_n) * BM, n0 = (tau % tiles_n) * BN;
    unsigned char* As = smem + (f & 1) * STAGE_BYTES;
    unsigned char* Bs = As + BM * BK;
    const int k0 = kb * BK;
#pragma unroll
    for (int i = 0; i < APT; ++i) {
      const int m = m0 + lrow + 64 * i;
      glds16_u8(m < p.M ? p.a + (long)m * p.lda + lp * 16 + k0 : zero, As + (i * 64 + wave * 8) * BK);
    }
#pragma unroll
    for (int i = 0; i < BPT; ++i)
      glds16_u8(p.b + (long)(n0 + lrow + 64 * i) * p.K + lp * 16 + k0, Bs + (i * 64 + wave * 8) * BK);
    if constexpr (MXA) {   // scale rows m0 .. m0 + BM - 1 (4 B each): wave w takes BM / 8 rows
      const int r0 = m0 + wave * (BM / 8);           // (the scale tensor holds M rounded up to 128 rows)
      const uint8_t* src = r0 < p.mxr ? p.amx + ((long)kb * p.mxr + r0) * 4 + lane * 16 : zero;
      if (lane < BM / 32) glds16_u8(src, As + TILE_BYTES + wave * (BM / 2));
    }
  };
  // per-row A scales of tile k, loaded one K block before they are used: branch-free buffer
  // loads (rows past M read out of range -> 0); no per-row scales -> 1, applied at the use
  const __amdgpu_buffer_rsrc_t rsa = __builtin_amdgcn_make_buffer_rsrc((void*)p.sa, (short)0,
                                                                       p.sa ? p.M * 4 : 0, 0x00020000);
  auto load_rs = [&](int k, float (&r)[MI]) {
    const int m0 = ((lid + k * G) / tiles_n) * BM;
#pragma unroll
    for (int i = 0; i < MI; ++i)
      r[i] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rsa, (m0 + wr * WM + i * 16 + fr) * 4, 0, 0));
  };
  // LN 1: row partials out; LN 2: in (lane group g loads partial g of its row)
  const __amdgpu_buffer_rsrc_t rst = __builtin_amdgcn_make_buffer_rsrc(
      LN ? (void*)p.st : (void*)p.sb, (short)0, LN == 2 ? p.stp * p.sts * 8 : (LN == 1 ? 0x7ffffff0 : 0), 0x00020000);

  const __amdgpu_buffer_rsrc_t ry = __builtin_amdgcn_make_buffer_rsrc(MXO ? (void*)p.yq : (void*)p.y, (short)0,
                                                                      0x7ffffff0, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsc = __builtin_amdgcn_make_buffer_rsrc((MXO || LN == 1) ? (void*)p.ysc : (void*)p.y,
                                                                       (short)0, 0x7ffffff0, 0x00020000);
  const __amdgpu_buffer_rsrc_t rq = __builtin_amdgcn_make_buffer_rsrc(LN == 1 ? (void*)p.yq : (void*)p.y, (short)0,
                                                                      0x7ffffff0, 0x00020000);
  const __amdgpu_buffer_rsrc_t rres_rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)p.res, (short)0, 0x7ffffff0,
                                                                             0x00020000);
  const int off_lo = (fg ^ (fr & 7)) << 4, off_hi = ((fg + 4) ^ (fr & 7)) << 4;

  f32x4 acc[MI][NI];
  // MFMAs of flat K block f; Z: start from zero; pre(i) runs before fragment group i's MFMAs
  auto kblock = [&](int f, auto ztag, auto&& pre) {
    constexpr bool Z = decltype(ztag)::value;
    const uint32_t la = (uint32_t)reinterpret_cast<uintptr_t>(smem + (f & 1) * STAGE_BYTES + (wr * WM + fr) * BK);
    const uint32_t* scw = reinterpret_cast<const uint32_t*>(smem + (f & 1) * STAGE_BYTES + TILE_BYTES) + wr * WM + fr;
    const uint32_t lb = la + (uint32_t)(BM * BK + (wc * WN - wr * WM) * BK);
    const uint32_t alo = la + off_lo, ahi = la + off_hi, blo = lb + off_lo, bhi = lb + off_hi;
    u32x4 bl[NI], bh[NI], al[MI], ah[MI];
    fp8_static_for<0, NI>([&](auto J) {
      constexpr int j = decltype(J)::value;
      bl[j] = fp8_lds_rd128<j * 16 * BK>(blo);
      bh[j] = fp8_lds_rd128<j * 16 * BK>(bhi);
    });
    fp8_static_for<0, LA>([&](auto I) {
      constexpr int i = decltype(I)::value;
      al[i] = fp8_lds_rd128<i * 16 * BK>(alo);
      ah[i] = fp8_lds_rd128<i * 16 * BK>(ahi);
    });
    fp8_static_for<0, MI>([&](auto I) {
      constexpr int i = decltype(I)::value;
      constexpr int last = i + LA < MI ? i + LA : MI - 1;
      if constexpr (i + LA < MI) {
        al[i + LA] = fp8_lds_rd128<(i + LA) * 16 * BK>(alo);
        ah[i + LA] = fp8_lds_rd128<(i + LA) * 16 * BK>(ahi);
      }
      pre(I);
      if constexpr (i == 0) fp8_lgkm_tie<2 * (last - i)>(bl, bh, al[0], ah[0]);
      else fp8_lgkm_tie<2 * (last - i)>(al[i], ah[i]);
      const i32x8 af = fp8_frag(al[i], ah[i]);
      int asc = 127;                                 // E8M0 scale of this lane's A block (byte fg)
      if constexpr (MXA) asc = (int)(scw[i * 16] >> (8 * fg));
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int j = 0; j < NI; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(
            fp8_frag(bl[j], bh[j]), af, Z ? f32x4{0.f, 0.f, 0.f, 0.f} : acc[i][j], 0, 0, 0, 127, 0, asc);
      __builtin_amdgcn_s_setprio(0);
      // pin the previous group's MFMAs here (a use, 4 MFMAs after them: no wait states): in the
      // fused block their results are next read a K block later, and the compiler sank them
      // below the epilogue
      if constexpr (i > 0) fp8_pin(acc[i - 1]);
    });
    fp8_pin(acc[MI - 1]);
  };
  auto nop = [](auto) {};

  // LN 1: tile kp's row partials (its four column waves, in s_part since the barrier just passed)
  // -> st[tile_n][m]: two threads per row, the even one stores
  auto part_out = [&](int kp) {
    if constexpr (LN == 1) {
      const int tau = lid + kp * G;
      const int m = (tau / tiles_n) * BM + (tid >> 1);
      const f32x4 a = *reinterpret_cast<const f32x4*>(s_part + (tid >> 1) * 8 + (tid & 1) * 4);
      float t1 = a[0] + a[2], t2 = a[1] + a[3];
      t1 += dpp_f32<0xB1>(t1);
      t2 += dpp_f32<0xB1>(t2);
      typedef __attribute__((ext_vector_type(2))) unsigned u32x2v;
      const uint32_t off = (tid & 1) == 0 && m < p.M ? (uint32_t)(((long)(tau % tiles_n) * p.sts + m) * 8) : 0x80000000u;
      __builtin_amdgcn_raw_buffer_store_b64(u32x2v{__float_as_uint(t1), __float_as_uint(t2)}, rst, off, 0, 0);
    }
  };

  float rs[MI], rsn[MI];
  issue(0);
  fp8_wait_vm_barrier<0>();                          // block 0 landed; scale / bias table written
  load_rs(0, rs);
  issue(1);
  kblock(0, std::true_type{}, nop);
  for (int k = 0; k < my_tiles; ++k) {
    const int tau = lid + k * G;
    const int m0 = (tau / tiles_n) * BM, n0 = (tau % tiles_n) * BN;
    for (int kb = 1; kb < nkb; ++kb) {
      const int f = k * nkb + kb;
      if (kb == 1 && k > 0) {
        fp8_wait_vm_barrier<NST + NRL>();            // younger: the previous tile's stores and
        part_out(k - 1);                             // residual loads
      } else {
        fp8_wait_vm_barrier<0>();
      }
      if (kb == nkb - 1 && k + 1 < my_tiles) load_rs(k + 1, rsn);   // older than the next DMA
      issue(f + 1);
      kblock(f, std::false_type{}, nop);
    }
    const int mw = m0 + wr * WM + fr, nw = n0 + wc * WN;
    u32x4 rres[MI][2];                               // residual of fragment group i, loaded a group ahead
    [[maybe_unused]] float st1[MI], st2[MI];         // LN 2: row partials of group i, likewise
    auto ldres = [&](int i) {
      if constexpr (LN == 2) {
        const int m = mw + i * 16;
        const uint32_t off = fg < p.stp && m < p.M ? (uint32_t)((fg * p.sts + m) * 8) : 0x80000000u;
        const auto u = __builtin_amdgcn_raw_buffer_load_b64(rst, off, 0, 0);
        st1[i] = __uint_as_float(u[0]);
        st2[i] = __uint_as_float(u[1]);
      }
      if constexpr (RES) {
        const int m = mw + i * 16;
#pragma unroll
        for (int pp = 0; pp < 2; ++pp) {
          const uint32_t off = m < p.M ? (uint32_t)(((long)m * p.ldr + nw + pp * 32 + coff) * 2) : 0x80000000u;
          rres[i][pp] = __builtin_amdgcn_raw_buffer_load_b128(rres_rsrc, off, 0, 0);
        }
      }
    };
    auto epi = [&](auto I) {
      constexpr int i = decltype(I)::value;
      if constexpr (i + 1 < MI) ldres(i + 1);
      // MX-fp8 A carries its scales in the blocks (the host refuses sa with amx): with rs dead the
      // <256, MXA, RES> variant fits its 256 VGPRs (it spilled 24 B, and one reload's vmcnt(0)
      // inside the fused epilogue drained the next K block's DMA every tile)
      float r1 = !MXA && p.sa ? rs[i] : 1.f, r2 = 0.f;
      if constexpr (LN == 2) {                       // row statistics from the lane groups' partials
        float t1 = st1[i], t2 = st2[i];
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          float& u = t ? t2 : t1;
          const auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(u), __float_as_uint(u), false, false);
          u = __uint_as_float(a[0]) + __uint_as_float(a[1]);
          const auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(u), __float_as_uint(u), false, false);
          u = __uint_as_float(b[0]) + __uint_as_float(b[1]);
        }
        const float inv_d = 1.f / (float)p.ln_d;
        const float mean = t1 * inv_d;
        r1 = rsqrtf(fmaxf(t2 * inv_d - mean * mean, 0.f) + p.ln_eps);
        r2 = -mean * r1;
      }
      fp8_pers_epi<MXO, ACT, RES, LN>(p, acc[i], r1, r2, mw + i * 16, nw, coff, fg, s_sb, s_bias, ry, rsc, rres[i], rq,
                                      s_part + (wr * WM + i * 16 + fr) * 8 + wc * 2);
    };
    if (k + 1 < my_tiles) {                          // epilogue fused with the next tile's block 0
      const int f = (k + 1) * nkb;
      fp8_wait_vm_barrier<0>();
      issue(f + 1);
      ldres(0);
      kblock(f, std::true_type{}, epi);
#pragma unroll
      for (int i = 0; i < MI; ++i) rs[i] = rsn[i];
    } else {
      ldres(0);
      fp8_static_for<0, MI>(epi);
      if constexpr (LN == 1) {                       // the last tile's partials
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        part_out(k);
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// ---------------------------------------------------------------------------------------------
// Row-wise LayerNorm and/or fp8 quantisation, one wave per row (wave64 reductions):
//   z = gamma ? (x - mean) * rstd * gamma + beta : x
//   yb (optional) = bf16(z);  q (optional) = e4m3(z / s), s = amax(|z|) / 448 per row.
// Rows are read once with 16-byte loads and kept in registers (D <= 64 * 8 * MAXC).
// sum / max over a row's lane group: the whole wave (HALF = 0) or a 32-lane half (HALF = 1:
// DPP steps inside 16-lane rows, then v_permlane16_swap pairs rows 0-1 and 2-3 only)
template <int HALF>
__device__ __forceinline__ float group_sum(float v) {
  if constexpr (HALF == 0) {
    return wave_sum(v);
  } else {
    auto add = [](float x, float y) { return x + y; };
    v = add(v, dpp_f32<0xB1>(v));
    v = add(v, dpp_f32<0x4E>(v));
    v = add(v, dpp_f32<0x141>(v));
    v = add(v, dpp_f32<0x140>(v));
    const auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    return add(__uint_as_float(a[0]), __uint_as_float(a[1]));
  }
}

template <int HALF>
__device__ __forceinline__ float group_max(float v) {
  if constexpr (HALF == 0) {
    return wave_max(v);
  } else {
    auto mx = [](float x, float y) { return fmaxf(x, y); };
    v = mx(v, dpp_f32<0xB1>(v));
    v = mx(v, dpp_f32<0x4E>(v));
    v = mx(v, dpp_f32<0x141>(v));
    v = mx(v, dpp_f32<0x140>(v));
    const auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    return mx(__uint_as_float(a[0]), __uint_as_float(a[1]));
  }
}

// HALF = 1: two rows per wave, 32 lanes each (D <= 768: 96 chunks = 32 lanes x 3, no idle lanes
// in a second pass), reductions inside the 32-lane half
template <int MAXC, int HALF = 0>
__global__ __launch_bounds__(256) void rownorm_quant_kernel(
    const bf16_t* __restrict__ x, int ldx, const float* __restrict__ gamma,
    const float* __restrict__ beta, float eps, bf16_t* __restrict__ yb, int ldyb,
    uint8_t* __restrict__ q, int ldq, float* __restrict__ qs, int M, int D) {
  constexpr int G = 64 >> HALF;                  // lanes per row
  const int lane = threadIdx.x & (G - 1);
  const int row = blockIdx.x * (4 << HALF) + (threadIdx.x >> (6 - HALF));
  if (row >= M) return;
  const int nchunk = D >> 3;
  const bf16_t* src = x + (long)row * ldx;
  float v[MAXC][8];
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < MAXC; ++c) {
    const int ch = lane + G * c;
    if (ch < nchunk) {
      const u32x4 u = *reinterpret_cast<const u32x4*>(src + ch * 8);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        v[c][2 * e] = __uint_as_float(u[e] << 16);
        v[c][2 * e + 1] = __uint_as_float(u[e] & 0xffff0000u);
      }
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[c][e] = 0.f;
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) s += v[c][e];
  }
  if (gamma) {
    const float mean = group_sum<HALF>(s) / D;
    float ss = 0.f;
#pragma unroll
    for (int c = 0; c < MAXC; ++c) {
      if (lane + G * c < nchunk) {
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float d = v[c][e] - mean;
          ss += d * d;
        }
      }
    }
    const float rstd = rsqrtf(group_sum<HALF>(ss) / D + eps);
#pragma unroll
    for (int c = 0; c < MAXC; ++c) {
      const int ch = lane + G * c;
      if (ch < nchunk) {
#pragma unroll
        for (int e = 0; e < 8; ++e)
          v[c][e] = (v[c][e] - mean) * rstd * gamma[ch * 8 + e] + beta[ch * 8 + e];
      }
    }
  }
  if (yb) {
#pragma unroll
    for (int c = 0; c < MAXC; ++c) {
      const int ch = lane + G * c;
      if (ch < nchunk) {
        u32x4 o;
#pragma unroll
        for (int e = 0; e < 4; ++e) o[e] = pack2(v[c][2 * e], v[c][2 * e + 1]);
        *reinterpret_cast<u32x4*>(yb + (long)row * ldyb + ch * 8) = o;
      }
    }
  }
  if (q) {
    float amax = 0.f;
#pragma unroll
    for (int c = 0; c < MAXC; ++c)
      if (lane + G * c < nchunk) {
#pragma unroll
        for (int e = 0; e < 8; ++e) amax = fmaxf(amax, fabsf(v[c][e]));
      }
    amax = group_max<HALF>(amax);
    const float scale = amax > 0.f ? amax / 448.f : 1.f;
    const float inv = 1.f / scale;
    if (lane == 0) qs[row] = scale;        // lane = index inside the row's group
#pragma unroll
    for (int c = 0; c < MAXC; ++c) {
      const int ch = lane + G * c;
      if (ch < nchunk) {
        unsigned w0 = 0u, w1 = 0u;
        w0 = __builtin_amdgcn_cvt_pk_fp8_f32(fminf(fmaxf(v[c][0] * inv, -448.f), 448.f),
                                             fminf(fmaxf(v[c][1] * inv, -448.f), 448.f), w0, false);
        w0 = __builtin_amdgcn_cvt_pk_fp8_f32(fminf(fmaxf(v[c][2] * inv, -448.f), 448.f),
                                             fminf(fmaxf(v[c][3] * inv, -448.f), 448.f), w0, true);
        w1 = __builtin_amdgcn_cvt_pk_fp8_f32(fminf(fmaxf(v[c][4] * inv, -448.f), 448.f),
                                             fminf(fmaxf(v[c][5] * inv, -448.f), 448.f), w1, false);
        w1 = __builtin_amdgcn_cvt_pk_fp8_f32(fminf(fmaxf(v[c][6] * inv, -448.f), 448.f),
                                             fminf(fmaxf(v[c][7] * inv, -448.f), 448.f), w1, true);
        *reinterpret_cast<uint2*>(q + (long)row * ldq + ch * 8) = make_uint2(w0, w1);
      }
    }
  }
}

// Persistent LayerNorm + per-row e4m3 quantisation for D <= 32 * 8 * MAXC (two rows per wave, 32
// lanes x MAXC chunks of 8): rownorm_quant_kernel<3, 1> reloads gamma / beta (six 16-B loads per
// lane) for every row pair and launches one short wave per pair, so at the Whisper shapes
// (21014 x 768) it moved 48 MB in ~14 us (3.4 TB/s).  Here each wave keeps gamma / beta in
// registers for the whole launch, walks row pairs pr, pr + nwaves, ... (a wave-uniform loop, so
// the 32-lane DPP / permlane reductions always run with both halves active; a half past M reads
// zeros and stores nothing) and has the next pair's loads in flight while it reduces,
// normalises, quantises and stores the current one.
template <int MAXC>
__global__ __launch_bounds__(256) void rownorm_quant_pers_kernel(
    const bf16_t* __restrict__ x, int ldx, const float* __restrict__ gamma,
    const float* __restrict__ beta, float eps, bf16_t* __restrict__ yb, int ldyb,
    uint8_t* __restrict__ q, int ldq, float* __restrict__ qs, int M, int D) {
  const int lane = threadIdx.x & 31;
  const int half = (threadIdx.x >> 5) & 1;
  const int wave_g = (blockIdx.x * 256 + threadIdx.x) >> 6;
  const int nwaves = gridDim.x * 4;
  const int nchunk = D >> 3;
  const float inv_d = 1.f / (float)D;
  float g[MAXC][8], bt[MAXC][8];
#pragma unroll
  for (int c = 0; c < MAXC; ++c) {
    const int ch = lane + 32 * c;
#pragma unroll
    for (int e = 0; e < 8; ++e) g[c][e] = bt[c][e] = 0.f;
    if (gamma && ch < nchunk) {
      const f32x4 g0 = *reinterpret_cast<const f32x4*>(gamma + ch * 8);
      const f32x4 g1 = *reinterpret_cast<const f32x4*>(gamma + ch * 8 + 4);
      const f32x4 b0 = *reinterpret_cast<const f32x4*>(beta + ch * 8);
      const f32x4 b1 = *reinterpret_cast<const f32x4*>(beta + ch * 8 + 4);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        g[c][e] = g0[e]; g[c][e + 4] = g1[e];
        bt[c][e] = b0[e]; bt[c][e + 4] = b1[e];
      }
    }
  }
  auto load = [&](int pr, u32x4 (&u)[MAXC]) {
    const int row = 2 * pr + half;
#pragma unroll
    for (int c = 0; c < MAXC; ++c) {
      const int ch = lane + 32 * c;
      u[c] = u32x4{0u, 0u, 0u, 0u};
      if (row < M && ch < nchunk) u[c] = *reinterpret_cast<const u32x4*>(x + (long)row * ldx + ch * 8);
    }
  };
  u32x4 cur[MAXC], nxt[MAXC];
  int pr = wave_g;
  if (2 * pr < M) load(pr, cur);
  for (; 2 * pr < M; pr += nwaves) {
    const int row = 2 * pr + half;
    const bool live = row < M;
    if (2 * (pr + nwaves) < M) load(pr + nwaves, nxt);
    float v[MAXC][8];
    float s = 0.f;
#pragma unroll
    for (int c = 0; c < MAXC; ++c)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        v[c][2 * e] = __uint_as_float(cur[c][e] << 16);
        v[c][2 * e + 1] = __uint_as_float(cur[c][e] & 0xffff0000u);
        s += v[c][2 * e] + v[c][2 * e + 1];
      }
    if (gamma) {
      const float mean = group_sum<1>(s) * inv_d;
      float ss = 0.f;
#pragma unroll
      for (int c = 0; c < MAXC; ++c)
        if (lane + 32 * c < nchunk) {
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const float d = v[c][e] - mean;
            ss += d * d;
          }
        }
      const float rstd = rsqrtf(group_sum<1>(ss) * inv_d + eps);
#pragma unroll
      for (int c = 0; c < MAXC; ++c)
#pragma unroll
        for (int e = 0; e < 8; ++e) v[c][e] = (v[c][e] - mean) * rstd * g[c][e] + bt[c][e];
    }
    if (yb && live) {
#pragma unroll
      for (int c = 0; c < MAXC; ++c) {
        const int ch = lane + 32 * c;
        if (ch < nchunk) {
          u32x4 o;
#pragma unroll
          for (int e = 0; e < 4; ++e) o[e] = pack2(v[c][2 * e], v[c][2 * e + 1]);
          *reinterpret_cast<u32x4*>(yb + (long)row * ldyb + ch * 8) = o;
        }
      }
    }
    if (q) {
      float amax = 0.f;
#pragma unroll
      for (int c = 0; c < MAXC; ++c)
        if (lane + 32 * c < nchunk) {
#pragma unroll
          for (int e = 0; e < 8; ++e) amax = fmaxf(amax, fabsf(v[c][e]));
        }
      amax = group_max<1>(amax);
      const float scale = amax > 0.f ? amax / 448.f : 1.f;
      const float inv = 1.f / scale;
      if (live) {
        if (lane == 0) qs[row] = scale;
#pragma unroll
        for (int c = 0; c < MAXC; ++c) {
          const int ch = lane + 32 * c;
          if (ch < nchunk) {
            unsigned w0 = 0u, w1 = 0u;
            w0 = __builtin_amdgcn_cvt_pk_fp8_f32(fminf(fmaxf(v[c][0] * inv, -448.f), 448.f),
                                                 fminf(fmaxf(v[c][1] * inv, -448.f), 448.f), w0, false);
            w0 = __builtin_amdgcn_cvt_pk_fp8_f32(fminf(fmaxf(v[c][2] * inv, -448.f), 448.f),
                                                 fminf(fmaxf(v[c][3] * inv, -448.f), 448.f), w0, true);
            w1 = __builtin_amdgcn_cvt_pk_fp8_f32(fminf(fmaxf(v[c][4] * inv, -448.f), 448.f),
                                                 fminf(fmaxf(v[c][5] * inv, -448.f), 448.f), w1, false);
            w1 = __builtin_amdgcn_cvt_pk_fp8_f32(fminf(fmaxf(v[c][6] * inv, -448.f), 448.f),
                                                 fminf(fmaxf(v[c][7] * inv, -448.f), 448.f), w1, true);
            *reinterpret_cast<uint2*>(q + (long)row * ldq + ch * 8) = make_uint2(w0, w1);
          }
        }
      }
    }
#pragma unroll
    for (int c = 0; c < MAXC; ++c) cur[c] = nxt[c];
  }
}

}  // namespace aiko

extern "C" int aiko_gemm_fp8(const void* a, const void* b, const float* sa, const float* sb,
                             const float* bias, const void* res, void* y, int M, int N, int K,
                             int lda, int ldy, int ldr, int act, int bm, int bn, int variant,
                             const void* zero, const void* amx, int mxr, void* yq, void* ysc,
                             int ldq, int ysr, hipStream_t stream) {
  using namespace aiko;
  Fp8GemmParams p;
  p.amx = static_cast<const uint8_t*>(amx);
  p.mxr = mxr;
  p.yq = static_cast<uint8_t*>(yq);
  p.ysc = static_cast<uint8_t*>(ysc);
  p.ldq = ldq;
  p.ysr = ysr;
  if ((amx || yq) && variant != 1 && variant != 3 && variant != 4 && variant != 5) return -1;   // MX: LDS-DMA kernels
  if (amx && sa) return -1;                          // MX-fp8 A: block scales only, no per-row scales
  p.a = static_cast<const uint8_t*>(a);
  p.b = static_cast<const uint8_t*>(b);
  p.sa = sa; p.sb = sb; p.bias = bias;
  p.res = static_cast<const bf16_t*>(res);
  p.y = static_cast<bf16_t*>(y);
  p.M = M; p.N = N; p.K = K; p.lda = lda; p.ldy = ldy; p.ldr = ldr; p.act = act;
  dim3 grid(((M + bm - 1) / bm) * ((N + bn - 1) / bn)), block(256);
  if (variant == 4 || variant == 5) {   // persistent 256 x 256 / 128 x 256 (short-K encoder shapes)
    const uint8_t* z = static_cast<const uint8_t*>(zero);
    const int BMv = variant == 4 ? 256 : 128;
    const bool mxres = amx && res && act == 0 && !yq;   // MX-fp8 A + residual (out-proj, fc2)
    if (!z || bm != BMv || bn != 256 || N % 256 || N > 3072 || K % 128 || K < 256) return -1;
    if ((amx || res) && !mxres) return -1;
    if ((long)M * (yq ? ldq : 2L * ldy) >= 0x7ffffff0L || (yq && (long)(N / 128) * ysr * 4 >= 0x7ffffff0L)) return -1;
    if (res && ((long)M * ldr * 2 >= 0x7ffffff0L || ldr % 8 || reinterpret_cast<uintptr_t>(res) % 16)) return -1;
    if (!yq && (ldy % 8 || reinterpret_cast<uintptr_t>(y) % 16)) return -1;   // 16-B row stores
    static int cus = 0;
    if (cus == 0) {
      int dev = 0;
      (void)hipGetDevice(&dev);
      if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) cus = 256;
    }
    const int tiles_n = N / 256, ntiles = ((M + BMv - 1) / BMv) * tiles_n;
    const dim3 pg((unsigned)(ntiles < cus ? ntiles : cus));
    static const int diag = [] {                     // AIKO_FP8_DIAG: timing diagnostics only (1: no K-block DMAs
      const char* e = getenv("AIKO_FP8_DIAG");       // after the first two, 2: no epilogue stores, 4: no barrier,
      return e ? atoi(e) : 0;                        // 8: no epilogue) — wrong results by design
    }();
    static const bool ov = [] {                      // AIKO_FP8_OVERLAP=0: epilogue after the K
      const char* e = getenv("AIKO_FP8_OVERLAP");    // loop (gemm_fp8_pers_kernel, variant 4 only)
      return !(e && e[0] == '0');
    }();
    if (variant == 5) {
      if (mxres) gemm_fp8_pers2_kernel<128, false, 0, true, true><<<pg, 512, 0, stream>>>(p, z, tiles_n, ntiles, diag);
      else if (yq && act == 3) gemm_fp8_pers2_kernel<128, true, 3, false, false><<<pg, 512, 0, stream>>>(p, z, tiles_n, ntiles, diag);
      else if (!yq && act == 0) gemm_fp8_pers2_kernel<128, false, 0, false, false><<<pg, 512, 0, stream>>>(p, z, tiles_n, ntiles, diag);
      else if (!yq && act == 3) gemm_fp8_pers2_kernel<128, false, 3, false, false><<<pg, 512, 0, stream>>>(p, z, tiles_n, ntiles, diag);
      else return -1;
    } else if (mxres) {
      gemm_fp8_pers2_kernel<256, false, 0, true, true><<<pg, 512, 0, stream>>>(p, z, tiles_n, ntiles, diag);
    } else if (ov) {                                 // activation as a template argument: the
      auto go = [&](auto mxo, auto act) {            // epilogue's registers are those of one path
        gemm_fp8_pers2_kernel<256, decltype(mxo)::value, decltype(act)::value, false, false>
            <<<pg, 512, 0, stream>>>(p, z, tiles_n, ntiles, diag);
      };
      auto by_act = [&](auto mxo) {
        switch (p.act) {
          case 1: go(mxo, std::integral_constant<int, 1>{}); break;
          case 2: go(mxo, std::integral_constant<int, 2>{}); break;
          case 3: go(mxo, std::integral_constant<int, 3>{}); break;
          default: go(mxo, std::integral_constant<int, 0>{}); break;
        }
      };
      if (yq) by_act(std::true_type{});
      else by_act(std::false_type{});
    } else if (yq) gemm_fp8_pers_kernel<true><<<pg, 512, 0, stream>>>(p, z, tiles_n, ntiles, diag);
    else gemm_fp8_pers_kernel<false><<<pg, 512, 0, stream>>>(p, z, tiles_n, ntiles, diag);
    return (int)hipGetLastError();
  }
  if (variant == 3) {
    const uint8_t* z = static_cast<const uint8_t*>(zero);
    if (!z || bm != 256 || bn != 256) return -1;
    if ((amx || yq) && (N % 256 || K % 128)) return -1;
    if (amx && yq) gemm_fp8_big_kernel<true, true><<<grid, 512, 0, stream>>>(p, z);
    else if (amx) gemm_fp8_big_kernel<true, false><<<grid, 512, 0, stream>>>(p, z);
    else if (yq) gemm_fp8_big_kernel<false, true><<<grid, 512, 0, stream>>>(p, z);
    else gemm_fp8_big_kernel<false, false><<<grid, 512, 0, stream>>>(p, z);
    return (int)hipGetLastError();
  }
  if (variant == 2) {
    const uint8_t* z = static_cast<const uint8_t*>(zero);
    if (!z || bm != 256) return -1;
    if (bn == 128) {
      gemm_fp8_w8_kernel<128><<<grid, 512, 0, stream>>>(p, z);
    } else {
      return -1;
    }
    return (int)hipGetLastError();
  }
  if (variant == 1) {
    const uint8_t* z = static_cast<const uint8_t*>(zero);
    if (!z) return -1;
    if (amx || yq) {
      if (bn != 128 || (bm != 128 && bm != 64)) return -1;
      auto go = [&](auto mxa, auto mxo) {
        constexpr bool A = decltype(mxa)::value, O = decltype(mxo)::value;
        if (bm == 128) gemm_fp8_glds_kernel<128, 128, A, O><<<grid, block, 0, stream>>>(p, z);
        else gemm_fp8_glds_kernel<64, 128, A, O><<<grid, block, 0, stream>>>(p, z);
      };
      if (amx && yq) go(std::true_type{}, std::true_type{});
      else if (amx) go(std::true_type{}, std::false_type{});
      else go(std::false_type{}, std::true_type{});
      return (int)hipGetLastError();
    }
    if (bm == 128 && bn == 128) {
      gemm_fp8_glds_kernel<128, 128><<<grid, block, 0, stream>>>(p, z);
    } else if (bm == 128 && bn == 64) {
      gemm_fp8_glds_kernel<128, 64><<<grid, block, 0, stream>>>(p, z);
    } else if (bm == 64 && bn == 64) {
      gemm_fp8_glds_kernel<64, 64><<<grid, block, 0, stream>>>(p, z);
    } else if (bm == 64 && bn == 128) {
      gemm_fp8_glds_kernel<64, 128><<<grid, block, 0, stream>>>(p, z);
    } else {
      return -1;
    }
    return (int)hipGetLastError();
  }
  if (bm == 128 && bn == 128) {
    gemm_fp8_kernel<128, 128><<<grid, block, 0, stream>>>(p);
  } else if (bm == 128 && bn == 64) {
    gemm_fp8_kernel<128, 64><<<grid, block, 0, stream>>>(p);
  } else if (bm == 64 && bn == 64) {
    gemm_fp8_kernel<64, 64><<<grid, block, 0, stream>>>(p);
  } else if (bm == 64 && bn == 128) {
    gemm_fp8_kernel<64, 128><<<grid, block, 0, stream>>>(p);
  } else {
    return -1;
  }
  return (int)hipGetLastError();
}

extern "C" int aiko_rownorm_quant(const void* x, int ldx, const float* gamma, const float* beta,
                                  float eps, void* yb, int ldyb, void* q, int ldq, float* qs,
                                  int M, int D, hipStream_t stream) {
  using namespace aiko;
  dim3 grid((M + 3) / 4), block(256);
  const bf16_t* xp = static_cast<const bf16_t*>(x);
  bf16_t* yp = static_cast<bf16_t*>(yb);
  uint8_t* qp = static_cast<uint8_t*>(q);
  if (D <= 32 * 8 * 3) {               // 2 rows per wave, 32 lanes x <= 3 chunks each
    static const bool legacy = [] {
      const char* e = getenv("AIKO_ROWNORM_LEGACY");
      return e && e[0] == '1';
    }();
    if (!legacy) {                       // persistent: ~4 row pairs per wave at the Whisper shapes
      static int cus = 0;
      if (cus == 0) {
        int dev = 0;
        (void)hipGetDevice(&dev);
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) cus = 256;
      }
      const int pairs = (M + 1) / 2, need = (pairs + 3) / 4;
      const int blocks = need < cus * 4 ? need : cus * 4;
      rownorm_quant_pers_kernel<3><<<dim3(blocks), block, 0, stream>>>(xp, ldx, gamma, beta, eps, yp, ldyb, qp, ldq,
                                                                       qs, M, D);
      return (int)hipGetLastError();
    }
    rownorm_quant_kernel<3, 1><<<dim3((M + 7) / 8), block, 0, stream>>>(xp, ldx, gamma, beta, eps, yp, ldyb, qp, ldq,
                                                                       qs, M, D);
    return (int)hipGetLastError();
  }
  if (D <= 64 * 8 * 2) {
    rownorm_quant_kernel<2><<<grid, block, 0, stream>>>(xp, ldx, gamma, beta, eps, yp, ldyb, qp, ldq, qs, M, D);
  } else if (D <= 64 * 8 * 6) {
    rownorm_quant_kernel<6><<<grid, block, 0, stream>>>(xp, ldx, gamma, beta, eps, yp, ldyb, qp, ldq, qs, M, D);
  } else if (D <= 64 * 8 * 16) {
    rownorm_quant_kernel<16><<<grid, block, 0, stream>>>(xp, ldx, gamma, beta, eps, yp, ldyb, qp, ldq, qs, M, D);
  } else {
    return -1;
  }
  return (int)hipGetLastError();
}
