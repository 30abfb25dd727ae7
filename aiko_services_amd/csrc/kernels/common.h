// Shared device helpers for the aiko_services_amd CDNA4 (gfx950) kernel library.
//
// Everything here is written for wave64 + MFMA on MI355X; there is no other target.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace aiko {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;
typedef uint16_t bf16_t;  // raw bf16 bits in global memory

constexpr int kWave = 64;

__device__ __forceinline__ float bf2f(bf16_t v) {
  return __uint_as_float(((uint32_t)v) << 16);
}

// Round-to-nearest-even via the hardware convert (v_cvt_pk_bf16_f32 on gfx950).
__device__ __forceinline__ bf16_t f2bf(float f) {
  __bf16 b = (__bf16)f;
  return __builtin_bit_cast(bf16_t, b);
}

typedef __attribute__((ext_vector_type(2))) float f32x2;
typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2;

// two floats -> packed bf16 pair with ONE v_cvt_pk_bf16_f32 (RNE, NaN-preserving)
__device__ __forceinline__ uint32_t pack2(float lo, float hi) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(f32x2{lo, hi}, bf16x2));
}

// raw v_exp_f32 (2^x): no denormal-range fix-up sequence; results below 2^-126 flush to 0,
// which is what softmax wants
__device__ __forceinline__ float fast_exp2(float x) { return __builtin_amdgcn_exp2f(x); }

// Wave-wide reductions without the LDS crossbar (each ds_bpermute is an LDS round trip on the
// reduction's dependency chain): DPP quad_perm xor 1 / xor 2, DPP row_half_mirror / row_mirror
// (lane i <-> 7 - i, 15 - i inside each 16-lane row: after the quad steps this pairs whole quads
// and half-rows), then gfx950's v_permlane16_swap / v_permlane32_swap for the row pairs and the
// wave halves.  Every step adds / maxes the same two operands in every lane, so all 64 lanes end
// with the bit-identical result, like the xor butterfly this replaces.
template <int CTRL>
__device__ __forceinline__ float dpp_f32(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}

template <class Op>
__device__ __forceinline__ float wave_reduce(float v, Op op) {
  v = op(v, dpp_f32<0xB1>(v));     // quad_perm [1,0,3,2]
  v = op(v, dpp_f32<0x4E>(v));     // quad_perm [2,3,0,1]
  v = op(v, dpp_f32<0x141>(v));    // row_half_mirror
  v = op(v, dpp_f32<0x140>(v));    // row_mirror
  const auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = op(__uint_as_float(a[0]), __uint_as_float(a[1]));
  const auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return op(__uint_as_float(b[0]), __uint_as_float(b[1]));
}

__device__ __forceinline__ float wave_max(float v) {
  return wave_reduce(v, [](float x, float y) { return fmaxf(x, y); });
}

__device__ __forceinline__ float wave_sum(float v) {
  return wave_reduce(v, [](float x, float y) { return x + y; });
}

// 16-byte LDS-DMA (global_load_lds_dwordx4) issued through inline asm: the LDS destination is
// M0 (wave-uniform) + lane * 16.  Hidden from the compiler's waitcnt pass on purpose — where it
// cannot prove a later ds_read disjoint from a pending DMA it drains vmcnt to 0 before the read
// (seen in the attention loop), collapsing the ring to zero tiles in flight.  The caller owns
// every wait: counted `s_waitcnt vmcnt(N)` before the barrier that publishes a slot.  Only for
// loops with no other VMEM loads whose waits the compiler would then mis-count.
__device__ __forceinline__ void glds16_asm(const void* g, const void* lds_wave_base) {
  const uint32_t lds = __builtin_amdgcn_readfirstlane(
      static_cast<uint32_t>(reinterpret_cast<uintptr_t>(lds_wave_base)));
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off"
               :: "v"(g), "s"(lds) : "memory", "m0");
}

// E8M0 exponent of an MX-fp8 block with absolute maximum amax (so that amax / 2^e <= 448, the
// e4m3 range); shared by every epilogue that writes MX activations (fp8 GEMMs, attention)
__device__ __forceinline__ int mx_exponent(float amax) {
  const uint32_t bits = __float_as_uint(amax * (1.f / 448.f));
  int e = (int)((bits >> 23) & 255u) - 127 + ((bits & 0x7fffffu) != 0u);
  if (amax == 0.f) e = -126;
  return e < -126 ? -126 : (e > 127 ? 127 : e);
}

// Bijective XCD-aware remap of a linear workgroup id: consecutive logical ids land on the
// same XCD (blocks b and b+8 share an XCD under round-robin dispatch), so tiles that share
// an operand panel share an L2.  Speed only; correctness never depends on placement.
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int q = nwg >> 3, r = nwg & 7;
  const int xcd = bid & 7, idx = bid >> 3;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + idx;
}

// erf for every GELU epilogue (fp8 GEMMs, convs, decoder linears — one definition so fused and
// unfused paths agree): Abramowitz & Stegun 7.1.26, erf(|x|) = 1 - poly(t) e^{-x^2}, t = 1 / (1 +
// p |x|) — max abs error 1.5e-7, far below the bf16 / e4m3 outputs' resolution.  One v_rcp +
// 5 FMAs + one v_exp instead of OCML erff: the exact erff made the epilogue of the Whisper fc1
// GEMM (73.8M GELUs) cost 81 us on top of the 98 us GEMM (scripts/op_bench.py gemm_fc1 /
// fc1_gelu).
// SiLU for every epilogue: x * rcp(1 + e^-x) — v_rcp_f32 (1 ulp) instead of the IEEE division
// sequence (~10 VALU ops); the fused YOLO stem was VALU-issue bound (PMC: 819 VALU instructions
// per wave, 16 SiLUs per lane).  Limits as the division: -inf side -> -0, +inf side -> x.
__device__ __forceinline__ float silu(float x) {
  return x * __builtin_amdgcn_rcpf(1.f + __expf(-x));
}

// Every step is an explicit fmaf / mul so the scalar and the packed (two-lane) forms below
// round identically whatever the compiler contracts elsewhere.
__device__ __forceinline__ float gelu_erf(float x) {
  const float z = x * 0.70710678118654752f;
  const float az = fabsf(z);
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, az, 1.f));
  float poly = fmaf(1.061405429f, t, -1.453152027f);
  poly = fmaf(poly, t, 1.421413741f);
  poly = fmaf(poly, t, -0.284496736f);
  poly = fmaf(poly, t, 0.254829592f);
  const float e = __expf(-(az * az));
  const float erf = copysignf(fmaf(-(poly * t), e, 1.f), z);
  const float h = 0.5f * x;
  return fmaf(h, erf, h);
}

// two GELUs per packed-fp32 VALU op (v_pk_fma_f32 / v_pk_mul_f32) for the polynomial and
// scaling; only v_rcp / v_exp are per lane.  Bit-identical to gelu_erf (same op sequence).
__device__ __forceinline__ f32x2 gelu_erf2(f32x2 x) {
  const f32x2 z = x * f32x2{0.70710678118654752f, 0.70710678118654752f};
  const f32x2 az = {fabsf(z[0]), fabsf(z[1])};
  const f32x2 d = __builtin_elementwise_fma(f32x2{0.3275911f, 0.3275911f}, az, f32x2{1.f, 1.f});
  const f32x2 t = {__builtin_amdgcn_rcpf(d[0]), __builtin_amdgcn_rcpf(d[1])};
  f32x2 poly = __builtin_elementwise_fma(f32x2{1.061405429f, 1.061405429f}, t, f32x2{-1.453152027f, -1.453152027f});
  poly = __builtin_elementwise_fma(poly, t, f32x2{1.421413741f, 1.421413741f});
  poly = __builtin_elementwise_fma(poly, t, f32x2{-0.284496736f, -0.284496736f});
  poly = __builtin_elementwise_fma(poly, t, f32x2{0.254829592f, 0.254829592f});
  const f32x2 sq = az * az;
  const f32x2 e = {__expf(-sq[0]), __expf(-sq[1])};
  const f32x2 y = __builtin_elementwise_fma(-(poly * t), e, f32x2{1.f, 1.f});
  const f32x2 erf = {copysignf(y[0], z[0]), copysignf(y[1], z[1])};
  const f32x2 h = f32x2{0.5f, 0.5f} * x;
  return __builtin_elementwise_fma(h, erf, h);
}

// GELU with a transcendental-free erf, for epilogues that quantise to e4m3 right after (the
// fc1 -> fc2 MX-fp8 hand-off): erf(x / sqrt2) ~= xc Q(xc^2), xc = clamp(x, +-3 sqrt2), Q a
// degree-8 least-squares fit (|GELU error| <= 5.2e-5 absolute for every x in fp32 evaluation,
// far below e4m3's 2^-4 relative step).  Only packed-fp32 multiplies / FMAs: gelu_erf2 spends
// a v_rcp and a v_exp (quarter-rate transcendentals) per element, which made the fc1 epilogue
// VALU-bound.
__device__ __forceinline__ f32x2 gelu_poly2(f32x2 x) {
  constexpr float C = 4.242640687f;
  const f32x2 xc = {fminf(fmaxf(x[0], -C), C), fminf(fmaxf(x[1], -C), C)};
  const f32x2 s = xc * xc;
  f32x2 q = __builtin_elementwise_fma(f32x2{1.124738094e-10f, 1.124738094e-10f}, s,
                                      f32x2{-1.074885849e-08f, -1.074885849e-08f});
  q = __builtin_elementwise_fma(q, s, f32x2{4.542003143e-07f, 4.542003143e-07f});
  q = __builtin_elementwise_fma(q, s, f32x2{-1.130945777e-05f, -1.130945777e-05f});
  q = __builtin_elementwise_fma(q, s, f32x2{1.874421164e-04f, 1.874421164e-04f});
  q = __builtin_elementwise_fma(q, s, f32x2{-2.220934090e-03f, -2.220934090e-03f});
  q = __builtin_elementwise_fma(q, s, f32x2{1.964535859e-02f, 1.964535859e-02f});
  q = __builtin_elementwise_fma(q, s, f32x2{-1.327118241e-01f, -1.327118241e-01f});
  q = __builtin_elementwise_fma(q, s, f32x2{7.978177156e-01f, 7.978177156e-01f});
  const f32x2 h = f32x2{0.5f, 0.5f} * x;
  return __builtin_elementwise_fma(h, xc * q, h);
}

// gelu_poly2 over N independent pairs with the Horner steps interleaved across the pairs: a
// packed-fp32 op reading the previous one's result needs a wait state, so one chain at a time
// issued an s_nop after every FMA
template <int N>
__device__ __forceinline__ void gelu_poly_n(f32x2 (&x)[N]) {
  constexpr float C = 4.242640687f;
  constexpr float Q[9] = {7.978177156e-01f, -1.327118241e-01f, 1.964535859e-02f, -2.220934090e-03f,
                          1.874421164e-04f, -1.130945777e-05f, 4.542003143e-07f, -1.074885849e-08f,
                          1.124738094e-10f};
  f32x2 xc[N], s[N], q[N];
#pragma unroll
  for (int i = 0; i < N; ++i) {
    xc[i] = f32x2{fminf(fmaxf(x[i][0], -C), C), fminf(fmaxf(x[i][1], -C), C)};
    s[i] = xc[i] * xc[i];
  }
#pragma unroll
  for (int i = 0; i < N; ++i) q[i] = __builtin_elementwise_fma(f32x2{Q[8], Q[8]}, s[i], f32x2{Q[7], Q[7]});
#pragma unroll
  for (int k = 6; k >= 0; --k) {
    __builtin_amdgcn_sched_barrier(0);             // keep the steps interleaved (no per-chain nops)
#pragma unroll
    for (int i = 0; i < N; ++i) q[i] = __builtin_elementwise_fma(q[i], s[i], f32x2{Q[k], Q[k]});
  }
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int i = 0; i < N; ++i) {
    const f32x2 h = f32x2{0.5f, 0.5f} * x[i];
    x[i] = __builtin_elementwise_fma(h, xc[i] * q[i], h);
  }
}

}  // namespace aiko
