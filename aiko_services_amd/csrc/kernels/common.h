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

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
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

// Bijective XCD-aware remap of a linear workgroup id: consecutive logical ids land on the
// same XCD (blocks b and b+8 share an XCD under round-robin dispatch), so tiles that share
// an operand panel share an L2.  Speed only; correctness never depends on placement.
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int q = nwg >> 3, r = nwg & 7;
  const int xcd = bid & 7, idx = bid >> 3;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + idx;
}

}  // namespace aiko
