// Flash-attention forward (non-causal, head dim 64) for CDNA4 (gfx950), bf16 in / fp32 softmax.
//
// Built for the Whisper encoder (1500 tokens x 12 heads x 64): one 256-thread workgroup per
// (128-query block, head, sequence); each of the 4 waves owns 32 queries and streams the
// sequence's keys in 64-key tiles through a 2-deep LDS ring (K as [key][dh] with 16-B XOR
// swizzle, V transposed to [dh][key] with 8-B chunk swizzle).  The products are computed
// TRANSPOSED — S^T = K Q^T and O^T = V^T P^T with v_mfma_f32_16x16x32_bf16 — so that:
//   * each lane's accumulator column is one query: the online-softmax rescale of O^T is a
//     per-lane scalar, and row statistics need only 2 cross-lane shuffles (xor 16, 32);
//   * the bf16 probabilities P^T are consumed as the B operand straight from the S^T
//     accumulator registers (no LDS round trip): element j of lane group g of k-step s is key
//     32s + 16(j>>2) + 4g + (j&3), and the V^T fragment is read in that same key order.
// Q stays in registers for the whole key loop.  Sequences are rows b*Tpad .. b*Tpad+T-1 of
// q/k/v (any row pitch: q, k, v may be column slices of one fused QKV buffer).
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
};

constexpr int kQB = 128, kKB = 64, kDH = 64;

__device__ __forceinline__ bf16x8 as_bf16x8(u32x4 u) { return __builtin_bit_cast(bf16x8, u); }

__global__ __launch_bounds__(256, 2) void attn_fwd_kernel(AttnParams p) {
  __shared__ __attribute__((aligned(16))) bf16_t Ks[2][kKB * kDH];
  __shared__ __attribute__((aligned(16))) bf16_t Vt[2][kDH * kKB];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int fr = lane & 15, g = lane >> 4;
  const int h = blockIdx.y, b = blockIdx.z;
  const long seq0 = (long)b * p.Tpad;
  const int q0 = blockIdx.x * kQB + wave * 32;
  const int hc = h * kDH;

  // Q^T fragments (B operand): lane holds Q[q][ks*32 + 8g .. +7] for q = q0 + qt*16 + fr
  bf16x8 qf[2][2];
#pragma unroll
  for (int qt = 0; qt < 2; ++qt) {
    const int q = q0 + qt * 16 + fr;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      // rows past T are clamped to T-1 (their outputs are never written): no predicated loads
      const int qc = q < p.T ? q : p.T - 1;
      qf[qt][ks] = as_bf16x8(*reinterpret_cast<const u32x4*>(p.q + (seq0 + qc) * p.ldq + hc + ks * 32 + 8 * g));
    }
  }

  // staging: 2 x 16-B pieces of K and of V per thread per tile
  const int piece = tid & 7, prow = tid >> 3;  // rows prow, prow + 32
  u32x4 rk[2], rv[2];
  auto load_tile = [&](int t0) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      // keys past T read row T-1 (finite data): their scores are masked to -inf, so P = 0 and
      // the V rows contribute exactly 0 — unconditional loads keep the prefetch pipelined
      const int key = min(t0 + prow + 32 * i, p.T - 1);
      rk[i] = *reinterpret_cast<const u32x4*>(p.k + (seq0 + key) * p.ldk + hc + piece * 8);
      rv[i] = *reinterpret_cast<const u32x4*>(p.v + (seq0 + key) * p.ldv + hc + piece * 8);
    }
  };
  auto store_tile = [&](int slot) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int row = prow + 32 * i;
      *reinterpret_cast<u32x4*>(&Ks[slot][row * kDH + ((piece ^ (row & 7)) << 3)]) = rk[i];
      const int chunk = row >> 2, within = row & 3;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int d0 = piece * 8 + 2 * e, d1 = d0 + 1;
        Vt[slot][d0 * kKB + ((chunk ^ (d0 & 15)) << 2) + within] = (bf16_t)(rv[i][e] & 0xffffu);
        Vt[slot][d1 * kKB + ((chunk ^ (d1 & 15)) << 2) + within] = (bf16_t)(rv[i][e] >> 16);
      }
    }
  };

  f32x4 o[4][2];
#pragma unroll
  for (int d = 0; d < 4; ++d)
#pragma unroll
    for (int qt = 0; qt < 2; ++qt) o[d][qt] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m_run[2] = {-INFINITY, -INFINITY}, l_run[2] = {0.f, 0.f};

  const int ntiles = (p.T + kKB - 1) / kKB;
  load_tile(0);
  store_tile(0);
  __syncthreads();

  for (int it = 0; it < ntiles; ++it) {
    const int cur = it & 1;
    const int t0 = it * kKB;
    if (it + 1 < ntiles) load_tile(t0 + kKB);

    // S^T = K Q^T : 4 key tiles x 2 query tiles
    f32x4 s[4][2];
#pragma unroll
    for (int kt = 0; kt < 4; ++kt) {
#pragma unroll
      for (int qt = 0; qt < 2; ++qt) s[kt][qt] = f32x4{0.f, 0.f, 0.f, 0.f};
      const int row = kt * 16 + fr;
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const bf16x8 kf = *reinterpret_cast<const bf16x8*>(
            &Ks[cur][row * kDH + (((ks * 4 + g) ^ (row & 7)) << 3)]);
#pragma unroll
        for (int qt = 0; qt < 2; ++qt)
          s[kt][qt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf, qf[qt][ks], s[kt][qt], 0, 0, 0);
      }
    }

    // online softmax per query column; P^T packed to bf16 B fragments
    bf16x8 pf[2][2];
#pragma unroll
    for (int qt = 0; qt < 2; ++qt) {
      float mloc = -INFINITY;
#pragma unroll
      for (int kt = 0; kt < 4; ++kt)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int key = t0 + kt * 16 + 4 * g + j;
          const float v = key < p.T ? s[kt][qt][j] * p.scale_log2 : -INFINITY;
          s[kt][qt][j] = v;
          mloc = fmaxf(mloc, v);
        }
      mloc = fmaxf(mloc, __shfl_xor(mloc, 16, 64));
      mloc = fmaxf(mloc, __shfl_xor(mloc, 32, 64));
      const float m_new = fmaxf(m_run[qt], mloc);
      const float alpha = exp2f(m_run[qt] - m_new);
      m_run[qt] = m_new;
      float lsum = 0.f;
      float pv[4][4];
#pragma unroll
      for (int kt = 0; kt < 4; ++kt)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          pv[kt][j] = exp2f(s[kt][qt][j] - m_new);
          lsum += pv[kt][j];
        }
      l_run[qt] = l_run[qt] * alpha + lsum;
#pragma unroll
      for (int d = 0; d < 4; ++d) o[d][qt] *= alpha;
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        u32x4 u;
        u[0] = pack2(pv[2 * ks][0], pv[2 * ks][1]);
        u[1] = pack2(pv[2 * ks][2], pv[2 * ks][3]);
        u[2] = pack2(pv[2 * ks + 1][0], pv[2 * ks + 1][1]);
        u[3] = pack2(pv[2 * ks + 1][2], pv[2 * ks + 1][3]);
        pf[qt][ks] = as_bf16x8(u);
      }
    }

    // O^T += V^T P^T
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      const int dh = d * 16 + fr;
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const int c0 = 8 * ks + g, c1 = 8 * ks + 4 + g;
        const uint2 lo = *reinterpret_cast<const uint2*>(&Vt[cur][dh * kKB + ((c0 ^ (dh & 15)) << 2)]);
        const uint2 hi = *reinterpret_cast<const uint2*>(&Vt[cur][dh * kKB + ((c1 ^ (dh & 15)) << 2)]);
        const bf16x8 vf = as_bf16x8(u32x4{lo.x, lo.y, hi.x, hi.y});
#pragma unroll
        for (int qt = 0; qt < 2; ++qt)
          o[d][qt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vf, pf[qt][ks], o[d][qt], 0, 0, 0);
      }
    }

    if (it + 1 < ntiles) store_tile(cur ^ 1);
    __syncthreads();
  }

  // normalise and write O[q][dh]: lane holds dh = d*16 + 4g + j for its query
#pragma unroll
  for (int qt = 0; qt < 2; ++qt) {
    float l = l_run[qt];
    l += __shfl_xor(l, 16, 64);
    l += __shfl_xor(l, 32, 64);
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

extern "C" int aiko_attn_fwd(const void* q, const void* k, const void* v, void* o, int ldq, int ldk,
                             int ldv, int ldo, int B, int H, int T, int Tpad, int dh, float scale,
                             hipStream_t stream) {
  if (dh != aiko::kDH || T < 1 || Tpad < T) return -1;
  aiko::AttnParams p;
  p.q = static_cast<const aiko::bf16_t*>(q);
  p.k = static_cast<const aiko::bf16_t*>(k);
  p.v = static_cast<const aiko::bf16_t*>(v);
  p.o = static_cast<aiko::bf16_t*>(o);
  p.ldq = ldq; p.ldk = ldk; p.ldv = ldv; p.ldo = ldo;
  p.T = T; p.Tpad = Tpad; p.H = H;
  p.scale_log2 = scale * 1.4426950408889634f;
  dim3 grid((T + aiko::kQB - 1) / aiko::kQB, H, B), block(256);
  aiko::attn_fwd_kernel<<<grid, block, 0, stream>>>(p);
  return (int)hipGetLastError();
}
