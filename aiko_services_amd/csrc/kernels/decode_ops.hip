// Autoregressive decoder step kernels (gfx950, wave64) for the Whisper text decoder
// (the speech-to-text half of the reference's PE_WhisperX, examples/speech/
// speech_elements.py:203-262):
//
//   * embed_kernel        x[b] = tok_emb[ids[b]] + pos_emb[*pos]
//   * attn_decode_kernel  one query row per sequence against a KV cache: online softmax over
//                         256-key chunks, split over workgroups only when there are few
//                         sequences (then fp32 partials + attn_decode_combine).  In append
//                         mode the new key/value row (at *pos) is taken from the QKV GEMM
//                         output and written into the cache by the split that owns it
//   * dec_linear_kernel   LayerNorm + per-row e4m3 quantisation fused into a skinny-M fp8
//                         MFMA GEMM (bias, GELU, residual epilogue) for the decoder's B rows
//   * argmax_step_kernel  greedy next token per sequence (first index on ties), forced
//                         prompt prefix, sticky end-of-text, device-side position counter
//                         advanced by the last workgroup to finish (threadfence + counter)
//
// Every launch reads the step position from device memory, so a whole decoder step is one
// hipGraph replayed without host round trips.  The step is bandwidth / latency bound
// (cross-attention K/V and fp8 weights stream once per token): attention runs on VALU with
// coalesced 16-byte loads, the linears on MFMA with their normalisation fused in.
#include <hip/hip_runtime.h>

#include <math.h>

#include "common.h"

namespace aiko {

typedef __attribute__((ext_vector_type(8))) int i32x8;

constexpr int kDecKC = 256;    // keys per split (= threads per workgroup)
constexpr int kDecDh = 64;     // head dim

__device__ __forceinline__ void add_bf16x8(uint4& a, const uint4 e) {
  const uint32_t* ap = reinterpret_cast<const uint32_t*>(&a);
  const uint32_t* ep = reinterpret_cast<const uint32_t*>(&e);
  uint32_t r[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float lo = __uint_as_float(ap[i] << 16) + __uint_as_float(ep[i] << 16);
    const float hi = __uint_as_float(ap[i] & 0xffff0000u) + __uint_as_float(ep[i] & 0xffff0000u);
    r[i] = pack2(lo, hi);
  }
  a = make_uint4(r[0], r[1], r[2], r[3]);
}

__global__ void embed_kernel(const int* __restrict__ ids, const int* __restrict__ pos,
                             const bf16_t* __restrict__ tok, const bf16_t* __restrict__ pemb,
                             bf16_t* __restrict__ x, int d, int ldx, int vocab, int n_pos) {
  const int b = blockIdx.x;
  int id = ids[b];
  id = id < 0 ? 0 : (id >= vocab ? vocab - 1 : id);
  int p = *pos;
  p = p < 0 ? 0 : (p >= n_pos ? n_pos - 1 : p);
  for (int c = threadIdx.x * 8; c < d; c += blockDim.x * 8) {
    uint4 a = *reinterpret_cast<const uint4*>(tok + (long)id * d + c);
    const uint4 e = *reinterpret_cast<const uint4*>(pemb + (long)p * d + c);
    add_bf16x8(a, e);
    *reinterpret_cast<uint4*>(x + (long)b * ldx + c) = a;
  }
}

__device__ __forceinline__ float dot8(const uint4 k, const float* q) {
  const uint32_t* kp = reinterpret_cast<const uint32_t*>(&k);
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    s += __uint_as_float(kp[i] << 16) * q[2 * i];
    s += __uint_as_float(kp[i] & 0xffff0000u) * q[2 * i + 1];
  }
  return s;
}

// k/v: row j of sequence b at (b*S + j)*ld + h*64.  len = pos ? *pos + 1 : T.
// Workgroup (split, b*H+h) covers key chunks split, split + nsplit, ... of KC keys with an online
// softmax.  Thread t owns 16-byte column chunk c = t & 7 (head dims 8c .. 8c+7) of keys kg,
// kg + 32, ... of a chunk (kg = t >> 3): a score is an 8-lane shuffle reduction and every K/V
// load is a full 128-byte row segment shared by 8 consecutive lanes (the V loads are issued
// before the max reduction).  nsplit == 1 writes the output row; otherwise fp32 partials
// (max, sum, P.V) for attn_decode_combine — no device-scope fences inside the kernel.
__global__ __launch_bounds__(kDecKC) void attn_decode_kernel(
    const bf16_t* __restrict__ q, int ldq, bf16_t* k, bf16_t* v, int ldk, int ldv, int S,
    const int* __restrict__ pos, int T, const bf16_t* __restrict__ knew,
    const bf16_t* __restrict__ vnew, int ldnew, int H, int nsplit, float scale_log2,
    float* __restrict__ opart, float* __restrict__ mlpart, bf16_t* __restrict__ o, int ldo) {
  constexpr int KG = kDecKC / 8;               // key groups (32)
  constexpr int KPT = kDecKC / KG;             // keys per thread per chunk (8)
  __shared__ float red[2][kDecKC / kWave];
  __shared__ float accs[KG][kDecDh + 4];
  const int split = blockIdx.x, bh = blockIdx.y;
  const int b = bh / H, h = bh - b * H;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int c = tid & 7, kg = tid >> 3;
  const int papp = pos ? *pos : -1;            // appended position (append mode)
  const int len = pos ? papp + 1 : T;
  const long kb = (long)b * S;
  const bf16_t* knr = knew ? knew + (long)b * ldnew + h * kDecDh : nullptr;
  const bf16_t* vnr = vnew ? vnew + (long)b * ldnew + h * kDecDh : nullptr;
  // the split owning the appended row writes it into the cache (read by later steps only)
  if (knr && tid < 16 && (papp / kDecKC) % nsplit == split) {
    const int cc = (tid & 7) * 8;
    if (tid < 8)
      *reinterpret_cast<uint4*>(k + (kb + papp) * ldk + h * kDecDh + cc) = *reinterpret_cast<const uint4*>(knr + cc);
    else
      *reinterpret_cast<uint4*>(v + (kb + papp) * ldv + h * kDecDh + cc) = *reinterpret_cast<const uint4*>(vnr + cc);
  }
  float qv[8];
  {
    const uint4 u = *reinterpret_cast<const uint4*>(q + (long)b * ldq + h * kDecDh + c * 8);
    const uint32_t* up = reinterpret_cast<const uint32_t*>(&u);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      qv[2 * i] = __uint_as_float(up[i] << 16) * scale_log2;
      qv[2 * i + 1] = __uint_as_float(up[i] & 0xffff0000u) * scale_log2;
    }
  }
  float m = -INFINITY, ls = 0.f;               // running max (uniform), this thread's sum share
  float acc[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) acc[e] = 0.f;
  int par = 0;
  for (int start = split * kDecKC; start < len; start += nsplit * kDecKC, par ^= 1) {
    const int cnt = min(kDecKC, len - start);
    uint4 kr[KPT], vr[KPT];
#pragma unroll
    for (int i = 0; i < KPT; ++i) {
      const int jj = kg + KG * i, j = start + (jj < cnt ? jj : 0);
      const bf16_t* row = (j == papp && knr) ? knr : k + (kb + j) * ldk + h * kDecDh;
      kr[i] = *reinterpret_cast<const uint4*>(row + c * 8);
    }
#pragma unroll
    for (int i = 0; i < KPT; ++i) {
      const int jj = kg + KG * i, j = start + (jj < cnt ? jj : 0);
      const bf16_t* row = (j == papp && vnr) ? vnr : v + (kb + j) * ldv + h * kDecDh;
      vr[i] = *reinterpret_cast<const uint4*>(row + c * 8);
    }
    float sc[KPT], cm = -INFINITY;
#pragma unroll
    for (int i = 0; i < KPT; ++i) {
      float sv = dot8(kr[i], qv);
      sv += __shfl_xor(sv, 1, 64);
      sv += __shfl_xor(sv, 2, 64);
      sv += __shfl_xor(sv, 4, 64);
      sc[i] = kg + KG * i < cnt ? sv : -INFINITY;
      cm = fmaxf(cm, sc[i]);
    }
    cm = wave_max(cm);
    if (lane == 0) red[par][wave] = cm;        // double-buffered: no barrier before the write
    __syncthreads();
#pragma unroll
    for (int w = 0; w < kDecKC / kWave; ++w) cm = fmaxf(cm, red[par][w]);
    const float mn = fmaxf(m, cm);
    const float corr = fast_exp2(m - mn);      // m = -inf on the first chunk: corr = 0
    m = mn;
    ls *= corr;
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[e] *= corr;
#pragma unroll
    for (int i = 0; i < KPT; ++i) {
      const float p = fast_exp2(sc[i] - m);    // masked keys: exp2(-inf) = 0
      ls += p;
      const uint32_t* up = reinterpret_cast<const uint32_t*>(&vr[i]);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        acc[2 * e] += p * __uint_as_float(up[e] << 16);
        acc[2 * e + 1] += p * __uint_as_float(up[e] & 0xffff0000u);
      }
    }
  }
  // each key's p was added by its 8 column lanes: count one lane per key group
  float l = wave_sum(c == 0 ? ls : 0.f);
  __syncthreads();
  if (lane == 0) red[0][wave] = l;
#pragma unroll
  for (int e = 0; e < 8; ++e) accs[kg][c * 8 + e] = acc[e];
  __syncthreads();
  if (tid >= kDecDh) return;
  l = 0.f;
#pragma unroll
  for (int w = 0; w < kDecKC / kWave; ++w) l += red[0][w];
  float r = 0.f;
#pragma unroll 8
  for (int g = 0; g < KG; ++g) r += accs[g][tid];
  if (nsplit == 1) {
    o[(long)b * ldo + h * kDecDh + tid] = f2bf(l > 0.f ? r / l : 0.f);
    return;
  }
  opart[((long)bh * nsplit + split) * kDecDh + tid] = r;
  if (tid == 0) {
    mlpart[((long)bh * nsplit + split) * 2] = m;
    mlpart[((long)bh * nsplit + split) * 2 + 1] = l;
  }
}

__global__ void attn_decode_combine(const float* __restrict__ opart, const float* __restrict__ mlpart,
                                    bf16_t* __restrict__ o, int ldo, int H, int nsplit) {
  const int bh = blockIdx.x, b = bh / H, h = bh - b * H, d = threadIdx.x;
  const float* ml = mlpart + (long)bh * nsplit * 2;
  float M = -INFINITY;
  for (int s = 0; s < nsplit; ++s) M = fmaxf(M, ml[2 * s]);
  float L = 0.f, acc = 0.f;
  for (int s = 0; s < nsplit; ++s) {
    const float ms = ml[2 * s];
    if (ms == -INFINITY) continue;
    const float w = fast_exp2(ms - M);
    L += w * ml[2 * s + 1];
    acc += w * opart[((long)bh * nsplit + s) * kDecDh + d];
  }
  o[(long)b * ldo + h * kDecDh + d] = f2bf(L > 0.f ? acc / L : 0.f);
}

// ---------------------------------------------------------------------------------------------
// Decode linear layer: y = act(s_x[m] s_w[n] (e4m3(LN(x)) . W[n]) + bias) (+ residual) for a
// few rows (one token per sequence).  A workgroup owns 16 rows x (16 or 64) columns:
//   1. every load that does not depend on the activations is issued first — the wave's weight
//      fragments for all of its K blocks, its epilogue scale / bias / residual values, the
//      LayerNorm gamma / beta — together with the activation rows, so the kernel pays one HBM
//      round trip instead of a chain of them;
//   2. prologue: each wave normalises (optional LayerNorm) and quantises its 4 rows per row to
//      e4m3 (the rownorm_quant arithmetic, so results equal the unfused path) and writes the
//      bytes to LDS, XOR-swizzled like the fp8 GEMM;
//   3. v_mfma_scale_f32_16x16x128_f8f6f4 over the preloaded fragments (each lane holds 32 K
//      bytes of one row, pieces g and g + 4 of a 128-byte block).
// KS = 4: the four waves split K over a 16-column tile (partials meet in LDS) — small N.
// KS = 1 (large N, the vocabulary projection): a persistent grid; each workgroup quantises its
// rows once and then walks 64-column tiles (wave w owns columns 16w .. 16w+15 over all of K),
// double-buffering the next tile's weight fragments behind the current tile's MFMAs.
template <int MAXC, int KS, int KBW, bool LN>
__global__ __launch_bounds__(256) void dec_linear_kernel(
    const bf16_t* __restrict__ x, int ldx, const float* __restrict__ gamma, const float* __restrict__ beta,
    float eps, const uint8_t* __restrict__ w, const float* __restrict__ sw, const float* __restrict__ bias,
    const bf16_t* res, int ldr, bf16_t* y, int ldy, int M, int N, int K, int act) {
  constexpr int KMAX = MAXC * 512;
  constexpr int BN = 16 * (4 / KS);
  __shared__ __attribute__((aligned(16))) uint8_t As[16 * KMAX];
  __shared__ float sa[16];
  __shared__ float red[3][256];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int m0 = blockIdx.y * 16;
  const int fr = lane & 15, g = lane >> 4;
  const int nkb = K >> 7;
  const int kw = KS == 1 ? 0 : wave;           // this wave's first K block; stride KS
  const int ntiles = (N + BN - 1) / BN;
  int tile = blockIdx.x;
  auto col = [&](int t) { return t * BN + (KS == 1 ? wave * 16 : 0) + fr; };
  // ---- 1. independent loads in flight
  // two fragment buffers, always indexed by compile-time constants (register arrays)
  u32x4 bl0[KBW], bh0[KBW], bl1[KBW], bh1[KBW];
  auto load_w = [&](int t, u32x4 (&lo)[KBW], u32x4 (&hi)[KBW]) {
    const int n = col(t);
    const uint8_t* wr = w + (long)(n < N ? n : N - 1) * K + g * 16;
#pragma unroll
    for (int i = 0; i < KBW; ++i) {
      const int kb = kw + KS * i;
      if (kb < nkb) {
        lo[i] = *reinterpret_cast<const u32x4*>(wr + kb * 128);
        hi[i] = *reinterpret_cast<const u32x4*>(wr + kb * 128 + 64);
      }
    }
  };
  load_w(tile, bl0, bh0);
  const int nchunk = K >> 3;
  u32x4 raw[4][MAXC];
#pragma unroll
  for (int rr = 0; rr < 4; ++rr) {
    const int row = m0 + wave + 4 * rr;
#pragma unroll
    for (int cc = 0; cc < MAXC; ++cc) {
      const int ch = lane + 64 * cc;
      raw[rr][cc] = row < M && ch < nchunk ? *reinterpret_cast<const u32x4*>(x + (long)row * ldx + ch * 8)
                                           : u32x4{0u, 0u, 0u, 0u};
    }
  }
  f32x4 gm[MAXC][2], bt[MAXC][2];
  if constexpr (LN) {
#pragma unroll
    for (int cc = 0; cc < MAXC; ++cc) {
      const int ch = lane + 64 * cc < nchunk ? lane + 64 * cc : 0;
      gm[cc][0] = *reinterpret_cast<const f32x4*>(gamma + ch * 8);
      gm[cc][1] = *reinterpret_cast<const f32x4*>(gamma + ch * 8 + 4);
      bt[cc][0] = *reinterpret_cast<const f32x4*>(beta + ch * 8);
      bt[cc][1] = *reinterpret_cast<const f32x4*>(beta + ch * 8 + 4);
    }
  }
  // ---- 2. prologue: rows wave, wave + 4, wave + 8, wave + 12 of the tile
#pragma unroll
  for (int rr = 0; rr < 4; ++rr) {
    const int r = wave + 4 * rr, row = m0 + r;
    float vv[MAXC][8];
    float s = 0.f;
#pragma unroll
    for (int cc = 0; cc < MAXC; ++cc) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        vv[cc][2 * e] = __uint_as_float(raw[rr][cc][e] << 16);
        vv[cc][2 * e + 1] = __uint_as_float(raw[rr][cc][e] & 0xffff0000u);
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) s += vv[cc][e];
    }
    if constexpr (LN) {
      const float mean = wave_sum(s) / K;
      float ss = 0.f;
#pragma unroll
      for (int cc = 0; cc < MAXC; ++cc)
        if (lane + 64 * cc < nchunk) {
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const float d = vv[cc][e] - mean;
            ss += d * d;
          }
        }
      const float rstd = rsqrtf(wave_sum(ss) / K + eps);
#pragma unroll
      for (int cc = 0; cc < MAXC; ++cc) {
#pragma unroll
        for (int e = 0; e < 8; ++e) vv[cc][e] = (vv[cc][e] - mean) * rstd * gm[cc][e >> 2][e & 3] + bt[cc][e >> 2][e & 3];
      }
    }
    float amax = 0.f;
#pragma unroll
    for (int cc = 0; cc < MAXC; ++cc)
      if (lane + 64 * cc < nchunk) {
#pragma unroll
        for (int e = 0; e < 8; ++e) amax = fmaxf(amax, fabsf(vv[cc][e]));
      }
    amax = wave_max(amax);
    const float scale = amax > 0.f ? amax / 448.f : 1.f;
    const float inv = 1.f / scale;
    if (lane == 0) sa[r] = row < M ? scale : 0.f;
#pragma unroll
    for (int cc = 0; cc < MAXC; ++cc) {
      const int ch = lane + 64 * cc;
      if (ch < nchunk) {
        unsigned w0 = 0u, w1 = 0u;
        w0 = __builtin_amdgcn_cvt_pk_fp8_f32(fminf(fmaxf(vv[cc][0] * inv, -448.f), 448.f),
                                             fminf(fmaxf(vv[cc][1] * inv, -448.f), 448.f), w0, false);
        w0 = __builtin_amdgcn_cvt_pk_fp8_f32(fminf(fmaxf(vv[cc][2] * inv, -448.f), 448.f),
                                             fminf(fmaxf(vv[cc][3] * inv, -448.f), 448.f), w0, true);
        w1 = __builtin_amdgcn_cvt_pk_fp8_f32(fminf(fmaxf(vv[cc][4] * inv, -448.f), 448.f),
                                             fminf(fmaxf(vv[cc][5] * inv, -448.f), 448.f), w1, false);
        w1 = __builtin_amdgcn_cvt_pk_fp8_f32(fminf(fmaxf(vv[cc][6] * inv, -448.f), 448.f),
                                             fminf(fmaxf(vv[cc][7] * inv, -448.f), 448.f), w1, true);
        const int kbyte = ch * 8, piece = (kbyte & 127) >> 4;
        *reinterpret_cast<uint2*>(As + r * K + (kbyte & ~127) + ((piece ^ (r & 7)) << 4) + (kbyte & 8)) =
            make_uint2(w0, w1);
      }
    }
  }
  __syncthreads();
  // ---- 3. MFMA over the preloaded weight fragments, then the epilogue; KS == 1 loops tiles
  auto do_tile = [&](int t, const u32x4 (&lo)[KBW], const u32x4 (&hi)[KBW]) {
    const int n = col(t);
    float cs = 0.f, cb = 0.f, rv[4] = {0.f, 0.f, 0.f, 0.f};
    if (n < N) {
      cs = sw[n];
      cb = bias ? bias[n] : 0.f;
      if (res) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int m = m0 + g * 4 + e;
          if (m < M) rv[e] = bf2f(res[(long)m * ldr + n]);
        }
      }
    }
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int i = 0; i < KBW; ++i) {
      const int kb = kw + KS * i;
      if (kb < nkb) {
        const uint8_t* ar = As + fr * K + kb * 128;
        const u32x4 a0 = *reinterpret_cast<const u32x4*>(ar + ((g ^ (fr & 7)) << 4));
        const u32x4 a1 = *reinterpret_cast<const u32x4*>(ar + (((g + 4) ^ (fr & 7)) << 4));
        acc = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(
            i32x8{(int)a0[0], (int)a0[1], (int)a0[2], (int)a0[3], (int)a1[0], (int)a1[1], (int)a1[2], (int)a1[3]},
            i32x8{(int)lo[i][0], (int)lo[i][1], (int)lo[i][2], (int)lo[i][3], (int)hi[i][0], (int)hi[i][1],
                  (int)hi[i][2], (int)hi[i][3]},
            acc, 0, 0, 0, 127, 0, 127);
      }
    }
    if constexpr (KS == 4) {
      if (wave > 0) {
#pragma unroll
        for (int e = 0; e < 4; ++e) red[wave - 1][lane * 4 + e] = acc[e];
      }
      __syncthreads();
      if (wave > 0) return;
#pragma unroll
      for (int e = 0; e < 4; ++e) acc[e] += red[0][lane * 4 + e] + red[1][lane * 4 + e] + red[2][lane * 4 + e];
    }
    if (n < N) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int r = g * 4 + e, m = m0 + r;
        if (m >= M) continue;
        float val = acc[e] * sa[r] * cs + cb;
        if (act == 1) val = fmaxf(val, 0.f);
        else if (act == 2) val = silu(val);
        else if (act == 3) val = gelu_erf(val);
        y[(long)m * ldy + n] = f2bf(val + rv[e]);
      }
    }
  };
  if constexpr (KS == 4) {
    do_tile(tile, bl0, bh0);
  } else {
    const int step = gridDim.x;
    while (tile < ntiles) {                      // ping-pong: prefetch one tile ahead
      if (tile + step < ntiles) load_w(tile + step, bl1, bh1);
      do_tile(tile, bl0, bh0);
      tile += step;
      if (tile >= ntiles) break;
      if (tile + step < ntiles) load_w(tile + step, bl0, bh0);
      do_tile(tile, bl1, bh1);
      tile += step;
    }
  }
}

// greedy next token; one 1024-thread workgroup per sequence
__global__ __launch_bounds__(1024) void argmax_step_kernel(
    const bf16_t* __restrict__ logits, int ld, int V, int* __restrict__ ids, int* pos,
    int* __restrict__ out_tokens, int max_len, const int* __restrict__ forced, int n_forced, int eot,
    int* __restrict__ done, unsigned* counter) {
  __shared__ float bv[16];
  __shared__ int bi[16];
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int p = *pos;
  const bf16_t* row = logits + (long)b * ld;
  float best = -INFINITY;
  int besti = 0x7fffffff;
  const int n8 = (V + 7) / 8;
  for (int c = tid; c < n8; c += 1024) {
    const uint4 u = *reinterpret_cast<const uint4*>(row + c * 8);
    const uint32_t* up = reinterpret_cast<const uint32_t*>(&u);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int idx = c * 8 + i;
      const float val = __uint_as_float(i & 1 ? up[i >> 1] & 0xffff0000u : up[i >> 1] << 16);
      if (idx < V && val > best) { best = val; besti = idx; }   // ascending idx: first wins
    }
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const float ov = __shfl_xor(best, off, 64);
    const int oi = __shfl_xor(besti, off, 64);
    if (ov > best || (ov == best && oi < besti)) { best = ov; besti = oi; }
  }
  if (lane == 0) { bv[wave] = best; bi[wave] = besti; }
  __syncthreads();
  if (tid == 0) {
    for (int w = 1; w < 16; ++w)
      if (bv[w] > best || (bv[w] == best && bi[w] < besti)) { best = bv[w]; besti = bi[w]; }
    if (besti == 0x7fffffff) besti = eot;       // all NaN / -inf row
    int tok = besti;
    const int nxt = p + 1;
    if (done[b]) tok = eot;
    if (nxt < n_forced) tok = forced[nxt];
    if (nxt < max_len) out_tokens[(long)b * max_len + nxt] = tok;
    ids[b] = tok;
    if (tok == eot && nxt >= n_forced) done[b] = 1;
    __threadfence();
    if (atomicAdd(counter, 1u) == gridDim.x - 1) {   // last sequence of the step advances pos
      *pos = nxt;
      *counter = 0u;
    }
  }
}

}  // namespace aiko

extern "C" {

int aiko_embed_tokens(const int* ids, const int* pos, const void* tok, const void* pemb, void* x, int B,
                      int d, int ldx, int vocab, int n_pos, hipStream_t stream) {
  if (d % 8 || ldx % 8 || B <= 0) return -1;
  hipLaunchKernelGGL(aiko::embed_kernel, dim3(B), dim3(128), 0, stream, ids, pos,
                     (const aiko::bf16_t*)tok, (const aiko::bf16_t*)pemb, (aiko::bf16_t*)x, d, ldx,
                     vocab, n_pos);
  return (int)hipGetLastError();
}

// splits: one per (sequence, head) once there are enough of those to cover the CUs (the chunk
// loop streams the keys), more for few sequences (partials + combine launch)
static int attn_decode_splits(int B, int H, int maxlen) {
  const int chunks = (maxlen + aiko::kDecKC - 1) / aiko::kDecKC;
  const int bh = B * H;
  if (bh >= 128) return 1;
  const int want = (512 + bh - 1) / bh;
  return want < chunks ? want : chunks;
}

int aiko_attn_decode(const void* q, int ldq, void* k, void* v, int ldk, int ldv, int S, const int* pos,
                     int T, const void* knew, const void* vnew, int ldnew, void* o, int ldo, int B,
                     int H, float scale, float* work, long work_elems, hipStream_t stream) {
  const int maxlen = pos ? S : T;
  if (maxlen <= 0 || (!pos && T > S) || ldq % 8 || ldk % 8 || ldv % 8 || (pos && ldnew % 8)) return -1;
  const int nsplit = attn_decode_splits(B, H, maxlen);
  const long need = (long)B * H * nsplit * (aiko::kDecDh + 2);
  if (nsplit > 1 && need > work_elems) return -1;
  float* opart = work;
  float* mlpart = work + (long)B * H * nsplit * aiko::kDecDh;
  const float scale_log2 = scale * 1.4426950408889634f;
  hipLaunchKernelGGL(aiko::attn_decode_kernel, dim3(nsplit, B * H), dim3(aiko::kDecKC), 0, stream,
                     (const aiko::bf16_t*)q, ldq, (aiko::bf16_t*)k, (aiko::bf16_t*)v, ldk, ldv, S, pos, T,
                     (const aiko::bf16_t*)knew, (const aiko::bf16_t*)vnew, ldnew, H, nsplit, scale_log2,
                     opart, mlpart, (aiko::bf16_t*)o, ldo);
  if (nsplit > 1)
    hipLaunchKernelGGL(aiko::attn_decode_combine, dim3(B * H), dim3(aiko::kDecDh), 0, stream, opart, mlpart,
                       (aiko::bf16_t*)o, ldo, H, nsplit);
  return (int)hipGetLastError();
}

long aiko_attn_decode_work(int B, int H, int maxlen) {
  return (long)B * H * attn_decode_splits(B, H, maxlen) * (aiko::kDecDh + 2);
}

int aiko_dec_linear(const void* x, int ldx, const float* gamma, const float* beta, float eps, const void* w,
                    const float* sw, const float* bias, const void* res, int ldr, void* y, int ldy, int M, int N,
                    int K, int act, hipStream_t stream) {
  if (K % 128 || ldx % 8 || M <= 0 || N <= 0 || K > 3072) return -1;
  const aiko::bf16_t* xp = (const aiko::bf16_t*)x;
  const uint8_t* wp = (const uint8_t*)w;
  const aiko::bf16_t* rp = (const aiko::bf16_t*)res;
  aiko::bf16_t* yp = (aiko::bf16_t*)y;
  const int nkb = K / 128;
  const bool wide = N >= 8192 && nkb <= 8;      // vocabulary projection: persistent 64-column tiles
  const bool ln = gamma != nullptr;
  dim3 grid(wide ? min((N + 63) / 64, 512) : (N + 15) / 16, (M + 15) / 16), block(256);
#define AIKO_DEC_LIN(MC, KS, KBW)                                                                     \
  do {                                                                                               \
    if (ln)                                                                                          \
      hipLaunchKernelGGL((aiko::dec_linear_kernel<MC, KS, KBW, true>), grid, block, 0, stream, xp, ldx, \
                         gamma, beta, eps, wp, sw, bias, rp, ldr, yp, ldy, M, N, K, act);            \
    else                                                                                             \
      hipLaunchKernelGGL((aiko::dec_linear_kernel<MC, KS, KBW, false>), grid, block, 0, stream, xp, ldx, \
                         gamma, beta, eps, wp, sw, bias, rp, ldr, yp, ldy, M, N, K, act);            \
  } while (0)
  if (wide) {
    if (K <= 1024) AIKO_DEC_LIN(2, 1, 8);
    else return -1;
  } else if (K <= 1024) {
    AIKO_DEC_LIN(2, 4, 2);
  } else if (K <= 1536) {
    AIKO_DEC_LIN(3, 4, 3);
  } else {
    AIKO_DEC_LIN(6, 4, 6);
  }
#undef AIKO_DEC_LIN
  return (int)hipGetLastError();
}

int aiko_argmax_step(const void* logits, int ld, int V, int B, int* ids, int* pos, int* out_tokens,
                     int max_len, const int* forced, int n_forced, int eot, int* done, unsigned* counter,
                     hipStream_t stream) {
  if (ld % 8 || (V + 7) / 8 * 8 > ld || B <= 0) return -1;
  hipLaunchKernelGGL(aiko::argmax_step_kernel, dim3(B), dim3(1024), 0, stream, (const aiko::bf16_t*)logits,
                     ld, V, ids, pos, out_tokens, max_len, forced, n_forced, eot, done, counter);
  return (int)hipGetLastError();
}

}  // extern "C"
