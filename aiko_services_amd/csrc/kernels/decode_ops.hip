// Autoregressive decoder step kernels (gfx950, wave64) for the Whisper text decoder
// (the speech-to-text half of the reference's PE_WhisperX, examples/speech/
// speech_elements.py:203-262):
//
//   * embed_kernel        x[b] = tok_emb[ids[b]] + pos_emb[*pos]
//   * attn_decode_partial one query row per sequence against a KV cache, flash-decoding
//                         split: workgroup (split, b*H+h) scores KC keys, keeps its own
//                         running max / sum / P·V in fp32 and writes one partial; in append
//                         mode the new key/value row (at *pos) is taken from the QKV GEMM
//                         output and written into the cache by the split that owns it
//   * attn_decode_combine merges the per-split partials (log2-domain maxima) -> bf16 row
//   * argmax_step_kernel  greedy next token per sequence (first index on ties), forced
//                         prompt prefix, sticky end-of-text, device-side position counter
//                         advanced by the last workgroup to finish (threadfence + counter)
//
// Every launch reads the step position from device memory, so a whole decoder step is one
// hipGraph replayed without host round trips.  The step is bandwidth bound (cross-attention
// K/V and fp8 weights stream once per token); scores/values run on VALU with 16-byte loads.
#include <hip/hip_runtime.h>

#include <math.h>

#include "common.h"

namespace aiko {

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
__global__ __launch_bounds__(kDecKC) void attn_decode_partial(
    const bf16_t* __restrict__ q, int ldq, bf16_t* k, bf16_t* v, int ldk, int ldv, int S,
    const int* __restrict__ pos, int T, const bf16_t* __restrict__ knew,
    const bf16_t* __restrict__ vnew, int ldnew, int H, int nsplit, float scale_log2,
    float* __restrict__ opart, float* __restrict__ mlpart) {
  __shared__ float qs[kDecDh];
  __shared__ float ps[kDecKC];
  __shared__ float red[kDecKC / kWave];
  __shared__ float accs[kDecKC / kDecDh][kDecDh];
  const int split = blockIdx.x, bh = blockIdx.y;
  const int b = bh / H, h = bh - b * H;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int papp = pos ? *pos : -1;            // appended position (append mode)
  const int len = pos ? papp + 1 : T;
  const int start = split * kDecKC;
  const int cnt = min(kDecKC, len - start);
  float* op = opart + ((long)bh * nsplit + split) * kDecDh;
  float* ml = mlpart + ((long)bh * nsplit + split) * 2;
  if (cnt <= 0) {                              // uniform: nothing to attend in this split
    if (tid < kDecDh) op[tid] = 0.f;
    if (tid == 0) { ml[0] = -INFINITY; ml[1] = 0.f; }
    return;
  }
  const long kb = (long)b * S;
  const bf16_t* knr = knew ? knew + (long)b * ldnew + h * kDecDh : nullptr;
  const bf16_t* vnr = vnew ? vnew + (long)b * ldnew + h * kDecDh : nullptr;
  if (tid < kDecDh) qs[tid] = bf2f(q[(long)b * ldq + h * kDecDh + tid]) * scale_log2;
  // the split owning the appended row writes it into the cache (read by later steps only)
  if (knr && papp >= start && papp < start + kDecKC && tid < 16) {
    const int c = (tid & 7) * 8;
    if (tid < 8)
      *reinterpret_cast<uint4*>(k + (kb + papp) * ldk + h * kDecDh + c) = *reinterpret_cast<const uint4*>(knr + c);
    else
      *reinterpret_cast<uint4*>(v + (kb + papp) * ldv + h * kDecDh + c) = *reinterpret_cast<const uint4*>(vnr + c);
  }
  __syncthreads();
  // ---- scores: one key per thread
  const int j = start + tid;
  float s = -INFINITY;
  if (tid < cnt) {
    const bf16_t* kr = (j == papp && knr) ? knr : k + (kb + j) * ldk + h * kDecDh;
    float acc = 0.f;
#pragma unroll
    for (int c = 0; c < 8; ++c) acc += dot8(*reinterpret_cast<const uint4*>(kr + c * 8), qs + c * 8);
    s = acc;
  }
  float m = wave_max(s);
  if (lane == 0) red[wave] = m;
  __syncthreads();
  m = red[0];
#pragma unroll
  for (int w = 1; w < kDecKC / kWave; ++w) m = fmaxf(m, red[w]);
  const float p = tid < cnt ? fast_exp2(s - m) : 0.f;
  ps[tid] = p;
  float l = wave_sum(p);
  __syncthreads();                              // red[] reads done before reuse; ps[] visible
  if (lane == 0) red[wave] = l;
  // ---- P·V: lane = dim, wave = key phase
  float o = 0.f;
  for (int jj = wave; jj < cnt; jj += kDecKC / kDecDh) {
    const int jg = start + jj;
    const bf16_t* vr = (jg == papp && vnr) ? vnr : v + (kb + jg) * ldv + h * kDecDh;
    o += ps[jj] * bf2f(vr[lane]);
  }
  accs[wave][lane] = o;
  __syncthreads();
  if (tid < kDecDh) {
    float r = accs[0][tid];
#pragma unroll
    for (int w = 1; w < kDecKC / kDecDh; ++w) r += accs[w][tid];
    op[tid] = r;
  }
  if (tid == 0) {
    float lt = 0.f;
#pragma unroll
    for (int w = 0; w < kDecKC / kWave; ++w) lt += red[w];
    ml[0] = m;
    ml[1] = lt;
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

int aiko_attn_decode(const void* q, int ldq, void* k, void* v, int ldk, int ldv, int S, const int* pos,
                     int T, const void* knew, const void* vnew, int ldnew, void* o, int ldo, int B,
                     int H, float scale, float* work, long work_elems, hipStream_t stream) {
  const int maxlen = pos ? S : T;
  if (maxlen <= 0 || (!pos && T > S) || ldq % 8 || ldk % 8 || ldv % 8 || (pos && ldnew % 8)) return -1;
  const int nsplit = (maxlen + aiko::kDecKC - 1) / aiko::kDecKC;
  const long need = (long)B * H * nsplit * (aiko::kDecDh + 2);
  if (need > work_elems) return -1;
  float* opart = work;
  float* mlpart = work + (long)B * H * nsplit * aiko::kDecDh;
  const float scale_log2 = scale * 1.4426950408889634f;
  hipLaunchKernelGGL(aiko::attn_decode_partial, dim3(nsplit, B * H), dim3(aiko::kDecKC), 0, stream,
                     (const aiko::bf16_t*)q, ldq, (aiko::bf16_t*)k, (aiko::bf16_t*)v, ldk, ldv, S, pos, T,
                     (const aiko::bf16_t*)knew, (const aiko::bf16_t*)vnew, ldnew, H, nsplit, scale_log2,
                     opart, mlpart);
  hipLaunchKernelGGL(aiko::attn_decode_combine, dim3(B * H), dim3(aiko::kDecDh), 0, stream, opart, mlpart,
                     (aiko::bf16_t*)o, ldo, H, nsplit);
  return (int)hipGetLastError();
}

long aiko_attn_decode_work(int B, int H, int maxlen) {
  const int nsplit = (maxlen + aiko::kDecKC - 1) / aiko::kDecKC;
  return (long)B * H * nsplit * (aiko::kDecDh + 2);
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
