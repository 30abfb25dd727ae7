// Detection kernels for gfx950 (YOLOv8 family): nearest upsample into concat slices, the
// anchor-free DFL box decode, and a fused per-image "top-k candidates + class-aware NMS".
//
// top-k + NMS — three kernels.  Measured (rocprofv3, YOLOv8-n bench batch: B=64 x 8400 anchors,
// random weights, 1024 candidates per image): the former single 1024-thread workgroup per
// image took 246 us (IoU bitmask 130 us on 64 CUs, shuffle-bound greedy scan 86 us); now
// nms_select 24 us + nms_mask 31-32 us + nms_greedy 26 us = 83 us (scripts/nms_phases.py,
// per-phase stops: scripts/nms_stop.sh):
//   nms_select (one workgroup per image): keys (5 us), radix select (2 x 12-bit passes over
//              key - min key, skipped when every live key is a candidate), compaction, sort
//              (per-wave register bitonic + merge by rank), sorted candidates to a workspace;
//   nms_mask   (B x 136 waves, balanced): the IoU bitmask over the whole GPU, 4-compare overlap
//              gate before the exact IoU, plus the transposed diagonal words;
//   nms_greedy (one workgroup per image): upper-triangle masks staged in LDS (padded rows), the
//              scan per 64-candidate word as a ballot fixed point, output mapping.
// Phases:
//   1. scores above the confidence threshold -> 32-bit keys (float bits are monotone for
//      positive floats) in LDS;
//   2. radix select finds the K-th largest key, K = min(max_candidates, #above conf);
//   3. deterministic compaction (block-wide exclusive scan, ties -> lowest anchor index) and a
//      sort of the <= 1024 candidates by (score desc, index asc);
//   4. the IoU suppression bitmask (n x ceil(n/64) 64-bit words) — boxes are offset by
//      class * max_wh so one pass is class-aware;
//   5. one wave scans the bitmask 64 candidates at a time: inside a word the suppression chain
//      is resolved from the diagonal words, then the kept rows' words are OR-ed into the later
//      words lane-parallel; stops at max_det;
//   6. kept boxes are mapped back from letterbox to frame coordinates, clipped, and written
//      as fixed-size [max_det, 6] rows (x1, y1, x2, y2, score, class) + a count, so results can
//      be all-gathered over RCCL without a size exchange.
// AIKO_NMS_STOP=<phase> (profiling only) ends the kernels early: 1-4 inside nms_select (then
// nothing else runs), 5 / 6 inside nms_greedy.
#include "common.h"

namespace aiko {

// ---------------------------------------------------------------------------------------------
// Nearest 2x upsample, NHWC bf16 (C % 8 == 0), x / y may be channel slices (pixel pitches
// ldx / ldy): one thread per 8 channels of an input pixel, one 16-B load -> four 16-B stores.
// 2-D grid (y: image row b*H + h) so a thread only divides its in-row index by C/8 (32-bit);
// the flat grid-stride version spent four 64-bit div/mods per 16 bytes.  More than 65535 rows
// (B*H) stride over grid y.
__global__ __launch_bounds__(256) void upsample2x_kernel(const bf16_t* __restrict__ x, bf16_t* __restrict__ y,
                                                         int BH, int H, int W, int C, int ldx, int ldy) {
  const int C8 = C >> 3;
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= W * C8) return;
  const int w = i / C8, c8 = i - w * C8;
  const int Wo = 2 * W;
  for (int bh = blockIdx.y; bh < BH; bh += gridDim.y) {
    const int b = bh / H, h = bh - b * H;
    const u32x4 v = *reinterpret_cast<const u32x4*>(x + ((long)bh * W + w) * ldx + c8 * 8);
    bf16_t* o = y + (((long)b * 2 * H + 2 * h) * Wo + 2 * w) * ldy + c8 * 8;
    *reinterpret_cast<u32x4*>(o) = v;
    *reinterpret_cast<u32x4*>(o + ldy) = v;
    *reinterpret_cast<u32x4*>(o + (long)Wo * ldy) = v;
    *reinterpret_cast<u32x4*>(o + (long)Wo * ldy + ldy) = v;
  }
}

// ---------------------------------------------------------------------------------------------
// DFL decode: per anchor (all levels, all images) read the 4 x reg_max box logits and the nc
// class logits of its head pixel -> box xyxy (letterbox pixels), max class score, class id.
constexpr int kMaxLevels = 4;
constexpr int kRegMax = 16;   // DFL bins per box side (YOLOv8)

struct DecodeParams {
  const bf16_t* feat[kMaxLevels];  // [B, H, W, ld] bf16: box logits [0, 4*reg_max), cls after
  int H[kMaxLevels], W[kMaxLevels], stride[kMaxLevels], ld[kMaxLevels], start[kMaxLevels];
  int tstart[kMaxLevels];          // first 64-anchor tile of each level (tiled kernel)
  int nlev, B, A, nc, reg_max;
  float4* boxes;   // [B, A]
  float* scores;   // [B, A]
  int* cls;        // [B, A]
};

__global__ void yolo_decode_kernel(DecodeParams p) {
  const long total = (long)p.B * p.A;
  for (long idx = blockIdx.x * (long)blockDim.x + threadIdx.x; idx < total;
       idx += (long)gridDim.x * blockDim.x) {
    const int b = idx / p.A;
    const int a = idx - (long)b * p.A;
    int l = 0;
#pragma unroll
    for (int i = 1; i < kMaxLevels; ++i)
      if (i < p.nlev && a >= p.start[i]) l = i;
    const int r = a - p.start[l];
    const int h = r / p.W[l], w = r - h * p.W[l];
    const bf16_t* f = p.feat[l] + (((long)b * p.H[l] + h) * p.W[l] + w) * p.ld[l];
    float dist[4];
#pragma unroll
    for (int side = 0; side < 4; ++side) {
      const bf16_t* q = f + side * kRegMax;
      float v[kRegMax];
#pragma unroll
      for (int k = 0; k < kRegMax; k += 8) {
        const u32x4 u = *reinterpret_cast<const u32x4*>(q + k);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          v[k + 2 * e] = __uint_as_float(u[e] << 16);
          v[k + 2 * e + 1] = __uint_as_float(u[e] & 0xffff0000u);
        }
      }
      float m = v[0];
#pragma unroll
      for (int k = 1; k < kRegMax; ++k) m = fmaxf(m, v[k]);
      float se = 0.f, sk = 0.f;
#pragma unroll
      for (int k = 0; k < kRegMax; ++k) {
        const float e = __expf(v[k] - m);
        se += e;
        sk += e * k;
      }
      dist[side] = sk / se;
    }
    const bf16_t* c = f + 4 * kRegMax;
    float best = -INFINITY;
    int bi = 0;
    for (int k = 0; k < p.nc; k += 8) {
      const u32x4 u = *reinterpret_cast<const u32x4*>(c + k);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float v0 = __uint_as_float(u[e] << 16), v1 = __uint_as_float(u[e] & 0xffff0000u);
        if (v0 > best) { best = v0; bi = k + 2 * e; }
        if (v1 > best) { best = v1; bi = k + 2 * e + 1; }
      }
    }
    const float s = (float)p.stride[l];
    const float ax = w + 0.5f, ay = h + 0.5f;
    p.boxes[idx] = make_float4((ax - dist[0]) * s, (ay - dist[1]) * s, (ax + dist[2]) * s,
                               (ay + dist[3]) * s);
    p.scores[idx] = 1.f / (1.f + __expf(-best));
    p.cls[idx] = bi;
  }
}

// Coalesced variant: a 256-thread block takes 64 consecutive anchors of one level of one image
// (blockIdx.y = image, blockIdx.x = tile; tiles never straddle levels), copies their rows
// (contiguous [64, ld] in memory) into LDS with 16-byte loads, then a quad of lanes decodes each
// anchor: lane j takes DFL side j and class chunks j, j+4, j+8 (8 classes each), combined with
// quad DPP (max value, lowest index on ties).  The per-anchor thread version above reads 16 B at
// a 288 B lane stride, touching 64 lines per load instruction.  Same per-side arithmetic in the
// same order and an exact max, so the outputs are bit-identical to it.
template <int Q>
__device__ __forceinline__ int dpp_i32(int v) {
  return __builtin_amdgcn_update_dpp(0, v, Q, 0xF, 0xF, false);
}

__global__ __launch_bounds__(256) void yolo_decode_tiled_kernel(DecodeParams p) {
  extern __shared__ __attribute__((aligned(16))) bf16_t rows[];
  const int CH = 4 * kRegMax + p.nc, CHP = CH + 8, NCH = CH >> 3;
  const int b = blockIdx.y;
  int l = 0;
#pragma unroll
  for (int i = 1; i < kMaxLevels; ++i)
    if (i < p.nlev && (int)blockIdx.x >= p.tstart[i]) l = i;
  const int HW = p.H[l] * p.W[l];
  const int r0 = ((int)blockIdx.x - p.tstart[l]) * 64;
  const int n = min(64, HW - r0);
  const bf16_t* src = p.feat[l] + ((long)b * HW + r0) * p.ld[l];
  for (int i = threadIdx.x; i < n * NCH; i += 256) {
    const int row = i / NCH, ch = i - row * NCH;
    *reinterpret_cast<u32x4*>(rows + row * CHP + ch * 8) =
        *reinterpret_cast<const u32x4*>(src + (long)row * p.ld[l] + ch * 8);
  }
  __syncthreads();
  const int j = threadIdx.x & 3, ai = threadIdx.x >> 2;
  const bool live = ai < n;
  const bf16_t* f = rows + (live ? ai : 0) * CHP;
  float v[kRegMax];
#pragma unroll
  for (int k = 0; k < kRegMax; k += 8) {
    const u32x4 u = *reinterpret_cast<const u32x4*>(f + j * kRegMax + k);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      v[k + 2 * e] = __uint_as_float(u[e] << 16);
      v[k + 2 * e + 1] = __uint_as_float(u[e] & 0xffff0000u);
    }
  }
  float m = v[0];
#pragma unroll
  for (int k = 1; k < kRegMax; ++k) m = fmaxf(m, v[k]);
  float se = 0.f, sk = 0.f;
#pragma unroll
  for (int k = 0; k < kRegMax; ++k) {
    const float e = __expf(v[k] - m);
    se += e;
    sk += e * k;
  }
  const float dist = sk / se;
  const bf16_t* c = f + 4 * kRegMax;
  float best = -INFINITY;
  int bi = 0x7fffffff;
  for (int k = 8 * j; k < p.nc; k += 32) {
    const u32x4 u = *reinterpret_cast<const u32x4*>(c + k);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float v0 = __uint_as_float(u[e] << 16), v1 = __uint_as_float(u[e] & 0xffff0000u);
      if (v0 > best) { best = v0; bi = k + 2 * e; }
      if (v1 > best) { best = v1; bi = k + 2 * e + 1; }
    }
  }
  {
    const float ob = dpp_f32<0xB1>(best);
    const int oi = dpp_i32<0xB1>(bi);
    if (ob > best || (ob == best && oi < bi)) { best = ob; bi = oi; }
  }
  {
    const float ob = dpp_f32<0x4E>(best);
    const int oi = dpp_i32<0x4E>(bi);
    if (ob > best || (ob == best && oi < bi)) { best = ob; bi = oi; }
  }
  if (bi == 0x7fffffff) bi = 0;       // no logit above -INF: class 0, as the sequential scan gives
  const float d0 = dpp_f32<0x00>(dist), d1 = dpp_f32<0x55>(dist);
  const float d2 = dpp_f32<0xAA>(dist), d3 = dpp_f32<0xFF>(dist);
  if (live && j == 0) {
    const int r = r0 + ai;
    const int h = r / p.W[l], w = r - h * p.W[l];
    const float s = (float)p.stride[l];
    const float ax = w + 0.5f, ay = h + 0.5f;
    const long idx = (long)b * p.A + p.start[l] + r;
    p.boxes[idx] = make_float4((ax - d0) * s, (ay - d1) * s, (ax + d2) * s, (ay + d3) * s);
    p.scores[idx] = 1.f / (1.f + __expf(-best));
    p.cls[idx] = bi;
  }
}

// ---------------------------------------------------------------------------------------------
constexpr int kNmsThreads = 1024;
constexpr int kMaxCand = 1024;
constexpr int kMaxAnchors = 32768;
constexpr int kMaskWords = kMaxCand / 64;  // 16

struct NmsParams {
  const float4* boxes;
  const float* scores;
  const int* cls;
  int A, max_cand, max_det;
  float conf, iou, max_wh;
  float gain, pad_l, pad_t, img_w, img_h;  // letterbox -> frame mapping
  float* det;   // [B, max_det, 6]
  int* count;   // [B]
  int stop;     // profiling: end the kernels early at phase `stop` (99 = run everything)
};

__device__ __forceinline__ unsigned long long shfl64(unsigned long long v, int src) {
  const unsigned lo = __shfl((unsigned)(v & 0xffffffffull), src, 64);
  const unsigned hi = __shfl((unsigned)(v >> 32), src, 64);
  return ((unsigned long long)hi << 32) | lo;
}

__device__ __forceinline__ float box_iou(float4 a, float4 b) {
  const float iw = fmaxf(0.f, fminf(a.z, b.z) - fmaxf(a.x, b.x));
  const float ih = fmaxf(0.f, fminf(a.w, b.w) - fmaxf(a.y, b.y));
  const float inter = iw * ih;
  const float area_a = (a.z - a.x) * (a.w - a.y), area_b = (b.z - b.x) * (b.w - b.y);
  return inter / (area_a + area_b - inter);
}

// block-wide exclusive scan of one int per thread (1024 threads = 16 waves)
__device__ int block_exclusive_scan(int v, int* sh) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  int x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int t = __shfl_up(x, o, 64);
    if (lane >= o) x += t;
  }
  if (lane == 63) sh[wave] = x;
  __syncthreads();
  if (wave == 0) {
    int y = lane < 16 ? sh[lane] : 0;
    const int own = y;
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) {
      const int t = __shfl_up(y, o, 64);
      if (lane >= o) y += t;
    }
    if (lane < 16) sh[16 + lane] = y - own;
  }
  __syncthreads();
  return x - v + sh[16 + wave];
}

// Workspace of the three NMS kernels (global memory, per image b):
//   ckey[b][1024] u64 sorted candidate keys, cbox[b][1024] class-offset boxes, n[b] count,
//   mask[b][16][1024] u64 IoU suppression words, word-major (word w of row i at [w][i], so
//   consecutive rows store coalesced); only words on / right of the diagonal are written.
struct NmsWork {
  unsigned long long* ckey;
  float4* cbox;
  int* n;
  unsigned long long* mask;
  unsigned long long* low;   // [b][16][1024]: diagonal word, bits k < i (suppressors of i)
};

// 1. keys, radix select, deterministic compaction and bitonic sort — one 1024-thread
//    workgroup per image, keys in LDS; writes the sorted candidates to the workspace.
constexpr int kRadixBits = 12, kRadixBins = 1 << kRadixBits;   // 4096 bins = 4 per thread
__global__ __launch_bounds__(kNmsThreads) void nms_select_kernel(NmsParams p, NmsWork ws) {
  constexpr int REGION0 = kMaxAnchors * 4;
  __shared__ __attribute__((aligned(16))) unsigned char region0[REGION0];
  __shared__ unsigned long long ckey[kMaxCand];
  __shared__ unsigned hist[kRadixBins];
  __shared__ int sh[40];

  unsigned* keys = reinterpret_cast<unsigned*>(region0);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int b = blockIdx.x;
  const int A = p.A;
  const float* sc = p.scores + (long)b * A;
  const float4* bx = p.boxes + (long)b * A;
  const int* cl = p.cls + (long)b * A;

  if (tid == 0) {
    sh[32] = 0;
    sh[36] = 0;                      // max key
    sh[37] = (int)0xffffffffu;       // min live key (as unsigned)
  }
  __syncthreads();
  int cnt = 0;
  unsigned kmax = 0u, kmin = 0xffffffffu;
  // 16 independent loads in flight: one latency round covers A <= 16384 (YOLO VGA: 8400 / 6300)
  for (int i0 = 0; i0 < A; i0 += 16 * kNmsThreads) {
    float v[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const int i = i0 + u * kNmsThreads + tid;
      v[u] = i < A ? sc[i] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const int i = i0 + u * kNmsThreads + tid;
      if (i < A) {
        const unsigned k = v[u] > p.conf ? __float_as_uint(v[u]) : 0u;
        keys[i] = k;
        cnt += k != 0u;
        kmax = max(kmax, k);
        if (k != 0u) kmin = min(kmin, k);
      }
    }
  }
  for (int o = 32; o > 0; o >>= 1) {
    cnt += __shfl_xor(cnt, o, 64);
    kmax = max(kmax, (unsigned)__shfl_xor((int)kmax, o, 64));
    kmin = min(kmin, (unsigned)__shfl_xor((int)kmin, o, 64));
  }
  if (lane == 0) {
    atomicAdd(&sh[32], cnt);
    atomicMax(reinterpret_cast<unsigned*>(&sh[36]), kmax);
    atomicMin(reinterpret_cast<unsigned*>(&sh[37]), kmin);
  }
  __syncthreads();
  const int total = sh[32];
  const int K = min(p.max_cand, total);
  if (tid == 0) ws.n[b] = K;
  if (K == 0 || p.stop == 1) return;

  // radix select of the K-th largest key, on d = key - (min live key), 12-bit digits: only as
  // many as the live range needs (scores in (conf, 1) span ~24 bits -> 2 passes); skipped when
  // every live key is a candidate.  T = threshold key, remaining = candidates equal to T.
  const unsigned klo = (unsigned)sh[37];
  const unsigned range = (unsigned)sh[36] - klo;
  unsigned prefix = 0u, pmask = 0u;
  int remaining = K;
  const int nbits = range == 0u ? 0 : 32 - __clz((int)range);
  int shift = (total <= p.max_cand || nbits == 0) ? -1 : max(0, nbits - kRadixBits);
  while (shift >= 0) {
#pragma unroll
    for (int u = 0; u < kRadixBins / kNmsThreads; ++u) hist[u * kNmsThreads + tid] = 0u;
    __syncthreads();
    // scores cluster: most live keys of a wave often share a bin; a wave accumulates same-bin
    // ballots in a (wave-uniform) running count and issues one LDS atomic per bin change
    unsigned run_bin = 0u, run_cnt = 0u;
    for (int i0 = 0; i0 < A; i0 += kNmsThreads) {   // wave-uniform trip count (ballots below)
      const int i = i0 + tid;
      const unsigned k = i < A ? keys[i] : 0u;
      const unsigned d = k - klo;
      const bool live = k != 0u && (d & pmask) == prefix;
      const unsigned bin = (d >> shift) & (kRadixBins - 1u);
      const unsigned long long lm = __ballot(live);
      if (lm) {
        const int leader = __ffsll((long long)lm) - 1;
        const unsigned lbin = __shfl(bin, leader, 64);
        const unsigned long long same = __ballot(live && bin == lbin);
        if (same == lm) {
          if (lbin != run_bin) {
            if (lane == 0 && run_cnt) atomicAdd(&hist[run_bin], run_cnt);
            run_bin = lbin;
            run_cnt = 0u;
          }
          run_cnt += (unsigned)__popcll(lm);
        } else if (live) {
          atomicAdd(&hist[bin], 1u);
        }
      }
    }
    if (lane == 0 && run_cnt) atomicAdd(&hist[run_bin], run_cnt);
    __syncthreads();
    // thread t owns bins 4095-4t .. 4092-4t (descending): an exclusive scan of the per-thread
    // sums gives the count of keys in higher bins; the owner of the K-th key picks its bin
    const int top = kRadixBins - 1 - 4 * tid;
    const int h0 = hist[top], h1 = hist[top - 1], h2 = hist[top - 2], h3 = hist[top - 3];
    const int above = block_exclusive_scan(h0 + h1 + h2 + h3, sh);
    if (above < remaining && above + h0 + h1 + h2 + h3 >= remaining) {
      const int hs[4] = {h0, h1, h2, h3};
      int acc = above;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if (acc + hs[j] >= remaining) {
          sh[34] = top - j;
          sh[35] = remaining - acc;
          break;
        }
        acc += hs[j];
      }
    }
    __syncthreads();
    prefix |= (unsigned)sh[34] << shift;
    pmask |= (kRadixBins - 1u) << shift;
    remaining = sh[35];
    __syncthreads();
    shift = shift == 0 ? -1 : max(0, shift - kRadixBits);
  }
  // all live keys are candidates: threshold below every live key, none "equal"
  const bool take_all = total <= p.max_cand;
  const unsigned T = take_all ? 0u : klo + prefix;
  if (take_all) remaining = 0;
  const int n_gt = K - remaining;
  if (p.stop == 2) return;

  // deterministic compaction (contiguous chunks + block scan) and bitonic sort
  const int chunk = (A + kNmsThreads - 1) / kNmsThreads;
  const int i0 = tid * chunk, i1 = min(A, i0 + chunk);
  int gt = 0, eq = 0;
  for (int i = i0; i < i1; ++i) {
    const unsigned k = keys[i];
    gt += k > T;
    eq += k == T;
  }
  const int base = block_exclusive_scan(gt | (eq << 16), sh);
  int gpos = base & 0xffff, epos = base >> 16;
  for (int i = i0; i < i1; ++i) {
    const unsigned k = keys[i];
    const unsigned long long ck = ((unsigned long long)k << 32) | (0xffffffffu - (unsigned)i);
    if (k > T) {
      ckey[gpos++] = ck;
    } else if (k == T) {
      if (epos < remaining) ckey[n_gt + epos] = ck;
      ++epos;
    }
  }
  int NP = 1;
  while (NP < K) NP <<= 1;
  if (tid >= K && tid < NP) ckey[tid] = 0ull;
  __syncthreads();
  if (p.stop == 3) return;
  // sort = per-wave bitonic sort of 64 keys in registers (21 shuffle passes, no barrier) + merge
  // by rank: a key's final position is its place in its own wave's sorted list plus, for each of
  // the other lists, the number of keys greater than it (7-step binary search of the LDS copy;
  // the 15 searches are independent).  Keys are unique (index in the low word); padding keys
  // are 0 and are not written.  Two barriers instead of the 55-pass block-wide network's 20.
  {
    unsigned long long v = tid < NP ? ckey[tid] : 0ull;
    for (int size = 2; size <= 64; size <<= 1) {
      for (int stride = size >> 1; stride > 0; stride >>= 1) {
        const unsigned lo = __shfl_xor((unsigned)(v & 0xffffffffull), stride, 64);
        const unsigned hi = __shfl_xor((unsigned)(v >> 32), stride, 64);
        const unsigned long long c = ((unsigned long long)hi << 32) | lo;
        const bool desc = size == 64 || (lane & size) == 0, lower = (lane & stride) == 0;
        v = (desc == lower) ? (v > c ? v : c) : (v < c ? v : c);
      }
    }
    __syncthreads();
    ckey[tid] = v;                                   // [wave][64] sorted descending
    __syncthreads();
    int rank = lane;
    const int nl = (NP + 63) >> 6;
#pragma unroll 4
    for (int l = 0; l < nl; ++l) {
      if (l == wave) continue;
      const unsigned long long* L = ckey + l * 64;
      int pos = 0;
#pragma unroll
      for (int st = 32; st > 0; st >>= 1)
        if (L[pos + st - 1] > v) pos += st;
      rank += pos + (L[pos] > v ? 1 : 0);
    }
    __syncthreads();
    if (v != 0ull) ckey[rank] = v;
    __syncthreads();
  }
  if (p.stop == 4) return;
  // sorted keys + class-offset boxes to the workspace
  for (int i = tid; i < K; i += kNmsThreads) {
    const unsigned long long ck = ckey[i];
    const int idx = (int)(0xffffffffu - (unsigned)(ck & 0xffffffffull));
    const float off = cl[idx] * p.max_wh;
    const float4 q = bx[idx];
    ws.ckey[(long)b * kMaxCand + i] = ck;
    ws.cbox[(long)b * kMaxCand + i] = make_float4(q.x + off, q.y + off, q.z + off, q.w + off);
  }
}

// IoU > thr bits of row box bi against the 64 column boxes in LDS (bit jj = column jj), one
// fully unrolled pass: constant bit positions, broadcast LDS reads (FULL: all 64 columns valid,
// no per-column guard; NEG: negative threshold, every pair tested).  Measured alternatives, all
// slower on the bench inputs (most candidate pairs overlap, so the exact IoU math is the work):
// LDS reads issued 8 at a time 32.9 us, a division-free fma test with an exact 1-ulp fallback
// 35 us, a branch-free overlap pass + scalar loop over overlapping columns 50 us, 4 items per
// workgroup 33 us, partial unroll 33-38 us — against 30.7 us for this form.  A 4-compare overlap test on both axes (a superset of inter > 0)
// gates the exact intersection + IEEE division, so the decisions are box_iou() > thr bit for
// bit; most pairs (other classes sit max_wh apart) stop at the 4 compares.  The test is symmetric
// bit for bit (fminf / fmaxf and the area sum commute), so the diagonal word's transposed half
// comes out of the same pass.
template <bool FULL, bool NEG>
__device__ __forceinline__ unsigned long long mask_word(const float4* col, float4 bi, float area_i,
                                                        int je, float thr) {
  unsigned long long hit = 0ull;
#pragma unroll
  for (int jj = 0; jj < 64; ++jj) {
    if (FULL || jj < je) {                                  // wave-uniform
      const float4 c = col[jj];
      if (NEG || (bi.z > c.x && c.z > bi.x && bi.w > c.y && c.w > bi.y)) {
        const float iw = fmaxf(0.f, fminf(bi.z, c.z) - fmaxf(bi.x, c.x));
        const float ih = fmaxf(0.f, fminf(bi.w, c.w) - fmaxf(bi.y, c.y));
        const float inter = iw * ih;
        if (NEG || inter > 0.f) {
          const float iou = inter / (area_i + (c.z - c.x) * (c.w - c.y) - inter);
          if (iou > thr) hit |= 1ull << jj;
        }
      }
    }
  }
  return hit;
}

// 2. IoU suppression bitmask over the whole GPU: one wave per (image, 64-row block rb, word
//    w >= rb) — B x 136 equal-sized work items; lane = row, the 64 column boxes of word w sit in
//    LDS and are read as broadcasts.  The diagonal word also yields its transposed half (bits
//    k < i: the suppressors of row i inside the word) for the greedy kernel's fixed point.
constexpr int kMaskPairs = kMaskWords * (kMaskWords + 1) / 2;   // 136 (rb, w) with w >= rb
constexpr int kMaskWaves = 1;   // work items (waves) per workgroup
static_assert(kMaskPairs % kMaskWaves == 0, "items of an image fill whole workgroups");
__global__ __launch_bounds__(64 * kMaskWaves) void nms_mask_kernel(NmsParams p, NmsWork ws) {
  __shared__ float4 cols[kMaskWaves][64];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int item = blockIdx.x * kMaskWaves + wave;
  const int b = item / kMaskPairs;
  int q = item - b * kMaskPairs, rb = 0;
  while (q >= kMaskWords - rb) {                 // (rb, w) from the triangle index
    q -= kMaskWords - rb;
    ++rb;
  }
  const int w = rb + q;
  const int n = ws.n[b];
  const int r0 = rb * 64, j0 = w * 64;
  const bool work = r0 < n && j0 < n;            // wave-uniform; no return before the barrier
  float4* col = cols[wave];
  const float4* cb = ws.cbox + (long)b * kMaxCand;
  if (work && j0 + lane < n) col[lane] = cb[j0 + lane];
  const int i = r0 + lane;
  const float4 bi = work && i < n ? cb[i] : make_float4(0.f, 0.f, 0.f, 0.f);
  __syncthreads();
  if (!work || i >= n) return;
  const float area_i = (bi.z - bi.x) * (bi.w - bi.y);
  const int je = min(64, n - j0);
  const bool diag = w == rb;
  // (a negative threshold keeps every pair, disjoint ones included: the generic instantiation)
  const unsigned long long hit =
      p.iou < 0.f ? mask_word<false, true>(col, bi, area_i, je, p.iou)
                  : (je == 64 ? mask_word<true, false>(col, bi, area_i, je, p.iou)
                              : mask_word<false, false>(col, bi, area_i, je, p.iou));
  unsigned long long bits = hit;
  if (diag) {
    bits = lane == 63 ? 0ull : hit & (~0ull << (lane + 1));
    ws.low[((long)b * kMaskWords + w) * kMaxCand + i] = hit & ((1ull << lane) - 1ull);
  }
  ws.mask[((long)b * kMaskWords + w) * kMaxCand + i] = bits;
}

__device__ __forceinline__ unsigned long long readlane64(unsigned long long v, int l) {
  const unsigned lo = __builtin_amdgcn_readlane((unsigned)(v & 0xffffffffull), l);
  const unsigned hi = __builtin_amdgcn_readlane((unsigned)(v >> 32), l);
  return ((unsigned long long)hi << 32) | lo;
}

// 3. greedy scan per image.  The mask words at / right of the diagonal are staged into LDS
//    (row stride padded by one word: the scan's lane-parallel reads hit distinct banks).  (A
//    chunked variant — 256 rows at a time, next chunk loaded during the scan, stopping at
//    max_det — measured slower: 26.7 -> 31.6 us.)  The scan: lane w holds the "removed" word w;
//    inside a 64-candidate word the suppression chain is a ballot fixed point over the
//    transposed diagonal words, then the kept rows' words are OR-ed lane-parallel into the later
//    words.  Finally the kept boxes are mapped back from letterbox to frame coordinates.
constexpr int kGreedyThreads = 1024;
constexpr int kWordStride = kMaxCand + 1;   // padded: lane w's reads of words[w][row] hit distinct banks
__global__ __launch_bounds__(kGreedyThreads) void nms_greedy_kernel(NmsParams p, NmsWork ws) {
  __shared__ unsigned long long words[kMaskWords * kWordStride];  // [w][i]
  __shared__ unsigned long long lowd[kMaxCand];                  // row i's transposed diagonal word
  __shared__ int kept[kMaxCand];
  __shared__ int nk_sh;
  const int tid = threadIdx.x, lane = tid & 63;
  const int b = blockIdx.x;
  const int n = ws.n[b];
  const int W = (n + 63) >> 6;
  const unsigned long long* mk = ws.mask + (long)b * kMaxCand * kMaskWords;
  // staging: all 16 loads of a thread are issued before the first LDS store (a load -> store
  // loop would pay one HBM/L2 latency per word); only the words at / right of the diagonal
  // (w >= row block), the only ones the scan reads
  {
    static_assert(kGreedyThreads == kMaxCand, "one thread per candidate row");
    const int rb = tid >> 6;
    unsigned long long tmp[kMaskWords];
#pragma unroll
    for (int w = 0; w < kMaskWords; ++w)
      tmp[w] = (w >= rb && w < W && tid < n) ? mk[(long)w * kMaxCand + tid] : 0ull;
    const unsigned long long lw =
        tid < n ? ws.low[((long)b * kMaskWords + rb) * kMaxCand + tid] : 0ull;
#pragma unroll
    for (int w = 0; w < kMaskWords; ++w) words[w * kWordStride + tid] = tmp[w];
    lowd[tid] = lw;
  }
  if (tid == 0) nk_sh = 0;
  __syncthreads();
  if (p.stop == 5) return;
  if (tid < 64) {
    unsigned long long removed = 0ull;
    int nkept = 0;
    {
      for (int w = 0; w < W && nkept < p.max_det; ++w) {
        unsigned long long cur = readlane64(removed, w);
        const int row = w * 64 + lane;
        // suppressors of this lane's candidate inside the word (rows k < row, transposed diagonal)
        const unsigned long long low = row < n ? lowd[row] : 0ull;
        const int left = n - w * 64;
        const unsigned long long valid = left >= 64 ? ~0ull : ((1ull << left) - 1ull);
        const unsigned long long alive = ~cur & valid;
        const bool me_alive = (alive >> lane) & 1ull;
        // greedy inside the word as a fixed point: kept = alive minus those with a kept
        // suppressor.  Candidate c's status is final once all k < c are, so <= 64 rounds; the
        // first repeat is the (unique) greedy solution.  One ballot per round, not one
        // dependent step per candidate.
        unsigned long long keep = alive;
        for (int it = 0; it <= 64; ++it) {
          const unsigned long long nk = __ballot(me_alive && !(low & keep));
          if (nk == keep) break;
          keep = nk;
        }
        const int room = p.max_det - nkept;
        if (__popcll(keep) > room) {
          unsigned long long trimmed = 0ull, kk = keep;
          for (int r = 0; r < room; ++r) {
            const unsigned long long lowb = kk & (~kk + 1ull);
            trimmed |= lowb;
            kk ^= lowb;
          }
          keep = trimmed;
        }
        if ((keep >> lane) & 1ull) {
          const unsigned long long below = lane ? (keep & ((1ull << lane) - 1ull)) : 0ull;
          kept[nkept + __popcll(below)] = row;
        }
        nkept += __popcll(keep);
        // OR the kept rows' words into the later words: 8 LDS reads in flight per round (a
        // one-read-per-iteration loop exposes the LDS latency for every kept row)
        unsigned long long kk = keep;
        unsigned long long acc = 0ull;
        const bool mine = lane > w && lane < W;
        const unsigned long long* wl = words + lane * kWordStride + w * 64;
        while (kk) {
          int bsel[8];
#pragma unroll
          for (int u = 0; u < 8; ++u) {
            bsel[u] = kk ? __ffsll((long long)kk) - 1 : -1;
            kk &= kk - 1ull;
          }
          unsigned long long v[8];
#pragma unroll
          for (int u = 0; u < 8; ++u) v[u] = (mine && bsel[u] >= 0) ? wl[bsel[u]] : 0ull;
#pragma unroll
          for (int u = 0; u < 8; ++u) acc |= v[u];
        }
        removed |= acc;
      }
    }
    if (lane == 0) nk_sh = nkept;
  }
  __syncthreads();
  if (p.stop == 6) return;
  const int nk = nk_sh;
  const float4* bx = p.boxes + (long)b * p.A;
  const int* cl = p.cls + (long)b * p.A;
  const unsigned long long* ck_all = ws.ckey + (long)b * kMaxCand;
  const float inv = 1.f / p.gain;
  for (int r = tid; r < p.max_det; r += kGreedyThreads) {
    float* o = p.det + ((long)b * p.max_det + r) * 6;
    if (r < nk) {
      const unsigned long long ck = ck_all[kept[r]];
      const int idx = (int)(0xffffffffu - (unsigned)(ck & 0xffffffffull));
      const float4 q = bx[idx];
      o[0] = fminf(fmaxf((q.x - p.pad_l) * inv, 0.f), p.img_w);
      o[1] = fminf(fmaxf((q.y - p.pad_t) * inv, 0.f), p.img_h);
      o[2] = fminf(fmaxf((q.z - p.pad_l) * inv, 0.f), p.img_w);
      o[3] = fminf(fmaxf((q.w - p.pad_t) * inv, 0.f), p.img_h);
      o[4] = __uint_as_float((unsigned)(ck >> 32));
      o[5] = (float)cl[idx];
    } else {
      o[0] = o[1] = o[2] = o[3] = o[4] = 0.f;
      o[5] = -1.f;
    }
  }
  if (tid == 0) p.count[b] = nk;
}

}  // namespace aiko

static inline int grid_for_d(long total, int block) {
  long g = (total + block - 1) / block;
  if (g > 256 * 16) g = 256 * 16;
  if (g < 1) g = 1;
  return (int)g;
}

extern "C" int aiko_upsample2x(const void* x, void* y, int B, int H, int W, int C, int ldx,
                               int ldy, hipStream_t stream) {
  if ((long)B * H > (1L << 31) - 1 || (long)W * (C / 8) > (1L << 30)) return -1;
  const int gx = (W * (C / 8) + 255) / 256;
  const int BH = B * H;
  const int gy = BH < 65535 ? BH : 65535;
  aiko::upsample2x_kernel<<<dim3(gx, gy), 256, 0, stream>>>(
      static_cast<const aiko::bf16_t*>(x), static_cast<aiko::bf16_t*>(y), BH, H, W, C, ldx, ldy);
  return (int)hipGetLastError();
}

// levels: nlev entries of (feat ptr, H, W, stride, ld); outputs [B, A]
extern "C" int aiko_yolo_decode(const void* const* feats, const int* H, const int* W,
                                const int* strides, const int* ld, int nlev, int B, int nc,
                                int reg_max, void* boxes, float* scores, int* cls,
                                hipStream_t stream) {
  if (nlev < 1 || nlev > aiko::kMaxLevels || reg_max != aiko::kRegMax || nc % 8) return -1;
  aiko::DecodeParams p;
  int A = 0, tiles = 0;
  bool tiled = (4 * aiko::kRegMax + nc) * 2 * 64 + 16 * 64 <= 64 * 1024;
  for (int i = 0; i < aiko::kMaxLevels; ++i) {
    p.tstart[i] = tiles;
    if (i < nlev) {
      tiles += (H[i] * W[i] + 63) / 64;
      tiled = tiled && ld[i] % 8 == 0 && ld[i] >= 4 * aiko::kRegMax + nc &&
              reinterpret_cast<uintptr_t>(feats[i]) % 16 == 0;
    }
    p.feat[i] = i < nlev ? static_cast<const aiko::bf16_t*>(feats[i]) : nullptr;
    p.H[i] = i < nlev ? H[i] : 0;
    p.W[i] = i < nlev ? W[i] : 1;
    p.stride[i] = i < nlev ? strides[i] : 1;
    p.ld[i] = i < nlev ? ld[i] : 0;
    p.start[i] = A;
    if (i < nlev) A += H[i] * W[i];
  }
  p.nlev = nlev; p.B = B; p.A = A; p.nc = nc; p.reg_max = reg_max;
  p.boxes = static_cast<float4*>(boxes);
  p.scores = scores;
  p.cls = cls;
  // AIKO_DECODE_FLAT=1 selects the per-anchor kernel (read per call: the exactness test flips it)
  const char* flat = getenv("AIKO_DECODE_FLAT");
  if (tiled && B <= 65535 && !(flat && flat[0] == '1')) {
    const size_t lds = (size_t)64 * (4 * aiko::kRegMax + nc + 8) * sizeof(aiko::bf16_t);
    aiko::yolo_decode_tiled_kernel<<<dim3(tiles, B), 256, lds, stream>>>(p);
    return (int)hipGetLastError();
  }
  aiko::yolo_decode_kernel<<<grid_for_d((long)B * A, 256), 256, 0, stream>>>(p);
  return (int)hipGetLastError();
}

extern "C" size_t aiko_topk_nms_workspace(int B) {
  return (size_t)B * aiko::kMaxCand * (8 + 16 + 2 * aiko::kMaskWords * 8) + ((size_t)B * 4 + 255) / 256 * 256;
}

extern "C" int aiko_topk_nms(const void* boxes, const float* scores, const int* cls, int B, int A,
                             int max_cand, int max_det, float conf, float iou, float max_wh,
                             float gain, float pad_l, float pad_t, float img_w, float img_h,
                             float* det, int* count, void* workspace, hipStream_t stream) {
  if (A > aiko::kMaxAnchors || max_cand < 1 || max_cand > aiko::kMaxCand || max_det < 1 ||
      max_det > aiko::kMaxCand || workspace == nullptr)
    return -1;
  aiko::NmsParams p;
  p.boxes = static_cast<const float4*>(boxes);
  p.scores = scores;
  p.cls = cls;
  p.A = A; p.max_cand = max_cand; p.max_det = max_det;
  p.conf = conf; p.iou = iou; p.max_wh = max_wh;
  p.gain = gain; p.pad_l = pad_l; p.pad_t = pad_t; p.img_w = img_w; p.img_h = img_h;
  p.det = det;
  p.count = count;
  static const int stop = [] {                  // profiling hook (scripts/nms_stop.sh), read once
    const char* e = getenv("AIKO_NMS_STOP");
    return e ? atoi(e) : 99;
  }();
  p.stop = stop;
  char* w = static_cast<char*>(workspace);
  aiko::NmsWork ws;
  ws.mask = reinterpret_cast<unsigned long long*>(w);
  w += (size_t)B * aiko::kMaxCand * aiko::kMaskWords * 8;
  ws.ckey = reinterpret_cast<unsigned long long*>(w);
  w += (size_t)B * aiko::kMaxCand * 8;
  ws.cbox = reinterpret_cast<float4*>(w);
  w += (size_t)B * aiko::kMaxCand * 16;
  ws.n = reinterpret_cast<int*>(w);
  w += ((size_t)B * 4 + 255) / 256 * 256;
  ws.low = reinterpret_cast<unsigned long long*>(w);
  aiko::nms_select_kernel<<<B, aiko::kNmsThreads, 0, stream>>>(p, ws);
  if (p.stop < 5) return 0;
  aiko::nms_mask_kernel<<<B * aiko::kMaskPairs / aiko::kMaskWaves, 64 * aiko::kMaskWaves, 0, stream>>>(p, ws);
  aiko::nms_greedy_kernel<<<B, aiko::kGreedyThreads, 0, stream>>>(p, ws);
  return (int)hipGetLastError();
}
