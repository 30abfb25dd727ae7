// Detection kernels for gfx950 (YOLOv8 family): nearest upsample into concat slices, the
// anchor-free DFL box decode, and a fused per-image "top-k candidates + class-aware NMS".
//
// top-k + NMS: one launch, up to 4 workgroups per image, the IoU bitmask only where a class run
// needs it (nms_fused_kernel).  History (YOLOv8-n bench batch, B=64 x 8400 anchors, random
// weights, 1024 candidates per image): one workgroup per image over the full bitmask 246 us
// (round 2); three kernels with the full bitmask on the whole GPU, 24 + 31 + 26 = 83 us
// (rounds 3-5; profiles/nms_r2.md); this kernel 88 us at 4 workgroups per image on that input
// (3 classes among the candidates, 625 in the largest), far less where classes are many
// (profiles/nms_r6.md).
#include <cmath>
#include <cstdlib>
#include <cstring>

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
constexpr int kMaxItems = kMaskWords * (kMaskWords + 1) / 2;   // 136 (row block, word) pairs

struct NmsParams {
  const float4* boxes;
  const float* scores;
  const int* cls;
  int A, max_cand, max_det;
  float conf, iou, max_wh;
  float gain, pad_l, pad_t, img_w, img_h;  // letterbox -> frame mapping
  float* det;   // [B, max_det, 6]
  int* count;   // [B]
  double thr_m; // the division-free IoU threshold (mask_word)
  int thr_tie;
  // G > 1: G workgroups per image (each repeats the selection and computes every G-th mask
  // block into gmask / glow; the last to finish, counted in gcount, runs the scan)
  int G;
  unsigned long long* gmask;   // [B][136][64]
  unsigned long long* glow;    // [B][1024]
  int* gcount;                 // [B], zero before the launch; the last arriver re-zeroes it
};

// block-wide exclusive scan of one int per thread (1024 threads = 16 waves); sh[0..31] scratch
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
  const int r = x - v + sh[16 + wave];
  __syncthreads();                                 // sh reusable by the next scan
  return r;
}

// Sort buf[0 .. NP) (NP a power of two <= 1024, unique non-zero keys, zero padding) descending
// with all 1024 threads: a per-wave bitonic sort of 64 keys in registers (21 shuffle passes, no
// barrier), then a merge by rank — a key's final position is its place in its own wave's list
// plus, for each other list, the number of keys greater than it (7-step binary search of the
// LDS copy; the 15 searches are independent).  Padding keys are not written back.
__device__ void block_sort_desc(unsigned long long* buf, int NP) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  unsigned long long v = tid < NP ? buf[tid] : 0ull;
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
  buf[tid] = v;                                    // [wave][64] sorted descending
  __syncthreads();
  int rank = lane;
  const int nl = (NP + 63) >> 6;
#pragma unroll 4
  for (int l = 0; l < nl; ++l) {
    if (l == wave) continue;
    const unsigned long long* L = buf + l * 64;
    int pos = 0;
#pragma unroll
    for (int st = 32; st > 0; st >>= 1)
      if (L[pos + st - 1] > v) pos += st;
    rank += pos + (L[pos] > v ? 1 : 0);
  }
  __syncthreads();
  if (v != 0ull) buf[rank] = v;
  __syncthreads();
}

// v_min / v_max without the NaN canonicalisation fminf / fmaxf carry (two extra v_max per call):
// box coordinates are finite
__device__ __forceinline__ float vmin(float a, float b) {
  float r;
  asm("v_min_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ float vmax(float a, float b) {
  float r;
  asm("v_max_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}

struct IouThrHost {
  double m;
  bool tie_up;
};

__host__ inline IouThrHost iou_threshold(float t) {
  const float s = nextafterf(t, __builtin_inff());
  IouThrHost r;
  r.m = ((double)t + (double)s) * 0.5;
  uint32_t sb;
  memcpy(&sb, &s, 4);
  r.tie_up = (sb & 1u) == 0u;
  return r;
}

// The reference's decision RN(inter / union) > t (fp32 division, fp32 threshold t >= 0) without
// the division: with s = the next float above t and m = (t + s) / 2, RN(q) > t  <=>  q > m, or
// q == m where m rounds to s (ties to even: s's mantissa even).  m has 25 significant bits and
// union 24, so m * union is exact in double and the comparison inter <=> m * union is exact.
// (Host side: iou_threshold() below fills NmsParams.thr_m / thr_tie.)
//
// IoU > thr bits of row box bi against the 64 column boxes in LDS (bit jj = column jj), one
// fully unrolled pass: constant bit positions, broadcast LDS reads (FULL: all 64 columns valid,
// no per-column guard; NEG: negative threshold, every pair tested with the reference's division).
// A 4-compare overlap test on both axes gates the intersection; pairs of different classes
// (max_wh apart) stop there.  Products and sums are the reference's roundings (the product is
// made opaque before the union's subtraction: hipcc contracts a * b - c into an FMA even through
// __fmul_rn / __fsub_rn), column areas come precomputed, so each bit equals the reference's
// box_iou > thr.  The test is symmetric bit for bit (min / max and the area sum commute), so the
// diagonal word's transposed half comes out of the same pass.
template <bool FULL, bool NEG>
__device__ __forceinline__ unsigned long long mask_word(const float4* col, const float* carea, float4 bi,
                                                        float area_i, int je, double thr_m, bool thr_tie,
                                                        float thr) {
  unsigned long long hit = 0ull;
#pragma unroll
  for (int jj = 0; jj < 64; ++jj) {
    if (FULL || jj < je) {                                  // wave-uniform
      const float4 c = col[jj];
      if (NEG) {
        const float iw = fmaxf(0.f, __fsub_rn(fminf(bi.z, c.z), fmaxf(bi.x, c.x)));
        const float ih = fmaxf(0.f, __fsub_rn(fminf(bi.w, c.w), fmaxf(bi.y, c.y)));
        float inter = __fmul_rn(iw, ih);
        asm volatile("" : "+v"(inter));                     // no FMA contraction into the union
        const float iou = __fdiv_rn(inter, __fsub_rn(__fadd_rn(area_i, carea[jj]), inter));
        if (iou > thr) hit |= 1ull << jj;
      } else if (bi.z > c.x && c.z > bi.x && bi.w > c.y && c.w > bi.y) {
        const float iw = __fsub_rn(vmin(bi.z, c.z), vmax(bi.x, c.x));
        const float ih = __fsub_rn(vmin(bi.w, c.w), vmax(bi.y, c.y));
        if (iw > 0.f && ih > 0.f) {                         // else the reference's inter is 0
          float inter = __fmul_rn(iw, ih);
          asm volatile("" : "+v"(inter));                   // no FMA contraction into the union
          const float uni = __fsub_rn(__fadd_rn(area_i, carea[jj]), inter);
          const double d = thr_m * (double)uni;
          const double in = (double)inter;
          if (in > d || (thr_tie && in == d)) hit |= 1ull << jj;
        }
      }
    }
  }
  return hit;
}

__device__ __forceinline__ unsigned long long readlane64(unsigned long long v, int l) {
  const unsigned lo = __builtin_amdgcn_readlane((unsigned)(v & 0xffffffffull), l);
  const unsigned hi = __builtin_amdgcn_readlane((unsigned)(v >> 32), l);
  return ((unsigned long long)hi << 32) | lo;
}

// Top-k + class-aware greedy NMS, ONE launch: G 1024-thread workgroups per image (G = CUs / B,
// at most 4).  Each repeats steps 1-4 (cheaper than a hand-off: no workgroup ever waits for
// another) and computes every G-th mask block into a global workspace; the last to finish
// (agent-scope release / acquire around a per-image counter) loads all blocks into LDS and runs
// steps 6-7.  G = 1 keeps everything in LDS.
//
// Class-aware NMS with class-offset boxes (box + class * max_wh, the reference's one-pass trick)
// never suppresses across classes, so it is an independent greedy NMS per class; the first
// max_det kept boxes in score order are the same either way.  The kernel therefore re-sorts the
// score-sorted candidates by (class, score rank) and computes the IoU bitmask only for the
// 64 x 64 blocks (row block rb, word w >= rb) that hold a same-class pair — the diagonal blocks
// and, where a class spans blocks, the blocks of that run.  With 80 classes and 1024 candidates
// that is ~20-30 of the 136 blocks (the three-kernel predecessor computed all 136 on the whole
// GPU: 31 us of its 83 us); with one class it is all 136, spread over the 16 waves.
//   1. scores above the confidence threshold -> 32-bit keys (float bits are monotone for
//      positive floats) in LDS;
//   2. radix select of the K-th largest key, K = min(max_candidates, #above conf) (12-bit
//      digits over key - min live key: only as many passes as the live range needs; none when
//      every live key is a candidate);
//   3. deterministic compaction (block scan, ties -> lowest anchor index) and a sort of the
//      <= 1024 candidates by (score desc, index asc) — the score ranks;
//   4. a second sort by (class, rank): positions; class-offset boxes in position order;
//   5. the list of same-class (rb, w) blocks; each wave computes its blocks' 64 mask words
//      (lane = row), the diagonal blocks also the transposed half (suppressors of a row inside
//      its own block), with the exact division-free IoU test of mask_word;
//   6. one wave scans the positions 64 at a time: inside a block the suppression chain is a
//      ballot fixed point over the transposed diagonal words, then the kept rows' words are
//      OR-ed into the later blocks of the same class, lane-parallel (no max_det stop: kept
//      flags go to the score ranks);
//   7. a block scan over the ranks takes the first max_det kept boxes, maps them back from
//      letterbox to frame coordinates (clipped) and writes fixed-size [max_det, 6] rows
//      (x1, y1, x2, y2, score, class) + a count, so results can be all-gathered over RCCL
//      without a size exchange.
// A negative IoU threshold (every pair suppresses, across classes too) keeps one class run:
// the second sort then orders by rank alone.
constexpr int kRadixBits = 12, kRadixBins = 1 << kRadixBits;   // 4096 bins = 4 per thread
__global__ __launch_bounds__(kNmsThreads) void nms_fused_kernel(NmsParams p) {
  constexpr int REGION0 = kMaxAnchors * 4;
  __shared__ __attribute__((aligned(16))) unsigned char region0[REGION0];
  __shared__ unsigned long long ckey[kMaxCand];
  __shared__ __attribute__((aligned(16))) unsigned hist[kRadixBins];
  __shared__ int sh[48];

  unsigned* keys = reinterpret_cast<unsigned*>(region0);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int b = blockIdx.x / p.G, g = blockIdx.x - b * p.G;
  const int A = p.A;
  const float* sc = p.scores + (long)b * A;
  const float4* bx = p.boxes + (long)b * A;
  const int* cl = p.cls + (long)b * A;
  float* det = p.det + (long)b * p.max_det * 6;
  const float inv = 1.f / p.gain;

  // ---- 1. keys
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
  if (K == 0) {
    if (g != 0) return;
    for (int r = tid; r < p.max_det; r += kNmsThreads) {
      float* o = det + (long)r * 6;
      o[0] = o[1] = o[2] = o[3] = o[4] = 0.f;
      o[5] = -1.f;
    }
    if (tid == 0) p.count[b] = 0;
    return;
  }

  // ---- 2. radix select of the K-th largest key; T = threshold key, remaining = candidates
  // equal to T
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

  // ---- 3. deterministic compaction and the score sort (ranks)
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
  block_sort_desc(ckey, NP);                       // ckey[rank], rank 0 = best score

  // ---- 4. (class, rank) order.  region0 (the keys) is free from here:
  //   cbox   float4[1024]           class-offset boxes by position     16 KB
  //   masks  u64[136][64]           mask words of the listed blocks    68 KB
  //   lowd   u64[1024]              transposed diagonal word by row     8 KB
  //   sbuf   u64[1024]              the second sort's keys              8 KB
  //   krank  int[1024]              kept flag by score rank             4 KB
  //   carea  float[1024]            box areas by position               4 KB
  // and hist: pos_rank int[1024] (rank of position), pcls int[1024] (class of position),
  // item int[136] ((rb << 8) | w), item_id int[16][16] (-1: block pair without a class run)
  float4* cbox = reinterpret_cast<float4*>(region0);
  unsigned long long* masks = reinterpret_cast<unsigned long long*>(region0 + 16384);
  unsigned long long* lowd = masks + kMaxItems * 64;
  unsigned long long* sbuf = lowd + kMaxCand;
  int* krank = reinterpret_cast<int*>(sbuf + kMaxCand);
  float* carea = reinterpret_cast<float*>(krank + kMaxCand);
  int* pos_rank = reinterpret_cast<int*>(hist);
  int* pcls = pos_rank + kMaxCand;
  int* item = pcls + kMaxCand;
  int* item_id = item + 256;
  const bool neg = p.iou < 0.f;
  if (tid < NP) {
    unsigned long long k2 = 0ull;
    if (tid < K) {
      const int idx = (int)(0xffffffffu - (unsigned)(ckey[tid] & 0xffffffffull));
      const unsigned c = neg ? 0u : (unsigned)cl[idx];
      k2 = ~(((unsigned long long)c << 32) | (unsigned)tid);   // descending sort = (class, rank) ascending
    }
    sbuf[tid] = k2;
  }
  if (tid < 256) item_id[tid] = -1;
  __syncthreads();
  block_sort_desc(sbuf, NP);
  if (tid < K) {
    const int r = (int)(~sbuf[tid] & 0xffffffffull);
    const unsigned long long ck = ckey[r];
    const int idx = (int)(0xffffffffu - (unsigned)(ck & 0xffffffffull));
    const int c = cl[idx];
    float off = __fmul_rn((float)c, p.max_wh);
    asm volatile("" : "+v"(off));                     // the reference rounds the offset, then adds
    const float4 q = bx[idx];
    const float4 o4 = make_float4(__fadd_rn(q.x, off), __fadd_rn(q.y, off), __fadd_rn(q.z, off), __fadd_rn(q.w, off));
    cbox[tid] = o4;
    carea[tid] = __fmul_rn(__fsub_rn(o4.z, o4.x), __fsub_rn(o4.w, o4.y));   // (no add to contract)
    pos_rank[tid] = r;
    pcls[tid] = neg ? 0 : c;
    krank[tid] = 0;
  }
  __syncthreads();

  // ---- 5. same-class block pairs, then their mask words
  const int W = (K + 63) >> 6;
  const int npairs = W * (W + 1) / 2;
  int rb = 0, wq = 0;
  bool need = false;
  if (tid < npairs) {
    int q = tid;
    while (q >= W - rb) {
      q -= W - rb;
      ++rb;
    }
    wq = rb + q;
    need = wq == rb || pcls[wq * 64] == pcls[rb * 64 + 63];
  }
  const int slot = block_exclusive_scan(need ? 1 : 0, sh);
  if (need) {
    item[slot] = (rb << 8) | wq;
    item_id[rb * 16 + wq] = slot;
  }
  if (tid == npairs - 1) sh[40] = slot + (need ? 1 : 0);
  __syncthreads();
  const int nitems = sh[40];
  const bool split = p.G > 1;
  unsigned long long* gm = split ? p.gmask + (long)b * kMaxItems * 64 : nullptr;
  unsigned long long* gl = split ? p.glow + (long)b * kMaxCand : nullptr;
  for (int j = g + p.G * wave; j < nitems; j += p.G * (kNmsThreads / 64)) {
    const int rbj = item[j] >> 8, wj = item[j] & 0xff;
    const int i = rbj * 64 + lane;
    const int je = min(64, K - wj * 64);
    unsigned long long bits = 0ull;
    if (i < K) {
      const float4 bi = cbox[i];
      const float area_i = carea[i];
      const float4* col = cbox + wj * 64;
      const float* ca = carea + wj * 64;
      const unsigned long long hit =
          neg ? mask_word<false, true>(col, ca, bi, area_i, je, p.thr_m, p.thr_tie, p.iou)
              : (je == 64 ? mask_word<true, false>(col, ca, bi, area_i, je, p.thr_m, p.thr_tie, p.iou)
                          : mask_word<false, false>(col, ca, bi, area_i, je, p.thr_m, p.thr_tie, p.iou));
      bits = hit;
      if (wj == rbj) {
        bits = lane == 63 ? 0ull : hit & (~0ull << (lane + 1));
        const unsigned long long lw = hit & ((1ull << lane) - 1ull);
        if (split) gl[i] = lw;
        else lowd[i] = lw;
      }
    }
    if (split) gm[j * 64 + lane] = bits;
    else masks[j * 64 + lane] = bits;
  }
  if (split) {
    // publish this workgroup's blocks; the last of the image's G workgroups takes them all
    // (release: stores drained, fence, then the counter; acquire: fence, then plain loads)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      sh[42] = __hip_atomic_fetch_add(p.gcount + b, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    if (sh[42] != p.G - 1) return;
    if (tid == 0) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      __hip_atomic_store(p.gcount + b, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int t = tid; t < nitems * 64; t += kNmsThreads) masks[t] = gm[t];
    if (tid < K) lowd[tid] = gl[tid];
  }
  __syncthreads();

  // ---- 6. greedy scan over the positions (one wave; lane w holds the "removed" word w)
  if (tid < 64) {
    unsigned long long removed = 0ull;
    for (int w = 0; w < W; ++w) {
      const unsigned long long cur = readlane64(removed, w);
      const int row = w * 64 + lane;
      // suppressors of this lane's candidate inside the block (rows k < row, transposed diagonal)
      const unsigned long long low = row < K ? lowd[row] : 0ull;
      const int left = K - w * 64;
      const unsigned long long valid = left >= 64 ? ~0ull : ((1ull << left) - 1ull);
      const unsigned long long alive = ~cur & valid;
      const bool me_alive = (alive >> lane) & 1ull;
      // greedy inside the block as a fixed point: kept = alive minus those with a kept
      // suppressor.  Candidate c's status is final once all k < c are, so <= 64 rounds; the
      // first repeat is the (unique) greedy solution.  One ballot per round.
      unsigned long long keep = alive;
      for (int it = 0; it <= 64; ++it) {
        const unsigned long long nk = __ballot(me_alive && !(low & keep));
        if (nk == keep) break;
        keep = nk;
      }
      if ((keep >> lane) & 1ull) krank[pos_rank[row]] = 1;
      // OR the kept rows' words into the later blocks of the same class run: 8 LDS reads in
      // flight per round
      const int jl = lane > w && lane < W ? item_id[w * 16 + lane] : -1;
      if (__ballot(jl >= 0)) {
        unsigned long long kk = keep, acc = 0ull;
        const unsigned long long* wl = masks + (jl >= 0 ? jl : 0) * 64;
        while (kk) {
          int bsel[8];
#pragma unroll
          for (int u = 0; u < 8; ++u) {
            bsel[u] = kk ? __ffsll((long long)kk) - 1 : -1;
            kk &= kk - 1ull;
          }
          unsigned long long v[8];
#pragma unroll
          for (int u = 0; u < 8; ++u) v[u] = (jl >= 0 && bsel[u] >= 0) ? wl[bsel[u]] : 0ull;
#pragma unroll
          for (int u = 0; u < 8; ++u) acc |= v[u];
        }
        removed |= acc;
      }
    }
  }
  __syncthreads();

  // ---- 7. the first max_det kept boxes in score order -> frame coordinates
  const int kf = tid < K ? krank[tid] : 0;
  const int out = block_exclusive_scan(kf, sh);
  if (tid == kNmsThreads - 1) sh[41] = out + kf;
  __syncthreads();
  const int nk = min(sh[41], p.max_det);
  if (kf && out < p.max_det) {
    const unsigned long long ck = ckey[tid];
    const int idx = (int)(0xffffffffu - (unsigned)(ck & 0xffffffffull));
    const float4 q = bx[idx];
    float* o = det + (long)out * 6;
    o[0] = fminf(fmaxf((q.x - p.pad_l) * inv, 0.f), p.img_w);
    o[1] = fminf(fmaxf((q.y - p.pad_t) * inv, 0.f), p.img_h);
    o[2] = fminf(fmaxf((q.z - p.pad_l) * inv, 0.f), p.img_w);
    o[3] = fminf(fmaxf((q.w - p.pad_t) * inv, 0.f), p.img_h);
    o[4] = __uint_as_float((unsigned)(ck >> 32));
    o[5] = (float)cl[idx];
  }
  for (int r = nk + tid; r < p.max_det; r += kNmsThreads) {
    float* o = det + (long)r * 6;
    o[0] = o[1] = o[2] = o[3] = o[4] = 0.f;
    o[5] = -1.f;
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

// workgroups per image: enough to spread the images' mask blocks over the CUs (up to 4)
extern "C" int aiko_topk_nms_groups(int B) {
  static int cus = [] {
    int dev = 0, n = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
    return n;
  }();
  const int g = cus / (B > 0 ? B : 1);
  return g < 1 ? 1 : (g > 4 ? 4 : g);
}

// bytes of the G > 1 workspace (mask blocks, diagonal words, counters), 0 for G == 1; the
// counters (the last 4 B bytes) must be zero before the launch
extern "C" size_t aiko_topk_nms_workspace(int B) {
  if (aiko_topk_nms_groups(B) <= 1) return 0;
  return (size_t)B * (aiko::kMaxItems * 64 * 8 + aiko::kMaxCand * 8 + 4);
}

extern "C" int aiko_topk_nms(const void* boxes, const float* scores, const int* cls, int B, int A,
                             int max_cand, int max_det, float conf, float iou, float max_wh,
                             float gain, float pad_l, float pad_t, float img_w, float img_h,
                             float* det, int* count, void* workspace, hipStream_t stream) {
  if (A > aiko::kMaxAnchors || max_cand < 1 || max_cand > aiko::kMaxCand || max_det < 1 ||
      max_det > aiko::kMaxCand)
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
  const aiko::IouThrHost th = aiko::iou_threshold(iou);
  p.thr_m = th.m;
  p.thr_tie = th.tie_up;
  p.G = aiko_topk_nms_groups(B);
  p.gmask = static_cast<unsigned long long*>(workspace);
  p.glow = p.gmask ? p.gmask + (size_t)B * aiko::kMaxItems * 64 : nullptr;
  p.gcount = p.gmask ? reinterpret_cast<int*>(p.glow + (size_t)B * aiko::kMaxCand) : nullptr;
  if (p.G > 1 && workspace == nullptr) return -1;
  aiko::nms_fused_kernel<<<B * p.G, aiko::kNmsThreads, 0, stream>>>(p);
  return (int)hipGetLastError();
}
