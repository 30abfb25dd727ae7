// Fused ResNet stem: 7x7/s2 conv (+ folded BN bias) + ReLU + 3x3/s2/p1 max-pool in one kernel.
//
// Unfused, the stem writes a [B, 112, 112, 64] bf16 tensor (411 MB at B=256) that the max-pool
// reads straight back: ~0.8 GB of HBM traffic for a 103 MB result, and the stem's N=64 GEMM
// with K padded 147 -> 256 ran at ~376 TFLOP/s (280 us + 127 us for the pool on MI355X).  Here
// each workgroup owns an 8 x 14 tile of POOLED pixels of one image, i.e. a 17 x 29 region of
// stem pixels (10 % halo recompute), and never writes the stem activation to HBM:
//
//  1. the input patch the region needs — 39 rows x 64 pixels x 4 channels of the zero-bordered
//     preprocess buffer, 20 KB — is DMA'd into LDS (buffer_load ... lds, out-of-image chunks
//     read as zero); the folded weights [7][64][32] (28 KB) too, from a host-prepared image
//     whose 16-byte chunks are XOR-swizzled by (channel >> 2) & 2, which makes the A-fragment
//     ds_read_b128 conflict-free for its lane groups {0-3,12-15,20-27}, {4-11,16-19,28-31}, ...;
//  2. MFMA v_mfma_f32_16x16x32_bf16 with channels as the A rows and stem pixels as the B
//     columns: one K=32 step is exactly one filter row (8 pixels x 4 channels; pixel 7 and
//     channel 3 carry zero weights), so a B fragment is 16 contiguous bytes of one patch row —
//     an implicit GEMM with no im2col at all (stride 2 = 16-byte steps between pixels).
//     Each of the 4 waves computes 128 stem pixels x 64 channels (8 x 4 accumulator tiles);
//  3. epilogue: bias + ReLU, stem pixels outside the image forced to 0 (ReLU output >= 0, so 0
//     is a valid -inf for the pool), 4 channels packed per 8-byte LDS write into the stem tile
//     [px][64 ch + 8 B pad] (aliasing the patch/weights; the 136-B pitch spreads 16 pixels'
//     8-byte writes over all 32 write banks);
//  4. 3x3/s2 max over the LDS tile, 8 channels (16 B) per thread as packed u16 max on the
//     non-negative bf16 bit patterns, coalesced 16-byte stores.
//
// Rounding is identical to the unfused path: the stem value is rounded to bf16 before the max.
#include "common.h"

namespace aiko {

namespace {

constexpr int kTPH = 8;                                 // pooled tile rows
constexpr int kSRH = 2 * kTPH + 1;                      // stem region rows (17)
constexpr int kPatchH = 2 * (kSRH - 1) + 7;             // 39 input rows
constexpr int kWB = 7 * 64 * 64;                        // 28672 B of weights
constexpr int kSPitch = 136;                            // stem-tile pixel pitch: 64 ch + 8 B pad

// pooled tile width TPW: 14 -> 17 x 29 stem region, 4 waves x 128 pixels, 64 KB LDS (2 WG/CU);
//                         7 -> 17 x 15 stem region, 4 waves x 64 pixels, 39 KB LDS (4 WG/CU)
template <int TPW>
struct StemTile {
  static constexpr int SRW = 2 * TPW + 1;
  static constexpr int NPIX = kSRH * SRW;
  static constexpr int NB = TPW == 14 ? 8 : 4;          // 16-pixel blocks per wave
  static constexpr int PATCH_W = 2 * (SRW - 1) + 8;     // input pixels per patch row
  static constexpr int ROW_B = PATCH_W * 8;
  static constexpr int PATCH_CH = kPatchH * (PATCH_W / 2);              // 16-byte chunks
  static constexpr int PATCH_B = (PATCH_CH + 255) / 256 * 256 * 16;    // whole DMA rounds
  static constexpr int S_B = 4 * NB * 16 * kSPitch;     // stem tile, 136 B per pixel
  static constexpr int LDS_B = (PATCH_B + kWB) > S_B ? (PATCH_B + kWB) : S_B;
  static constexpr int WGS = TPW == 14 ? 2 : 4;
  static_assert(NPIX <= 4 * NB * 16, "4 waves cover the stem region");
};

typedef __attribute__((ext_vector_type(2))) unsigned short u16x2;

struct StemPoolParams {
  const bf16_t* x;      // [B, Hp, Wp, 4]
  const bf16_t* w;      // [7][64][4 x 16 B] pre-swizzled LDS image of the stem weights
  const float* bias;    // [64]
  bf16_t* y;            // [B, Hm, Wm, ldy]
  int B, Hp, Wp, Ho, Wo, Hm, Wm, ldy, tiles_h, tiles_w;
  // U8 variant: raw frames [B, Hi, Wi, 3] (the stem's image, no resize); the patch holds
  // c - 255 mean_c (bf16) and the weight image is pre-scaled by 1 / (255 std_c)
  const uint8_t* xu8;
  int Hi, Wi;
  float m0, m1, m2;
};

template <int TPW, bool U8 = false>
__global__ __launch_bounds__(256, StemTile<TPW>::WGS) void stem_pool_kernel(StemPoolParams p) {
  using T = StemTile<TPW>;
  constexpr int kTPW = TPW, kSRW = T::SRW, kNPix = T::NPIX, NB = T::NB;
  constexpr int kPatchW = T::PATCH_W, kPatchRowB = T::ROW_B;
  __shared__ __attribute__((aligned(16))) unsigned char smem[T::LDS_B];
  unsigned char* patch = smem;
  unsigned char* wl = smem + T::PATCH_B;
  unsigned char* st = smem;                             // stem tile, after the MFMAs

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int per_img = p.tiles_h * p.tiles_w;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int img = bid / per_img;
  const int t = bid - img * per_img;
  const int ty = t / p.tiles_w, tx = t - ty * p.tiles_w;
  const int py0 = ty * kTPH, px0 = tx * kTPW;
  const int sy0 = 2 * py0 - 1, sx0 = 2 * px0 - 1;      // stem region origin
  const int gy0 = 2 * sy0, gx0 = 2 * sx0;               // patch origin in the padded buffer

  // ---- 1. patch + weights -> LDS ----
  if constexpr (U8) {
    // U8: the patch straight from the uint8 frame — no bf16 stem buffer in HBM, no separate
    // pre-processing kernel.  Patch pixel (r, j) is image pixel (gy0 - 3 + r, gx0 - 3 + j)
    // (the padded buffer's border is 3); 4-pixel groups aligned in the image (three dword
    // loads), each pixel written as one 8-byte [c0 - m0, c1 - m1, c2 - m2, 0] entry; outside
    // the image: 0 (= the normalised conv padding).  The weights still come by DMA.
    const int xa = ((gx0 - 3) >> 2) << 2;                // floor to a 4-pixel boundary
    constexpr int G = kPatchW / 4 + 1;                   // groups per patch row
    const uint8_t* im = p.xu8 + (size_t)img * p.Hi * p.Wi * 3;
    for (int task = tid; task < kPatchH * G; task += 256) {
      const int r = task / G, gi = task - r * G;
      const int y = gy0 - 3 + r, x = xa + 4 * gi;
      float c[12];
#pragma unroll
      for (int e = 0; e < 12; ++e) c[e] = 0.f;
      const bool in = (unsigned)y < (unsigned)p.Hi && x >= 0 && x + 3 < p.Wi;
      if (in) {
        const uint32_t* src = reinterpret_cast<const uint32_t*>(im + ((size_t)y * p.Wi + x) * 3);
        const uint32_t wd[3] = {src[0], src[1], src[2]};
#pragma unroll
        for (int e = 0; e < 12; ++e) c[e] = (float)((wd[e >> 2] >> (8 * (e & 3))) & 0xFFu);
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int j = x + q - (gx0 - 3);
        if ((unsigned)j >= (unsigned)kPatchW) continue;
        uint2 o = {0u, 0u};
        if (in) o = make_uint2(pack2(c[3 * q] - p.m0, c[3 * q + 1] - p.m1), pack2(c[3 * q + 2] - p.m2, 0.f));
        *reinterpret_cast<uint2*>(patch + r * kPatchRowB + j * 8) = o;
      }
    }
    const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<bf16_t*>(p.w), (short)0, kWB, 0x00020000);
#pragma unroll
    for (int k = 0; k < kWB / 16 / 256; ++k)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rw, reinterpret_cast<__attribute__((address_space(3))) void*>(
                  reinterpret_cast<uintptr_t>(wl + (k * 4 + wave) * 1024)), 16,
          (uint32_t)(((k * 4 + wave) * 64 + lane) * 16), 0, 0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  } else
  // buffer DMA (no VGPR staging, no ds_write)
  // patch chunk i (row i / (W/2), 2 pixels) lands at LDS byte 16 i: one wave instruction
  // fills 64 consecutive chunks.  Chunks outside the image get an offset past num_records,
  // which the hardware reads as zero (conv padding / region beyond the image); the rounds
  // past the last chunk write zeros into the patch's own rounding slack.
  {
    const uint32_t img_bytes = (uint32_t)p.Hp * p.Wp * 8;
    const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<bf16_t*>(p.x + (size_t)img * p.Hp * p.Wp * 4), (short)0, (int)img_bytes, 0x00020000);
    constexpr int CPR = kPatchW / 2;                     // chunks per patch row
#pragma unroll
    for (int k = 0; k < T::PATCH_B / 16 / 256; ++k) {
      const int i = (k * 4 + wave) * 64 + lane;
      const int r = i / CPR, c = i - r * CPR;
      const int gy = gy0 + r, gx = gx0 + 2 * c;
      const bool ok = i < T::PATCH_CH && (unsigned)gy < (unsigned)p.Hp && gx >= 0 && gx + 1 < p.Wp;
      const uint32_t off = ok ? (uint32_t)(gy * p.Wp + gx) * 8 : 0x80000000u;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rx, reinterpret_cast<__attribute__((address_space(3))) void*>(
                  reinterpret_cast<uintptr_t>(patch + (k * 4 + wave) * 1024)), 16, off, 0, 0, 0);
    }
    const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<bf16_t*>(p.w), (short)0, kWB, 0x00020000);
#pragma unroll
    for (int k = 0; k < kWB / 16 / 256; ++k)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rw, reinterpret_cast<__attribute__((address_space(3))) void*>(
                  reinterpret_cast<uintptr_t>(wl + (k * 4 + wave) * 1024)), 16,
          (uint32_t)(((k * 4 + wave) * 64 + lane) * 16), 0, 0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();

  // ---- 2. MFMA: channels (A rows) x stem pixels (B columns), one filter row per K step ----
  const int fr = lane & 15, fq = lane >> 4;
  int b_off[NB];
#pragma unroll
  for (int nb = 0; nb < NB; ++nb) {
    int n = wave * NB * 16 + nb * 16 + fr;
    if (n >= kNPix) n = 0;                               // dummy column, result discarded
    const int ly = n / kSRW, lx = n - ly * kSRW;
    b_off[nb] = 2 * ly * kPatchRowB + (2 * lx) * 8 + fq * 16;
  }
  int a_off[4];
#pragma unroll
  for (int mb = 0; mb < 4; ++mb) {
    const int o = mb * 16 + fr;
    a_off[mb] = (o * 4 + (fq ^ ((o >> 2) & 2))) * 16;
  }
  f32x4 acc[4][NB];
#pragma unroll
  for (int mb = 0; mb < 4; ++mb)
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) acc[mb][nb] = f32x4{0.f, 0.f, 0.f, 0.f};

#pragma unroll
  for (int r = 0; r < 7; ++r) {
    bf16x8 af[4];
#pragma unroll
    for (int mb = 0; mb < 4; ++mb)
      af[mb] = *reinterpret_cast<const bf16x8*>(wl + r * 64 * 64 + a_off[mb]);
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) {
      const bf16x8 bfr = *reinterpret_cast<const bf16x8*>(patch + r * kPatchRowB + b_off[nb]);
#pragma unroll
      for (int mb = 0; mb < 4; ++mb)
        acc[mb][nb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[mb], bfr, acc[mb][nb], 0, 0, 0);
    }
  }
  float bias[4][4];
#pragma unroll
  for (int mb = 0; mb < 4; ++mb) {
    const f32x4 b = *reinterpret_cast<const f32x4*>(p.bias + mb * 16 + fq * 4);
    bias[mb][0] = b[0]; bias[mb][1] = b[1]; bias[mb][2] = b[2]; bias[mb][3] = b[3];
  }
  __syncthreads();                                       // patch/weights dead: reuse as stem tile

  // ---- 3. bias + ReLU -> bf16 stem tile in LDS ----
  // Tiles whose whole stem region lies inside the image (most of them) skip the per-pixel
  // validity test (a workgroup-uniform branch).
  const bool interior = sy0 >= 0 && sx0 >= 0 && sy0 + kSRH <= p.Ho && sx0 + kSRW <= p.Wo;
#pragma unroll
  for (int nb = 0; nb < NB; ++nb) {
    const int n = wave * NB * 16 + nb * 16 + fr;
    if (n >= kNPix) continue;
    bool valid = true;
    if (!interior) {
      const int ly = n / kSRW, lx = n - ly * kSRW;
      valid = (unsigned)(sy0 + ly) < (unsigned)p.Ho && (unsigned)(sx0 + lx) < (unsigned)p.Wo;
    }
#pragma unroll
    for (int mb = 0; mb < 4; ++mb) {
      // acc + bias in packed fp32; max(., 0) gives +0 for non-positive sums (acc starts at +0,
      // so the sum is never -0) — the pool below compares bit patterns
      const f32x2 a01 = f32x2{acc[mb][nb][0], acc[mb][nb][1]} + f32x2{bias[mb][0], bias[mb][1]};
      const f32x2 a23 = f32x2{acc[mb][nb][2], acc[mb][nb][3]} + f32x2{bias[mb][2], bias[mb][3]};
      uint2 o2;
      o2.x = valid ? pack2(fmaxf(a01[0], 0.f), fmaxf(a01[1], 0.f)) : 0u;
      o2.y = valid ? pack2(fmaxf(a23[0], 0.f), fmaxf(a23[1], 0.f)) : 0u;
      *reinterpret_cast<uint2*>(st + n * kSPitch + (mb * 4 + fq) * 8) = o2;
    }
  }
  __syncthreads();

  // ---- 4. 3x3/s2 max-pool from LDS, 8 channels per item ----
  // Every value is a ReLU output (+0 or positive; the epilogue never produces -0), so the max
  // of the bf16 bit patterns as unsigned 16-bit integers is the float max: v_pk_max_u16 on
  // packed pairs, no unpacking.  The 9 reads are immediate offsets from one base address.
  for (int it = tid; it < kTPH * kTPW * 8; it += 256) {
    const int pp = it >> 3, g = it & 7;
    const int py = pp / kTPW, px = pp - py * kTPW;
    const int gy = py0 + py, gx = px0 + px;
    if (gy >= p.Hm || gx >= p.Wm) continue;
    const unsigned char* base = st + ((2 * py) * kSRW + 2 * px) * kSPitch + g * 16;
    u16x2 m[4] = {u16x2{0, 0}, u16x2{0, 0}, u16x2{0, 0}, u16x2{0, 0}};
#pragma unroll
    for (int dy = 0; dy < 3; ++dy)
#pragma unroll
      for (int dx = 0; dx < 3; ++dx) {
        const unsigned char* q = base + (dy * kSRW + dx) * kSPitch;
        const uint2 lo = *reinterpret_cast<const uint2*>(q);
        const uint2 hi = *reinterpret_cast<const uint2*>(q + 8);
        m[0] = __builtin_elementwise_max(m[0], __builtin_bit_cast(u16x2, lo.x));
        m[1] = __builtin_elementwise_max(m[1], __builtin_bit_cast(u16x2, lo.y));
        m[2] = __builtin_elementwise_max(m[2], __builtin_bit_cast(u16x2, hi.x));
        m[3] = __builtin_elementwise_max(m[3], __builtin_bit_cast(u16x2, hi.y));
      }
    u32x4 o;
#pragma unroll
    for (int e = 0; e < 4; ++e) o[e] = __builtin_bit_cast(uint32_t, m[e]);
    *reinterpret_cast<u32x4*>(p.y + ((size_t)(img * p.Hm + gy) * p.Wm + gx) * p.ldy + g * 8) = o;
  }
}


// ---- strip variant (uint8 frames): one workgroup walks a 7-wide column of pooled tiles ----
//
// The tile kernel above re-loads the 28 KB weight image into LDS for every 8 x 7 pooled tile,
// re-reads the A fragments from LDS for every wave, recomputes a one-row stem halo per tile and
// pools from a full 17 x 15 stem tile (9 LDS reads per output).  By LDS traffic it is bound
// well before its MFMAs (~370 KB of LDS reads/writes per 448 MFMAs).  Here:
//  * a workgroup owns one strip — all Hm/8 pooled tiles of 7 columns of one image — and keeps
//    the A fragments (7 filter rows x 4 channel blocks, 112 VGPRs) in registers for the whole
//    strip: weights are read once per strip, from L2, never through LDS;
//  * each tile computes exactly the 16 new stem rows 2 py0 .. 2 py0 + 15 (one 16-column stem row
//    per MFMA column block, wave w rows 4w .. 4w + 3); the pool's upper halo row is the previous
//    tile's last stem row, still in the other half of the double-buffered pool tile (zeros above
//    the image: ReLU outputs are >= 0, so 0 is a valid -inf for the max);
//  * the horizontal 3-wide / stride-2 max runs in registers: stem column fr sits in lane fr of a
//    16-lane DPP row, so max(v[fr-1], v[fr], v[fr+1]) is two row_shr / row_shl moves; only the
//    7 odd lanes store, into a 16-row x 7-pixel tile (pixel pitch 144 B: the 7 pixels' 8-byte
//    writes land in disjoint bank octets), and the vertical max reads 3 rows per output;
//  * the next tile's uint8 patch is loaded into registers before this tile's MFMAs and written
//    to the other patch buffer after the epilogue: one global-load latency per tile is hidden.
// Bit-identical to the tile kernel (same patch values, same MFMA order per accumulator).
constexpr int kSpRows = 16;                              // stem rows per tile
constexpr int kSpCols = 16;                              // stem columns per strip (15 used)
constexpr int kSpPW = 2 * (kSpCols - 1) + 8;             // 38 patch pixels per row
constexpr int kSpPH = 2 * (kSpRows - 1) + 7;             // 37 patch rows
constexpr int kSpRowB = kSpPW * 8;                       // 304 B
constexpr int kSpPatchB = kSpPH * kSpRowB;               // 11248 B
constexpr int kSpHpPitch = 144;                          // pool-tile pixel pitch
constexpr int kSpHpRowB = 7 * kSpHpPitch;                // 1008 B
constexpr int kSpHpB = kSpRows * kSpHpRowB;              // 16128 B
constexpr int kSpGroups = kSpPW / 4 + 2;                 // 4-pixel groups per patch row (11)
constexpr int kSpTasks = kSpPH * kSpGroups;              // 407
constexpr int kSpTaskIt = (kSpTasks + 255) / 256;        // 2

__device__ __forceinline__ uint32_t sp_dpp_shr1(uint32_t v) {       // lane i <- lane i - 1 (16-lane rows)
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xF, 0xF, true);
}
__device__ __forceinline__ uint32_t sp_dpp_shl1(uint32_t v) {       // lane i <- lane i + 1
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x101, 0xF, 0xF, true);
}

// (a helper, not __builtin_elementwise_max on u32x4 subscripts inside a loop: hipcc folded that
// form to element 0 broadcast into all four dwords)
__device__ __forceinline__ uint32_t sp_max3_u16x2(uint32_t a, uint32_t b, uint32_t c) {
  const u16x2 m = __builtin_elementwise_max(__builtin_elementwise_max(__builtin_bit_cast(u16x2, a),
                                                                      __builtin_bit_cast(u16x2, b)),
                                            __builtin_bit_cast(u16x2, c));
  return __builtin_bit_cast(uint32_t, m);
}

__global__ __launch_bounds__(256, 2) void stem_pool_strip_kernel(StemPoolParams p) {
  __shared__ __attribute__((aligned(16))) unsigned char smem[2 * kSpPatchB + 2 * kSpHpB];
  __shared__ __attribute__((aligned(16))) float bias_l[64];
  unsigned char* patch0 = smem;
  unsigned char* hp0 = smem + 2 * kSpPatchB;
  if (threadIdx.x < 16)
    *reinterpret_cast<f32x4*>(bias_l + 4 * threadIdx.x) = *reinterpret_cast<const f32x4*>(p.bias + 4 * threadIdx.x);

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int strips = p.tiles_w;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int img = bid / strips;
  const int sj = bid - img * strips;
  const int px0 = sj * 7;                                // first pooled column
  const int sx0 = 2 * px0 - 1;                           // first stem column
  const int ix0 = 2 * sx0 - 3;                           // patch column 0 in the image
  const int xa = ix0 >= 0 ? (ix0 & ~3) : -((3 - ix0) & ~3);   // floor to a 4-pixel boundary
  const uint8_t* im = p.xu8 + (size_t)img * p.Hi * p.Wi * 3;
  const int fr = lane & 15, fq = lane >> 4;

  // ---- A fragments: the whole weight image in registers for the strip ----
  bf16x8 af[7][4];
#pragma unroll
  for (int r = 0; r < 7; ++r)
#pragma unroll
    for (int mb = 0; mb < 4; ++mb) {
      const int o = mb * 16 + fr;
      af[r][mb] = *reinterpret_cast<const bf16x8*>(
          reinterpret_cast<const unsigned char*>(p.w) + r * 64 * 64 + (o * 4 + (fq ^ ((o >> 2) & 2))) * 16);
    }

  // ---- uint8 patch fill: load (registers) then store (LDS, normalised bf16) ----
  uint32_t pre[kSpTaskIt][3];
  auto load_patch = [&](int py0) {
    const int iy0 = 4 * py0 - 3;                          // image row of patch row 0
#pragma unroll
    for (int k = 0; k < kSpTaskIt; ++k) {
      const int task = tid + k * 256;
      const int r = task / kSpGroups, gi = task - r * kSpGroups;
      const int y = iy0 + r, x = xa + 4 * gi;
      pre[k][0] = pre[k][1] = pre[k][2] = 0u;
      if (task < kSpTasks && (unsigned)y < (unsigned)p.Hi && x >= 0 && x + 3 < p.Wi) {
        const uint32_t* src = reinterpret_cast<const uint32_t*>(im + ((size_t)y * p.Wi + x) * 3);
        pre[k][0] = __builtin_nontemporal_load(src);
        pre[k][1] = __builtin_nontemporal_load(src + 1);
        pre[k][2] = __builtin_nontemporal_load(src + 2);
      }
    }
  };
  auto store_patch = [&](unsigned char* patch, int py0) {
    const int iy0 = 4 * py0 - 3;
#pragma unroll
    for (int k = 0; k < kSpTaskIt; ++k) {
      const int task = tid + k * 256;
      if (task >= kSpTasks) continue;
      const int r = task / kSpGroups, gi = task - r * kSpGroups;
      const int y = iy0 + r, x = xa + 4 * gi;
      const bool in = (unsigned)y < (unsigned)p.Hi && x >= 0 && x + 3 < p.Wi;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int j = x + q - ix0;
        if ((unsigned)j >= (unsigned)kSpPW) continue;
        uint2 o = {0u, 0u};
        if (in) {
          const int e = 3 * q;
          const float c0 = (float)((pre[k][e >> 2] >> (8 * (e & 3))) & 0xFFu);
          const float c1 = (float)((pre[k][(e + 1) >> 2] >> (8 * ((e + 1) & 3))) & 0xFFu);
          const float c2 = (float)((pre[k][(e + 2) >> 2] >> (8 * ((e + 2) & 3))) & 0xFFu);
          o = make_uint2(pack2(c0 - p.m0, c1 - p.m1), pack2(c2 - p.m2, 0.f));
        }
        *reinterpret_cast<uint2*>(patch + r * kSpRowB + j * 8) = o;
      }
    }
  };

  int b_off[4];
#pragma unroll
  for (int nb = 0; nb < 4; ++nb) b_off[nb] = 2 * (wave * 4 + nb) * kSpRowB + 16 * fr + 16 * fq;
  const bool col_ok = (unsigned)(sx0 + fr) < (unsigned)p.Wo;
  const bool store_lane = (fr & 1) && fr < 15;
  const int hp_lane = ((fr - 1) >> 1) * kSpHpPitch + fq * 8;

  load_patch(0);
  store_patch(patch0, 0);
  __syncthreads();

  for (int t = 0; t < p.tiles_h; ++t) {
    const int py0 = t * 8;
    const int sy0 = 2 * py0;
    unsigned char* patch = patch0 + (t & 1) * kSpPatchB;
    unsigned char* hp = hp0 + (t & 1) * kSpHpB;
    const unsigned char* hprev = hp0 + ((t + 1) & 1) * kSpHpB;
    const bool more = t + 1 < p.tiles_h;
    if (more) load_patch(py0 + 8);

    // two stem rows (column blocks) at a time: 32 accumulator VGPRs beside the 112 of A
    // fragments (with all four rows live the compiler re-loaded the weights every tile)
#pragma unroll
    for (int np = 0; np < 2; ++np) {
      f32x4 acc[4][2];
#pragma unroll
      for (int mb = 0; mb < 4; ++mb) acc[mb][0] = acc[mb][1] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int r = 0; r < 7; ++r)
#pragma unroll
        for (int nj = 0; nj < 2; ++nj) {
          const bf16x8 bfr = *reinterpret_cast<const bf16x8*>(patch + r * kSpRowB + b_off[2 * np + nj]);
#pragma unroll
          for (int mb = 0; mb < 4; ++mb)
            acc[mb][nj] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[r][mb], bfr, acc[mb][nj], 0, 0, 0);
        }
      if (np == 0) __syncthreads();                      // pool(t - 1) is done with hp / hprev

      // ---- epilogue: bias + ReLU (v_med3 against 0 and a per-lane ceiling: 0 for stem pixels
      // outside the image, so they act as the pool's -inf), bf16 pack, then the 3-wide
      // horizontal max on the packed bit patterns (values >= 0): two row_shr / row_shl DPP
      // moves and two v_pk_max_u16 per dword; the 7 odd lanes store ----
#pragma unroll
      for (int nj = 0; nj < 2; ++nj) {
        const int row = wave * 4 + 2 * np + nj;
        const float hi = (col_ok && sy0 + row < p.Ho) ? __builtin_inff() : 0.f;
#pragma unroll
        for (int mb = 0; mb < 4; ++mb) {
          const f32x4 bias = *reinterpret_cast<const f32x4*>(bias_l + mb * 16 + fq * 4);
          const f32x2 s01 = f32x2{acc[mb][nj][0], acc[mb][nj][1]} + f32x2{bias[0], bias[1]};
          const f32x2 s23 = f32x2{acc[mb][nj][2], acc[mb][nj][3]} + f32x2{bias[2], bias[3]};
          const uint32_t w01 = pack2(__builtin_amdgcn_fmed3f(s01[0], 0.f, hi), __builtin_amdgcn_fmed3f(s01[1], 0.f, hi));
          const uint32_t w23 = pack2(__builtin_amdgcn_fmed3f(s23[0], 0.f, hi), __builtin_amdgcn_fmed3f(s23[1], 0.f, hi));
          const uint32_t h01 = sp_max3_u16x2(w01, sp_dpp_shr1(w01), sp_dpp_shl1(w01));
          const uint32_t h23 = sp_max3_u16x2(w23, sp_dpp_shr1(w23), sp_dpp_shl1(w23));
          if (store_lane)
            *reinterpret_cast<uint2*>(hp + row * kSpHpRowB + hp_lane + mb * 32) = make_uint2(h01, h23);
        }
      }
    }
    if (more) store_patch(patch0 + ((t + 1) & 1) * kSpPatchB, py0 + 8);
    __syncthreads();

    // ---- vertical 3 / stride-2 max: pooled row i = stem rows 2i - 1 (previous tile's 15 for
    // i = 0, zeros above the image), 2i, 2i + 1; packed u16 max of the bf16 bit patterns ----
    for (int it = tid; it < 8 * 7 * 8; it += 256) {
      const int pp = it >> 3, g = it & 7;
      const int i = pp / 7, jx = pp - i * 7;
      const int gy = py0 + i, gx = px0 + jx;
      if (gy >= p.Hm || gx >= p.Wm) continue;
      const int off = jx * kSpHpPitch + g * 16;
      const u32x4 a = *reinterpret_cast<const u32x4*>(hp + (2 * i) * kSpHpRowB + off);
      const u32x4 b = *reinterpret_cast<const u32x4*>(hp + (2 * i + 1) * kSpHpRowB + off);
      u32x4 c = u32x4{0u, 0u, 0u, 0u};
      if (i > 0)
        c = *reinterpret_cast<const u32x4*>(hp + (2 * i - 1) * kSpHpRowB + off);
      else if (t > 0)
        c = *reinterpret_cast<const u32x4*>(hprev + 15 * kSpHpRowB + off);
      const u32x4 o = u32x4{sp_max3_u16x2(a.x, b.x, c.x), sp_max3_u16x2(a.y, b.y, c.y),
                            sp_max3_u16x2(a.z, b.z, c.z), sp_max3_u16x2(a.w, b.w, c.w)};
      *reinterpret_cast<u32x4*>(p.y + ((size_t)(img * p.Hm + gy) * p.Wm + gx) * p.ldy + g * 8) = o;
    }
  }
}

// ---- strip variant with half-channel waves (variants 3 / 4): occupancy for lane overlap ----
//
// The strip kernel above holds all 64 channels' A fragments per wave (112 VGPRs, 214 in all)
// and 55 KB of LDS: two workgroups per CU, and while the stem runs (4 rounds of long-lived
// strips) the other frame lane's conv tiles cannot be resident beside it — the bench measured
// the stem costing ~170 us of wall time per batch against its 127 us of kernel time.  Here a
// wave owns 32 channels (2 channel blocks: 56 VGPRs of A fragments) x 8 stem rows instead of
// 64 channels x 4 rows — the same 112 MFMAs per wave and tile, the same accumulation order per
// output (so bit-identical to variants 0-2), twice the B-fragment reads (still < half the LDS
// rate) — and the pool tile is single-buffered with the previous tile's last stem row carried
// in a 2 x 1 KB side buffer: 40.6 KB of LDS and 124 VGPRs, so 4 workgroups fit a CU (variant 3,
// two stem rows per MFMA group) and the kernel leaves registers / LDS for a co-resident lane;
// variant 4 groups four rows (8 accumulators in flight, 3 workgroups per CU).
constexpr int kSp2HpB = kSpRows * kSpHpRowB;             // 16128 B, single buffer
constexpr int kSp2CarryB = kSpHpRowB;                    // 1008 B: one stem row of 7 pixels

template <int WGS, int RP>
__global__ __launch_bounds__(256, WGS) void stem_pool_strip2_kernel(StemPoolParams p) {
  __shared__ __attribute__((aligned(16))) unsigned char smem[2 * kSpPatchB + kSp2HpB + 2 * kSp2CarryB];
  unsigned char* patch0 = smem;
  unsigned char* hp = smem + 2 * kSpPatchB;
  unsigned char* carry0 = hp + kSp2HpB;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int chh = wave & 1;                              // channel half: blocks 2 chh, 2 chh + 1
  const int rh = wave >> 1;                              // stem rows 8 rh .. 8 rh + 7 of a tile
  const int strips = p.tiles_w;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int img = bid / strips;
  const int sj = bid - img * strips;
  const int px0 = sj * 7;
  const int sx0 = 2 * px0 - 1;
  const int ix0 = 2 * sx0 - 3;
  const int xa = ix0 >= 0 ? (ix0 & ~3) : -((3 - ix0) & ~3);
  const uint8_t* im = p.xu8 + (size_t)img * p.Hi * p.Wi * 3;
  const int fr = lane & 15, fq = lane >> 4;

  bf16x8 af[7][2];
  f32x4 bias[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int mb = 2 * chh + j;
    const int o = mb * 16 + fr;
#pragma unroll
    for (int r = 0; r < 7; ++r)
      af[r][j] = *reinterpret_cast<const bf16x8*>(
          reinterpret_cast<const unsigned char*>(p.w) + r * 64 * 64 + (o * 4 + (fq ^ ((o >> 2) & 2))) * 16);
    bias[j] = *reinterpret_cast<const f32x4*>(p.bias + mb * 16 + fq * 4);
  }

  uint32_t pre[kSpTaskIt][3];
  auto load_patch = [&](int py0) {
    const int iy0 = 4 * py0 - 3;
#pragma unroll
    for (int k = 0; k < kSpTaskIt; ++k) {
      const int task = tid + k * 256;
      const int r = task / kSpGroups, gi = task - r * kSpGroups;
      const int y = iy0 + r, x = xa + 4 * gi;
      pre[k][0] = pre[k][1] = pre[k][2] = 0u;
      if (task < kSpTasks && (unsigned)y < (unsigned)p.Hi && x >= 0 && x + 3 < p.Wi) {
        const uint32_t* src = reinterpret_cast<const uint32_t*>(im + ((size_t)y * p.Wi + x) * 3);
        pre[k][0] = __builtin_nontemporal_load(src);
        pre[k][1] = __builtin_nontemporal_load(src + 1);
        pre[k][2] = __builtin_nontemporal_load(src + 2);
      }
    }
  };
  auto store_patch = [&](unsigned char* patch, int py0) {
    const int iy0 = 4 * py0 - 3;
#pragma unroll
    for (int k = 0; k < kSpTaskIt; ++k) {
      const int task = tid + k * 256;
      if (task >= kSpTasks) continue;
      const int r = task / kSpGroups, gi = task - r * kSpGroups;
      const int y = iy0 + r, x = xa + 4 * gi;
      const bool in = (unsigned)y < (unsigned)p.Hi && x >= 0 && x + 3 < p.Wi;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int j = x + q - ix0;
        if ((unsigned)j >= (unsigned)kSpPW) continue;
        uint2 o = {0u, 0u};
        if (in) {
          const int e = 3 * q;
          const float c0 = (float)((pre[k][e >> 2] >> (8 * (e & 3))) & 0xFFu);
          const float c1 = (float)((pre[k][(e + 1) >> 2] >> (8 * ((e + 1) & 3))) & 0xFFu);
          const float c2 = (float)((pre[k][(e + 2) >> 2] >> (8 * ((e + 2) & 3))) & 0xFFu);
          o = make_uint2(pack2(c0 - p.m0, c1 - p.m1), pack2(c2 - p.m2, 0.f));
        }
        *reinterpret_cast<uint2*>(patch + r * kSpRowB + j * 8) = o;
      }
    }
  };

  const int b_base = 2 * (8 * rh) * kSpRowB + 16 * fr + 16 * fq;
  const bool col_ok = (unsigned)(sx0 + fr) < (unsigned)p.Wo;
  const bool store_lane = (fr & 1) && fr < 15;
  const int hp_lane = ((fr - 1) >> 1) * kSpHpPitch + fq * 8 + chh * 64;

  load_patch(0);
  store_patch(patch0, 0);
  __syncthreads();

  for (int t = 0; t < p.tiles_h; ++t) {
    const int py0 = t * 8;
    const int sy0 = 2 * py0;
    const unsigned char* patch = patch0 + (t & 1) * kSpPatchB + b_base;
    const bool more = t + 1 < p.tiles_h;
    if (more) load_patch(py0 + 8);

    // RP stem rows at a time: 2 RP accumulators (RP rows x 2 channel blocks)
#pragma unroll
    for (int np = 0; np < 8 / RP; ++np) {
      f32x4 acc[2][RP];
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int nj = 0; nj < RP; ++nj) acc[j][nj] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int r = 0; r < 7; ++r)
#pragma unroll
        for (int nj = 0; nj < RP; ++nj) {
          const bf16x8 bfr = *reinterpret_cast<const bf16x8*>(patch + (2 * (RP * np + nj) + r) * kSpRowB);
#pragma unroll
          for (int j = 0; j < 2; ++j)
            acc[j][nj] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[r][j], bfr, acc[j][nj], 0, 0, 0);
        }
      if (np == 0) __syncthreads();                      // pool(t - 1) is done with hp

#pragma unroll
      for (int nj = 0; nj < RP; ++nj) {
        const int row = 8 * rh + RP * np + nj;
        const float hi = (col_ok && sy0 + row < p.Ho) ? __builtin_inff() : 0.f;
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const f32x2 s01 = f32x2{acc[j][nj][0], acc[j][nj][1]} + f32x2{bias[j][0], bias[j][1]};
          const f32x2 s23 = f32x2{acc[j][nj][2], acc[j][nj][3]} + f32x2{bias[j][2], bias[j][3]};
          const uint32_t w01 = pack2(__builtin_amdgcn_fmed3f(s01[0], 0.f, hi), __builtin_amdgcn_fmed3f(s01[1], 0.f, hi));
          const uint32_t w23 = pack2(__builtin_amdgcn_fmed3f(s23[0], 0.f, hi), __builtin_amdgcn_fmed3f(s23[1], 0.f, hi));
          const uint32_t h01 = sp_max3_u16x2(w01, sp_dpp_shr1(w01), sp_dpp_shl1(w01));
          const uint32_t h23 = sp_max3_u16x2(w23, sp_dpp_shr1(w23), sp_dpp_shl1(w23));
          if (store_lane)
            *reinterpret_cast<uint2*>(hp + row * kSpHpRowB + hp_lane + j * 32) = make_uint2(h01, h23);
        }
      }
    }
    if (more) store_patch(patch0 + ((t + 1) & 1) * kSpPatchB, py0 + 8);
    __syncthreads();

    // vertical max; the thread that reads stem row 15 (pooled row 7) also copies it into the
    // carry buffer the next tile's pooled row 0 reads (double-buffered by tile parity)
    const unsigned char* cin = carry0 + (t & 1) * kSp2CarryB;
    unsigned char* cout_ = carry0 + ((t + 1) & 1) * kSp2CarryB;
    for (int it = tid; it < 8 * 7 * 8; it += 256) {
      const int pp = it >> 3, g = it & 7;
      const int i = pp / 7, jx = pp - i * 7;
      const int gy = py0 + i, gx = px0 + jx;
      const int off = jx * kSpHpPitch + g * 16;
      const u32x4 a = *reinterpret_cast<const u32x4*>(hp + (2 * i) * kSpHpRowB + off);
      const u32x4 b = *reinterpret_cast<const u32x4*>(hp + (2 * i + 1) * kSpHpRowB + off);
      u32x4 c = u32x4{0u, 0u, 0u, 0u};
      if (i > 0)
        c = *reinterpret_cast<const u32x4*>(hp + (2 * i - 1) * kSpHpRowB + off);
      else if (t > 0)
        c = *reinterpret_cast<const u32x4*>(cin + off);
      if (i == 7) *reinterpret_cast<u32x4*>(cout_ + off) = b;
      if (gy >= p.Hm || gx >= p.Wm) continue;
      const u32x4 o = u32x4{sp_max3_u16x2(a.x, b.x, c.x), sp_max3_u16x2(a.y, b.y, c.y),
                            sp_max3_u16x2(a.z, b.z, c.z), sp_max3_u16x2(a.w, b.w, c.w)};
      *reinterpret_cast<u32x4*>(p.y + ((size_t)(img * p.Hm + gy) * p.Wm + gx) * p.ldy + g * 8) = o;
    }
  }
}

}  // namespace

}  // namespace aiko

// x: zero-bordered stem input [B, Hp, Wp, 4] bf16 (image at (3, 3)); w: packed stem weights
// [64, 256] (make_stem_spec: 7 filter rows x 8 pixels x 4 channels, K padded to 256); y: pooled
// [B, Hm, Wm, >= 64] (pixel pitch ldy).  Host preconditions (binding): Cout 64, 7x7/s2 stem,
// Hp >= 2 * Ho + 5, Wp >= 2 * Wo + 6, Hm/Wm = pool(Ho/Wo), 16-byte alignment.  variant 0: 8x7
// pooled tiles (4 WG/CU), 1: 8x14 (2 WG/CU, less halo recompute).
extern "C" int aiko_stem_pool(const void* x, const void* w, const float* bias, void* y, int B, int Hp,
                              int Wp, int Ho, int Wo, int Hm, int Wm, int ldy, int variant,
                              hipStream_t stream) {
  using namespace aiko;
  StemPoolParams p;
  p.xu8 = nullptr;
  p.Hi = p.Wi = 0;
  p.m0 = p.m1 = p.m2 = 0.f;
  p.x = static_cast<const bf16_t*>(x);
  p.w = static_cast<const bf16_t*>(w);
  p.bias = bias;
  p.y = static_cast<bf16_t*>(y);
  p.B = B; p.Hp = Hp; p.Wp = Wp; p.Ho = Ho; p.Wo = Wo; p.Hm = Hm; p.Wm = Wm; p.ldy = ldy;
  const int tpw = variant == 1 ? 14 : 7;
  p.tiles_h = (Hm + kTPH - 1) / kTPH;
  p.tiles_w = (Wm + tpw - 1) / tpw;
  const long grid = (long)B * p.tiles_h * p.tiles_w;
  if (grid <= 0 || grid > 0x7fffffffL) return -1;
  if (tpw == 14)
    stem_pool_kernel<14><<<dim3((unsigned)grid), dim3(256), 0, stream>>>(p);
  else
    stem_pool_kernel<7><<<dim3((unsigned)grid), dim3(256), 0, stream>>>(p);
  return (int)hipGetLastError();
}

// uint8 frames [B, Hi, Wi, 3] (Wi % 4 == 0) straight into the fused stem + pool: ``w`` is the
// weight image pre-scaled by 1 / (255 std_c), ``mean255`` the per-channel 255 * mean.
extern "C" int aiko_stem_pool_u8(const void* frames, const void* w, const float* bias, void* y, int B, int Hi,
                                 int Wi, int Ho, int Wo, int Hm, int Wm, int ldy, const float* mean255,
                                 int variant, hipStream_t stream) {
  using namespace aiko;
  if (Wi % 4 || B <= 0) return -1;
  StemPoolParams p;
  p.x = nullptr;
  p.xu8 = static_cast<const uint8_t*>(frames);
  p.Hi = Hi; p.Wi = Wi;
  p.m0 = mean255[0]; p.m1 = mean255[1]; p.m2 = mean255[2];
  p.w = static_cast<const bf16_t*>(w);
  p.bias = bias;
  p.y = static_cast<bf16_t*>(y);
  p.B = B; p.Hp = Hi + 6; p.Wp = Wi + 6; p.Ho = Ho; p.Wo = Wo; p.Hm = Hm; p.Wm = Wm; p.ldy = ldy;
  if (variant >= 2 && variant <= 4) {
    // strip kernels: stem rows 2 py0 .. 2 py0 + 15 of every pooled tile must exist in the stem
    // geometry the pool expects (Ho = 2 Hm or 2 Hm - 1; stem rows past Ho read as zeros)
    p.tiles_h = (Hm + 7) / 8;
    p.tiles_w = (Wm + 6) / 7;
    const long grid = (long)B * p.tiles_w;
    if (grid <= 0 || grid > 0x7fffffffL) return -1;
    if (variant == 2)
      stem_pool_strip_kernel<<<dim3((unsigned)grid), dim3(256), 0, stream>>>(p);
    else if (variant == 3)
      stem_pool_strip2_kernel<4, 2><<<dim3((unsigned)grid), dim3(256), 0, stream>>>(p);
    else
      stem_pool_strip2_kernel<3, 4><<<dim3((unsigned)grid), dim3(256), 0, stream>>>(p);
    return (int)hipGetLastError();
  }
  const int tpw = variant == 1 ? 14 : 7;
  p.tiles_h = (Hm + kTPH - 1) / kTPH;
  p.tiles_w = (Wm + tpw - 1) / tpw;
  const long grid = (long)B * p.tiles_h * p.tiles_w;
  if (grid <= 0 || grid > 0x7fffffffL) return -1;
  if (tpw == 14)
    stem_pool_kernel<14, true><<<dim3((unsigned)grid), dim3(256), 0, stream>>>(p);
  else
    stem_pool_kernel<7, true><<<dim3((unsigned)grid), dim3(256), 0, stream>>>(p);
  return (int)hipGetLastError();
}
