// 3x3 / stride 1 / pad 1 convolution, 32 -> 32 channels, as a persistent ROW STREAM (tuner
// variant 17): YOLOv8-n's 80-wide C2f bottleneck convs (M = B * 6400, ~1.5 MFLOP per output row).
//
// These layers carry ~26 MB in and ~26 MB out for almost no arithmetic, so they are an HBM
// stream: the tiled direct kernel (conv_narrow.hip, 8 / 16 x 32 output tiles) re-reads a 2-row /
// 2-column halo per tile and serialises each tile's load behind the previous one's stores, and
// ran at 1.8-2.2 TB/s.  Here a workgroup of W / 16 waves owns a contiguous range of output rows of
// the flattened [B * H] row space and streams INPUT ROWS through an 8-slot LDS ring (each row read
// once; image boundaries are a per-row tap mask, so a range crosses images freely): output row v
// needs input rows v - 1 .. v + 1, and rows up to v + 7 are in flight.  The row image is the
// conv_patch.hip layout (64 B per pixel, 16-B slot k of pixel q holds channel chunk
// k ^ (((q >> 2) & 1) << 1), one zero pixel each side).  The 18 weight fragments (9 taps x two
// 16-channel blocks) stay in registers; per output row a wave does 9 ds_read_b128 + 18 MFMAs for
// its 16 pixels (weights on the MFMA A side) and one 16-B store per lane (8 consecutive channels of
// one pixel after a v_permlane16_swap).  An optional residual row (the C2f shortcut, added before
// or after the activation) streams through its own ring in the same DMA order.  Every wave issues
// the same op sequence (rows past the range read out-of-range = zero), so each vmcnt is an exact
// compile-time count (rows_young below).
#include <utility>

#include "common.h"

namespace aiko {

namespace rows {
constexpr int C = 32, NS = 8;
constexpr int IA = NS - 2;                       // input rows issued this far ahead of the output row
constexpr int RA = IA - 1;                       // residual rows ahead
constexpr uint32_t kOOB = 0x80000000u;
constexpr uint32_t kRecords = 0x7ffffff0u;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* base) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)kRecords, 0x00020000);
}
__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t r, uint32_t voff, void* lds) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(
      r, reinterpret_cast<__attribute__((address_space(3))) void*>(reinterpret_cast<uintptr_t>(lds)), 16,
      voff, 0, 0, 0);
}
template <int Nn>
__device__ __forceinline__ void vm_barrier() {
  asm volatile("s_waitcnt vmcnt(%0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::"n"(Nn) : "memory");
}

// Per-wave op order: prologue = input rows v0 - 1 .. v0 + IA - 1 (IOPS each), then (RES) residual
// rows v0 .. v0 + RA - 1 (1 op each); step s (output row v0 + s) issues input row v0 + s + IA,
// residual row v0 + s + RA, and after its MFMAs one store.  young(s) = ops issued after the newer
// of {input row v0 + s + 1, residual row v0 + s} and before step s's wait.
template <int IOPS, bool RES>
__host__ __device__ constexpr int young(int s) {
  // sequence positions: prologue, then per step [IN][RES][ST]
  int pos = 0, target = -1;
  const int in_need = s + 1;                     // input row index (relative to v0) needed
  const int res_need = s;
  // prologue input rows -1 .. IA - 1
  for (int r = -1; r < IA; ++r) {
    pos += IOPS;
    if (r == in_need) target = pos;
  }
  if (RES)
    for (int r = 0; r < RA; ++r) {
      pos += 1;
      if (r == res_need && pos > target) target = pos;
    }
  for (int t = 0; t < s; ++t) {
    pos += IOPS;
    if (t + IA == in_need && pos > target) target = pos;
    if (RES) {
      pos += 1;
      if (t + RA == res_need && pos > target) target = pos;
    }
    pos += 1;                                    // the step's store
  }
  return pos - target;
}
}  // namespace rows

template <int W, bool RES>
__global__ __launch_bounds__(W / 16 * 64, 1) void conv3x3_rows_kernel(
    const bf16_t* __restrict__ x, const bf16_t* __restrict__ wimg, const float* __restrict__ bias,
    const bf16_t* __restrict__ res, bf16_t* __restrict__ y, int rows_total, int H, int ldx, int ldy, int ldr,
    int act, int rows_per_wg, int rows_rem) {
  using namespace rows;
  constexpr int NW = W / 16;                      // waves: one 16-pixel block each
  constexpr int PW = W + 8;                       // pixels per LDS row (1 zero pixel left, >= 1 right)
  constexpr int IOPS = (PW * 4 + NW * 64 - 1) / (NW * 64);   // input-row DMA ops per wave
  constexpr int ROWB = IOPS * NW * 1024;          // slot stride: every op's 1 KB lands inside its slot
  constexpr int RESB = W * 64;                    // residual row image (plain: pixel-major, 4 chunks)
  static_assert(W % 16 == 0 && (W * 4) % (NW * 64) == 0, "one residual op per wave");
  __shared__ __attribute__((aligned(16))) unsigned char ring[NS * ROWB + (RES ? NS * RESB : 16)];
  unsigned char* const rring = ring + NS * ROWB;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int fr = lane & 15, fq = lane >> 4;
  const int coff = ((fq & 1) << 4) | ((fq >> 1) << 3);
  const int g = blockIdx.x;
  const int v0 = g * rows_per_wg + min(g, rows_rem);
  const int nrows = rows_per_wg + (g < rows_rem ? 1 : 0);
  if (nrows <= 0) return;
  const __amdgpu_buffer_rsrc_t rx = rsrc(x), rw = rsrc(wimg), ry = rsrc(y), rr = rsrc(RES ? res : x);

  // weights: fragment image [tap 9][block 2][lane 64][8] bf16, lane-linear 16-B loads
  bf16x8 wf[9][2];
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int j = 0; j < 2; ++j) wf[t][j] = *reinterpret_cast<const bf16x8*>(wimg + ((t * 2 + j) * 64 + lane) * 8);
  float bb[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) bb[e] = bias ? bias[coff + e] : 0.f;
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int j = 0; j < 2; ++j) asm volatile("" ::"v"(wf[t][j]));   // retired before the stream starts
#pragma unroll
  for (int e = 0; e < 8; ++e) asm volatile("" ::"v"(bb[e]));

  auto issue_in = [&](int r) {                    // global input row r (any value: out of range -> zeros)
    unsigned char* dst = ring + (((r % NS) + NS) % NS) * ROWB;
    const bool live = r >= 0 && r < rows_total;
#pragma unroll
    for (int k = 0; k < IOPS; ++k) {
      const int pi = (k * NW + wave) * 64 + lane;   // 16-B piece of the row image
      const int q = pi >> 2, slot = pi & 3;
      const int chunk = slot ^ (((q >> 2) & 1) << 1);
      const bool ok = live && q >= 1 && q <= W && pi < PW * 4;
      const uint32_t off = ok ? (uint32_t)(((r * W + (q - 1)) * ldx + chunk * 8) * 2) : kOOB;
      dma16(rx, off, dst + (k * NW + wave) * 1024);
    }
  };
  auto issue_res = [&](int r) {
    if constexpr (RES) {
      unsigned char* dst = rring + (((r % NS) + NS) % NS) * RESB;
      const bool live = r >= 0 && r < rows_total;
      const int pi = wave * 64 + lane;
      const int q = pi >> 2, chunk = pi & 3;
      const uint32_t off = live ? (uint32_t)(((r * W + q) * ldr + chunk * 8) * 2) : kOOB;
      dma16(rr, off, dst + wave * 1024);
    }
  };

  // this lane's B-fragment addresses for column shifts -1 / 0 / +1 (row image pixel q = 1 + p + dc)
  const int p = wave * 16 + fr;
  int addr[3];
#pragma unroll
  for (int dc = 0; dc < 3; ++dc) {
    const int q = p + dc;                          // = 1 + p + (dc - 1)
    addr[dc] = q * 64 + ((fq ^ (((q >> 2) & 1) << 1)) << 4);
  }

  // prologue
  for (int r = -1; r < IA; ++r) issue_in(v0 + r);
  if constexpr (RES)
    for (int r = 0; r < RA; ++r) issue_res(v0 + r);

  const bool post = (act & 16) != 0;
  const int a = act & 15;
  auto step = [&](int s, auto young_tag) {
    constexpr int YG = decltype(young_tag)::value;
    vm_barrier<YG>();
    const int v = v0 + s;
    issue_in(v + IA);
    issue_res(v + RA);
    const int h = v % H;
    f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int dr = 0; dr < 3; ++dr) {
      const int hh = h + dr - 1;
      if (hh < 0 || hh >= H) continue;             // image border: a zero row (wave-uniform)
      const unsigned char* rowp = ring + ((((v + dr - 1) % NS) + NS) % NS) * ROWB;
#pragma unroll
      for (int dc = 0; dc < 3; ++dc) {
        const bf16x8 xf = *reinterpret_cast<const bf16x8*>(rowp + addr[dc]);
        acc0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[dr * 3 + dc][0], xf, acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[dr * 3 + dc][1], xf, acc1, 0, 0, 0);
      }
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const auto sw = __builtin_amdgcn_permlane16_swap(__float_as_uint(acc0[e]), __float_as_uint(acc1[e]), false, false);
      acc0[e] = __uint_as_float(sw[0]);
      acc1[e] = __uint_as_float(sw[1]);
    }
    float o[8] = {acc0[0] + bb[0], acc0[1] + bb[1], acc0[2] + bb[2], acc0[3] + bb[3],
                  acc1[0] + bb[4], acc1[1] + bb[5], acc1[2] + bb[6], acc1[3] + bb[7]};
    u32x4 rv = {0u, 0u, 0u, 0u};
    if constexpr (RES) rv = *reinterpret_cast<const u32x4*>(rring + (((v % NS) + NS) % NS) * RESB + (p * 4 + (coff >> 3)) * 16);
    if (RES && !post) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        o[2 * e] += __uint_as_float(rv[e] << 16);
        o[2 * e + 1] += __uint_as_float(rv[e] & 0xffff0000u);
      }
    }
    if (a == 1) {
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = fmaxf(o[e], 0.f);
    } else if (a == 2) {
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = silu(o[e]);
    }
    if (RES && post) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        o[2 * e] += __uint_as_float(rv[e] << 16);
        o[2 * e + 1] += __uint_as_float(rv[e] & 0xffff0000u);
      }
    }
    u32x4 ov;
#pragma unroll
    for (int e = 0; e < 4; ++e) ov[e] = pack2(o[2 * e], o[2 * e + 1]);
    __builtin_amdgcn_raw_buffer_store_b128(ov, ry, (uint32_t)(((v * W + p) * ldy + coff) * 2), 0, 0);
  };
  // the first IA steps have prologue-dependent wait counts, the rest the steady count
  using Y0 = std::integral_constant<int, young<IOPS, RES>(0)>;
  using Y1 = std::integral_constant<int, young<IOPS, RES>(1)>;
  using Y2 = std::integral_constant<int, young<IOPS, RES>(2)>;
  using Y3 = std::integral_constant<int, young<IOPS, RES>(3)>;
  using Y4 = std::integral_constant<int, young<IOPS, RES>(4)>;
  using Y5 = std::integral_constant<int, young<IOPS, RES>(5)>;
  using YS = std::integral_constant<int, young<IOPS, RES>(6)>;
  static_assert(young<IOPS, RES>(6) == young<IOPS, RES>(7) && young<IOPS, RES>(7) == young<IOPS, RES>(12),
                "steady state from step 6");
  for (int s = 0; s < nrows; ++s) {
    if (s == 0) step(s, Y0{});
    else if (s == 1) step(s, Y1{});
    else if (s == 2) step(s, Y2{});
    else if (s == 3) step(s, Y3{});
    else if (s == 4) step(s, Y4{});
    else if (s == 5) step(s, Y5{});
    else step(s, YS{});
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // DMAs into LDS land before the workgroup ends
}

}  // namespace aiko

// x [B*H rows][W][>= 32] bf16 (pixel pitch ldx); wimg [9][2][64][8] bf16 fragment image
// (ops.conv.rows_weight); res (optional) with pixel pitch ldr; y pixel pitch ldy.  W = 80.  act
// bits 0-3: 0 none / 1 ReLU / 2 SiLU, bit 4: residual after the activation.  ``grid`` workgroups
// (<= 0: one per CU), each a contiguous range of the B * H output rows.
extern "C" int aiko_conv3x3_rows(const void* x, const void* wimg, const float* bias, const void* res, void* y, int B,
                                 int H, int W, int ldx, int ldy, int ldr, int act, int grid, hipStream_t stream) {
  using namespace aiko;
  if (W != 80 || B < 1 || H < 1 || ldx % 8 || ldy % 8 || (res && ldr % 8) || ldx < 32 || ldy < 32) return -1;
  const int rows_total = B * H;
  if (grid <= 0) {
    int dev = 0, cus = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) cus = 256;
    grid = cus;
  }
  if (grid > rows_total) grid = rows_total;
  const int per = rows_total / grid, rem = rows_total % grid;
  auto xp = static_cast<const bf16_t*>(x);
  auto wp = static_cast<const bf16_t*>(wimg);
  auto rp = static_cast<const bf16_t*>(res);
  auto yp = static_cast<bf16_t*>(y);
  if (res)
    hipLaunchKernelGGL((conv3x3_rows_kernel<80, true>), dim3(grid), dim3(320), 0, stream, xp, wp, bias, rp, yp,
                       rows_total, H, ldx, ldy, ldr, act, per, rem);
  else
    hipLaunchKernelGGL((conv3x3_rows_kernel<80, false>), dim3(grid), dim3(320), 0, stream, xp, wp, bias, rp, yp,
                       rows_total, H, ldx, ldy, ldr, act, per, rem);
  return (int)hipGetLastError();
}
