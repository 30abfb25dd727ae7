// Whole ResNet-50 stage-1 bottleneck in ONE launch (gfx950, wave64, v_mfma_f32_16x16x32_bf16):
//
//   t1 = relu(x . W1^T + b1)              1x1, CIN -> 64
//   t2 = relu(conv3x3(t1) . W2^T + b2)     3x3 pad 1, 64 -> 64
//   y  = relu(t2 . W3^T + b3 + x)          1x1, 64 -> 256, identity residual          (CIN = 256)
//   y  = relu([t2 | x] . W3^T + b3)        conv3 and the 1x1 projection shortcut
//                                          K-concatenated (ops.conv.fuse_shortcut)    (CIN = 64)
//
// Stage 1 (56x56) is memory-bound: at B=320 every 256-channel activation is 514 MB.  Unfused,
// a block moves x, t1, t2 and y through HBM several times (conv_chain + conv3x3_patch: ~1.5 GB
// per identity block); here only x is read (plus a 2-row halo per band) and y written, ~1.1 GB.
//
// Work decomposition: a persistent grid, one workgroup per CU (8 waves, two per SIMD, ~154 KB
// LDS).  The B * H output rows, flattened image-major, are split into one contiguous range per
// workgroup (consecutive logical ids on one XCD: xcd_remap, so neighbouring ranges share halo
// rows in that XCD's L2).  A workgroup streams its range with a rolling window that runs across
// image boundaries, so weights are loaded and the DMA pipeline filled once per CU, not per band.
// The x rows it needs form a "virtual row" sequence v: image n0 + v / (H + 2), row
// v % (H + 2) - 1 — every image contributes its rows plus a zero halo row above and below —
// and output row (n, h) is centred on v = (n - n0) (H + 2) + h + 1:
//   * x rows stream into a 4-slot LDS ring (slot v & 3) by LDS-DMA (global_load_lds_dwordx4):
//     rows v_c (conv3's residual / projection input) and v_c + 2 (conv1's input) in use,
//     v_c + 3 in flight;
//   * conv1 turns x rows into a 3-row t1 LDS ring (slot v % 3; 64 pixel slots per row: slots
//     56..63 and halo rows are zeros, which IS the 3x3's zero padding);
//   * conv2 reads the three t1 rows v_c - 1 .. v_c + 1 (im2col by address arithmetic) into t2;
//   * conv3 (+ residual / projection, bias, ReLU) writes y's row straight from the
//     accumulators with 16-byte stores.
//   Two barriers per row: phase A = conv2; phase B = conv3 and conv1(v_c + 2) (independent:
//   conv1 overwrites the t1 slot of v_c - 1, which only phase A read).  Where v_c jumps by 3
//   (an image boundary) an extra phase first converts the new image's first two rows.
//
// Every product is computed TRANSPOSED (weights on the MFMA A side, 16 output channels x 16
// pixels per tile) so the weights stay in VGPRs for the whole band — wave w & 3 owns one slice of
// every weight matrix (W1 16 ch x CIN, W2 16 ch x 576, W3 64 ch x K3) and wave w >> 2 one half of
// the row's pixel tiles — and the pixel-side fragments are 16-byte ds_read_b128s of channel runs.
// For conv3 the A rows are permuted (MFMA row 4q + e of tile t <- channel 8q + 4t + e) so each
// lane ends with 8 consecutive channels of one pixel: store needs no shuffle.
//
// The loop is VALU-lean by construction (the first version spent 5 VALU per MFMA on address
// arithmetic and epilogues and was issue-bound at a quarter of MFMA peak):
//   * LDS images are laid out so every fragment address is a per-lane base + an immediate:
//     t1 / t2 rows are channel-chunk planes of 64 pixel slots ([chunk][slot], 16 B units; a
//     read's 16-lane group then covers 16 consecutive slots = 16 distinct bank groups, no
//     swizzle needed); x rows stay NHWC (so each 1-KB LDS-DMA instruction reads ~2 whole
//     pixels, coalesced — a chunk-planar x image made every DMA a 16-B-per-line gather and cost
//     a third of the row time) with a pixel pitch of CIN/8 + 2 units, which spreads a lane
//     group's 16 (pixel, chunk) reads over 16 distinct bank groups;
//   * biases enter as the MFMA accumulator input (C operand), the identity residual as one
//     extra k-step against a one-hot A fragment (x's own bf16 fragment is the B operand), and
//     ReLU runs on the packed bf16 pair (v_pk_max_i16 against 0: a negative bf16 is a negative
//     int16) — the conv3 epilogue is 2 VALU per output dword.
//
// Synchronisation: raw s_barriers; LDS-DMA completion is a counted `s_waitcnt vmcnt(N)` where
// N = the wave's VMEM ops issued after the awaited DMA (the previous row's y stores and the next
// row's DMAs — the stores are inline asm too, so the count is exact and the compiler inserts no
// vmcnt(0) drains of its own).
#include <cstdlib>
#include <type_traits>

#include "conv_common.h"

namespace aiko {

namespace {

constexpr int kBnW = 56;            // image width / height of ResNet stage 1
constexpr int kBnMid = 64;          // bottleneck width
constexpr int kBnOut = 256;         // block output channels
constexpr int kBnNW = 8;            // waves per workgroup: 4 channel slices x 2 pixel halves
constexpr int kBnTPW = 2;           // 16-pixel tiles per wave (64 slots / 16 / 2)
// t1 / t2 row: 8 chunk planes x 64 slots (16 B units) + a zero guard unit in front (slot -1 of
// plane 0; slot -1 of plane c > 0 is plane c-1's slot 63, a zero pad) + a tail unit (slot 64
// of plane 7, read only for the discarded output slot 63)
constexpr int kBnTU = 8 * 64 + 8;   // units per t1 / t2 row (guard, 512, tail, padding to 16 B x 8)
constexpr int kBnTB = kBnTU * 16;

struct BnParams {
  const bf16_t* x;      // [B][H][56][CIN]
  const bf16_t* w1;     // [64][CIN]
  const float* b1;      // [64]
  const bf16_t* w2;     // [64][9 * 64]  (tap-major, channel-minor: ops.conv.make_conv_spec)
  const float* b2;      // [64]
  const bf16_t* w3;     // [256][K3]     K3 = 64 (identity) or 128 (conv3 | projection)
  const float* b3;      // [256]
  bf16_t* y;            // [B][H][56][256]
  int B, H;
  int rows_per_wg, rows_rem;   // output rows R = B * H split into contiguous per-workgroup ranges
  unsigned* dbg;        // diagnostic s_memtime stamps of wave 0, [G][rows_per_wg + 1][8] (null: off)
  int mode;             // schedule / ablation bits (AIKO_BN_MODE; default 1024 = split conv2 schedule)
};

__device__ __forceinline__ void bn_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// s_waitcnt vmcnt(n) for a wave-uniform n (the immediate must be a constant)
__device__ __forceinline__ void bn_vm_wait(int n) {
  switch (n) {
#define BN_W(k) case k: asm volatile("s_waitcnt vmcnt(" #k ")" ::: "memory"); break;
    BN_W(1) BN_W(2) BN_W(3) BN_W(4) BN_W(5) BN_W(6) BN_W(7) BN_W(8) BN_W(9) BN_W(10) BN_W(11) BN_W(12)
    BN_W(13) BN_W(14) BN_W(15) BN_W(16) BN_W(17) BN_W(18) BN_W(19) BN_W(20) BN_W(21) BN_W(22) BN_W(23)
    BN_W(24) BN_W(25) BN_W(26) BN_W(27) BN_W(28)
#undef BN_W
    default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
  }
}

// Software pipeline of an unrolled k loop (one scheduling region): the fragments of the first
// D k-steps are read up front, then every k-step's R MFMAs are followed by the reads of the
// k-step D ahead — D x R ds_read_b128 in flight behind the matrix pipe instead of the
// compiler's read -> wait -> MFMA pairs.
template <int KS, int R, int D>
__device__ __forceinline__ void bn_pipeline() {
  __builtin_amdgcn_sched_group_barrier(0x100, R * D, 0);      // DS_READ
#pragma unroll
  for (int k = 0; k < KS - D; ++k) {
    __builtin_amdgcn_sched_group_barrier(0x008, R, 0);        // MFMA
    __builtin_amdgcn_sched_group_barrier(0x100, R, 0);        // DS_READ
  }
  __builtin_amdgcn_sched_group_barrier(0x008, R * D, 0);
}

// the compiler's hazard recognizer does not see that this asm is a 128-bit store, so it does not
// keep the next VALU write off the data VGPRs while the store still reads them (observed: the
// first data dword of some lanes overwritten): the s_nop supplies those wait states
__device__ __forceinline__ void bn_store16(bf16_t* p, u32x4 v) {
  asm volatile("global_store_dwordx4 %0, %1, off\n\ts_nop 1" :: "v"(p), "v"(v) : "memory");
}

template <int OFF>
__device__ __forceinline__ bf16x8 bn_ld(const unsigned char* base) {
  return *reinterpret_cast<const bf16x8*>(base + OFF);
}

// relu on a packed bf16 pair: a negative bf16 (sign bit set) is a negative int16
__device__ __forceinline__ uint32_t bn_relu2(uint32_t v) {
  typedef short s16x2 __attribute__((ext_vector_type(2)));
  const s16x2 r = __builtin_elementwise_max(__builtin_bit_cast(s16x2, v), s16x2{0, 0});
  return __builtin_bit_cast(uint32_t, r);
}

template <int CIN>
__global__ __launch_bounds__(64 * kBnNW, 1) void bneck_fused_kernel(BnParams p) {
  constexpr bool DUAL = CIN == 64;                 // projection block (stage-1 entry)
  constexpr int NC = CIN / 8;                      // 16-byte channel chunks per pixel
  // x row image: NHWC with a pixel pitch of NC + 2 units (NC = 32 or 8: pitch = 2 mod 8, so
  // the 16 (pixel, chunk) pairs one ds_read_b128 lane group reads hit 16 distinct bank groups)
  // — the LDS-DMA fills it from contiguous global runs, one 1-KB instruction = ~2 pixels
  constexpr int XPU = NC + 2;
  constexpr int XU = kBnW * XPU;                   // 16-byte units per x row image
  constexpr int XB = XU * 16;                      // bytes per x ring slot
  constexpr int NI = (XU + 63) / 64;               // 1-KB DMA wave-instructions per x row
  constexpr int DQ = (NI + kBnNW - 1) / kBnNW;
  constexpr int KS1 = CIN / 32, KS2 = 9 * kBnMid / 32, K3 = DUAL ? 2 * kBnMid : kBnMid, KS3 = K3 / 32;
  constexpr int ST = 2 * kBnTPW;                   // y stores per wave per row
  constexpr int X_BYTES = 4 * XB, T1_BYTES = 3 * kBnTB;
  constexpr int LDS_BYTES = X_BYTES + T1_BYTES + kBnTB;
  // conv1 / conv3 read x units up to 7 past a row image (odd chunk, pixel slots 56..63): for the
  // last ring slot they fall into the t1 ring, still inside the allocation
  static_assert(LDS_BYTES <= 160 * 1024, "LDS");
  __shared__ __attribute__((aligned(16))) unsigned char lds[LDS_BYTES];
  unsigned char* const xr = lds;
  unsigned char* const t1r = lds + X_BYTES;
  unsigned char* const t2b = lds + X_BYTES + T1_BYTES;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int cg = wv & 3;                           // channel slice: 16 of conv1 / conv2, 64 of conv3
  const int pt0 = (wv >> 2) * kBnTPW;              // first 16-pixel tile of this wave
  const int fr = lane & 15, fq = lane >> 4;

  const int lid = xcd_remap(blockIdx.x, gridDim.x);
  const int H = p.H, HV = H + 2;
  const int R0 = lid * p.rows_per_wg + min(lid, p.rows_rem);
  const int nrows = p.rows_per_wg + (lid < p.rows_rem ? 1 : 0);
  if (nrows <= 0) return;
  const int n0 = R0 / H, h0 = R0 - n0 * H;

  // ---- weights into registers (one slice per wave), biases into registers / LDS
  bf16x8 w1f[KS1], w2f[KS2], w3f[4][KS3];
#pragma unroll
  for (int ks = 0; ks < KS1; ++ks)
    w1f[ks] = *reinterpret_cast<const bf16x8*>(p.w1 + (16 * cg + fr) * CIN + 32 * ks + 8 * fq);
#pragma unroll
  for (int ks = 0; ks < KS2; ++ks)
    w2f[ks] = *reinterpret_cast<const bf16x8*>(p.w2 + (16 * cg + fr) * (9 * kBnMid) + 32 * ks + 8 * fq);
#pragma unroll
  for (int t = 0; t < 4; ++t) {                    // tile t: channels 64 cg + 32 (t >> 1) + 8 q + 4 (t & 1) + e
    const int row = 64 * cg + 32 * (t >> 1) + 8 * (fr >> 2) + 4 * (t & 1) + (fr & 3);
#pragma unroll
    for (int ks = 0; ks < KS3; ++ks)
      w3f[t][ks] = *reinterpret_cast<const bf16x8*>(p.w3 + row * K3 + 32 * ks + 8 * fq);
  }
  f32x4 bias1, bias2;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    bias1[e] = p.b1[16 * cg + 4 * fq + e];
    bias2[e] = p.b2[16 * cg + 4 * fq + e];
  }
  // conv3's bias: the C input of each tile's first MFMA, held in registers (an LDS re-read per
  // pixel tile cost 8 ds_read_b128 per wave and row in the LDS-bound phase B)
  f32x4 bias3[4];
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int e = 0; e < 4; ++e) bias3[t][e] = p.b3[64 * cg + 32 * (t >> 1) + 8 * fq + 4 * (t & 1) + e];
  // one-hot A fragments of the identity residual (tile parity tp): row 4q + e of the tile is
  // channel 8q + 4tp + e of the 32-channel slice the B fragment (x's chunk run) holds
  bf16x8 eye[2];
#pragma unroll
  for (int tp = 0; tp < 2; ++tp)
#pragma unroll
    for (int i = 0; i < 8; ++i)
      eye[tp][i] = (fq == (fr >> 2) && i == 4 * tp + (fr & 3)) ? (bf16_t)1.0f : (bf16_t)0.0f;
  // zero guard unit (slot -1 of plane 0) of every t1 row
  if (tid < 3) *reinterpret_cast<u32x4*>(t1r + tid * kBnTB) = u32x4{0u, 0u, 0u, 0u};
  // the builtin (not asm): the compiler's waitcnt pass then knows these loads are done and
  // inserts no vmcnt waits of its own inside the loop, where only DMAs / stores are counted
  __builtin_amdgcn_s_waitcnt(0x0f70);              // vmcnt(0)

  // ---- per-lane DMA source offsets: unit u of the x row image <- (chunk c, pixel s) of x
  int goff[DQ];
  bool gok[DQ];
#pragma unroll
  for (int q = 0; q < DQ; ++q) {
    const int u = (wv + kBnNW * q) * 64 + lane;
    const int s = min(u / XPU, kBnW - 1);
    const int c = min(u - (u / XPU) * XPU, NC - 1);           // the pad units: a duplicate chunk
    goff[q] = s * CIN * 2 + c * 16;
    gok[q] = u < XU && wv + kBnNW * q < NI && u - (u / XPU) * XPU < NC;   // no request for pad units
  }
  int dw = 0;                                      // this wave's DMA instructions per row
#pragma unroll
  for (int q = 0; q < DQ; ++q) dw += wv + kBnNW * q < NI ? 1 : 0;

  // per-lane fragment bases (bytes): every read below adds only an immediate
  //   x:      unit s * XPU + c,                       c = 4 ks + fq (+ 8 cg + 4 h for the residual)
  //   t1, t2: unit 1 + c * 64 + s,                    c = 4 hk + fq
  const int xlb = ((16 * pt0 + fr) * XPU + fq) * 16;
  const int tlb = (fq * 64 + fr + 16 * pt0) * 16;
  //   t1 / t2 writes: lane holds channels 16 cg + 4 fq .. + 3 of pixel s: chunk 2 cg + fq / 2
  const int twb = ((2 * cg + (fq >> 1)) * 64 + fr + 16 * pt0) * 16 + (fq & 1) * 8;

  constexpr long XROWG = (long)kBnW * CIN * 2;    // bytes of one x row in global memory
  // virtual row v: image n0 + v / HV, row v % HV - 1 (-1 and H are the zero halo rows)
  // the last virtual row this workgroup needs: one past the centre of its last output row
  const int nl = (R0 + nrows - 1) / H;
  const int vlast = (nl - n0) * HV + (R0 + nrows - 1 - nl * H) + 2;
  // VMEM ops this wave has issued (DMAs and y stores; wave-uniform): a DMA issued when the count
  // became m has landed once vmcnt <= ops - m.  The marks of the last four virtual rows brought in
  // (vdma - 1 - d in field d) live in ONE 64-bit register, 16 bits each: bit 15 = a DMA was
  // issued (clear: a zero halo row, nothing to wait for; conv1 then writes zeros), bits 0..14 =
  // m mod 2^15 (ops - m is < 64, so the difference mod 2^15 is exact).  Four separate marks
  // read through the lambdas' captured references were folded into a select of pointers, which
  // put them in scratch — and the scratch load's vmcnt(0) drained every in-flight DMA at each
  // wait (rounds 3-5)
  int ops = 0;
  unsigned long long marks = 0;
  int vdma = h0, dn = n0, dr = h0 - 1;             // next virtual row to bring in = (image, row)
  auto dma_next = [&]() {                          // x row vdma -> ring slot vdma & 3
    const int v = vdma++;
    int m = -1;
    if (dr >= 0 && dr < H) {
      const unsigned char* src = reinterpret_cast<const unsigned char*>(p.x) + ((long)dn * H + dr) * XROWG;
      unsigned char* dst = xr + (v & 3) * XB;
#pragma unroll
      for (int q = 0; q < DQ; ++q) {
        const int j = wv + kBnNW * q;
        if (gok[q]) glds16_asm(src + goff[q], dst + j * 1024);
      }
      ops += dw;
      m = ops;
    }
    if (++dr > H) {                                // past the bottom halo: next image's top halo
      dr = -1;
      ++dn;
    }
    marks = (marks << 16) | (m >= 0 ? 0x8000ull | (unsigned)(m & 0x7fff) : 0ull);
  };
  auto slot_mark = [&](int v) {                    // v in [vdma - 4, vdma)
    return (unsigned)(marks >> (16 * (vdma - 1 - v))) & 0xffffu;
  };
  auto row_valid = [&](int v) { return (slot_mark(v) & 0x8000u) != 0; };    // v is in the ring
  auto wait_row = [&](int v) {                     // this wave's DMA of x row v has landed
    const unsigned mk = slot_mark(v);
    if (mk & 0x8000u) bn_vm_wait(__builtin_amdgcn_readfirstlane((int)(((unsigned)ops - mk) & 0x7fffu)));
  };

  // conv1: x row v -> t1 slot v % 3 (a zero row for the halo rows)
  auto conv1 = [&](int k) {
    unsigned char* t1w = t1r + (k % 3) * kBnTB + twb;
    if (!row_valid(k)) {
#pragma unroll
      for (int t = 0; t < kBnTPW; ++t) *reinterpret_cast<uint2*>(t1w + (1 + 16 * t) * 16) = uint2{0u, 0u};
      return;
    }
    const unsigned char* xs = xr + (k & 3) * XB + xlb;
    f32x4 a1[kBnTPW];
#pragma unroll
    for (int ks = 0; ks < KS1; ++ks) {
      bf16x8 bf[kBnTPW];
#pragma unroll
      for (int t = 0; t < kBnTPW; ++t)
        bf[t] = *reinterpret_cast<const bf16x8*>(xs + (16 * t * XPU + 4 * ks) * 16);
#pragma unroll
      for (int t = 0; t < kBnTPW; ++t)
        a1[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w1f[ks], bf[t], ks == 0 ? bias1 : a1[t], 0, 0, 0);
    }
    bn_pipeline<KS1, kBnTPW, KS1 >= 4 ? 3 : 1>();
#pragma unroll
    for (int t = 0; t < kBnTPW; ++t) {
      uint2 pk{bn_relu2(pack2(a1[t][0], a1[t][1])), bn_relu2(pack2(a1[t][2], a1[t][3]))};
      if (pt0 + t == 3 && fr >= kBnW - 48) pk = uint2{0u, 0u};   // pixel slots 56..63: zero pad
      *reinterpret_cast<uint2*>(t1w + (1 + 16 * t) * 16) = pk;
    }
  };

  // conv2 of the output row centred on virtual row vc: t1 slots of vc - 1, vc, vc + 1 -> t2.
  // k-steps [KB, KE) only, into a2n (ks 0 .. 11 are the taps of rows vc - 1 and vc, 12 .. 17 those
  // of row vc + 1): the split schedule runs the first part for the NEXT row inside phase B, whose
  // MFMA pipe the stores / packing of conv3 leave half idle, and only the last taps in phase A
  f32x4 a2n[kBnTPW];
  auto conv2_part = [&](int vc, auto kb, auto ke) __attribute__((always_inline)) {
    constexpr int KB = decltype(kb)::value, KE = decltype(ke)::value;
    const unsigned char* tr[3] = {t1r + ((vc - 1) % 3) * kBnTB + tlb, t1r + (vc % 3) * kBnTB + tlb,
                                  t1r + ((vc + 1) % 3) * kBnTB + tlb};
#pragma unroll
    for (int ks = KB; ks < KE; ++ks) {
      const int tap = ks >> 1, dy = tap / 3, dx = tap % 3 - 1, hk = ks & 1;
      bf16x8 bf[kBnTPW];
#pragma unroll
      for (int t = 0; t < kBnTPW; ++t)
        bf[t] = *reinterpret_cast<const bf16x8*>(tr[dy] + (1 + 256 * hk + 16 * t + dx) * 16);
#pragma unroll
      for (int t = 0; t < kBnTPW; ++t)
        a2n[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w2f[ks], bf[t], ks == 0 ? bias2 : a2n[t], 0, 0, 0);
    }
    bn_pipeline<KE - KB, kBnTPW, 4>();
  };
  auto conv2_store = [&]() __attribute__((always_inline)) {
    unsigned char* t2w = t2b + twb;
#pragma unroll
    for (int t = 0; t < kBnTPW; ++t) {
      const uint2 pk{bn_relu2(pack2(a2n[t][0], a2n[t][1])), bn_relu2(pack2(a2n[t][2], a2n[t][3]))};
      *reinterpret_cast<uint2*>(t2w + (1 + 16 * t) * 16) = pk;
    }
  };
  using KB0 = std::integral_constant<int, 0>;
  using KBS = std::integral_constant<int, 12>;
  using KBE = std::integral_constant<int, KS2>;

  // conv3 (+ residual / projection of x row vc) -> y row (n, r), centred on virtual row vc
  auto conv3 = [&](int vc, int n, int r) {
    const unsigned char* xres = xr + (vc & 3) * XB + xlb;
    const unsigned char* t2r = t2b + tlb;
    bf16_t* yrow = p.y + ((long)(n * H + r) * kBnW + 16 * pt0 + fr) * kBnOut + 64 * cg + 8 * fq;
#pragma unroll
    for (int t8 = 0; t8 < kBnTPW; ++t8) {          // pixel tile pt0 + t8
      bf16x8 bf[KS3];
#pragma unroll
      for (int ks = 0; ks < KS3; ++ks)
        bf[ks] = ks < 2 ? *reinterpret_cast<const bf16x8*>(t2r + (1 + 256 * ks + 16 * t8) * 16)
                        : *reinterpret_cast<const bf16x8*>(xres + (16 * t8 * XPU + 4 * (ks - 2)) * 16);
      bf16x8 rv[2];                                // x chunks 8 cg + 4 h + fq: the residual's B side
      if constexpr (!DUAL) {
#pragma unroll
        for (int h = 0; h < 2; ++h)
          rv[h] = *reinterpret_cast<const bf16x8*>(xres + (16 * t8 * XPU + 8 * cg + 4 * h) * 16);
      }
      f32x4 a3[4];
#pragma unroll
      for (int ks = 0; ks < KS3; ++ks)
#pragma unroll
        for (int t = 0; t < 4; ++t)
          a3[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w3f[t][ks], bf[ks], ks == 0 ? bias3[t] : a3[t], 0, 0, 0);
      if constexpr (!DUAL) {
#pragma unroll
        for (int t = 0; t < 4; ++t) a3[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(eye[t & 1], rv[t >> 1], a3[t], 0, 0, 0);
      }
#pragma unroll
      for (int h = 0; h < 2; ++h) {                // channels 64 cg + 32 h + 8 fq .. + 7
        const u32x4 ov{bn_relu2(pack2(a3[2 * h][0], a3[2 * h][1])), bn_relu2(pack2(a3[2 * h][2], a3[2 * h][3])),
                       bn_relu2(pack2(a3[2 * h + 1][0], a3[2 * h + 1][1])),
                       bn_relu2(pack2(a3[2 * h + 1][2], a3[2 * h + 1][3]))};
        if (p.mode & 128) {                        // ablation: no store (keep the values live)
          if (ov[0] == 0x7fc07fc0u && ov[1] == ov[2] && ov[3] == 1u) bn_store16(yrow, ov);
        } else if (p.mode & 256) {                 // ablation: same bytes, lane-contiguous addresses
          bf16_t* yr = p.y + ((long)(n * H + r) * kBnW) * kBnOut;
          bn_store16(yr + (long)(((cg * 2 + (pt0 >> 1)) * 4 + t8 * 2 + h) % 28) * 512 + lane * 8, ov);
        } else if (16 * (pt0 + t8) + fr < kBnW) {
          bn_store16(yrow + 16 * t8 * kBnOut + 32 * h, ov);
        }
      }
    }
    ops += ST;
  };

  // ---- prologue: virtual rows h0 .. h0 + 3 in flight, t1 rows of h0 .. h0 + 2 (the first
  //      output row is centred on vc = h0 + 1)
  while (vdma <= min(h0 + 3, vlast)) dma_next();
  wait_row(min(h0 + 2, vlast));
  wait_row(h0 + 1);
  wait_row(h0);
  bn_barrier();
  conv1(h0);
  conv1(h0 + 1);
  if (h0 + 2 <= vlast) conv1(h0 + 2);
  bn_barrier();

  // ---- one output row per iteration, two barriers:
  //   A: conv2(vc) -> t2                          | DMA of x row vc + 3 in flight
  //   B: conv3(vc) (reads t2, x row vc) and conv1 of x row vc + 2 (-> t1 slot of vc - 1, which
  //      conv2 read in A); the x slot of vc - 1 was last read by conv3 in the previous B
  int n = n0, r = h0, vc = h0 + 1;
  const bool stamps = p.dbg != nullptr && wv == 0;
  unsigned st[8];
  bool pre = false;                                // a2n holds this row's first conv2 taps
  auto stamp = [&](int i) {
    if (stamps) st[i] = (unsigned)__builtin_amdgcn_s_memtime();
  };
  for (int j = 0; j < nrows; ++j) {
    stamp(0);
    if (j > 0) {                                   // advance the output row
      if (++r == H) {
        r = 0;
        ++n;
        vc += 3;                                   // skip the bottom halo of image n-1, top of n
      } else {
        ++vc;
      }
    }
    while (!(p.mode & 32) && vdma <= min(vc + 3, vlast)) dma_next();
    stamp(1);
    if (j > 0 && r == 0) {                         // image boundary: t1 rows of vc and vc + 1 first
      wait_row(vc + 1);
      wait_row(vc);
      bn_barrier();
      conv1(vc);
      conv1(vc + 1);
      bn_barrier();
    }
    if (!(p.mode & 1)) {
      if (pre) conv2_part(vc, KBS{}, KBE{});       // rows vc - 1, vc were done in the last phase B
      else conv2_part(vc, KB0{}, KBE{});
      conv2_store();
    }
    stamp(2);
    if (!(p.mode & 8) && vc + 2 <= vlast) wait_row(vc + 2);
    stamp(3);
    if (!(p.mode & 16)) bn_barrier();
    stamp(4);
    // split schedule: the next output row's first conv2 taps (t1 rows vc, vc + 1, both complete;
    // conv1 below writes the slot of vc - 1) when it is in the same image
    const bool split = (p.mode & 3072) && j + 1 < nrows && r + 1 < H;
    if (split && (p.mode & 2048)) conv2_part(vc + 1, KB0{}, KBS{});
    if (p.mode & 512) {                            // A/B: conv3 (and its stores) first
      if (!(p.mode & 4)) conv3(vc, n, r);
      stamp(5);
      if (!(p.mode & 2) && vc + 2 <= vlast) conv1(vc + 2);
    } else {
      if (!(p.mode & 2) && vc + 2 <= vlast) conv1(vc + 2);
      stamp(5);
      if (!(p.mode & 4)) conv3(vc, n, r);
    }
    if (split && !(p.mode & 2048)) conv2_part(vc + 1, KB0{}, KBS{});
    pre = split;
    stamp(6);
    if (!(p.mode & 16)) bn_barrier();
    stamp(7);
    if (stamps) {                                  // two counted stores (vmcnt bookkeeping)
      unsigned* d = p.dbg + ((long)lid * (p.rows_per_wg + 1) + j) * 8;
      if (lane == 0) {
        bn_store16(reinterpret_cast<bf16_t*>(d), u32x4{st[0], st[1], st[2], st[3]});
        bn_store16(reinterpret_cast<bf16_t*>(d + 4), u32x4{st[4], st[5], st[6], st[7]});
      }
      ops += 2;
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

}  // namespace

}  // namespace aiko

static int bn_cu_count() {
  static int n = 0;
  if (n == 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
      n = 256;
  }
  return n;
}

// x [B][H][56][cin] (cin 256: identity block, 64: projection block with w3 = [conv3 | shortcut]),
// y [B][H][56][256]; grid = workgroups (0: one per CU), each streaming a contiguous range of the
// B * H output rows; dbg: null, or [G][R / G + 1][8] uint32 for wave 0's per-row s_memtime
// stamps (diagnostics).  Returns 0 or a HIP error / -1.
extern "C" int aiko_bneck_fused(const void* x, const void* w1, const float* b1, const void* w2, const float* b2,
                                const void* w3, const float* b3, void* y, int B, int H, int W, int cin, int grid,
                                unsigned* dbg, hipStream_t stream) {
  using namespace aiko;
  if (W != kBnW || (cin != 64 && cin != 256) || B <= 0 || H <= 0) return -1;
  const int R = B * H;
  int G = grid > 0 ? grid : bn_cu_count();
  G = G < R ? G : R;
  BnParams p;
  p.x = static_cast<const bf16_t*>(x);
  p.w1 = static_cast<const bf16_t*>(w1);
  p.b1 = b1;
  p.w2 = static_cast<const bf16_t*>(w2);
  p.b2 = b2;
  p.w3 = static_cast<const bf16_t*>(w3);
  p.b3 = b3;
  p.y = static_cast<bf16_t*>(y);
  p.B = B;
  p.H = H;
  p.rows_per_wg = R / G;
  p.rows_rem = R % G;
  p.dbg = dbg;
  // default 1024 = the split conv2 schedule (the next row's first 12 k-steps at the end of phase
  // B): neutral while every wait drained to vmcnt(0) (round 5), 3 % faster isolated once the
  // counted waits worked (round 6: 544 vs 561 us identity, 475 vs 486 us projection at B=640)
  const char* mode = getenv("AIKO_BN_MODE");
  p.mode = mode ? atoi(mode) : 1024;
  if (cin == 256)
    hipLaunchKernelGGL(bneck_fused_kernel<256>, dim3(G), dim3(64 * kBnNW), 0, stream, p);
  else
    hipLaunchKernelGGL(bneck_fused_kernel<64>, dim3(G), dim3(64 * kBnNW), 0, stream, p);
  return (int)hipGetLastError();
}
