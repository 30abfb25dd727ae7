// Implicit-GEMM convolution / GEMM for CDNA4 (gfx950), bf16 in, fp32 MFMA accumulate, bf16 out.
//
//   y[m, n] = act( sum_k A[m, k] * Wt[n, k] + bias[n] (+ residual[m, n]) )
//
// A is never materialised: row m is an output pixel (img, oh, ow) of an NHWC activation and
// column k walks the filter taps (r, s) and a contiguous channel run of length Cc (multiple
// of 8; K is zero-padded to a multiple of 64).  For every 64-wide K block a thread's 16-byte piece therefore maps to ONE tap and one
// contiguous 8-channel run of one input pixel, so the gather is a set of 16-byte loads with a
// per-row bounds predicate (zero fill = conv zero padding).  The same kernel is a plain GEMM
// (R = S = H = W = 1) and covers ResNet-50's 7x7/s2 stem through a pre-padded 4-channel input
// where a chunk of 32 elements spans 8 consecutive pixels of one input row (see ops/conv.py).
//
// Tiling (MI355X): 256 threads = 4 waves (2 x 2), block tile BM x BN x 64, every wave owns a
// (BM/2) x (BN/2) sub-tile computed with v_mfma_f32_16x16x32_bf16.  Operands are staged
// global -> VGPR -> LDS with a 2-deep LDS ring (the next K block's global loads are issued
// before the current block's MFMAs, written after them: one barrier per K block).  LDS tiles
// are [rows][64] bf16 (128-B rows) with the 16-B piece index XOR-swizzled by (row & 7), which
// makes every ds_read_b128 fragment read conflict-free (checked with the gfx950 lane-group
// rule).  The epilogue stages the fp32 accumulators through (padded) LDS so that bias,
// residual add, ReLU/SiLU and the bf16 store all run on 16-byte contiguous row pieces.
// Workgroup ids are remapped XCD-aware so that the N tiles of one M panel share an L2.
#include "conv_common.h"

namespace aiko {

// ConvParams: conv_common.h


// Occupancy per tile shape (waves per SIMD = resident 256-thread blocks per CU), bounded by LDS
// (2-deep ring + epilogue tile) and by the VGPR cap the launch bound imposes (512 / w):
// narrow / small tiles are latency-bound on low-K layers and need more resident blocks.
template <int BM, int BN>
constexpr int conv_occupancy() {
  return (BM * BN <= 64 * 64 || (BM == 128 && BN == 32)) ? 4 : (BM * BN <= 128 * 64 ? 3 : 2);
}

template <int BM, int BN>
__global__ __launch_bounds__(256, (conv_occupancy<BM, BN>())) void conv_igemm_kernel(ConvParams p) {
  constexpr int BK = 64;
  constexpr int WM = BM / 2, WN = BN / 2;      // per-wave tile
  constexpr int MI = WM / 16, NI = WN / 16;    // 16x16 MFMA tiles per wave
  constexpr int APT = BM / 32, BPT = BN / 32;  // 16-B pieces per thread per K block
  constexpr int STAGE_ELEMS = (BM + BN) * BK;  // one ring slot, bf16 elements
  constexpr int CPAD = 4;                      // fp32 pad per epilogue row (bank spread)
  constexpr int EPI_BYTES = BM * (BN + CPAD) * 4;
  constexpr int RING_BYTES = 2 * STAGE_ELEMS * 2;
  constexpr int LDS_BYTES = EPI_BYTES > RING_BYTES ? EPI_BYTES : RING_BYTES;
  __shared__ __attribute__((aligned(16))) unsigned char smem[LDS_BYTES];
  bf16_t* ring = reinterpret_cast<bf16_t*>(smem);

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wr = wave >> 1, wc = wave & 1;

  const int ntn = (p.Cout + BN - 1) / BN;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int tile_n = bid % ntn;
  const int tile_m = bid / ntn;
  const int m0 = tile_m * BM, n0 = tile_n * BN;

  // ---- per-thread gather setup ----
  const int piece = tid & 7;       // which 16-B piece of the 64-wide K block
  const int prow = tid >> 3;       // base row (0..31)
  const int HoWo = p.Ho * p.Wo;
  int a_base[APT], a_ih[APT], a_iw[APT];
#pragma unroll
  for (int i = 0; i < APT; ++i) {
    const int m = m0 + prow + 32 * i;
    if (m < p.M) {
      const int img = fdiv(m, p.mHoWo, p.lHoWo);
      const int rem = m - img * HoWo;
      const int oh = fdiv(rem, p.mWo, p.lWo);
      const int ow = rem - oh * p.Wo;
      a_ih[i] = oh * p.stride - p.pad;
      a_iw[i] = ow * p.stride - p.pad;
      a_base[i] = ((img * p.H + a_ih[i]) * p.W + a_iw[i]) * p.C;
    } else {
      a_ih[i] = -(1 << 28);  // never in bounds
      a_iw[i] = 0;
      a_base[i] = 0;
    }
  }
  int a2_base[APT];
  if (p.x2) {
#pragma unroll
    for (int i = 0; i < APT; ++i) {
      const int m = m0 + prow + 32 * i;
      if (m < p.M) {
        const int img = fdiv(m, p.mHoWo, p.lHoWo);
        const int rem = m - img * HoWo;
        const int oh = fdiv(rem, p.mWo, p.lWo);
        const int ow = rem - oh * p.Wo;
        a2_base[i] = ((img * p.H2 + oh * p.stride2) * p.W2 + ow * p.stride2) * p.C2;
      } else {
        a2_base[i] = -1;
      }
    }
  }

  // ---- epilogue operands prefetched now: their HBM latency hides under the K loop ----
  constexpr int CPR = BN / 8;             // 8-wide chunks per output row
  constexpr int CHUNKS = BM * CPR;
  constexpr int CPT = CHUNKS / 256;       // chunks per thread
  static_assert(CHUNKS % 256 == 0, "tile must give every thread whole chunks");
  const int e_cc = tid % CPR;             // this thread's column chunk (fixed: 256 % CPR == 0)
  const int e_row0 = tid / CPR;
  constexpr int E_ROWS = 256 / CPR;       // row stride between a thread's chunks
  const int e_n = n0 + e_cc * 8;
  float e_bias[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) e_bias[e] = 0.f;
  if (p.bias && e_n < p.Cout) {
    const f32x4 b0 = *reinterpret_cast<const f32x4*>(p.bias + e_n);
    const f32x4 b1 = *reinterpret_cast<const f32x4*>(p.bias + e_n + 4);
    e_bias[0] = b0[0]; e_bias[1] = b0[1]; e_bias[2] = b0[2]; e_bias[3] = b0[3];
    e_bias[4] = b1[0]; e_bias[5] = b1[1]; e_bias[6] = b1[2]; e_bias[7] = b1[3];
  }
  u32x4 e_res[CPT];
  if (p.res) {
#pragma unroll
    for (int i = 0; i < CPT; ++i) {
      const int m = m0 + e_row0 + E_ROWS * i;
      if (m < p.M && e_n < p.Cout) {
        e_res[i] = *reinterpret_cast<const u32x4*>(p.res + (size_t)m * p.ldr + e_n);
      } else {
        e_res[i] = u32x4{0u, 0u, 0u, 0u};
      }
    }
  }

  int b_off[BPT];
  bool b_ok[BPT];
#pragma unroll
  for (int i = 0; i < BPT; ++i) {
    const int n = n0 + prow + 32 * i;
    b_ok[i] = n < p.Cout;
    b_off[i] = (b_ok[i] ? n : 0) * p.K + piece * 8;
  }

  u32x4 ra[APT], rb[BPT];
  auto load_global = [&](int kb) {
    if (p.x2 && kb * BK >= p.K1) {          // block-uniform: second source (1x1 shortcut)
      const int c2 = kb * BK - p.K1 + piece * 8;
#pragma unroll
      for (int i = 0; i < APT; ++i) {
        if (a2_base[i] >= 0) {
          ra[i] = *reinterpret_cast<const u32x4*>(p.x2 + (a2_base[i] + c2));
        } else {
          ra[i] = u32x4{0u, 0u, 0u, 0u};
        }
      }
#pragma unroll
      for (int i = 0; i < BPT; ++i) {
        rb[i] = b_ok[i] ? *reinterpret_cast<const u32x4*>(p.w + (b_off[i] + kb * BK)) : u32x4{0u, 0u, 0u, 0u};
      }
      return;
    }
    const int koff = kb * BK + piece * 8;
    const int tap = fdiv(koff, p.mCc, p.lCc);  // K may be zero-padded past R*S*Cc: taps >= R*S meet zero weights
    const int c = koff - tap * p.Cc;
    const int r = fdiv(tap, p.mS, p.lS);
    const int s = tap - r * p.S;
    const int tap_off = (r * p.W + s) * p.C + c;
#pragma unroll
    for (int i = 0; i < APT; ++i) {
      const int ih = a_ih[i] + r, iw = a_iw[i] + s;
      const bool ok = (unsigned)ih < (unsigned)p.H && (unsigned)iw < (unsigned)p.W;
      if (ok) {
        ra[i] = *reinterpret_cast<const u32x4*>(p.x + (a_base[i] + tap_off));
      } else {
        ra[i] = u32x4{0u, 0u, 0u, 0u};
      }
    }
#pragma unroll
    for (int i = 0; i < BPT; ++i) {
      if (b_ok[i]) {
        rb[i] = *reinterpret_cast<const u32x4*>(p.w + (b_off[i] + kb * BK));
      } else {
        rb[i] = u32x4{0u, 0u, 0u, 0u};
      }
    }
  };

  auto store_lds = [&](int slot) {
    bf16_t* As = ring + slot * STAGE_ELEMS;
    bf16_t* Bs = As + BM * BK;
#pragma unroll
    for (int i = 0; i < APT; ++i) {
      const int row = prow + 32 * i;
      *reinterpret_cast<u32x4*>(As + row * BK + ((piece ^ (row & 7)) << 3)) = ra[i];
    }
#pragma unroll
    for (int i = 0; i < BPT; ++i) {
      const int row = prow + 32 * i;
      *reinterpret_cast<u32x4*>(Bs + row * BK + ((piece ^ (row & 7)) << 3)) = rb[i];
    }
  };

  f32x4 acc[MI][NI];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nkb = p.K / BK;
  load_global(0);
  store_lds(0);
  __syncthreads();

  const int fr = lane & 15;  // fragment row
  const int fq = lane >> 4;  // k quad

  for (int kb = 0; kb < nkb; ++kb) {
    const int cur = kb & 1;
    if (kb + 1 < nkb) load_global(kb + 1);
    const bf16_t* As = ring + cur * STAGE_ELEMS;
    const bf16_t* Bs = As + BM * BK;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8 af[MI], bfr[NI];
      const int pc = fq + 4 * kk;
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        const int row = wr * WM + i * 16 + fr;
        af[i] = *reinterpret_cast<const bf16x8*>(As + row * BK + ((pc ^ (row & 7)) << 3));
      }
#pragma unroll
      for (int j = 0; j < NI; ++j) {
        const int row = wc * WN + j * 16 + fr;
        bfr[j] = *reinterpret_cast<const bf16x8*>(Bs + row * BK + ((pc ^ (row & 7)) << 3));
      }
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NI; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    if (kb + 1 < nkb) store_lds(cur ^ 1);
    __syncthreads();
  }

  // ---- epilogue: accumulators -> padded fp32 LDS tile -> fused bias/residual/act -> bf16 ----
  float* Cs = reinterpret_cast<float*>(smem);
  constexpr int LDC = BN + CPAD;
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j) {
      const int col = wc * WN + j * 16 + fr;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int row = wr * WM + i * 16 + fq * 4 + e;
        Cs[row * LDC + col] = acc[i][j][e];
      }
    }
  __syncthreads();

#pragma unroll
  for (int i = 0; i < CPT; ++i) {
    const int row = e_row0 + E_ROWS * i;
    const int m = m0 + row;
    if (m >= p.M || e_n >= p.Cout) continue;
    const f32x4 v0 = *reinterpret_cast<const f32x4*>(Cs + row * LDC + e_cc * 8);
    const f32x4 v1 = *reinterpret_cast<const f32x4*>(Cs + row * LDC + e_cc * 8 + 4);
    float v[8] = {v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] += e_bias[e];
    const bool post = (p.act & 16) != 0;
    if (p.res && !post) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        v[2 * e] += __uint_as_float(e_res[i][e] << 16);
        v[2 * e + 1] += __uint_as_float(e_res[i][e] & 0xffff0000u);
      }
    }
    const int act = p.act & 15;
    if (act == 1) {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = fmaxf(v[e], 0.f);
    } else if (act == 2) {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = silu(v[e]);
    } else if (act == 3) {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = gelu_erf(v[e]);
    }
    if (p.res && post) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        v[2 * e] += __uint_as_float(e_res[i][e] << 16);
        v[2 * e + 1] += __uint_as_float(e_res[i][e] & 0xffff0000u);
      }
    }
    u32x4 o;
#pragma unroll
    for (int e = 0; e < 4; ++e) o[e] = pack2(v[2 * e], v[2 * e + 1]);
    *reinterpret_cast<u32x4*>(p.y + (size_t)m * p.ldy + e_n) = o;
  }
}

}  // namespace aiko

extern "C" int aiko_conv_igemm(const void* x, const void* w, const float* bias, const void* res,
                               void* y, int H, int W, int C, int Cc, int R, int S,
                               int stride, int pad, int Ho, int Wo, int M, int Cout, int K,
                               int act, int ldy, int ldr, int bm, int bn, const void* x2, int K1,
                               int H2, int W2, int C2, int stride2, hipStream_t stream) {
  using namespace aiko;
  ConvParams p;
  p.x = static_cast<const bf16_t*>(x);
  p.w = static_cast<const bf16_t*>(w);
  p.bias = bias;
  p.res = static_cast<const bf16_t*>(res);
  p.y = static_cast<bf16_t*>(y);
  p.H = H; p.W = W; p.C = C; p.Cc = Cc; p.R = R; p.S = S;
  p.stride = stride; p.pad = pad; p.Ho = Ho; p.Wo = Wo; p.M = M; p.Cout = Cout; p.K = K;
  p.act = act; p.ldy = ldy; p.ldr = ldr;
  p.x2 = static_cast<const bf16_t*>(x2);
  p.K1 = x2 ? K1 : K; p.H2 = H2; p.W2 = W2; p.C2 = C2; p.stride2 = stride2;
  conv_params_finalize(p);
  const int ntm = (M + bm - 1) / bm;
  const int ntn = (Cout + bn - 1) / bn;
  dim3 grid(ntm * ntn), block(256);
  if (bm == 128 && bn == 128) {
    conv_igemm_kernel<128, 128><<<grid, block, 0, stream>>>(p);
  } else if (bm == 128 && bn == 64) {
    conv_igemm_kernel<128, 64><<<grid, block, 0, stream>>>(p);
  } else if (bm == 64 && bn == 64) {
    conv_igemm_kernel<64, 64><<<grid, block, 0, stream>>>(p);
  } else if (bm == 64 && bn == 128) {
    conv_igemm_kernel<64, 128><<<grid, block, 0, stream>>>(p);
  } else if (bm == 128 && bn == 32) {
    conv_igemm_kernel<128, 32><<<grid, block, 0, stream>>>(p);
  } else if (bm == 256 && bn == 32) {
    conv_igemm_kernel<256, 32><<<grid, block, 0, stream>>>(p);
  } else {
    return -1;
  }
  return (int)hipGetLastError();
}
