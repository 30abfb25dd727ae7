// Torch operator registrations for the aiko_services_amd native library (torch.ops.aiko.*).
//
// Kernels live in csrc/kernels/*.hip behind plain extern "C" launchers (no torch headers in
// device code); this file validates shapes/dtypes/devices on the host — failing loudly, never
// falling back — and launches on the caller's current HIP stream so every op is capturable in
// a hipGraph (no allocation, no synchronisation inside a launch).
#include <ATen/ATen.h>
#include <c10/hip/HIPStream.h>
#include <torch/library.h>

#include <hip/hip_runtime.h>

#include <climits>
#include <vector>

extern "C" {
int aiko_conv_igemm(const void* x, const void* w, const float* bias, const void* res, void* y,
                    int H, int W, int C, int Cc, int R, int S, int stride, int pad, int Ho,
                    int Wo, int M, int Cout, int K, int act, int ldy, int ldr, int bm, int bn,
                    const void* x2, int K1, int H2, int W2, int C2, int stride2, hipStream_t stream);
int aiko_conv_buf(const void* x, const void* w, const float* bias, const void* res, void* y,
                  int H, int W, int C, int Cc, int R, int S, int stride, int pad, int Ho, int Wo,
                  int M, int Cout, int K, int act, int ldy, int ldr, int bm, int bn, const void* x2,
                  int K1, int H2, int W2, int C2, int stride2, int occ, int mf32, hipStream_t stream);
int aiko_conv_wide(const void* x, const void* w, const float* bias, const void* res, void* y,
                   int H, int W, int C, int Cc, int R, int S, int stride, int pad, int Ho, int Wo,
                   int M, int Cout, int K, int act, int ldy, int ldr, int bm, int bn, const void* x2,
                   int K1, int H2, int W2, int C2, int stride2, int occ, hipStream_t stream);
int aiko_conv_pw(const void* x, const void* w, const float* bias, const void* res, void* y, int M, int N,
                 int K, int ldx, int ldy, int ldr, int act, int cus, int mode, hipStream_t stream);
int aiko_conv_pw_dual(const void* x, const void* x2, const void* w, const float* bias, void* y, int M, int N,
                      int ldx, int ldx2, int ldy, int act, int Ho, int Wo, int H2, int W2, int s2, int cus,
                      hipStream_t stream);
int aiko_conv_persist(const void* x, const void* w, const float* bias, const void* res, void* y,
                      int H, int W, int C, int Cc, int R, int S, int stride, int pad, int Ho, int Wo,
                      int M, int Cout, int K, int act, int ldy, int ldr, int bm, int bn, const void* x2,
                      int K1, int H2, int W2, int C2, int stride2, hipStream_t stream);
int aiko_conv_glds_tail(const void* x, const void* w, const float* bias, int H, int W, int C, int Cc, int R, int S,
                        int stride, int pad, int Ho, int Wo, int M, int K, int N, int act, const void* w2, const float* b2,
                        void* y2, int ldy2, int ldw2, int act2, const void* zero, const int* dec, void* boxes,
                        float* scores, int* cls, hipStream_t stream);
int aiko_conv_glds(const void* x, const void* w, const float* bias, const void* res, void* y,
                   int H, int W, int C, int Cc, int R, int S, int stride, int pad, int Ho,
                   int Wo, int M, int Cout, int K, int act, int ldy, int ldr, int bm, int bn,
                   const void* x2, int K1, int H2, int W2, int C2, int stride2, const void* zero,
                   hipStream_t stream);
int aiko_preprocess(const void* in, void* out, int B, int Hin, int Win, int Ho, int Wo, int Hp,
                    int Wp, int pad_t, int pad_l, int Hc, int Wc, int off_t, int off_l, float fill,
                    const float* mean, const float* std, int bgr, hipStream_t stream);
int aiko_stem_direct(const void* in, void* out, const void* w, const float* bias, int B, int Hin, int Win,
                     int Ho, int Wo, int Hc, int Wc, int off_t, int off_l, float fill, const float* mean,
                     const float* std, int bgr, int H1, int W1, int Cout, int ldo, int k, int stride, int pad,
                     int act, hipStream_t stream);
int aiko_conv3x3_rows(const void* x, const void* wimg, const float* bias, const void* res, void* y, int B, int H,
                      int W, int ldx, int ldy, int ldr, int act, int grid, hipStream_t stream);
int aiko_conv3x3_patchw(const void* x, const void* wimg, const float* bias, void* y, int B, int H, int W, int ldx,
                        int ldy, int act, int grid, hipStream_t stream);
int aiko_conv3x3_patch(const void* x, const void* wimg, const float* bias, void* y, int B, int H, int W, int ldy,
                       int act, int grid, hipStream_t stream);
int aiko_bneck_fused(const void* x, const void* w1, const float* b1, const void* w2, const float* b2,
                     const void* w3, const float* b3, void* y, int B, int H, int W, int cin, int grid,
                     unsigned* dbg, hipStream_t stream);
int aiko_conv_chain(const void* A, const void* W1, const float* b1, const void* R, void* Y, const void* W2,
                    const float* b2, void* Z, const void* A2, int M, int K1, int N1, int N2, int grid,
                    hipStream_t stream);
int aiko_maxpool(const void* x, void* y, int B, int H, int W, int C, int Ho, int Wo, int k,
                 int s, int p, int ldx, int ldy, hipStream_t stream);
int aiko_resize_u8(const void* in, void* out, int B, int Hin, int Win, int Ho, int Wo, hipStream_t stream);
int aiko_batchnorm(const void* x, void* y, const float* scale, const float* shift, long P, int C, int ldx,
                   int ldy, int act, hipStream_t stream);
int aiko_upsample2x(const void* x, void* y, int B, int H, int W, int C, int ldx, int ldy,
                    hipStream_t stream);
int aiko_yolo_decode(const void* const* feats, const int* H, const int* W, const int* strides,
                     const int* ld, int nlev, int B, int nc, int reg_max, void* boxes,
                     float* scores, int* cls, hipStream_t stream);
int aiko_gemm_fp8(const void* a, const void* b, const float* sa, const float* sb, const float* bias,
                  const void* res, void* y, int M, int N, int K, int lda, int ldy, int ldr, int act,
                  int bm, int bn, int variant, const void* zero, const void* amx, int mxr, void* yq, void* ysc, int ldq, int ysr,
                  hipStream_t stream);
int aiko_rownorm_quant(const void* x, int ldx, const float* gamma, const float* beta, float eps,
                       void* yb, int ldyb, void* q, int ldq, float* qs, int M, int D, hipStream_t stream);
int aiko_c2f_fused(const void* x, int ldx, const void* w1, const float* b1, int k1, const void* wa, const float* ba,
                   int ka, const void* wb, const float* bb, int kb, const void* w2, const float* b2, int k2, void* y, int ldy,
                   int B, int H, int W, int CI, int C, int CO, int shortcut, int rb, const void* xu, int ldxu, int cu, hipStream_t stream);
int aiko_c2f_bneck(const void* x, int ldx, const void* wa, const float* ba, int ka, const void* wb, const float* bb,
                   int kb, void* y, int ldy, int B, int H, int W, int C, int shortcut, int rb, hipStream_t stream);
int aiko_linear_splitk(const void* x, const void* w, const float* bias, float* part, void* y, int M, int N, int K,
                       int ldx, int ldw, int ldy, int S, hipStream_t stream);
int aiko_attn_fwd(const void* q, const void* k, const void* v, void* o, int ldq, int ldk, int ldv,
                  int ldo, int B, int H, int T, int Tpad, int dh, float scale, void* work, long work_bytes,
                  void* oq, void* osc, int ldoq, int osr, hipStream_t stream);
int aiko_logmel(const float* audio, int B, int N, const float* mel, int n_mels, const int* mel_range,
                int n_fft, int hop, int F, float* logmel, int* gmax, void* dst, int rows, int pad, int ld,
                hipStream_t stream);
int aiko_topk_nms(const void* boxes, const float* scores, const int* cls, int B, int A,
                  int max_cand, int max_det, float conf, float iou, float max_wh, float gain,
                  float pad_l, float pad_t, float img_w, float img_h, float* det, int* count,
                  void* workspace, hipStream_t stream);
size_t aiko_topk_nms_workspace(int B);
int aiko_avgpool(const void* x, void* y, int B, int HW, int C, hipStream_t stream);
int aiko_mean_rows_f32(const void* x, float* y, int B, int T, int C, long ldb, hipStream_t stream);
int aiko_zero_border_rows(void* x, int B, int rows, int C, hipStream_t stream);
int aiko_sppf_pool(void* x, int B, int H, int W, int ld, int c, int k, hipStream_t stream);
int aiko_window_shift(const float* src, const float* chunk, float* dst, int B, int W, int n, hipStream_t stream);
int aiko_conv_narrow(const void* x, const void* w, const float* bias, const void* res, void* y, int H, int W, int C,
                     int Cc, int R, int S, int stride, int pad, int Ho, int Wo, int M, int Cout, int K, int act,
                     int ldy, int ldr, int th, int wreg, hipStream_t stream);
int aiko_stem_pool_u8(const void* frames, const void* w, const float* bias, void* y, int B, int Hi, int Wi,
                      int Ho, int Wo, int Hm, int Wm, int ldy, const float* mean255, int variant, hipStream_t stream);
int aiko_stem_pool(const void* x, const void* w, const float* bias, void* y, int B, int Hp, int Wp,
                   int Ho, int Wo, int Hm, int Wm, int ldy, int variant, hipStream_t stream);
int aiko_softmax_topk(const void* logits, float* prob, int* index, int B, int N, int k,
                      hipStream_t stream);
int aiko_embed_tokens(const int* ids, const int* pos, const void* tok, const void* pemb, void* x, int B,
                      int d, int ldx, int vocab, int n_pos, hipStream_t stream);
int aiko_attn_decode(const void* q, int ldq, void* k, void* v, int ldk, int ldv, int S, const int* pos,
                     int T, const void* knew, const void* vnew, int ldnew, void* o, int ldo, int B,
                     int H, float scale, float* work, long work_elems, hipStream_t stream);
long aiko_attn_decode_work(int B, int H, int maxlen);
int aiko_dec_linear(const void* x, int ldx, const float* gamma, const float* beta, float eps, const void* w,
                    const float* sw, const float* bias, const void* res, int ldr, void* y, int ldy, int M, int N,
                    int K, int act, hipStream_t stream);
int aiko_argmax_step(const void* logits, int ld, int V, int B, int* ids, int* pos, int* out_tokens,
                     int max_len, const int* forced, int n_forced, int eot, int* done, unsigned* counter,
                     hipStream_t stream);
}

namespace {

hipStream_t cur_stream() { return c10::hip::getCurrentHIPStream().stream(); }

void check_cuda(const at::Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda(), "aiko: ", name, " must be a GPU tensor");
}

// elements addressable from t.data_ptr() to the end of its storage
int64_t avail_elems(const at::Tensor& t) {
  return (int64_t)(t.storage().nbytes() / t.element_size()) - t.storage_offset();
}

void check_launch(int rc, const char* what) {
  TORCH_CHECK(rc == 0, "aiko: launch of ", what, " failed: ",
              rc < 0 ? "unsupported configuration" : hipGetErrorString((hipError_t)rc));
}

// geom = [H, W, C, Cc, R, S, stride, pad, Ho, Wo, M, act, ldy, ldr, bm, bn,
//         K1, H2, W2, C2, stride2 (the optional second source x2), [variant]]
// variant 0: register-staged kernel (conv_igemm.hip); 1: LDS-DMA kernel (conv_glds.hip), which
// needs ``zero`` (>= 16 B of zeros on the device) as the source of conv padding; 2: buffer
// LDS-DMA kernel (conv_buf.hip, padding by out-of-range buffer reads); 3 / 5 / 6: conv_buf at high
// occupancy / on 32x32x16 MFMA / as 4-wave wide tiles; 4: persistent conv_buf; 7: direct 3x3 kernel
// for narrow layers (conv_narrow.hip); 8: 8-wave wide tiles with a register-direct epilogue
// (conv_wide.hip); 9: the same kernel at several workgroups per CU; 18: conv_wide with exact-N
// tiles (BN = 80 or 144 channels computed per tile).
void conv_igemm_out(const at::Tensor& x, const c10::optional<at::Tensor>& x2, const at::Tensor& w,
                    const c10::optional<at::Tensor>& bias, const c10::optional<at::Tensor>& res,
                    at::Tensor& y, at::IntArrayRef geom, const c10::optional<at::Tensor>& zero) {
  TORCH_CHECK(geom.size() == 21 || geom.size() == 22, "aiko.conv_igemm_out: geom needs 21 or 22 ints");
  const int64_t variant = geom.size() == 22 ? geom[21] : 0;
  const int64_t H = geom[0], W = geom[1], C = geom[2], Cc = geom[3], R = geom[4], S = geom[5];
  const int64_t stride = geom[6], pad = geom[7], Ho = geom[8], Wo = geom[9], M = geom[10];
  const int64_t act = geom[11], ldy = geom[12], ldr = geom[13], bm = geom[14], bn = geom[15];
  const int64_t K1 = geom[16], H2 = geom[17], W2 = geom[18], C2 = geom[19], stride2 = geom[20];
  check_cuda(x, "x");
  check_cuda(w, "w");
  check_cuda(y, "y");
  TORCH_CHECK(x.scalar_type() == at::kBFloat16 && w.scalar_type() == at::kBFloat16 &&
                  y.scalar_type() == at::kBFloat16,
              "aiko.conv_igemm_out: x, w, y must be bfloat16");
  TORCH_CHECK(w.dim() == 2 && w.is_contiguous(), "aiko.conv_igemm_out: w must be [Cout, K] contiguous");
  const int64_t Cout = w.size(0), K = w.size(1);
  const bool dual = x2.has_value() && x2->defined();
  const int64_t Kmain = dual ? K1 : K;
  TORCH_CHECK(Kmain >= R * S * Cc && Kmain % 64 == 0 && Kmain - R * S * Cc < 64, "aiko.conv_igemm_out: K=",
              Kmain, " must be R*S*Cc rounded up to a multiple of 64");
  const void* x2ptr = nullptr;
  if (dual) {
    check_cuda(*x2, "x2");
    TORCH_CHECK(x2->scalar_type() == at::kBFloat16, "aiko.conv_igemm_out: x2 must be bf16");
    TORCH_CHECK((K - K1) % 64 == 0 && K - K1 <= C2 && C2 % 8 == 0 && K1 > 0,
                "aiko.conv_igemm_out: second source needs K-K1 (multiple of 64) <= C2");
    TORCH_CHECK(reinterpret_cast<uintptr_t>(x2->data_ptr()) % 16 == 0, "aiko.conv_igemm_out: x2 alignment");
    TORCH_CHECK(M % (Ho * Wo) == 0 && (Ho - 1) * stride2 < H2 && (Wo - 1) * stride2 < W2 &&
                    avail_elems(*x2) >= (M / (Ho * Wo)) * H2 * W2 * C2,
                "aiko.conv_igemm_out: x2 too small for the output geometry");
    x2ptr = x2->data_ptr();
  }
  TORCH_CHECK(Cc % 8 == 0 && (Cc <= C || C == 4), "aiko.conv_igemm_out: Cc must be a multiple of 8 within the pixel pitch (or span pixels of a 4-channel stem input)");
  TORCH_CHECK(Cout % 8 == 0, "aiko.conv_igemm_out: Cout must be a multiple of 8");
  TORCH_CHECK(C % 8 == 0 || (C == 4 && Cc % 8 == 0), "aiko.conv_igemm_out: pixel pitch must keep 16-B alignment");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0 &&
                  reinterpret_cast<uintptr_t>(y.data_ptr()) % 16 == 0,
              "aiko.conv_igemm_out: x and y must be 16-byte aligned");
  // x / y / residual may be channel-slice views (concat buffers): bound by storage extent
  const int64_t x_extent = avail_elems(x);
  TORCH_CHECK(x_extent < INT_MAX && w.numel() < INT_MAX, "aiko.conv_igemm_out: tensor too large for 32-bit offsets");
  TORCH_CHECK(ldy % 8 == 0 && ldy >= Cout, "aiko.conv_igemm_out: bad ldy");
  TORCH_CHECK(avail_elems(y) >= (M - 1) * ldy + Cout, "aiko.conv_igemm_out: y too small");
  const int64_t img_elems = H * W * C;
  // (the stem's 32-element chunks span pixels inside a row; its geometry keeps them in-row)
  const int64_t tail = Cc <= C ? Cc : C;
  TORCH_CHECK(M % (Ho * Wo) == 0 && x_extent >= (M / (Ho * Wo) - 1) * img_elems + (H * W - 1) * C + tail,
              "aiko.conv_igemm_out: x too small for M");
  const float* bptr = nullptr;
  if (bias.has_value() && bias->defined()) {
    check_cuda(*bias, "bias");
    TORCH_CHECK(bias->scalar_type() == at::kFloat && bias->numel() == Cout && bias->is_contiguous(),
                "aiko.conv_igemm_out: bias must be fp32 [Cout]");
    bptr = bias->data_ptr<float>();
  }
  const void* rptr = nullptr;
  if (res.has_value() && res->defined()) {
    check_cuda(*res, "residual");
    TORCH_CHECK(res->scalar_type() == at::kBFloat16, "aiko.conv_igemm_out: residual must be bf16");
    TORCH_CHECK(ldr % 8 == 0 && avail_elems(*res) >= (M - 1) * ldr + Cout, "aiko.conv_igemm_out: bad residual");
    rptr = res->data_ptr();
  }
  int rc;
  if (variant == 7) {
    // direct 3x3 kernel for narrow layers (conv_narrow.hip): Cc, Cout in {16, 32}, pad 1, stride 1/2
    TORCH_CHECK(!dual && ((R == 3 && S == 3 && pad == 1 && (stride == 1 || stride == 2)) ||
                          (R == 1 && S == 1 && pad == 0 && stride == 1)) &&
                    (Cc == 16 || Cc == 32) && (Cout == 16 || Cout == 32),
                "aiko.conv_igemm_out: variant 7 needs a 3x3 / pad 1 / stride 1-2 or 1x1 / stride 1 conv with Cc, Cout in {16, 32}");
    rc = aiko_conv_narrow(x.data_ptr(), w.data_ptr(), bptr, rptr, y.data_ptr(), H, W, C, Cc, R, S, stride, pad, Ho,
                          Wo, M, Cout, K, act, ldy, ldr, bm == 16 ? 16 : 8, bn == 64 ? 1 : 0, cur_stream());
  } else if (variant == 8 || variant == 9 || variant == 11 || variant == 18 || variant == 19 || variant == 20) {
    // 8-wave wide tiles, transposed product, register-direct epilogue (conv_wide.hip)
    TORCH_CHECK(Cc % 64 == 0 && R * S <= 32 && x_extent * 2 < (1LL << 31) - 64 && w.numel() * 2 < (1LL << 31),
                "aiko.conv_igemm_out: variant 8 needs Cc % 64 == 0, R*S <= 32 and operands < 2 GiB");
    TORCH_CHECK(!dual || avail_elems(*x2) * 2 < (1LL << 31) - 64, "aiko.conv_igemm_out: x2 too large for variant 8");
    TORCH_CHECK(ldy % 8 == 0 && (!rptr || (ldr % 8 == 0 && reinterpret_cast<uintptr_t>(rptr) % 16 == 0)),
                "aiko.conv_igemm_out: variant 8 needs 16-B aligned rows");
    rc = aiko_conv_wide(x.data_ptr(), w.data_ptr(), bptr, rptr, y.data_ptr(), H, W, C, Cc, R, S, stride,
                        pad, Ho, Wo, M, Cout, K, act, ldy, ldr, bm, bn, x2ptr, K1, H2, W2, C2, stride2,
                        variant == 18 ? 18 : variant == 19 ? 19 : variant == 20 ? 20 : variant == 11 ? 11 : (variant == 9 ? 2 : 1), cur_stream());
  } else if (variant == 13 && dual) {
    // fused projection on the resident-weight pointwise kernel (conv_pw.hip): 1x1 main source of
    // 128 channels + a 1x1 / stride-s2 second source of 256 channels
    TORCH_CHECK(R == 1 && S == 1 && stride == 1 && pad == 0 && Cc == 128 && K1 == 128 && K == 384 &&
                    Cout % 128 == 0 && C % 8 == 0 && !rptr && x_extent * 2 < (1LL << 31) - 64 &&
                    avail_elems(*x2) * 2 < (1LL << 31) - 64 && avail_elems(y) * 2 < (1LL << 31) && ldy % 8 == 0,
                "aiko.conv_igemm_out: variant 13 with a second source needs a 128 + 256 column 1x1 projection, "
                "Cout % 128 == 0, no residual and operands < 2 GiB");
    TORCH_CHECK(!bptr || reinterpret_cast<uintptr_t>(bptr) % 16 == 0, "aiko.conv_igemm_out: bias alignment");
    int dev = 0, cus = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) cus = 256;
    rc = aiko_conv_pw_dual(x.data_ptr(), x2ptr, w.data_ptr(), bptr, y.data_ptr(), M, Cout, C, C2, ldy, act, Ho, Wo,
                           H2, W2, stride2, cus, cur_stream());
  } else if (variant == 12 || variant == 13 || variant == 14) {
    // persistent pointwise GEMM (conv_pw.hip): 1x1 / stride 1 / one source, K % 256 == 0,
    // Cout % 128 == 0, x rows = pixels at pitch C
    const bool pw_shape = variant == 12 ? (K % 256 == 0 && Cout % 128 == 0)
                                        : ((K == 128 && Cout % 256 == 0) || (K == 256 && Cout % 128 == 0) ||
                                           (K == 512 && Cout % 64 == 0));
    TORCH_CHECK(!dual && R == 1 && S == 1 && stride == 1 && pad == 0 && Cc == K && pw_shape &&
                    C % 8 == 0 && x_extent * 2 < (1LL << 31) - 64 && w.numel() * 2 < (1LL << 31) &&
                    avail_elems(y) * 2 < (1LL << 31),
                "aiko.conv_igemm_out: variants 12/13 need a 1x1/s1 single-source conv with K % 256 == 0 "
                "(13: K = 128 / 256 / 512), Cout a multiple of the channel block and operands < 2 GiB");
    TORCH_CHECK(ldy % 8 == 0 && (!rptr || (ldr % 8 == 0 && reinterpret_cast<uintptr_t>(rptr) % 16 == 0 &&
                                          avail_elems(*res) * 2 < (1LL << 31) - 64)),
                "aiko.conv_igemm_out: variant 12 needs 16-B aligned rows");
    TORCH_CHECK(!bptr || reinterpret_cast<uintptr_t>(bptr) % 16 == 0, "aiko.conv_igemm_out: bias alignment");
    static int cus = 0;
    if (cus == 0) {
      int dev = 0, n = 0;
      (void)hipGetDevice(&dev);
      if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
      cus = n;
    }
    rc = aiko_conv_pw(x.data_ptr(), w.data_ptr(), bptr, rptr, y.data_ptr(), M, Cout, K, C, ldy, ldr, act, cus,
                      variant == 13 ? 1 : variant == 14 ? 2 : 0, cur_stream());
  } else if (variant == 4) {
    // persistent buffer-LDS-DMA kernel: one K-block stream across each workgroup's run of tiles
    TORCH_CHECK(Cc % 64 == 0 && R * S <= 32 && K % 64 == 0 && x_extent * 2 < (1LL << 31) - 64 &&
                    w.numel() * 2 < (1LL << 31),
                "aiko.conv_igemm_out: variant 4 needs Cc % 64 == 0, R*S <= 32 and operands < 2 GiB");
    TORCH_CHECK(!dual || avail_elems(*x2) * 2 < (1LL << 31) - 64, "aiko.conv_igemm_out: x2 too large for variant 4");
    rc = aiko_conv_persist(x.data_ptr(), w.data_ptr(), bptr, rptr, y.data_ptr(), H, W, C, Cc, R, S, stride,
                           pad, Ho, Wo, M, Cout, K, act, ldy, ldr, bm, bn, x2ptr, K1, H2, W2, C2, stride2,
                           cur_stream());
  } else if (variant == 2 || variant == 3 || variant == 5 || variant == 6) {
    // buffer-LDS-DMA kernel: 64-channel K blocks inside one tap, byte offsets in 31 bits;
    // variant 3 = the same kernel at forced high occupancy (64x64: 5, 64x128 / 128x64: 3 WG/CU)
    TORCH_CHECK(Cc % 64 == 0 && R * S <= 32 && x_extent * 2 < (1LL << 31) - 64 && w.numel() * 2 < (1LL << 31),
                "aiko.conv_igemm_out: variant 2 needs Cc % 64 == 0, R*S <= 32 and operands < 2 GiB");
    TORCH_CHECK(!dual || avail_elems(*x2) * 2 < (1LL << 31) - 64, "aiko.conv_igemm_out: x2 too large for variant 2");
    rc = aiko_conv_buf(x.data_ptr(), w.data_ptr(), bptr, rptr, y.data_ptr(), H, W, C, Cc, R, S, stride,
                       pad, Ho, Wo, M, Cout, K, act, ldy, ldr, bm, bn, x2ptr, K1, H2, W2, C2, stride2,
                       variant == 3 ? (bm == 64 && bn == 64 ? 5 : 3) : (variant == 6 ? 1 : 0), variant == 5 ? 1 : 0,
                       cur_stream());
  } else if (variant == 1) {
    TORCH_CHECK(zero.has_value() && zero->defined() && zero->is_cuda() && zero->nbytes() >= 16 &&
                    reinterpret_cast<uintptr_t>(zero->data_ptr()) % 16 == 0,
                "aiko.conv_igemm_out: the LDS-DMA variant needs a zero page tensor (>= 16 B)");
    rc = aiko_conv_glds(x.data_ptr(), w.data_ptr(), bptr, rptr, y.data_ptr(), H, W, C, Cc, R, S, stride,
                        pad, Ho, Wo, M, Cout, K, act, ldy, ldr, bm, bn, x2ptr, K1, H2, W2, C2, stride2,
                        zero->data_ptr(), cur_stream());
  } else {
    rc = aiko_conv_igemm(x.data_ptr(), w.data_ptr(), bptr, rptr, y.data_ptr(), H, W, C, Cc, R, S, stride,
                         pad, Ho, Wo, M, Cout, K, act, ldy, ldr, bm, bn, x2ptr, K1, H2, W2, C2, stride2,
                         cur_stream());
  }
  check_launch(rc, "conv_igemm");
}

// canvas = [Hc, Wc, off_t, off_l, fill]: the frame is resized to (Ho, Wo) and placed at
// (off_t, off_l) inside an Hc x Wc canvas of colour ``fill`` at (pad_t, pad_l) of ``out``.
void preprocess_out(const at::Tensor& frames, at::Tensor& out, int64_t Ho, int64_t Wo,
                    int64_t pad_t, int64_t pad_l, at::ArrayRef<double> mean,
                    at::ArrayRef<double> std, bool bgr, at::ArrayRef<double> canvas) {
  check_cuda(frames, "frames");
  check_cuda(out, "out");
  TORCH_CHECK(frames.scalar_type() == at::kByte && frames.dim() == 4 && frames.size(3) == 3 &&
                  frames.is_contiguous(),
              "aiko.preprocess_out: frames must be uint8 [B, H, W, 3] contiguous");
  TORCH_CHECK(out.scalar_type() == at::kBFloat16 && out.dim() == 4 && out.size(3) == 4 &&
                  out.is_contiguous() && out.size(0) == frames.size(0),
              "aiko.preprocess_out: out must be bf16 [B, Hp, Wp, 4] contiguous");
  TORCH_CHECK(mean.size() == 3 && std.size() == 3, "aiko.preprocess_out: mean/std need 3 values");
  int64_t Hc = Ho, Wc = Wo, off_t = 0, off_l = 0;
  double fill = 0.0;
  if (!canvas.empty()) {
    TORCH_CHECK(canvas.size() == 5, "aiko.preprocess_out: canvas = [Hc, Wc, off_t, off_l, fill]");
    Hc = (int64_t)canvas[0]; Wc = (int64_t)canvas[1];
    off_t = (int64_t)canvas[2]; off_l = (int64_t)canvas[3]; fill = canvas[4];
  }
  TORCH_CHECK(off_t >= 0 && off_l >= 0 && off_t + Ho <= Hc && off_l + Wo <= Wc,
              "aiko.preprocess_out: image must lie inside the canvas");
  TORCH_CHECK(pad_t + Hc <= out.size(1) && pad_l + Wc <= out.size(2), "aiko.preprocess_out: out too small");
  float m[3] = {(float)mean[0], (float)mean[1], (float)mean[2]};
  float s[3] = {(float)std[0], (float)std[1], (float)std[2]};
  const int rc = aiko_preprocess(frames.data_ptr(), out.data_ptr(), frames.size(0), frames.size(1),
                                 frames.size(2), Ho, Wo, out.size(1), out.size(2), pad_t, pad_l,
                                 Hc, Wc, off_t, off_l, (float)fill, m, s, bgr ? 1 : 0, cur_stream());
  check_launch(rc, "preprocess");
}

int64_t pixel_pitch(const at::Tensor& t, const char* op);

// 3x3 / stride 1 / pad 1 conv, 64 -> 64 channels, with an LDS-resident input patch (conv_patch.hip).
// x [B, H, W, 64] contiguous; wimg the [9, 2, 4, 64, 8] fragment image (ops.conv.patch_weight);
// y [B, H, W, >= 64] NHWC with unit channel stride (a channel slice of a wider buffer is fine).
void conv3x3_patch_out(const at::Tensor& x, const at::Tensor& wimg, const c10::optional<at::Tensor>& bias,
                       at::Tensor& y, int64_t act, int64_t grid) {
  check_cuda(x, "x");
  check_cuda(wimg, "wimg");
  check_cuda(y, "y");
  TORCH_CHECK(x.scalar_type() == at::kBFloat16 && wimg.scalar_type() == at::kBFloat16 && y.scalar_type() == at::kBFloat16,
              "aiko.conv3x3_patch_out: bf16 tensors");
  TORCH_CHECK(x.dim() == 4 && x.size(3) == 64 && x.is_contiguous(), "aiko.conv3x3_patch_out: x must be [B, H, W, 64] contiguous");
  TORCH_CHECK(wimg.is_contiguous() && wimg.numel() == 9 * 64 * 64, "aiko.conv3x3_patch_out: wimg must be the 36864-element image");
  const int64_t B = x.size(0), H = x.size(1), W = x.size(2);
  TORCH_CHECK(W + 8 <= 64, "aiko.conv3x3_patch_out: W <= 56");
  TORCH_CHECK(y.dim() == 4 && y.size(0) == B && y.size(1) == H && y.size(2) == W && y.size(3) == 64 && y.stride(3) == 1 &&
                  y.stride(2) % 8 == 0 && y.stride(1) == W * y.stride(2) && y.stride(0) == H * W * y.stride(2) &&
                  reinterpret_cast<uintptr_t>(y.data_ptr()) % 16 == 0,
              "aiko.conv3x3_patch_out: y must be [B, H, W, 64] NHWC (16-B aligned pixel pitch)");
  TORCH_CHECK(x.numel() * 2 < (1LL << 31) - 64 && avail_elems(y) * 2 < (1LL << 31) - 64,
              "aiko.conv3x3_patch_out: tensors too large for 32-bit offsets");
  TORCH_CHECK(act == 0 || act == 1 || act == 2, "aiko.conv3x3_patch_out: act none / relu / silu");
  const float* bptr = nullptr;
  if (bias.has_value() && bias->defined()) {
    check_cuda(*bias, "bias");
    TORCH_CHECK(bias->scalar_type() == at::kFloat && bias->numel() == 64, "aiko.conv3x3_patch_out: bias fp32 [64]");
    bptr = bias->data_ptr<float>();
  }
  check_launch(aiko_conv3x3_patch(x.data_ptr(), wimg.data_ptr(), bptr, y.data_ptr(), (int)B, (int)H, (int)W,
                                  (int)y.stride(2), (int)act, (int)grid, cur_stream()),
               "conv3x3_patch");
}

// 3x3 / stride 1 / pad 1 conv, 128 -> 128 channels, W = 28, patch per 14-row tile with streamed
// weights (conv_patchw.hip).  x [B, H, 28, >= 128] NHWC (16-B aligned pixel pitch); wimg the
// [4, 9, 8, 64, 8] fragment image (ops.conv.patchw_weight); y [B, H, 28, >= 128] NHWC.
void conv3x3_patchw_out(const at::Tensor& x, const at::Tensor& wimg, const c10::optional<at::Tensor>& bias,
                        at::Tensor& y, int64_t act, int64_t grid) {
  check_cuda(x, "x");
  check_cuda(wimg, "wimg");
  check_cuda(y, "y");
  TORCH_CHECK(x.scalar_type() == at::kBFloat16 && wimg.scalar_type() == at::kBFloat16 && y.scalar_type() == at::kBFloat16,
              "aiko.conv3x3_patchw_out: bf16 tensors");
  TORCH_CHECK(x.dim() == 4 && x.size(3) >= 128 && x.size(2) == 28 && x.stride(3) == 1 && x.stride(2) % 8 == 0 &&
                  x.stride(1) == 28 * x.stride(2) && x.stride(0) == x.size(1) * x.stride(1) &&
                  reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0,
              "aiko.conv3x3_patchw_out: x must be [B, H, 28, >= 128] NHWC with a 16-B aligned pixel pitch");
  TORCH_CHECK(wimg.is_contiguous() && wimg.numel() == 9 * 128 * 128, "aiko.conv3x3_patchw_out: wimg must be the 147456-element image");
  const int64_t B = x.size(0), H = x.size(1), W = x.size(2);
  TORCH_CHECK(y.dim() == 4 && y.size(0) == B && y.size(1) == H && y.size(2) == W && y.size(3) == 128 && y.stride(3) == 1 &&
                  y.stride(2) % 8 == 0 && y.stride(1) == W * y.stride(2) && y.stride(0) == H * W * y.stride(2) &&
                  reinterpret_cast<uintptr_t>(y.data_ptr()) % 16 == 0,
              "aiko.conv3x3_patchw_out: y must be [B, H, 28, 128] NHWC (16-B aligned pixel pitch)");
  TORCH_CHECK(avail_elems(x) * 2 < (1LL << 31) - 64 && avail_elems(y) * 2 < (1LL << 31) - 64,
              "aiko.conv3x3_patchw_out: tensors too large for 32-bit offsets");
  TORCH_CHECK(act == 0 || act == 1, "aiko.conv3x3_patchw_out: act none / relu");
  const float* bptr = nullptr;
  if (bias.has_value() && bias->defined()) {
    check_cuda(*bias, "bias");
    TORCH_CHECK(bias->scalar_type() == at::kFloat && bias->numel() == 128, "aiko.conv3x3_patchw_out: bias fp32 [128]");
    bptr = bias->data_ptr<float>();
  }
  check_launch(aiko_conv3x3_patchw(x.data_ptr(), wimg.data_ptr(), bptr, y.data_ptr(), (int)B, (int)H, (int)W,
                                   (int)x.stride(2), (int)y.stride(2), (int)act, (int)grid, cur_stream()),
               "conv3x3_patchw");
}

// 3x3 / stride 1 / pad 1 conv, 32 -> 32 channels, W = 80, as a persistent row stream
// (conv_rows.hip).  x / res / y: [B, H, 80, >= 32] NHWC views whose rows are uniformly strided
// (channel slices of wider buffers are fine); wimg the [9, 2, 64, 8] fragment image
// (ops.conv.rows_weight).  act bits 0-3: none / ReLU / SiLU, bit 4: residual after the activation.
void conv3x3_rows_out(const at::Tensor& x, const at::Tensor& wimg, const c10::optional<at::Tensor>& bias,
                      const c10::optional<at::Tensor>& res, at::Tensor& y, int64_t act, int64_t grid) {
  check_cuda(x, "x");
  check_cuda(wimg, "wimg");
  check_cuda(y, "y");
  auto rows_ok = [](const at::Tensor& t, int64_t B, int64_t H) {
    return t.dim() == 4 && t.size(0) == B && t.size(1) == H && t.size(2) == 80 && t.size(3) >= 32 && t.stride(3) == 1 &&
           t.stride(2) % 8 == 0 && t.stride(1) == 80 * t.stride(2) && t.stride(0) == H * t.stride(1) &&
           reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0 && t.scalar_type() == at::kBFloat16 &&
           avail_elems(t) * 2 < (1LL << 31) - 64;
  };
  const int64_t B = x.size(0), H = x.size(1);
  TORCH_CHECK(rows_ok(x, B, H), "aiko.conv3x3_rows_out: x must be [B, H, 80, >= 32] bf16 with uniformly strided rows");
  TORCH_CHECK(rows_ok(y, B, H) && y.size(3) == 32, "aiko.conv3x3_rows_out: y must be [B, H, 80, 32] bf16 (a slice is fine)");
  TORCH_CHECK(wimg.is_contiguous() && wimg.numel() == 9 * 32 * 32 && wimg.scalar_type() == at::kBFloat16,
              "aiko.conv3x3_rows_out: wimg must be the 9216-element bf16 image");
  const void* rptr = nullptr;
  int64_t ldr = 0;
  if (res.has_value() && res->defined()) {
    check_cuda(*res, "res");
    TORCH_CHECK(rows_ok(*res, B, H), "aiko.conv3x3_rows_out: res must be [B, H, 80, >= 32] bf16 with uniformly strided rows");
    rptr = res->data_ptr();
    ldr = res->stride(2);
  }
  TORCH_CHECK((act & 15) <= 2 && (act & ~31) == 0, "aiko.conv3x3_rows_out: act none / relu / silu (+16: residual after)");
  const float* bptr = nullptr;
  if (bias.has_value() && bias->defined()) {
    check_cuda(*bias, "bias");
    TORCH_CHECK(bias->scalar_type() == at::kFloat && bias->numel() == 32, "aiko.conv3x3_rows_out: bias fp32 [32]");
    bptr = bias->data_ptr<float>();
  }
  check_launch(aiko_conv3x3_rows(x.data_ptr(), wimg.data_ptr(), bptr, rptr, y.data_ptr(), (int)B, (int)H, 80,
                                 (int)x.stride(2), (int)y.stride(2), (int)ldr, (int)act, (int)grid, cur_stream()),
               "conv3x3_rows");
}

// Chained 1x1 convs at a bottleneck boundary (conv_chain.hip):
//   Y = relu(A W1^T + b1 + R) [M, N1],  Z = relu(Y W2^T + b2) [M, N2]
//   (K1, N1, N2) in {(64, 256, 64), (64, 256, 128), (128, 512, 128), (128, 512, 256)}
void conv_chain_out(const at::Tensor& A, const at::Tensor& W1, const at::Tensor& b1, const c10::optional<at::Tensor>& R_opt,
                    at::Tensor& Y, const at::Tensor& W2, const at::Tensor& b2, at::Tensor& Z, int64_t grid,
                    const c10::optional<at::Tensor>& A2_opt) {
  const bool dual = A2_opt.has_value() && A2_opt->defined();
  TORCH_CHECK(dual != (R_opt.has_value() && R_opt->defined()),
              "aiko.conv_chain_out: exactly one of R (identity residual) and A2 (fused projection shortcut)");
  const at::Tensor& R = dual ? *A2_opt : *R_opt;   // (validated by the dual branch below when dual)
  for (const at::Tensor* t : {&A, &W1, &b1, &R, (const at::Tensor*)&Y, &W2, &b2, (const at::Tensor*)&Z}) {
    check_cuda(*t, "conv_chain operand");
    TORCH_CHECK(t->is_contiguous() && reinterpret_cast<uintptr_t>(t->data_ptr()) % 16 == 0,
                "aiko.conv_chain_out: operands must be contiguous and 16-byte aligned");
  }
  for (const at::Tensor* t : {&A, &W1, &R, (const at::Tensor*)&Y, &W2, (const at::Tensor*)&Z})
    TORCH_CHECK(t->scalar_type() == at::kBFloat16, "aiko.conv_chain_out: bf16 activations / weights");
  TORCH_CHECK(b1.scalar_type() == at::kFloat && b2.scalar_type() == at::kFloat, "aiko.conv_chain_out: fp32 biases");
  TORCH_CHECK(W1.dim() == 2 && W2.dim() == 2, "aiko.conv_chain_out: W1 / W2 [Cout, K]");
  const int64_t N1 = W1.size(0), K1 = W1.size(1), N2 = W2.size(0);
  const bool shape_ok = dual ? (K1 == 128 && N1 == 256 && N2 == 64)
                             : ((K1 == 64 && N1 == 256 && (N2 == 64 || N2 == 128)) ||
                                (K1 == 128 && N1 == 512 && (N2 == 128 || N2 == 256)) ||
                                (K1 == 256 && N1 == 1024 && N2 == 256));
  TORCH_CHECK(shape_ok, "aiko.conv_chain_out: unsupported (K1, N1, N2) = (", K1, ", ", N1, ", ", N2, ")", dual ? " dual" : "");
  const int64_t ka = dual ? K1 / 2 : K1;           // width of each A source
  const int64_t M = A.numel() / ka;
  TORCH_CHECK(A.size(-1) == ka && b1.numel() == N1 && W2.size(1) == N1 && b2.numel() == N2,
              "aiko.conv_chain_out: A [.., K1 (or K1/2 per source)], b1 [N1], W2 [N2, N1], b2 [N2]");
  if (dual) {
    TORCH_CHECK(R.numel() == M * ka && R.size(-1) == ka, "aiko.conv_chain_out: A2 [M, K1/2]");
  } else {
    TORCH_CHECK(R.numel() == M * N1 && R.size(-1) == N1, "aiko.conv_chain_out: R [M, N1]");
  }
  TORCH_CHECK(Y.numel() == M * N1 && Y.size(-1) == N1 && Z.numel() == M * N2 && Z.size(-1) == N2,
              "aiko.conv_chain_out: Y [M, N1], Z [M, N2]");
  TORCH_CHECK(M % 64 == 0, "aiko.conv_chain_out: M must be a multiple of 64");
  check_launch(aiko_conv_chain(A.data_ptr(), W1.data_ptr(), b1.data_ptr<float>(), dual ? nullptr : R.data_ptr(),
                               Y.data_ptr(), W2.data_ptr(), b2.data_ptr<float>(), Z.data_ptr(),
                               dual ? R.data_ptr() : nullptr, M, K1, N1, N2, grid, cur_stream()),
               "conv_chain");
}

// A YOLOv8 C2f block with one bottleneck in one launch (c2f_fused.hip): x [B, H, W, >= CI] ->
// y [B, H, W, >= CO]; weights / biases as the four ConvSpecs hold them (cv1, conv a, conv b, cv2:
// [Cout, K padded] bf16 + fp32 biases, SiLU everywhere).  Shapes without an instantiation fail.
void c2f_fused_out(const at::Tensor& x, const at::Tensor& w1, const at::Tensor& b1, const at::Tensor& wa,
                   const at::Tensor& ba, const at::Tensor& wb, const at::Tensor& bb, const at::Tensor& w2,
                   const at::Tensor& b2, at::Tensor& y, int64_t ci, bool shortcut, int64_t rb,
                   const c10::optional<at::Tensor>& xu_opt) {
  for (const at::Tensor* t : {&x, &w1, &b1, &wa, &ba, &wb, &bb, &w2, &b2, (const at::Tensor*)&y}) check_cuda(*t, "c2f operand");
  for (const at::Tensor* t : {&x, &w1, &wa, &wb, &w2, (const at::Tensor*)&y})
    TORCH_CHECK(t->scalar_type() == at::kBFloat16, "aiko.c2f_fused_out: bf16 activations / weights");
  for (const at::Tensor* t : {&b1, &ba, &bb, &b2})
    TORCH_CHECK(t->scalar_type() == at::kFloat && t->is_contiguous(), "aiko.c2f_fused_out: fp32 contiguous biases");
  for (const at::Tensor* t : {&w1, &wa, &wb, &w2})
    TORCH_CHECK(t->dim() == 2 && t->is_contiguous() && t->size(1) % 8 == 0, "aiko.c2f_fused_out: weights [Cout, K] contiguous");
  TORCH_CHECK(x.dim() == 4 && y.dim() == 4 && x.size(0) == y.size(0) && x.size(1) == y.size(1) && x.size(2) == y.size(2),
              "aiko.c2f_fused_out: x, y [B, H, W, C]");
  const int64_t B = x.size(0), H = x.size(1), W = x.size(2);
  const int64_t C = wa.size(0), CO = w2.size(0), CI = ci;
  TORCH_CHECK(CI % 32 == 0 && w1.size(1) >= CI, "aiko.c2f_fused_out: cv1 K (input channels) a multiple of 32");
  TORCH_CHECK(w1.size(0) == 2 * C && wb.size(0) == C && wa.size(1) >= 9 * C && wb.size(1) >= 9 * C &&
                  ((9 * C + 31) / 32) * 32 <= wa.size(1) && ((9 * C + 31) / 32) * 32 <= wb.size(1) && w2.size(1) >= 3 * C &&
                  b1.numel() == 2 * C && ba.numel() == C && bb.numel() == C && b2.numel() == CO,
              "aiko.c2f_fused_out: inconsistent cv1 / bottleneck / cv2 shapes");
  const int64_t ldx = x.stride(2), ldy = y.stride(2);
  TORCH_CHECK(x.stride(3) == 1 && y.stride(3) == 1 && x.stride(2) == ldx && y.stride(2) == ldy &&
                  x.stride(1) == W * ldx && y.stride(1) == W * ldy && x.stride(0) == H * W * ldx &&
                  y.stride(0) == H * W * ldy && ldx % 8 == 0 && ldy % 4 == 0 && x.size(3) >= CI && y.size(3) >= CO &&
                  reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0 && reinterpret_cast<uintptr_t>(y.data_ptr()) % 8 == 0,
              "aiko.c2f_fused_out: NHWC views with 16-B aligned pixels");
  // optional in-place 2x upsample source for input channels [0, cu): xu [B, H/2, W/2, cu] (NHWC view)
  const void* xup = nullptr;
  int64_t ldxu = 0, cu = 0;
  if (xu_opt.has_value() && xu_opt->defined()) {
    const at::Tensor& xu = *xu_opt;
    check_cuda(xu, "c2f upsample source");
    TORCH_CHECK(xu.scalar_type() == at::kBFloat16 && xu.dim() == 4 && xu.size(0) == B && 2 * xu.size(1) == H &&
                    2 * xu.size(2) == W && xu.stride(3) == 1 && xu.stride(1) == xu.size(2) * xu.stride(2) &&
                    xu.stride(0) == xu.size(1) * xu.stride(1) && xu.stride(2) % 8 == 0 &&
                    reinterpret_cast<uintptr_t>(xu.data_ptr()) % 16 == 0,
                "aiko.c2f_fused_out: xu must be an NHWC [B, H/2, W/2, cu] view with 16-B aligned pixels");
    cu = xu.size(3);
    TORCH_CHECK(cu % 32 == 0 && cu < CI, "aiko.c2f_fused_out: xu channels a multiple of 32 below ci");
    xup = xu.data_ptr();
    ldxu = xu.stride(2);
  }
  check_launch(aiko_c2f_fused(x.data_ptr(), (int)ldx, w1.data_ptr(), b1.data_ptr<float>(), (int)w1.size(1), wa.data_ptr(),
                              ba.data_ptr<float>(), (int)wa.size(1), wb.data_ptr(), bb.data_ptr<float>(), (int)wb.size(1),
                              w2.data_ptr(), b2.data_ptr<float>(), (int)w2.size(1), y.data_ptr(), (int)ldy, (int)B, (int)H,
                              (int)W, (int)CI, (int)C, (int)CO, shortcut ? 1 : 0, (int)rb, xup, (int)ldxu, (int)cu,
                              cur_stream()),
               "c2f_fused");
}


// One YOLOv8 C2f bottleneck (3x3 C -> C twice + shortcut) in one launch (c2f_fused.hip):
// x = s, y = c as NHWC channel-slice views of the C2f's concat buffer.
void c2f_bneck_out(const at::Tensor& x, const at::Tensor& wa, const at::Tensor& ba, const at::Tensor& wb,
                   const at::Tensor& bb, at::Tensor& y, bool shortcut, int64_t rb) {
  for (const at::Tensor* t : {&x, &wa, &ba, &wb, &bb, (const at::Tensor*)&y}) check_cuda(*t, "c2f bottleneck operand");
  for (const at::Tensor* t : {&x, &wa, &wb, (const at::Tensor*)&y})
    TORCH_CHECK(t->scalar_type() == at::kBFloat16, "aiko.c2f_bneck_out: bf16 activations / weights");
  TORCH_CHECK(ba.scalar_type() == at::kFloat && bb.scalar_type() == at::kFloat && ba.is_contiguous() && bb.is_contiguous(),
              "aiko.c2f_bneck_out: fp32 biases");
  const int64_t C = wa.size(0);
  TORCH_CHECK(wa.dim() == 2 && wb.dim() == 2 && wa.is_contiguous() && wb.is_contiguous() && wb.size(0) == C &&
                  wa.size(1) >= 9 * C && wb.size(1) >= 9 * C && wa.size(1) % 8 == 0 && wb.size(1) % 8 == 0 &&
                  ba.numel() == C && bb.numel() == C,
              "aiko.c2f_bneck_out: 3x3 weights [C, >= 9C]");
  TORCH_CHECK(x.dim() == 4 && y.dim() == 4 && x.sizes() == y.sizes() && x.size(3) == C, "aiko.c2f_bneck_out: x, y [B, H, W, C]");
  const int64_t B = x.size(0), H = x.size(1), W = x.size(2), ldx = x.stride(2), ldy = y.stride(2);
  TORCH_CHECK(x.stride(3) == 1 && y.stride(3) == 1 && x.stride(1) == W * ldx && y.stride(1) == W * ldy &&
                  x.stride(0) == H * W * ldx && y.stride(0) == H * W * ldy && ldx % 8 == 0 && ldy % 4 == 0 &&
                  reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0 && reinterpret_cast<uintptr_t>(y.data_ptr()) % 8 == 0,
              "aiko.c2f_bneck_out: NHWC channel-slice views, 16-B aligned pixels");
  check_launch(aiko_c2f_bneck(x.data_ptr(), (int)ldx, wa.data_ptr(), ba.data_ptr<float>(), (int)wa.size(1), wb.data_ptr(),
                              bb.data_ptr<float>(), (int)wb.size(1), y.data_ptr(), (int)ldy, (int)B, (int)H, (int)W, (int)C,
                              shortcut ? 1 : 0, (int)rb, cur_stream()),
               "c2f_bneck");
}

// R x R conv (Cout N = 64, 80 or 128, exact-N tile, LDS-DMA kernel) with a fused trailing 1x1 N -> N + bias
// (conv_glds.hip, TAIL): y2 = act2((act(conv(x) + bias)) . w2[:, :N]^T + b2).  x, y2: NHWC channel-slice
// views; w [N, K] and w2 [N, >= ceil32(N)] with zero K padding (conv spec layout).
void conv_glds_tail_out(const at::Tensor& x, const at::Tensor& w, const at::Tensor& bias, const at::Tensor& w2,
                        const at::Tensor& b2, at::Tensor& y2, int64_t R, int64_t stride, int64_t pad, int64_t act,
                        int64_t act2, const at::Tensor& zero) {
  TORCH_CHECK(act2 == 0 || act2 == 2, "aiko.conv_glds_tail_out: act2 = 0 (none) or 2 (SiLU)");
  for (const at::Tensor* t : {&x, &w, &bias, &w2, &b2, (const at::Tensor*)&y2, &zero}) check_cuda(*t, "conv tail operand");
  for (const at::Tensor* t : {&x, &w, &w2, (const at::Tensor*)&y2})
    TORCH_CHECK(t->scalar_type() == at::kBFloat16, "aiko.conv_glds_tail_out: bf16 activations / weights");
  const int64_t N = w.size(0);
  TORCH_CHECK(N == 64 || N == 80 || N == 128, "aiko.conv_glds_tail_out: N = 64, 80 or 128");
  TORCH_CHECK(bias.scalar_type() == at::kFloat && b2.scalar_type() == at::kFloat && bias.numel() == N &&
                  b2.numel() == N && bias.is_contiguous() && b2.is_contiguous(),
              "aiko.conv_glds_tail_out: fp32 biases [N]");
  TORCH_CHECK(x.dim() == 4 && y2.dim() == 4 && x.stride(3) == 1 && y2.stride(3) == 1, "aiko.conv_glds_tail_out: NHWC");
  const int64_t B = x.size(0), H = x.size(1), W = x.size(2), Cc = x.size(3), C = x.stride(2);
  TORCH_CHECK(x.stride(1) == W * C && x.stride(0) == H * W * C && C % 8 == 0 && Cc % 8 == 0 &&
                  reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0,
              "aiko.conv_glds_tail_out: x must be an NHWC (channel-slice) view with 16-B aligned pixels");
  const int64_t K = (R * R * Cc + 63) / 64 * 64;
  TORCH_CHECK(w.dim() == 2 && w.is_contiguous() && w.size(1) == K,
              "aiko.conv_glds_tail_out: w must be [N, ceil64(R*R*Cc)]");
  TORCH_CHECK(w2.dim() == 2 && w2.is_contiguous() && w2.size(0) == N && w2.size(1) >= (N + 31) / 32 * 32 &&
                  w2.size(1) % 8 == 0,
              "aiko.conv_glds_tail_out: w2 must be [N, >= ceil32(N)] (zero past column N)");
  const int64_t Ho = (H + 2 * pad - R) / stride + 1, Wo = (W + 2 * pad - R) / stride + 1;
  const int64_t ldy2 = y2.stride(2);
  TORCH_CHECK(y2.size(0) == B && y2.size(1) == Ho && y2.size(2) == Wo && y2.size(3) == N &&
                  y2.stride(1) == Wo * ldy2 && y2.stride(0) == Ho * Wo * ldy2 && ldy2 % 8 == 0 &&
                  reinterpret_cast<uintptr_t>(y2.data_ptr()) % 16 == 0,
              "aiko.conv_glds_tail_out: y2 must be an NHWC [B, Ho, Wo, N] (channel-slice) view");
  const int64_t M = B * Ho * Wo;
  TORCH_CHECK(avail_elems(x) < INT_MAX && avail_elems(y2) < INT_MAX, "aiko.conv_glds_tail_out: 32-bit offsets");
  check_launch(aiko_conv_glds_tail(x.data_ptr(), w.data_ptr(), bias.data_ptr<float>(), (int)H, (int)W, (int)C, (int)Cc,
                                   (int)R, (int)R, (int)stride, (int)pad, (int)Ho, (int)Wo, (int)M, (int)K, (int)N, (int)act,
                                   w2.data_ptr(), b2.data_ptr<float>(), y2.data_ptr(), (int)ldy2, (int)w2.size(1),
                                   (int)act2, zero.data_ptr(), nullptr, nullptr, nullptr, nullptr, cur_stream()),
               "conv_glds_tail");
}

// The detect head's box / class branch (R x R conv + 1x1 as above) with the YOLOv8 decode in the
// epilogue instead of a stored head output: mode 1 (N = 64, 4 x 16 DFL bins) writes xyxy boxes
// [B, A] float4 at anchors astart + h * W + w, mode 2 (N = 80) sigmoid(max logit over the first nc)
// and its class into scores / cls [B, A] (ops.detect.yolo_decode semantics, bf16-rounded inputs).
void conv_glds_tail_decode_out(const at::Tensor& x, const at::Tensor& w, const at::Tensor& bias, const at::Tensor& w2,
                               const at::Tensor& b2, at::Tensor& boxes, at::Tensor& scores, at::Tensor& cls, int64_t R,
                               int64_t pad, int64_t act, int64_t mode, int64_t nc, int64_t level_stride, int64_t astart,
                               const at::Tensor& zero) {
  for (const at::Tensor* t : {&x, &w, &bias, &w2, &b2, (const at::Tensor*)&boxes, (const at::Tensor*)&scores,
                              (const at::Tensor*)&cls, &zero})
    check_cuda(*t, "conv tail decode operand");
  TORCH_CHECK(x.scalar_type() == at::kBFloat16 && w.scalar_type() == at::kBFloat16 && w2.scalar_type() == at::kBFloat16,
              "aiko.conv_glds_tail_decode_out: bf16 activations / weights");
  TORCH_CHECK(bias.scalar_type() == at::kFloat && b2.scalar_type() == at::kFloat && bias.is_contiguous() && b2.is_contiguous(),
              "aiko.conv_glds_tail_decode_out: fp32 biases");
  const int64_t N = w.size(0);
  TORCH_CHECK((mode == 1 && N == 64) || (mode == 2 && N == 80), "aiko.conv_glds_tail_decode_out: mode 1 needs N = 64, mode 2 N = 80");
  TORCH_CHECK(bias.numel() == N && b2.numel() == N && nc >= 1 && nc <= N, "aiko.conv_glds_tail_decode_out: biases [N], 1 <= nc <= N");
  TORCH_CHECK(x.dim() == 4 && x.stride(3) == 1, "aiko.conv_glds_tail_decode_out: NHWC x");
  const int64_t B = x.size(0), H = x.size(1), W = x.size(2), Cc = x.size(3), C = x.stride(2);
  TORCH_CHECK(x.stride(1) == W * C && x.stride(0) == H * W * C && C % 8 == 0 && Cc % 8 == 0 &&
                  reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0,
              "aiko.conv_glds_tail_decode_out: x must be an NHWC (channel-slice) view with 16-B aligned pixels");
  const int64_t K = (R * R * Cc + 63) / 64 * 64;
  TORCH_CHECK(w.dim() == 2 && w.is_contiguous() && w.size(1) == K, "aiko.conv_glds_tail_decode_out: w [N, ceil64(R*R*Cc)]");
  TORCH_CHECK(w2.dim() == 2 && w2.is_contiguous() && w2.size(0) == N && w2.size(1) >= (N + 31) / 32 * 32 && w2.size(1) % 8 == 0,
              "aiko.conv_glds_tail_decode_out: w2 [N, >= ceil32(N)]");
  const int64_t Ho = H + 2 * pad - R + 1, Wo = W + 2 * pad - R + 1;
  TORCH_CHECK(boxes.scalar_type() == at::kFloat && boxes.dim() == 3 && boxes.size(0) == B && boxes.size(2) == 4 &&
                  boxes.is_contiguous() && scores.scalar_type() == at::kFloat && scores.dim() == 2 && scores.is_contiguous() &&
                  cls.scalar_type() == at::kInt && cls.dim() == 2 && cls.is_contiguous() && scores.size(0) == B &&
                  cls.size(0) == B && scores.size(1) == boxes.size(1) && cls.size(1) == boxes.size(1) &&
                  astart >= 0 && astart + Ho * Wo <= boxes.size(1),
              "aiko.conv_glds_tail_decode_out: boxes [B, A, 4] f32, scores [B, A] f32, cls [B, A] i32 covering the level");
  const int dec[5] = {(int)mode, (int)nc, (int)level_stride, (int)astart, (int)boxes.size(1)};
  check_launch(aiko_conv_glds_tail(x.data_ptr(), w.data_ptr(), bias.data_ptr<float>(), (int)H, (int)W, (int)C, (int)Cc,
                                   (int)R, (int)R, 1, (int)pad, (int)Ho, (int)Wo, (int)(B * Ho * Wo), (int)K, (int)N, (int)act,
                                   w2.data_ptr(), b2.data_ptr<float>(), nullptr, 0, (int)w2.size(1), 0, zero.data_ptr(), dec,
                                   boxes.data_ptr(), scores.data_ptr<float>(), cls.data_ptr<int>(), cur_stream()),
               "conv_glds_tail_decode");
}


// A whole ResNet stage-1 bottleneck in one launch (bneck_fused.hip): x [B, H, 56, cin] ->
// y [B, H, 56, 256]; cin 256 = identity block (w3 [256, 64]), cin 64 = projection block with
// w3 = [conv3 | shortcut] [256, 128] (K-concatenated, ops.conv.fuse_shortcut).
void bneck_fused_out(const at::Tensor& x, const at::Tensor& w1, const at::Tensor& b1, const at::Tensor& w2,
                     const at::Tensor& b2, const at::Tensor& w3, const at::Tensor& b3, at::Tensor& y, int64_t grid,
                     const c10::optional<at::Tensor>& dbg) {
  for (const at::Tensor* t : {&x, &w1, &b1, &w2, &b2, &w3, &b3, (const at::Tensor*)&y}) {
    check_cuda(*t, "bneck_fused operand");
    TORCH_CHECK(t->is_contiguous() && reinterpret_cast<uintptr_t>(t->data_ptr()) % 16 == 0,
                "aiko.bneck_fused_out: operands must be contiguous and 16-byte aligned");
  }
  for (const at::Tensor* t : {&x, &w1, &w2, &w3, (const at::Tensor*)&y})
    TORCH_CHECK(t->scalar_type() == at::kBFloat16, "aiko.bneck_fused_out: bf16 activations / weights");
  for (const at::Tensor* t : {&b1, &b2, &b3})
    TORCH_CHECK(t->scalar_type() == at::kFloat, "aiko.bneck_fused_out: fp32 biases");
  TORCH_CHECK(x.dim() == 4 && y.dim() == 4, "aiko.bneck_fused_out: x / y NHWC");
  const int64_t B = x.size(0), H = x.size(1), W = x.size(2), cin = x.size(3);
  TORCH_CHECK(W == 56 && (cin == 256 || cin == 64), "aiko.bneck_fused_out: x must be [B, H, 56, 256 | 64]");
  TORCH_CHECK(y.size(0) == B && y.size(1) == H && y.size(2) == W && y.size(3) == 256,
              "aiko.bneck_fused_out: y must be [B, H, 56, 256]");
  const int64_t k3 = cin == 64 ? 128 : 64;
  TORCH_CHECK(w1.dim() == 2 && w1.size(0) == 64 && w1.size(1) == cin, "aiko.bneck_fused_out: w1 [64, cin]");
  TORCH_CHECK(w2.dim() == 2 && w2.size(0) == 64 && w2.size(1) == 576, "aiko.bneck_fused_out: w2 [64, 576] (3x3, tap-major)");
  TORCH_CHECK(w3.dim() == 2 && w3.size(0) == 256 && w3.size(1) == k3, "aiko.bneck_fused_out: w3 [256, ", k3, "]");
  TORCH_CHECK(b1.numel() == 64 && b2.numel() == 64 && b3.numel() == 256, "aiko.bneck_fused_out: biases [64], [64], [256]");
  TORCH_CHECK(x.data_ptr() != y.data_ptr(), "aiko.bneck_fused_out: in place is not supported");
  TORCH_CHECK(grid >= 0, "aiko.bneck_fused_out: grid must be >= 0 (0: one workgroup per CU)");
  unsigned* dbg_ptr = nullptr;
  if (dbg.has_value()) {                // diagnostics: [grid, B * H / grid + 1, 8] int32 stamps
    check_cuda(*dbg, "bneck_fused dbg");
    TORCH_CHECK(grid > 0 && dbg->scalar_type() == at::kInt && dbg->is_contiguous() &&
                    dbg->numel() >= grid * ((x.size(0) * x.size(1)) / grid + 1) * 8,
                "aiko.bneck_fused_out: dbg must be int32 [grid, B*H/grid + 1, 8] with an explicit grid");
    dbg_ptr = reinterpret_cast<unsigned*>(dbg->data_ptr());
  }
  TORCH_CHECK(B * H * W * 256 < INT_MAX, "aiko.bneck_fused_out: batch too large for 32-bit pixel indices");
  check_launch(aiko_bneck_fused(x.data_ptr(), w1.data_ptr(), b1.data_ptr<float>(), w2.data_ptr(), b2.data_ptr<float>(),
                                w3.data_ptr(), b3.data_ptr<float>(), y.data_ptr(), (int)B, (int)H, (int)W, (int)cin,
                                (int)grid, dbg_ptr, cur_stream()),
               "bneck_fused");
}

// uint8 frames -> letterbox/normalise -> k x k stem conv (+bias, act) -> bf16 NHWC ``out``
// [B, H1, W1, Cout]; w bf16 [Cout, 64] (k = tap * 4 + channel, zero padded); geom = [Ho, Wo, Hc, Wc, off_t, off_l, k, stride, pad, act]
void stem_direct_out(const at::Tensor& frames, const at::Tensor& w, const c10::optional<at::Tensor>& bias,
                     at::Tensor& out, at::IntArrayRef geom, double fill, at::ArrayRef<double> mean,
                     at::ArrayRef<double> std, bool bgr) {
  check_cuda(frames, "frames");
  check_cuda(w, "w");
  check_cuda(out, "out");
  TORCH_CHECK(frames.scalar_type() == at::kByte && frames.dim() == 4 && frames.size(3) == 3 && frames.is_contiguous(),
              "aiko.stem_direct_out: frames must be uint8 [B, H, W, 3] contiguous");
  TORCH_CHECK(geom.size() == 10, "aiko.stem_direct_out: geom = [Ho, Wo, Hc, Wc, off_t, off_l, k, stride, pad, act]");
  const int64_t Ho = geom[0], Wo = geom[1], Hc = geom[2], Wc = geom[3], off_t = geom[4], off_l = geom[5];
  const int64_t k = geom[6], stride = geom[7], pad = geom[8], act = geom[9];
  TORCH_CHECK(off_t >= 0 && off_l >= 0 && off_t + Ho <= Hc && off_l + Wo <= Wc,
              "aiko.stem_direct_out: image must lie inside the canvas");
  const int64_t B = frames.size(0), Cout = out.size(3);
  const int64_t H1 = (Hc + 2 * pad - k) / stride + 1, W1 = (Wc + 2 * pad - k) / stride + 1;
  TORCH_CHECK(out.size(0) == B && out.size(1) == H1 && out.size(2) == W1, "aiko.stem_direct_out: out must be [B, ",
              H1, ", ", W1, ", Cout]");
  const int64_t ldo = pixel_pitch(out, "stem_direct_out");
  TORCH_CHECK(w.scalar_type() == at::kBFloat16 && w.is_contiguous() && w.dim() == 2 && w.size(0) == Cout &&
                  w.size(1) == 64 && k * k * 4 <= 64 && Cout % 16 == 0,
              "aiko.stem_direct_out: w bf16 [Cout, 64] contiguous (k <= 4, Cout % 16 == 0)");
  const float* bp = nullptr;
  if (bias.has_value() && bias->defined()) {
    check_cuda(*bias, "bias");
    TORCH_CHECK(bias->scalar_type() == at::kFloat && bias->numel() == Cout && bias->is_contiguous(), "aiko.stem_direct_out: bias fp32 [Cout]");
    bp = bias->data_ptr<float>();
  }
  TORCH_CHECK(mean.size() == 3 && std.size() == 3, "aiko.stem_direct_out: mean/std need 3 values");
  float m[3] = {(float)mean[0], (float)mean[1], (float)mean[2]};
  float s[3] = {(float)std[0], (float)std[1], (float)std[2]};
  check_launch(aiko_stem_direct(frames.data_ptr(), out.data_ptr(), w.data_ptr(), bp, B, frames.size(1),
                                frames.size(2), Ho, Wo, Hc, Wc, off_t, off_l, (float)fill, m, s, bgr ? 1 : 0, H1, W1,
                                Cout, ldo, k, stride, pad, act, cur_stream()),
               "stem_direct");
}

// NHWC bf16 tensor whose channels may be a slice of a wider buffer: returns the pixel pitch
int64_t pixel_pitch(const at::Tensor& t, const char* op) {
  TORCH_CHECK(t.scalar_type() == at::kBFloat16 && t.dim() == 4, "aiko.", op, ": NHWC bf16 tensors required");
  const int64_t C = t.size(3), ld = t.stride(2);
  TORCH_CHECK(t.stride(3) == 1 && t.stride(1) == t.size(2) * ld && t.stride(0) == t.size(1) * t.stride(1) &&
                  ld % 8 == 0 && C % 8 == 0 && reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0,
              "aiko.", op, ": tensor must be NHWC with unit channel stride, C and pitch multiples of 8");
  TORCH_CHECK(avail_elems(t) >= (t.size(0) * t.size(1) * t.size(2) - 1) * ld + C, "aiko.", op, ": storage too small");
  return ld;
}

void maxpool_out(const at::Tensor& x, at::Tensor& y, int64_t k, int64_t s, int64_t p) {
  check_cuda(x, "x");
  check_cuda(y, "y");
  const int64_t ldx = pixel_pitch(x, "maxpool_out"), ldy = pixel_pitch(y, "maxpool_out");
  const int64_t B = x.size(0), H = x.size(1), W = x.size(2), C = x.size(3);
  TORCH_CHECK(y.size(0) == B && y.size(3) == C, "aiko.maxpool_out: bad shapes");
  const int64_t Ho = (H + 2 * p - k) / s + 1, Wo = (W + 2 * p - k) / s + 1;
  TORCH_CHECK(y.size(1) == Ho && y.size(2) == Wo, "aiko.maxpool_out: y must be [B, ", Ho, ", ", Wo, ", C]");
  check_launch(aiko_maxpool(x.data_ptr(), y.data_ptr(), B, H, W, C, Ho, Wo, k, s, p, ldx, ldy,
                            cur_stream()),
               "maxpool");
}

// Fused 7x7/s2 stem conv + bias + ReLU + 3x3/s2/p1 max-pool (stem_pool.hip).  x: the zero-bordered
// [B, Hp, Wp, 4] preprocess buffer; w: [7, 64, 32] LDS image of the stem weights (16-byte chunks
// XOR-swizzled by channel >> 2, built by ops.conv.stem_pool); y: [B, Hm, Wm, 64] (slice ok).
void stem_pool_out(const at::Tensor& x, const at::Tensor& w, const at::Tensor& bias, at::Tensor& y,
                   int64_t Ho, int64_t Wo, int64_t variant) {
  check_cuda(x, "x");
  check_cuda(w, "w");
  check_cuda(bias, "bias");
  check_cuda(y, "y");
  TORCH_CHECK(x.scalar_type() == at::kBFloat16 && x.dim() == 4 && x.size(3) == 4 && x.is_contiguous(),
              "aiko.stem_pool_out: x must be a contiguous [B, Hp, Wp, 4] bf16 stem buffer");
  TORCH_CHECK(w.scalar_type() == at::kBFloat16 && w.dim() == 3 && w.size(0) == 7 && w.size(1) == 64 &&
                  w.size(2) == 32 && w.is_contiguous(),
              "aiko.stem_pool_out: w must be the [7, 64, 32] swizzled stem weight image (ops.conv.stem_pool)");
  TORCH_CHECK(bias.scalar_type() == at::kFloat && bias.numel() == 64 && bias.is_contiguous(),
              "aiko.stem_pool_out: bias must be fp32 [64]");
  const int64_t ldy = pixel_pitch(y, "stem_pool_out");
  const int64_t B = x.size(0), Hp = x.size(1), Wp = x.size(2);
  const int64_t Hm = (Ho + 2 - 3) / 2 + 1, Wm = (Wo + 2 - 3) / 2 + 1;
  TORCH_CHECK(Ho > 0 && Wo > 0 && Hp >= 2 * (Ho - 1) + 7 && Wp >= 2 * (Wo - 1) + 8,
              "aiko.stem_pool_out: stem buffer too small for a ", Ho, "x", Wo, " stem output");
  TORCH_CHECK(y.size(0) == B && y.size(1) == Hm && y.size(2) == Wm && y.size(3) == 64,
              "aiko.stem_pool_out: y must be [B, ", Hm, ", ", Wm, ", 64]");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0 &&
                  reinterpret_cast<uintptr_t>(w.data_ptr()) % 16 == 0 &&
                  reinterpret_cast<uintptr_t>(bias.data_ptr()) % 16 == 0,
              "aiko.stem_pool_out: operands must be 16-byte aligned");
  check_launch(aiko_stem_pool(x.data_ptr(), w.data_ptr(), bias.data_ptr<float>(), y.data_ptr(), B, Hp, Wp,
                              Ho, Wo, Hm, Wm, ldy, (int)variant, cur_stream()),
               "stem_pool");
}

// The same fused stem fed with uint8 frames [B, Hi, Wi, 3] (Wi % 4 == 0) — no pre-processing
// kernel, no bf16 stem buffer: w is the weight image scaled by 1 / (255 std_c)
// (ops.conv.stem_pool_u8), mean255 the per-channel 255 * mean subtracted in the kernel.
void stem_pool_u8_out(const at::Tensor& frames, const at::Tensor& w, const at::Tensor& bias, at::Tensor& y,
                      at::ArrayRef<double> mean255, int64_t variant) {
  check_cuda(frames, "frames");
  check_cuda(w, "w");
  check_cuda(bias, "bias");
  check_cuda(y, "y");
  TORCH_CHECK(frames.scalar_type() == at::kByte && frames.dim() == 4 && frames.size(3) == 3 && frames.is_contiguous() &&
                  frames.size(2) % 4 == 0,
              "aiko.stem_pool_u8_out: frames must be contiguous uint8 [B, H, W, 3] with W % 4 == 0");
  TORCH_CHECK(w.scalar_type() == at::kBFloat16 && w.dim() == 3 && w.size(0) == 7 && w.size(1) == 64 &&
                  w.size(2) == 32 && w.is_contiguous(),
              "aiko.stem_pool_u8_out: w must be the [7, 64, 32] swizzled stem weight image");
  TORCH_CHECK(bias.scalar_type() == at::kFloat && bias.numel() == 64 && bias.is_contiguous(),
              "aiko.stem_pool_u8_out: bias must be fp32 [64]");
  TORCH_CHECK(mean255.size() == 3, "aiko.stem_pool_u8_out: mean255 has 3 values");
  const int64_t B = frames.size(0), Hi = frames.size(1), Wi = frames.size(2);
  const int64_t Ho = (Hi + 6 - 7) / 2 + 1, Wo = (Wi + 6 - 7) / 2 + 1;
  const int64_t Hm = (Ho + 2 - 3) / 2 + 1, Wm = (Wo + 2 - 3) / 2 + 1;
  const int64_t ldy = pixel_pitch(y, "stem_pool_u8_out");
  TORCH_CHECK(y.size(0) == B && y.size(1) == Hm && y.size(2) == Wm && y.size(3) == 64,
              "aiko.stem_pool_u8_out: y must be [B, ", Hm, ", ", Wm, ", 64]");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(frames.data_ptr()) % 4 == 0 &&
                  reinterpret_cast<uintptr_t>(w.data_ptr()) % 16 == 0 &&
                  reinterpret_cast<uintptr_t>(bias.data_ptr()) % 16 == 0,
              "aiko.stem_pool_u8_out: frames 4-byte, w / bias 16-byte aligned");
  const float m[3] = {(float)mean255[0], (float)mean255[1], (float)mean255[2]};
  check_launch(aiko_stem_pool_u8(frames.data_ptr(), w.data_ptr(), bias.data_ptr<float>(), y.data_ptr(), B, Hi, Wi,
                                 Ho, Wo, Hm, Wm, ldy, m, (int)variant, cur_stream()),
               "stem_pool_u8");
}

void resize_u8_out(const at::Tensor& x, at::Tensor& y) {
  check_cuda(x, "x");
  check_cuda(y, "y");
  TORCH_CHECK(x.scalar_type() == at::kByte && y.scalar_type() == at::kByte && x.dim() == 4 && y.dim() == 4 &&
                  x.size(3) == 3 && y.size(3) == 3 && x.is_contiguous() && y.is_contiguous() && x.size(0) == y.size(0),
              "aiko.resize_u8_out: uint8 [B, H, W, 3] contiguous tensors required");
  check_launch(aiko_resize_u8(x.data_ptr(), y.data_ptr(), x.size(0), x.size(1), x.size(2), y.size(1), y.size(2),
                              cur_stream()),
               "resize_u8");
}

void batchnorm_out(const at::Tensor& x, const at::Tensor& scale, const at::Tensor& shift, at::Tensor& y, int64_t act) {
  check_cuda(x, "x");
  check_cuda(y, "y");
  check_cuda(scale, "scale");
  check_cuda(shift, "shift");
  const int64_t ldx = pixel_pitch(x, "batchnorm_out"), ldy = pixel_pitch(y, "batchnorm_out");
  const int64_t C = x.size(3);
  TORCH_CHECK(y.sizes() == x.sizes(), "aiko.batchnorm_out: y must match x");
  TORCH_CHECK(scale.scalar_type() == at::kFloat && shift.scalar_type() == at::kFloat && scale.numel() == C &&
                  shift.numel() == C && scale.is_contiguous() && shift.is_contiguous(),
              "aiko.batchnorm_out: scale/shift fp32 [C]");
  check_launch(aiko_batchnorm(x.data_ptr(), y.data_ptr(), scale.data_ptr<float>(), shift.data_ptr<float>(),
                              x.size(0) * x.size(1) * x.size(2), C, ldx, ldy, act, cur_stream()),
               "batchnorm");
}

void upsample2x_out(const at::Tensor& x, at::Tensor& y) {
  check_cuda(x, "x");
  check_cuda(y, "y");
  const int64_t ldx = pixel_pitch(x, "upsample2x_out"), ldy = pixel_pitch(y, "upsample2x_out");
  TORCH_CHECK(y.size(0) == x.size(0) && y.size(1) == 2 * x.size(1) && y.size(2) == 2 * x.size(2) &&
                  y.size(3) == x.size(3),
              "aiko.upsample2x_out: y must be [B, 2H, 2W, C]");
  check_launch(aiko_upsample2x(x.data_ptr(), y.data_ptr(), x.size(0), x.size(1), x.size(2), x.size(3),
                               ldx, ldy, cur_stream()),
               "upsample2x");
}

// feats: per level [B, H, W, 4*reg_max + nc] bf16 (channel slices allowed), strides per level
void yolo_decode_out(at::TensorList feats, at::IntArrayRef strides, int64_t nc, int64_t reg_max,
                     at::Tensor& boxes, at::Tensor& scores, at::Tensor& cls) {
  const int nlev = (int)feats.size();
  TORCH_CHECK(nlev >= 1 && nlev <= 4 && (int)strides.size() == nlev, "aiko.yolo_decode_out: 1..4 levels");
  TORCH_CHECK(reg_max == 16 && nc % 8 == 0, "aiko.yolo_decode_out: reg_max 16, nc % 8 == 0");
  const void* ptrs[4] = {nullptr, nullptr, nullptr, nullptr};
  int H[4] = {0, 0, 0, 0}, W[4] = {1, 1, 1, 1}, st[4] = {1, 1, 1, 1}, ld[4] = {0, 0, 0, 0};
  const int64_t B = feats[0].size(0);
  int64_t A = 0;
  for (int i = 0; i < nlev; ++i) {
    check_cuda(feats[i], "feat");
    ld[i] = (int)pixel_pitch(feats[i], "yolo_decode_out");
    TORCH_CHECK(feats[i].size(0) == B && feats[i].size(3) == 4 * reg_max + nc,
                "aiko.yolo_decode_out: level channels must be 4*reg_max + nc");
    ptrs[i] = feats[i].data_ptr();
    H[i] = feats[i].size(1); W[i] = feats[i].size(2); st[i] = strides[i];
    A += H[i] * W[i];
  }
  check_cuda(boxes, "boxes");
  check_cuda(scores, "scores");
  check_cuda(cls, "cls");
  TORCH_CHECK(boxes.scalar_type() == at::kFloat && boxes.is_contiguous() && boxes.numel() == B * A * 4 &&
                  scores.scalar_type() == at::kFloat && scores.is_contiguous() && scores.numel() == B * A &&
                  cls.scalar_type() == at::kInt && cls.is_contiguous() && cls.numel() == B * A,
              "aiko.yolo_decode_out: outputs boxes fp32 [B, A, 4], scores fp32 [B, A], cls int32 [B, A]");
  check_launch(aiko_yolo_decode(ptrs, H, W, st, ld, nlev, B, nc, reg_max, boxes.data_ptr(),
                                scores.data_ptr<float>(), cls.data_ptr<int>(), cur_stream()),
               "yolo_decode");
}

// params = [conf, iou, max_wh, gain, pad_l, pad_t, img_w, img_h]
void topk_nms_out(const at::Tensor& boxes, const at::Tensor& scores, const at::Tensor& cls,
                  int64_t max_cand, at::ArrayRef<double> params, at::Tensor& det, at::Tensor& count) {
  check_cuda(boxes, "boxes");
  check_cuda(scores, "scores");
  check_cuda(cls, "cls");
  check_cuda(det, "det");
  check_cuda(count, "count");
  TORCH_CHECK(params.size() == 8, "aiko.topk_nms_out: params = [conf, iou, max_wh, gain, pad_l, pad_t, img_w, img_h]");
  TORCH_CHECK(scores.scalar_type() == at::kFloat && scores.dim() == 2 && scores.is_contiguous(),
              "aiko.topk_nms_out: scores fp32 [B, A]");
  const int64_t B = scores.size(0), A = scores.size(1);
  TORCH_CHECK(A <= 32768, "aiko.topk_nms_out: at most 32768 anchors per image");
  TORCH_CHECK(boxes.scalar_type() == at::kFloat && boxes.is_contiguous() && boxes.numel() == B * A * 4,
              "aiko.topk_nms_out: boxes fp32 [B, A, 4]");
  TORCH_CHECK(cls.scalar_type() == at::kInt && cls.is_contiguous() && cls.numel() == B * A,
              "aiko.topk_nms_out: cls int32 [B, A]");
  TORCH_CHECK(det.scalar_type() == at::kFloat && det.dim() == 3 && det.size(0) == B && det.size(2) == 6 &&
                  det.is_contiguous(),
              "aiko.topk_nms_out: det fp32 [B, max_det, 6]");
  const int64_t max_det = det.size(1);
  TORCH_CHECK(max_cand >= 1 && max_cand <= 1024 && max_det >= 1 && max_det <= 1024,
              "aiko.topk_nms_out: 1 <= max_candidates, max_det <= 1024");
  TORCH_CHECK(count.scalar_type() == at::kInt && count.numel() == B && count.is_contiguous(),
              "aiko.topk_nms_out: count int32 [B]");
  // G > 1 workgroups per image: mask-block workspace + zeroed counters from the caching
  // allocator (graph-capture safe: the memset is a node of the captured graph)
  const size_t wsb = aiko_topk_nms_workspace((int)B);
  at::Tensor ws;
  if (wsb) {
    ws = at::empty({(int64_t)wsb}, scores.options().dtype(at::kByte));
    ws.narrow(0, (int64_t)wsb - 4 * B, 4 * B).zero_();
  }
  check_launch(aiko_topk_nms(boxes.data_ptr(), scores.data_ptr<float>(), cls.data_ptr<int>(), B, A,
                             max_cand, max_det, params[0], params[1], params[2], params[3], params[4],
                             params[5], params[6], params[7], det.data_ptr<float>(),
                             count.data_ptr<int>(), wsb ? ws.data_ptr() : nullptr, cur_stream()),
               "topk_nms");
}

void mean_rows_out(const at::Tensor& x, at::Tensor& y) {
  check_cuda(x, "x");
  check_cuda(y, "y");
  // x may be a T-prefix view of a [B, Tp, C] buffer: rows contiguous, any batch pitch >= T*C
  TORCH_CHECK(x.scalar_type() == at::kBFloat16 && x.dim() == 3 && x.stride(2) == 1 &&
                  x.stride(1) == x.size(2) && x.stride(0) >= x.size(1) * x.size(2) &&
                  y.scalar_type() == at::kFloat && y.is_contiguous(),
              "aiko.mean_rows_out: x bf16 [B, T, C] with contiguous rows, y fp32 [B, C]");
  const int64_t B = x.size(0), T = x.size(1), C = x.size(2);
  TORCH_CHECK(C % 8 == 0 && y.numel() == B * C, "aiko.mean_rows_out: C % 8 == 0, y [B, C]");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0 && x.stride(0) % 8 == 0,
              "aiko.mean_rows_out: 16-byte aligned rows");
  TORCH_CHECK(avail_elems(x) >= (B - 1) * x.stride(0) + T * C, "aiko.mean_rows_out: x storage too small");
  check_launch(aiko_mean_rows_f32(x.data_ptr(), y.data_ptr<float>(), B, T, C, (long)x.stride(0), cur_stream()),
               "mean_rows");
}

// SPPF: slices 1..3 of the [B, H, W, >= 4c] concat buffer = chained k x k / 1 max pools of slice 0
void sppf_pool_(at::Tensor& cat, int64_t c, int64_t k) {
  check_cuda(cat, "cat");
  const int64_t ld = pixel_pitch(cat, "sppf_pool_");
  TORCH_CHECK(c % 8 == 0 && 4 * c <= cat.size(3) && k % 2 == 1 && cat.size(1) * cat.size(2) <= 2048,
              "aiko.sppf_pool_: c % 8 == 0, 4c <= C, odd k, H*W <= 2048");
  check_launch(aiko_sppf_pool(cat.data_ptr(), cat.size(0), cat.size(1), cat.size(2), (int)ld, (int)c, (int)k,
                              cur_stream()), "sppf_pool");
}

void zero_border_rows_(at::Tensor& x, int64_t rows) {
  check_cuda(x, "x");
  TORCH_CHECK(x.scalar_type() == at::kBFloat16 && x.dim() == 2 && x.is_contiguous() && x.size(1) % 8 == 0 &&
                  rows >= 2 && x.size(0) % rows == 0,
              "aiko.zero_border_rows_: x bf16 [B*rows, C] contiguous, C % 8 == 0");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0, "aiko.zero_border_rows_: alignment");
  check_launch(aiko_zero_border_rows(x.data_ptr(), x.size(0) / rows, rows, x.size(1), cur_stream()),
               "zero_border_rows");
}

void window_shift_out(const at::Tensor& src, const at::Tensor& chunk, at::Tensor& dst) {
  check_cuda(src, "src");
  check_cuda(chunk, "chunk");
  check_cuda(dst, "dst");
  TORCH_CHECK(src.scalar_type() == at::kFloat && chunk.scalar_type() == at::kFloat && dst.scalar_type() == at::kFloat &&
                  src.dim() == 2 && chunk.dim() == 2 && src.sizes() == dst.sizes() && src.is_contiguous() &&
                  chunk.is_contiguous() && dst.is_contiguous() && chunk.size(0) == src.size(0),
              "aiko.window_shift_out: fp32 contiguous src / dst [B, W], chunk [B, n]");
  TORCH_CHECK(src.data_ptr() != dst.data_ptr(), "aiko.window_shift_out: dst must not alias src");
  const int64_t B = src.size(0), W = src.size(1), n = chunk.size(1);
  TORCH_CHECK(n <= W && W % 4 == 0 && n % 4 == 0, "aiko.window_shift_out: n <= W, both multiples of 4");
  check_launch(aiko_window_shift(src.data_ptr<float>(), chunk.data_ptr<float>(), dst.data_ptr<float>(), B, W, n,
                                 cur_stream()), "window_shift");
}

void avgpool_out(const at::Tensor& x, at::Tensor& y) {
  check_cuda(x, "x");
  check_cuda(y, "y");
  TORCH_CHECK(x.scalar_type() == at::kBFloat16 && y.scalar_type() == at::kBFloat16 &&
                  x.dim() == 4 && x.is_contiguous() && y.is_contiguous(),
              "aiko.avgpool_out: NHWC bf16 contiguous tensors required");
  const int64_t B = x.size(0), C = x.size(3);
  TORCH_CHECK(C % 8 == 0 && y.numel() == B * C, "aiko.avgpool_out: bad shapes");
  check_launch(aiko_avgpool(x.data_ptr(), y.data_ptr(), B, x.size(1) * x.size(2), C, cur_stream()),
               "avgpool");
}

void softmax_topk_out(const at::Tensor& logits, at::Tensor& prob, at::Tensor& index, int64_t k) {
  check_cuda(logits, "logits");
  check_cuda(prob, "prob");
  check_cuda(index, "index");
  TORCH_CHECK(logits.scalar_type() == at::kBFloat16 && logits.dim() == 2 && logits.is_contiguous(),
              "aiko.softmax_topk_out: logits must be bf16 [B, N] contiguous");
  TORCH_CHECK(prob.scalar_type() == at::kFloat && index.scalar_type() == at::kInt,
              "aiko.softmax_topk_out: prob fp32, index int32");
  const int64_t B = logits.size(0), N = logits.size(1);
  TORCH_CHECK(k >= 1 && k <= 8 && k <= N, "aiko.softmax_topk_out: 1 <= k <= min(8, N)");
  TORCH_CHECK(prob.numel() == B * k && index.numel() == B * k, "aiko.softmax_topk_out: outputs must hold B*k");
  check_launch(aiko_softmax_topk(logits.data_ptr(), prob.data_ptr<float>(), index.data_ptr<int>(),
                                 B, N, k, cur_stream()),
               "softmax_topk");
}

// ---- transformer / fp8 ------------------------------------------------------------------------

int64_t row_pitch(const at::Tensor& t, int64_t cols, const char* op, const char* name) {
  TORCH_CHECK(t.dim() == 2 && t.stride(1) == 1 && t.size(1) == cols && t.stride(0) >= cols,
              "aiko.", op, ": ", name, " must be a row-major [rows, ", cols, "] matrix (row slices / column slices allowed)");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0 && (t.stride(0) * t.element_size()) % 16 == 0,
              "aiko.", op, ": ", name, " rows must be 16-byte aligned");
  TORCH_CHECK(avail_elems(t) >= (t.size(0) - 1) * t.stride(0) + cols, "aiko.", op, ": ", name, " storage too small");
  return t.stride(0);
}

// y = act(sa[m] * sb[n] * (A @ B^T) + bias) + residual ; A fp8 [M, K] (uint8 storage), B fp8 [N, K].
// MX-fp8 options (LDS-DMA kernel, variant 1): ``amx`` uint8 [K/128, R, 4] E8M0 block scales of A
// (replaces ``sa``); ``yq`` uint8 [M, N] + ``ysc`` uint8 [N/128, R2, 4]: quantise the output to
// MX-fp8 instead of writing bf16 ``y`` (then ``y`` may be omitted).
void gemm_fp8_out(const at::Tensor& a, const c10::optional<at::Tensor>& sa_opt, const at::Tensor& b,
                  const at::Tensor& sb, const c10::optional<at::Tensor>& bias,
                  const c10::optional<at::Tensor>& res, const c10::optional<at::Tensor>& y_opt, int64_t act,
                  int64_t bm, int64_t bn, int64_t variant, const c10::optional<at::Tensor>& zero,
                  const c10::optional<at::Tensor>& amx, const c10::optional<at::Tensor>& yq,
                  const c10::optional<at::Tensor>& ysc) {
  for (const at::Tensor* t : {&a, &b, &sb}) check_cuda(*t, "operand");
  TORCH_CHECK(a.element_size() == 1 && b.element_size() == 1, "aiko.gemm_fp8_out: A and B must be 1-byte fp8 storage");
  const int64_t M = a.size(0), K = a.size(1), N = b.size(0);
  TORCH_CHECK(K % 128 == 0 && b.dim() == 2 && b.size(1) == K && b.is_contiguous(),
              "aiko.gemm_fp8_out: K must be a multiple of 128 and B [N, K] contiguous");
  TORCH_CHECK(N % 8 == 0, "aiko.gemm_fp8_out: N must be a multiple of 8");
  const int64_t lda = row_pitch(a, K, "gemm_fp8_out", "A");
  TORCH_CHECK(sb.scalar_type() == at::kFloat && sb.numel() == N && sb.is_contiguous(), "aiko.gemm_fp8_out: sb fp32 [N]");
  const bool mx_in = amx.has_value() && amx->defined();
  const bool mx_out = yq.has_value() && yq->defined();
  const float* sap = nullptr;
  if (!mx_in) {
    TORCH_CHECK(sa_opt.has_value() && sa_opt->defined(), "aiko.gemm_fp8_out: sa needed without amx");
    const at::Tensor& sa = *sa_opt;
    check_cuda(sa, "sa");
    TORCH_CHECK(sa.scalar_type() == at::kFloat && sa.numel() >= M && sa.is_contiguous(), "aiko.gemm_fp8_out: sa fp32 [M]");
    sap = sa.data_ptr<float>();
  }
  const void* amxp = nullptr;
  int64_t mxr = 0;
  if (mx_in) {
    check_cuda(*amx, "amx");
    TORCH_CHECK(amx->element_size() == 1 && amx->dim() == 3 && amx->size(0) == K / 128 && amx->size(2) == 4 &&
                    amx->is_contiguous() && amx->size(1) >= ((M + 127) / 128) * 128,
                "aiko.gemm_fp8_out: amx must be uint8 [K/128, rows >= M rounded to 128, 4]");
    amxp = amx->data_ptr();
    mxr = amx->size(1);
  }
  void* yp = nullptr;
  int64_t ldy = 0;
  if (y_opt.has_value() && y_opt->defined()) {
    check_cuda(*y_opt, "y");
    TORCH_CHECK(y_opt->scalar_type() == at::kBFloat16 && y_opt->size(0) == M, "aiko.gemm_fp8_out: y must be bf16 [M, N]");
    ldy = row_pitch(*y_opt, N, "gemm_fp8_out", "y");
    yp = y_opt->data_ptr();
  }
  void* yqp = nullptr;
  void* yscp = nullptr;
  int64_t ldq = 0, ysr = 0;
  if (mx_out) {
    check_cuda(*yq, "yq");
    TORCH_CHECK(ysc.has_value() && ysc->defined(), "aiko.gemm_fp8_out: yq needs ysc");
    check_cuda(*ysc, "ysc");
    TORCH_CHECK(yq->element_size() == 1 && yq->size(0) == M && N % 128 == 0, "aiko.gemm_fp8_out: yq uint8 [M, N], N % 128 == 0");
    ldq = row_pitch(*yq, N, "gemm_fp8_out", "yq");
    TORCH_CHECK(ysc->element_size() == 1 && ysc->dim() == 3 && ysc->size(0) == N / 128 && ysc->size(1) >= M &&
                    ysc->size(2) == 4 && ysc->is_contiguous(),
                "aiko.gemm_fp8_out: ysc must be uint8 [N/128, rows >= M, 4]");
    TORCH_CHECK(!(res.has_value() && res->defined()), "aiko.gemm_fp8_out: no residual with MX output");
    yqp = yq->data_ptr();
    yscp = ysc->data_ptr();
    ysr = ysc->size(1);
  } else {
    TORCH_CHECK(yp != nullptr, "aiko.gemm_fp8_out: y (or yq) required");
  }
  TORCH_CHECK(!(mx_in || mx_out) || (variant == 1 && bn == 128) || (variant == 3 && bm == 256 && bn == 256 && N % 256 == 0) ||
                  (variant == 4 && bm == 256 && bn == 256 && N % 256 == 0) ||
                  (variant == 5 && bm == 128 && bn == 256 && N % 256 == 0),
              "aiko.gemm_fp8_out: MX paths need variant 1 with BN 128, variant 3 (256 x 256, N % 256 == 0), "
              "variant 4 (persistent 256 x 256) or variant 5 (persistent 128 x 256)");
  const float* bp = nullptr;
  if (bias.has_value() && bias->defined()) {
    check_cuda(*bias, "bias");
    TORCH_CHECK(bias->scalar_type() == at::kFloat && bias->numel() == N && bias->is_contiguous(), "aiko.gemm_fp8_out: bias fp32 [N]");
    bp = bias->data_ptr<float>();
  }
  const void* rp = nullptr;
  int64_t ldr = 0;
  if (res.has_value() && res->defined()) {
    check_cuda(*res, "residual");
    TORCH_CHECK(res->scalar_type() == at::kBFloat16 && res->size(0) == M, "aiko.gemm_fp8_out: residual bf16 [M, N]");
    ldr = row_pitch(*res, N, "gemm_fp8_out", "residual");
    rp = res->data_ptr();
  }
  TORCH_CHECK(lda * M < INT_MAX * 2L, "aiko.gemm_fp8_out: A too large");
  const void* zp = nullptr;
  if (variant >= 1) {
    TORCH_CHECK(zero.has_value() && zero->defined() && zero->is_cuda() && zero->nbytes() >= 16 &&
                    reinterpret_cast<uintptr_t>(zero->data_ptr()) % 16 == 0,
                "aiko.gemm_fp8_out: the LDS-DMA variants need a zero page tensor (>= 16 B)");
    TORCH_CHECK(reinterpret_cast<uintptr_t>(a.data_ptr()) % 16 == 0 && reinterpret_cast<uintptr_t>(b.data_ptr()) % 16 == 0,
                "aiko.gemm_fp8_out: operands must be 16-byte aligned");
    zp = zero->data_ptr();
  }
  check_launch(aiko_gemm_fp8(a.data_ptr(), b.data_ptr(), sap, sb.data_ptr<float>(), bp, rp, yp, M, N, K, lda,
                             ldy, ldr, act, bm, bn, (int)variant, zp, amxp, (int)mxr, yqp, yscp, (int)ldq,
                             (int)ysr, cur_stream()),
               "gemm_fp8");
}

// LayerNorm (gamma/beta given) and/or per-row fp8 quantisation of bf16 rows x [M, D]
void rownorm_quant_out(const at::Tensor& x, const c10::optional<at::Tensor>& gamma,
                       const c10::optional<at::Tensor>& beta, double eps,
                       const c10::optional<at::Tensor>& yb, const c10::optional<at::Tensor>& q,
                       const c10::optional<at::Tensor>& qs) {
  check_cuda(x, "x");
  TORCH_CHECK(x.scalar_type() == at::kBFloat16, "aiko.rownorm_quant_out: x must be bf16");
  const int64_t M = x.size(0), D = x.size(1);
  TORCH_CHECK(D % 8 == 0 && D <= 8192, "aiko.rownorm_quant_out: D % 8 == 0, D <= 8192");
  const int64_t ldx = row_pitch(x, D, "rownorm_quant_out", "x");
  const float *g = nullptr, *be = nullptr;
  if (gamma.has_value() && gamma->defined()) {
    TORCH_CHECK(beta.has_value() && beta->defined(), "aiko.rownorm_quant_out: gamma needs beta");
    check_cuda(*gamma, "gamma");
    check_cuda(*beta, "beta");
    TORCH_CHECK(gamma->scalar_type() == at::kFloat && beta->scalar_type() == at::kFloat && gamma->numel() == D &&
                    beta->numel() == D && gamma->is_contiguous() && beta->is_contiguous(),
                "aiko.rownorm_quant_out: gamma/beta fp32 [D]");
    g = gamma->data_ptr<float>();
    be = beta->data_ptr<float>();
  }
  void* yp = nullptr;
  int64_t ldyb = 0;
  if (yb.has_value() && yb->defined()) {
    check_cuda(*yb, "yb");
    TORCH_CHECK(yb->scalar_type() == at::kBFloat16 && yb->size(0) == M, "aiko.rownorm_quant_out: yb bf16 [M, D]");
    ldyb = row_pitch(*yb, D, "rownorm_quant_out", "yb");
    yp = yb->data_ptr();
  }
  void* qp = nullptr;
  float* sp = nullptr;
  int64_t ldq = 0;
  if (q.has_value() && q->defined()) {
    TORCH_CHECK(qs.has_value() && qs->defined(), "aiko.rownorm_quant_out: q needs qs");
    check_cuda(*q, "q");
    check_cuda(*qs, "qs");
    TORCH_CHECK(q->element_size() == 1 && q->size(0) == M, "aiko.rownorm_quant_out: q fp8 [M, D]");
    ldq = row_pitch(*q, D, "rownorm_quant_out", "q");
    TORCH_CHECK(qs->scalar_type() == at::kFloat && qs->numel() >= M && qs->is_contiguous(), "aiko.rownorm_quant_out: qs fp32 [M]");
    qp = q->data_ptr();
    sp = qs->data_ptr<float>();
  }
  TORCH_CHECK(yp || qp, "aiko.rownorm_quant_out: nothing to write");
  check_launch(aiko_rownorm_quant(x.data_ptr(), ldx, g, be, (float)eps, yp, ldyb, qp, ldq, sp, M, D, cur_stream()),
               "rownorm_quant");
}



// Split-K linear (linear_splitk.hip): x [M, >= K] bf16, w [N, >= K] bf16 (row pitch w.stride(0)),
// bias fp32 [N] or None, part fp32 with >= S*M*N elements, y [M, >= N] bf16.
void linear_splitk_out(const at::Tensor& x, const at::Tensor& w, const c10::optional<at::Tensor>& bias,
                       at::Tensor& part, at::Tensor& y, int64_t K, int64_t S) {
  for (const at::Tensor* t : {&x, &w, (const at::Tensor*)&part, (const at::Tensor*)&y}) check_cuda(*t, "x/w/part/y");
  TORCH_CHECK(x.scalar_type() == at::kBFloat16 && w.scalar_type() == at::kBFloat16 && y.scalar_type() == at::kBFloat16,
              "aiko.linear_splitk_out: x, w, y must be bf16");
  TORCH_CHECK(part.scalar_type() == at::kFloat && part.is_contiguous(), "aiko.linear_splitk_out: part must be contiguous fp32");
  TORCH_CHECK(x.dim() == 2 && w.dim() == 2 && y.dim() == 2 && x.stride(1) == 1 && w.stride(1) == 1 && y.stride(1) == 1,
              "aiko.linear_splitk_out: row-major 2-D operands");
  const int64_t M = x.size(0), N = w.size(0);
  TORCH_CHECK(y.size(0) == M && y.size(1) == N && x.size(1) >= K && w.size(1) >= K, "aiko.linear_splitk_out: shapes");
  TORCH_CHECK(S >= 1 && K % (32 * S) == 0 && N % 4 == 0, "aiko.linear_splitk_out: K % (32 S) == 0 and N % 4 == 0");
  TORCH_CHECK(x.stride(0) % 8 == 0 && w.stride(0) % 8 == 0 && y.stride(0) % 4 == 0 &&
                  reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0 && reinterpret_cast<uintptr_t>(w.data_ptr()) % 16 == 0 &&
                  reinterpret_cast<uintptr_t>(y.data_ptr()) % 8 == 0 && reinterpret_cast<uintptr_t>(part.data_ptr()) % 16 == 0,
              "aiko.linear_splitk_out: 16-B aligned operand rows");
  TORCH_CHECK(part.numel() >= S * M * N, "aiko.linear_splitk_out: part too small");
  const float* bp = nullptr;
  if (bias.has_value() && bias->defined()) {
    check_cuda(*bias, "bias");
    TORCH_CHECK(bias->scalar_type() == at::kFloat && bias->numel() == N && bias->is_contiguous(),
                "aiko.linear_splitk_out: bias must be fp32 [N]");
    bp = bias->data_ptr<float>();
  }
  check_launch(aiko_linear_splitk(x.data_ptr(), w.data_ptr(), bp, part.data_ptr<float>(), y.data_ptr(), (int)M, (int)N,
                                  (int)K, (int)x.stride(0), (int)w.stride(0), (int)y.stride(0), (int)S, cur_stream()),
               "linear_splitk");
}

// q/k/v/o: [B*Tpad, >= H*64] row-major (column slices of a fused QKV buffer allowed)
void attn_fwd_out(const at::Tensor& q, const at::Tensor& k, const at::Tensor& v, at::Tensor& o,
                  int64_t B, int64_t H, int64_t T, int64_t Tpad, double scale,
                  const c10::optional<at::Tensor>& work, const c10::optional<at::Tensor>& oq,
                  const c10::optional<at::Tensor>& osc) {
  for (const at::Tensor* t : {&q, &k, &v, (const at::Tensor*)&o}) {
    check_cuda(*t, "q/k/v/o");
    TORCH_CHECK(t->scalar_type() == at::kBFloat16, "aiko.attn_fwd_out: bf16 tensors required");
    TORCH_CHECK(t->size(0) == B * Tpad, "aiko.attn_fwd_out: tensors need B*Tpad rows");
    row_pitch(*t, H * 64, "attn_fwd_out", "q/k/v/o");
  }
  TORCH_CHECK(T >= 1 && T <= Tpad, "aiko.attn_fwd_out: 1 <= T <= Tpad");
  void* wp = nullptr;
  long wb = 0;
  if (work.has_value() && work->defined()) {
    check_cuda(*work, "work");
    TORCH_CHECK(work->is_contiguous() && reinterpret_cast<uintptr_t>(work->data_ptr()) % 256 == 0,
                "aiko.attn_fwd_out: work must be a contiguous, 256-byte aligned (zero-initialised) buffer");
    wp = work->data_ptr();
    wb = (long)(work->numel() * work->element_size());
  }
  // MX-fp8 output (ops.transformer.mx_buffers layout): e4m3 [B*Tpad, >= H*64] + E8M0 scales
  // [H*64/128][rows >= B*Tpad][4]; o is then not written
  void* qp = nullptr;
  void* sp = nullptr;
  int ldoq = 0, osr = 0;
  if (oq.has_value() && oq->defined()) {
    TORCH_CHECK(osc.has_value() && osc->defined(), "aiko.attn_fwd_out: oq needs osc");
    check_cuda(*oq, "oq");
    check_cuda(*osc, "osc");
    TORCH_CHECK(oq->scalar_type() == at::kByte && oq->dim() == 2 && oq->stride(1) == 1 && oq->size(0) == B * Tpad &&
                    oq->size(1) >= H * 64 && oq->stride(0) % 4 == 0,
                "aiko.attn_fwd_out: oq uint8 [B*Tpad, >= H*64] with a 4-byte row pitch");
    TORCH_CHECK((H * 64) % 128 == 0 && osc->scalar_type() == at::kByte && osc->is_contiguous() && osc->dim() == 3 &&
                    osc->size(0) == H * 64 / 128 && osc->size(1) >= B * Tpad && osc->size(2) == 4,
                "aiko.attn_fwd_out: osc uint8 [H*64/128, rows >= B*Tpad, 4]");
    qp = oq->data_ptr();
    sp = osc->data_ptr();
    ldoq = (int)oq->stride(0);
    osr = (int)osc->size(1);
  }
  check_launch(aiko_attn_fwd(q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), q.stride(0), k.stride(0),
                             v.stride(0), o.stride(0), B, H, T, Tpad, 64, (float)scale, wp, wb, qp, sp, ldoq, osr,
                             cur_stream()),
               "attn_fwd");
}

// audio fp32 [B, N] -> bf16 log-mel rows [B*rows, n_mels] (frame t at row b*rows + pad + t)
void logmel_out(const at::Tensor& audio, const at::Tensor& mel, const at::Tensor& mel_range, int64_t n_fft,
                int64_t hop, int64_t F, at::Tensor& work, at::Tensor& gmax, at::Tensor& dst, int64_t rows,
                int64_t pad) {
  for (const at::Tensor* t : {&audio, &mel, (const at::Tensor*)&work, (const at::Tensor*)&gmax, (const at::Tensor*)&dst})
    check_cuda(*t, "logmel operand");
  TORCH_CHECK(audio.scalar_type() == at::kFloat && audio.dim() == 2 && audio.is_contiguous(), "aiko.logmel_out: audio fp32 [B, N]");
  const int64_t B = audio.size(0), N = audio.size(1), n_mels = mel.size(0);
  TORCH_CHECK(mel.scalar_type() == at::kFloat && mel.is_contiguous() && mel.size(1) == n_fft / 2 + 1,
              "aiko.logmel_out: mel filters fp32 [n_mels, n_fft/2+1]");
  check_cuda(mel_range, "mel_range");
  TORCH_CHECK(mel_range.scalar_type() == at::kInt && mel_range.is_contiguous() && mel_range.numel() == n_mels * 3 &&
                  n_mels <= 128,
              "aiko.logmel_out: mel_range int32 [n_mels, 3] (lo, len, offset), n_mels <= 128");
  TORCH_CHECK(N > n_fft / 2 && F >= 1 && (F - 1) * hop - n_fft / 2 < N, "aiko.logmel_out: bad frame count");
  TORCH_CHECK(work.scalar_type() == at::kFloat && work.numel() >= B * F * n_mels, "aiko.logmel_out: work fp32 [B*F*n_mels]");
  TORCH_CHECK(gmax.scalar_type() == at::kInt && gmax.numel() >= B, "aiko.logmel_out: gmax int32 [B]");
  TORCH_CHECK(dst.scalar_type() == at::kBFloat16 && dst.dim() == 2 && dst.size(1) == n_mels && dst.stride(1) == 1 &&
                  dst.size(0) == B * rows && rows >= F + pad,
              "aiko.logmel_out: dst bf16 [B*rows, n_mels]");
  check_launch(aiko_logmel(audio.data_ptr<float>(), B, N, mel.data_ptr<float>(), n_mels,
                           mel_range.data_ptr<int>(), n_fft, hop, F,
                           work.data_ptr<float>(), gmax.data_ptr<int>(), dst.data_ptr(), rows, pad, dst.stride(0),
                           cur_stream()),
               "logmel");
}

// ---- decoder step ops (decode_ops.hip) ----------------------------------------------------------

void check_i32(const at::Tensor& t, int64_t n, const char* what) {
  check_cuda(t, what);
  TORCH_CHECK(t.scalar_type() == at::kInt && t.is_contiguous() && t.numel() >= n, "aiko: ", what,
              " must be contiguous int32 with >= ", n, " elements");
}

// x[b] = tok[ids[b]] + pemb[pos[0]]; tok bf16 [V, d], pemb bf16 [P, d], x bf16 [B, d]
void embed_tokens_out(const at::Tensor& ids, const at::Tensor& pos, const at::Tensor& tok, const at::Tensor& pemb,
                      at::Tensor& x) {
  const int64_t B = x.size(0), d = x.size(1);
  check_i32(ids, B, "ids");
  check_i32(pos, 1, "pos");
  for (const at::Tensor* t : {&tok, &pemb, (const at::Tensor*)&x}) {
    check_cuda(*t, "embedding operand");
    TORCH_CHECK(t->scalar_type() == at::kBFloat16 && t->dim() == 2 && t->size(1) == d,
                "aiko.embed_tokens_out: bf16 [*, d] tensors required");
  }
  TORCH_CHECK(tok.is_contiguous() && pemb.is_contiguous() && d % 8 == 0, "aiko.embed_tokens_out: contiguous tables, d % 8 == 0");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0, "aiko.embed_tokens_out: x alignment");
  const int64_t ldx = row_pitch(x, d, "embed_tokens_out", "x");
  check_launch(aiko_embed_tokens(ids.data_ptr<int>(), pos.data_ptr<int>(), tok.data_ptr(), pemb.data_ptr(), x.data_ptr(),
                                 B, d, ldx, tok.size(0), pemb.size(0), cur_stream()),
               "embed_tokens");
}

// One query row per sequence against K/V rows [B*S, >= H*64] (sequence b's key j at row b*S+j).
// With ``pos`` (device int32 [1]) the step appends ``knew``/``vnew`` [B, >= H*64] at row pos of
// every sequence and attends keys 0..pos; otherwise it attends keys 0..T-1.
void attn_decode_out(const at::Tensor& q, at::Tensor& k, at::Tensor& v, at::Tensor& o, int64_t B, int64_t H,
                     int64_t S, int64_t T, const c10::optional<at::Tensor>& pos,
                     const c10::optional<at::Tensor>& knew, const c10::optional<at::Tensor>& vnew, double scale,
                     at::Tensor& work) {
  const bool app = pos.has_value() && pos->defined();
  for (const at::Tensor* t : {&q, (const at::Tensor*)&k, (const at::Tensor*)&v, (const at::Tensor*)&o}) {
    check_cuda(*t, "q/k/v/o");
    TORCH_CHECK(t->scalar_type() == at::kBFloat16 && t->dim() == 2, "aiko.attn_decode_out: bf16 2-D tensors required");
    row_pitch(*t, H * 64, "attn_decode_out", "q/k/v/o");
    TORCH_CHECK(reinterpret_cast<uintptr_t>(t->data_ptr()) % 16 == 0, "aiko.attn_decode_out: 16-byte alignment");
  }
  TORCH_CHECK(q.size(0) == B && o.size(0) == B, "aiko.attn_decode_out: q/o need B rows");
  TORCH_CHECK(k.size(0) == B * S && v.size(0) == B * S, "aiko.attn_decode_out: k/v need B*S rows");
  const void *kn = nullptr, *vn = nullptr;
  int64_t ldnew = 0;
  const int* pp = nullptr;
  if (app) {
    check_i32(*pos, 1, "pos");
    pp = pos->data_ptr<int>();
    TORCH_CHECK(knew.has_value() && knew->defined() && vnew.has_value() && vnew->defined(),
                "aiko.attn_decode_out: append mode needs knew and vnew");
    for (const at::Tensor* t : {&*knew, &*vnew}) {
      check_cuda(*t, "knew/vnew");
      TORCH_CHECK(t->scalar_type() == at::kBFloat16 && t->size(0) == B &&
                      reinterpret_cast<uintptr_t>(t->data_ptr()) % 16 == 0,
                  "aiko.attn_decode_out: knew/vnew bf16 [B, >= H*64], 16-byte aligned");
      row_pitch(*t, H * 64, "attn_decode_out", "knew/vnew");
    }
    TORCH_CHECK(knew->stride(0) == vnew->stride(0), "aiko.attn_decode_out: knew/vnew must share a row pitch");
    kn = knew->data_ptr();
    vn = vnew->data_ptr();
    ldnew = knew->stride(0);
  } else {
    TORCH_CHECK(T >= 1 && T <= S, "aiko.attn_decode_out: 1 <= T <= S");
  }
  check_cuda(work, "work");
  TORCH_CHECK(work.scalar_type() == at::kFloat && work.is_contiguous(), "aiko.attn_decode_out: work fp32");
  TORCH_CHECK(work.numel() >= aiko_attn_decode_work(B, H, app ? S : T), "aiko.attn_decode_out: work too small");
  check_launch(aiko_attn_decode(q.data_ptr(), q.stride(0), k.data_ptr(), v.data_ptr(), k.stride(0), v.stride(0), S, pp,
                                T, kn, vn, ldnew, o.data_ptr(), o.stride(0), B, H, (float)scale,
                                work.data_ptr<float>(), work.numel(), cur_stream()),
               "attn_decode");
}


// y = act(LN?(x) quantised per row to e4m3 @ W^T * scales + bias) (+ res): the decoder's fused
// skinny-M linear (x bf16 [M, K], K % 128 == 0, K <= 3072; W e4m3 [N, K])
void dec_linear_out(const at::Tensor& x, const c10::optional<at::Tensor>& gamma, const c10::optional<at::Tensor>& beta,
                    double eps, const at::Tensor& w, const at::Tensor& sw, const c10::optional<at::Tensor>& bias,
                    const c10::optional<at::Tensor>& res, at::Tensor& y, int64_t act) {
  for (const at::Tensor* t : {&x, &w, &sw, (const at::Tensor*)&y}) check_cuda(*t, "dec_linear operand");
  TORCH_CHECK(x.scalar_type() == at::kBFloat16 && y.scalar_type() == at::kBFloat16, "aiko.dec_linear_out: bf16 x / y");
  const int64_t M = x.size(0), K = x.size(1), N = w.size(0);
  TORCH_CHECK(w.element_size() == 1 && w.dim() == 2 && w.size(1) == K && w.is_contiguous(),
              "aiko.dec_linear_out: w e4m3 [N, K] contiguous with K == x width");
  TORCH_CHECK(K % 128 == 0 && K <= 3072, "aiko.dec_linear_out: K % 128 == 0 and K <= 3072");
  TORCH_CHECK(sw.scalar_type() == at::kFloat && sw.numel() == N && sw.is_contiguous(), "aiko.dec_linear_out: sw fp32 [N]");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0 && reinterpret_cast<uintptr_t>(w.data_ptr()) % 16 == 0,
              "aiko.dec_linear_out: x / w 16-byte alignment");
  const int64_t ldx = row_pitch(x, K, "dec_linear_out", "x");
  TORCH_CHECK(y.size(0) == M, "aiko.dec_linear_out: y [M, N]");
  const int64_t ldy = row_pitch(y, N, "dec_linear_out", "y");
  const float *g = nullptr, *be = nullptr, *bp = nullptr;
  if (gamma.has_value() && gamma->defined()) {
    TORCH_CHECK(beta.has_value() && beta->defined(), "aiko.dec_linear_out: gamma needs beta");
    for (const at::Tensor* t : {&*gamma, &*beta}) {
      check_cuda(*t, "gamma/beta");
      TORCH_CHECK(t->scalar_type() == at::kFloat && t->numel() == K && t->is_contiguous(), "aiko.dec_linear_out: gamma/beta fp32 [K]");
    }
    g = gamma->data_ptr<float>();
    be = beta->data_ptr<float>();
  }
  if (bias.has_value() && bias->defined()) {
    check_cuda(*bias, "bias");
    TORCH_CHECK(bias->scalar_type() == at::kFloat && bias->numel() == N && bias->is_contiguous(), "aiko.dec_linear_out: bias fp32 [N]");
    bp = bias->data_ptr<float>();
  }
  const void* rp = nullptr;
  int64_t ldr = 0;
  if (res.has_value() && res->defined()) {
    check_cuda(*res, "residual");
    TORCH_CHECK(res->scalar_type() == at::kBFloat16 && res->size(0) == M, "aiko.dec_linear_out: residual bf16 [M, N]");
    ldr = row_pitch(*res, N, "dec_linear_out", "residual");
    rp = res->data_ptr();
  }
  check_launch(aiko_dec_linear(x.data_ptr(), ldx, g, be, (float)eps, w.data_ptr(), sw.data_ptr<float>(), bp, rp, ldr,
                               y.data_ptr(), ldy, M, N, K, act, cur_stream()),
               "dec_linear");
}

// greedy next token per sequence; advances pos[0] on the device (see decode_ops.hip)
void argmax_step_out(const at::Tensor& logits, int64_t V, at::Tensor& ids, at::Tensor& pos, at::Tensor& out_tokens,
                     const at::Tensor& forced, int64_t eot, at::Tensor& done, at::Tensor& counter) {
  check_cuda(logits, "logits");
  TORCH_CHECK(logits.scalar_type() == at::kBFloat16 && logits.dim() == 2 && logits.stride(1) == 1 &&
                  reinterpret_cast<uintptr_t>(logits.data_ptr()) % 16 == 0,
              "aiko.argmax_step_out: logits bf16 [B, >= V], 16-byte aligned rows");
  const int64_t B = logits.size(0);
  check_i32(ids, B, "ids");
  check_i32(pos, 1, "pos");
  check_i32(done, B, "done");
  check_i32(counter, 1, "counter");
  check_cuda(out_tokens, "out_tokens");
  TORCH_CHECK(out_tokens.scalar_type() == at::kInt && out_tokens.dim() == 2 && out_tokens.size(0) == B &&
                  out_tokens.is_contiguous(),
              "aiko.argmax_step_out: out_tokens int32 [B, max_len]");
  check_i32(forced, 1, "forced");
  check_launch(aiko_argmax_step(logits.data_ptr(), logits.stride(0), V, B, ids.data_ptr<int>(), pos.data_ptr<int>(),
                                out_tokens.data_ptr<int>(), out_tokens.size(1), forced.data_ptr<int>(), forced.numel(),
                                eot, done.data_ptr<int>(), reinterpret_cast<unsigned*>(counter.data_ptr<int>()),
                                cur_stream()),
               "argmax_step");
}

}  // namespace

TORCH_LIBRARY(aiko, m) {
  m.def("conv_igemm_out(Tensor x, Tensor? x2, Tensor w, Tensor? bias, Tensor? res, Tensor(a!) y, int[] geom, Tensor? zero=None) -> ()");
  m.def("preprocess_out(Tensor frames, Tensor(a!) out, int Ho, int Wo, int pad_t, int pad_l, float[] mean, float[] std, bool bgr, float[] canvas=[]) -> ()");
  m.def("upsample2x_out(Tensor x, Tensor(a!) y) -> ()");
  m.def("resize_u8_out(Tensor x, Tensor(a!) y) -> ()");
  m.def("batchnorm_out(Tensor x, Tensor scale, Tensor shift, Tensor(a!) y, int act) -> ()");
  m.def("yolo_decode_out(Tensor[] feats, int[] strides, int nc, int reg_max, Tensor(a!) boxes, Tensor(b!) scores, Tensor(c!) cls) -> ()");
  m.def("topk_nms_out(Tensor boxes, Tensor scores, Tensor cls, int max_cand, float[] params, Tensor(a!) det, Tensor(b!) count) -> ()");
  m.def("stem_direct_out(Tensor frames, Tensor w, Tensor? bias, Tensor(a!) out, int[] geom, float fill, float[] mean, float[] std, bool bgr) -> ()");
  m.def("conv3x3_patch_out(Tensor x, Tensor wimg, Tensor? bias, Tensor(a!) y, int act, int grid=0) -> ()");
  m.def("conv3x3_patchw_out(Tensor x, Tensor wimg, Tensor? bias, Tensor(a!) y, int act, int grid=0) -> ()");
  m.def("conv3x3_rows_out(Tensor x, Tensor wimg, Tensor? bias, Tensor? res, Tensor(a!) y, int act, int grid=0) -> ()");
  m.def("conv_chain_out(Tensor A, Tensor W1, Tensor b1, Tensor? R, Tensor(a!) Y, Tensor W2, Tensor b2, Tensor(b!) Z, int grid=0, Tensor? A2=None) -> ()");
  m.def("bneck_fused_out(Tensor x, Tensor w1, Tensor b1, Tensor w2, Tensor b2, Tensor w3, Tensor b3, Tensor(a!) y, int grid=0, Tensor? dbg=None) -> ()");
  m.def("maxpool_out(Tensor x, Tensor(a!) y, int k, int s, int p) -> ()");
  m.def("avgpool_out(Tensor x, Tensor(a!) y) -> ()");
  m.def("mean_rows_out(Tensor x, Tensor(a!) y) -> ()");
  m.def("window_shift_out(Tensor src, Tensor chunk, Tensor(a!) dst) -> ()");
  m.def("zero_border_rows_(Tensor(a!) x, int rows) -> ()");
  m.def("sppf_pool_(Tensor(a!) cat, int c, int k) -> ()");
  m.def("stem_pool_out(Tensor x, Tensor w, Tensor bias, Tensor(a!) y, int Ho, int Wo, int variant=0) -> ()");
  m.def("stem_pool_u8_out(Tensor frames, Tensor w, Tensor bias, Tensor(a!) y, float[] mean255, int variant=0) -> ()");
  m.def("gemm_fp8_out(Tensor a, Tensor? sa, Tensor b, Tensor sb, Tensor? bias, Tensor? res, Tensor(a!)? y, int act, int bm, int bn, int variant=0, Tensor? zero=None, Tensor? amx=None, Tensor(b!)? yq=None, Tensor(c!)? ysc=None) -> ()");
  m.def("rownorm_quant_out(Tensor x, Tensor? gamma, Tensor? beta, float eps, Tensor(a!)? yb, Tensor(b!)? q, Tensor(c!)? qs) -> ()");
  m.def("c2f_fused_out(Tensor x, Tensor w1, Tensor b1, Tensor wa, Tensor ba, Tensor wb, Tensor bb, Tensor w2, Tensor b2, Tensor(a!) y, int ci, bool shortcut, int rb, Tensor? xu=None) -> ()");
  m.def("c2f_bneck_out(Tensor x, Tensor wa, Tensor ba, Tensor wb, Tensor bb, Tensor(a!) y, bool shortcut, int rb) -> ()");
  m.def("conv_glds_tail_decode_out(Tensor x, Tensor w, Tensor bias, Tensor w2, Tensor b2, Tensor(a!) boxes, Tensor(b!) scores, Tensor(c!) cls, int R, int pad, int act, int mode, int nc, int level_stride, int astart, Tensor zero) -> ()");
  m.def("conv_glds_tail_out(Tensor x, Tensor w, Tensor bias, Tensor w2, Tensor b2, Tensor(a!) y2, int R, int stride, int pad, int act, int act2, Tensor zero) -> ()");
  m.def("linear_splitk_out(Tensor x, Tensor w, Tensor? bias, Tensor(a!) part, Tensor(b!) y, int K, int S) -> ()");
  m.def("attn_fwd_out(Tensor q, Tensor k, Tensor v, Tensor(a!) o, int B, int H, int T, int Tpad, float scale, Tensor(b!)? work=None, Tensor(c!)? oq=None, Tensor(d!)? osc=None) -> ()");
  m.def("logmel_out(Tensor audio, Tensor mel, Tensor mel_range, int n_fft, int hop, int F, Tensor(a!) work, Tensor(b!) gmax, Tensor(c!) dst, int rows, int pad) -> ()");
  m.def("softmax_topk_out(Tensor logits, Tensor(a!) prob, Tensor(b!) index, int k) -> ()");
  m.def("embed_tokens_out(Tensor ids, Tensor pos, Tensor tok, Tensor pemb, Tensor(a!) x) -> ()");
  m.def("attn_decode_out(Tensor q, Tensor(a!) k, Tensor(b!) v, Tensor(c!) o, int B, int H, int S, int T, Tensor? pos, Tensor? knew, Tensor? vnew, float scale, Tensor(d!) work) -> ()");
  m.def("dec_linear_out(Tensor x, Tensor? gamma, Tensor? beta, float eps, Tensor w, Tensor sw, Tensor? bias, Tensor? res, Tensor(a!) y, int act) -> ()");
  m.def("argmax_step_out(Tensor logits, int V, Tensor(a!) ids, Tensor(b!) pos, Tensor(c!) out_tokens, Tensor forced, int eot, Tensor(d!) done, Tensor(e!) counter) -> ()");
}

TORCH_LIBRARY_IMPL(aiko, CUDA, m) {
  m.impl("conv_igemm_out", &conv_igemm_out);
  m.impl("preprocess_out", &preprocess_out);
  m.impl("maxpool_out", &maxpool_out);
  m.impl("conv_chain_out", &conv_chain_out);
  m.impl("bneck_fused_out", &bneck_fused_out);
  m.impl("conv3x3_patch_out", &conv3x3_patch_out);
  m.impl("conv3x3_patchw_out", &conv3x3_patchw_out);
  m.impl("conv3x3_rows_out", &conv3x3_rows_out);
  m.impl("stem_direct_out", &stem_direct_out);
  m.impl("upsample2x_out", &upsample2x_out);
  m.impl("resize_u8_out", &resize_u8_out);
  m.impl("batchnorm_out", &batchnorm_out);
  m.impl("yolo_decode_out", &yolo_decode_out);
  m.impl("topk_nms_out", &topk_nms_out);
  m.impl("avgpool_out", &avgpool_out);
  m.impl("mean_rows_out", &mean_rows_out);
  m.impl("window_shift_out", &window_shift_out);
  m.impl("zero_border_rows_", &zero_border_rows_);
  m.impl("sppf_pool_", &sppf_pool_);
  m.impl("stem_pool_out", &stem_pool_out);
  m.impl("stem_pool_u8_out", &stem_pool_u8_out);
  m.impl("softmax_topk_out", &softmax_topk_out);
  m.impl("gemm_fp8_out", &gemm_fp8_out);
  m.impl("rownorm_quant_out", &rownorm_quant_out);
  m.impl("c2f_fused_out", &c2f_fused_out);
  m.impl("c2f_bneck_out", &c2f_bneck_out);
  m.impl("conv_glds_tail_out", &conv_glds_tail_out);
  m.impl("conv_glds_tail_decode_out", &conv_glds_tail_decode_out);
  m.impl("attn_fwd_out", &attn_fwd_out);
  m.impl("linear_splitk_out", &linear_splitk_out);
  m.impl("logmel_out", &logmel_out);
  m.impl("embed_tokens_out", &embed_tokens_out);
  m.impl("attn_decode_out", &attn_decode_out);
  m.impl("argmax_step_out", &argmax_step_out);
  m.impl("dec_linear_out", &dec_linear_out);
}
