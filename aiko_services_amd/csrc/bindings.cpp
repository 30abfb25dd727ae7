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
int aiko_preprocess(const void* in, void* out, int B, int Hin, int Win, int Ho, int Wo, int Hp,
                    int Wp, int pad_t, int pad_l, const float* mean, const float* std, int bgr,
                    hipStream_t stream);
int aiko_maxpool(const void* x, void* y, int B, int H, int W, int C, int Ho, int Wo, int k,
                 int s, int p, hipStream_t stream);
int aiko_avgpool(const void* x, void* y, int B, int HW, int C, hipStream_t stream);
int aiko_softmax_topk(const void* logits, float* prob, int* index, int B, int N, int k,
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
//         K1, H2, W2, C2, stride2]   (the last five describe the optional second source x2)
void conv_igemm_out(const at::Tensor& x, const c10::optional<at::Tensor>& x2, const at::Tensor& w,
                    const c10::optional<at::Tensor>& bias, const c10::optional<at::Tensor>& res,
                    at::Tensor& y, at::IntArrayRef geom) {
  TORCH_CHECK(geom.size() == 21, "aiko.conv_igemm_out: geom needs 21 ints");
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
  TORCH_CHECK(Cc % 8 == 0 && Cc <= C || (C == 4 && Cc == 32), "aiko.conv_igemm_out: Cc must be a multiple of 8 within the pixel pitch");
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
  const int rc = aiko_conv_igemm(x.data_ptr(), w.data_ptr(), bptr, rptr, y.data_ptr(), H, W, C,
                                 Cc, R, S, stride, pad, Ho, Wo, M, Cout, K, act, ldy,
                                 ldr, bm, bn, x2ptr, K1, H2, W2, C2, stride2, cur_stream());
  check_launch(rc, "conv_igemm");
}

void preprocess_out(const at::Tensor& frames, at::Tensor& out, int64_t Ho, int64_t Wo,
                    int64_t pad_t, int64_t pad_l, at::ArrayRef<double> mean,
                    at::ArrayRef<double> std, bool bgr) {
  check_cuda(frames, "frames");
  check_cuda(out, "out");
  TORCH_CHECK(frames.scalar_type() == at::kByte && frames.dim() == 4 && frames.size(3) == 3 &&
                  frames.is_contiguous(),
              "aiko.preprocess_out: frames must be uint8 [B, H, W, 3] contiguous");
  TORCH_CHECK(out.scalar_type() == at::kBFloat16 && out.dim() == 4 && out.size(3) == 4 &&
                  out.is_contiguous() && out.size(0) == frames.size(0),
              "aiko.preprocess_out: out must be bf16 [B, Hp, Wp, 4] contiguous");
  TORCH_CHECK(mean.size() == 3 && std.size() == 3, "aiko.preprocess_out: mean/std need 3 values");
  TORCH_CHECK(pad_t + Ho <= out.size(1) && pad_l + Wo <= out.size(2), "aiko.preprocess_out: out too small");
  float m[3] = {(float)mean[0], (float)mean[1], (float)mean[2]};
  float s[3] = {(float)std[0], (float)std[1], (float)std[2]};
  const int rc = aiko_preprocess(frames.data_ptr(), out.data_ptr(), frames.size(0), frames.size(1),
                                 frames.size(2), Ho, Wo, out.size(1), out.size(2), pad_t, pad_l, m,
                                 s, bgr ? 1 : 0, cur_stream());
  check_launch(rc, "preprocess");
}

void maxpool_out(const at::Tensor& x, at::Tensor& y, int64_t k, int64_t s, int64_t p) {
  check_cuda(x, "x");
  check_cuda(y, "y");
  TORCH_CHECK(x.scalar_type() == at::kBFloat16 && y.scalar_type() == at::kBFloat16 &&
                  x.dim() == 4 && y.dim() == 4 && x.is_contiguous() && y.is_contiguous(),
              "aiko.maxpool_out: NHWC bf16 contiguous tensors required");
  const int64_t B = x.size(0), H = x.size(1), W = x.size(2), C = x.size(3);
  TORCH_CHECK(C % 8 == 0 && y.size(0) == B && y.size(3) == C, "aiko.maxpool_out: bad shapes");
  const int64_t Ho = (H + 2 * p - k) / s + 1, Wo = (W + 2 * p - k) / s + 1;
  TORCH_CHECK(y.size(1) == Ho && y.size(2) == Wo, "aiko.maxpool_out: y must be [B, ", Ho, ", ", Wo, ", C]");
  check_launch(aiko_maxpool(x.data_ptr(), y.data_ptr(), B, H, W, C, Ho, Wo, k, s, p, cur_stream()),
               "maxpool");
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

}  // namespace

TORCH_LIBRARY(aiko, m) {
  m.def("conv_igemm_out(Tensor x, Tensor? x2, Tensor w, Tensor? bias, Tensor? res, Tensor(a!) y, int[] geom) -> ()");
  m.def("preprocess_out(Tensor frames, Tensor(a!) out, int Ho, int Wo, int pad_t, int pad_l, float[] mean, float[] std, bool bgr) -> ()");
  m.def("maxpool_out(Tensor x, Tensor(a!) y, int k, int s, int p) -> ()");
  m.def("avgpool_out(Tensor x, Tensor(a!) y) -> ()");
  m.def("softmax_topk_out(Tensor logits, Tensor(a!) prob, Tensor(b!) index, int k) -> ()");
}

TORCH_LIBRARY_IMPL(aiko, CUDA, m) {
  m.impl("conv_igemm_out", &conv_igemm_out);
  m.impl("preprocess_out", &preprocess_out);
  m.impl("maxpool_out", &maxpool_out);
  m.impl("avgpool_out", &avgpool_out);
  m.impl("softmax_topk_out", &softmax_topk_out);
}
