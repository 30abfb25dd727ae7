// Whisper front end for gfx950: log-mel spectrogram of 16 kHz audio, fully on the GPU.
//
// logmel_kernel: one 256-thread workgroup per 16 STFT frames of one clip.  Frames (n_fft 400,
// hop 160, centred with reflect padding, periodic Hann window) are staged in LDS; the 201-bin
// power spectrum is a direct DFT against an LDS twiddle table (0.26 MFLOP per frame: a few
// microseconds for a 30 s clip, not worth an FFT's passes at this size); the mel filterbank
// (80 x 201, in L2) maps it to mel energies; log10(max(e, 1e-10)) is written and the clip's
// maximum is kept with an order-preserving integer atomicMax.
// logmel_finalize_kernel: Whisper's dynamic-range clamp max(x, max - 8), (x + 4) / 4, written
// as bf16 straight into the zero-bordered [rows][80] buffer the first conv reads.
#include "common.h"

namespace aiko {

constexpr int kFPB = 16;         // frames per workgroup
constexpr int kMaxFFT = 400;
constexpr int kMaxBins = kMaxFFT / 2 + 1;

__device__ __forceinline__ int float_order_key(float f) {
  const int i = __float_as_int(f);
  return i >= 0 ? i : i ^ 0x7fffffff;
}
__device__ __forceinline__ float float_from_key(int k) {
  return __int_as_float(k >= 0 ? k : k ^ 0x7fffffff);
}

__global__ __launch_bounds__(256) void logmel_kernel(const float* __restrict__ audio, int N,
                                                      const float* __restrict__ mel, int n_mels,
                                                      int n_fft, int hop, int F,
                                                      float* __restrict__ out, int* __restrict__ gmax) {
  __shared__ float tw_c[kMaxFFT], tw_s[kMaxFFT];
  __shared__ float frame[kFPB][kMaxFFT];
  __shared__ float power[kFPB][kMaxBins];
  __shared__ float red[4];
  const int tid = threadIdx.x;
  const int b = blockIdx.y;
  const int f0 = blockIdx.x * kFPB;
  const int nbins = n_fft / 2 + 1;
  const float* x = audio + (long)b * N;
  for (int n = tid; n < n_fft; n += 256) {
    float s, c;
    sincosf(6.283185307179586f * n / n_fft, &s, &c);
    tw_c[n] = c;
    tw_s[n] = s;
  }
  for (int i = tid; i < kFPB * n_fft; i += 256) {
    const int f = i / n_fft, n = i - f * n_fft;
    float v = 0.f;
    if (f0 + f < F) {
      int idx = (f0 + f) * hop - n_fft / 2 + n;
      if (idx < 0) idx = -idx;
      if (idx >= N) idx = 2 * (N - 1) - idx;
      const float w = 0.5f - 0.5f * cospif(2.f * n / n_fft);
      v = x[idx] * w;
    }
    frame[f][n] = v;
  }
  __syncthreads();
  // one thread per frequency bin, all kFPB frames at once: each twiddle gather from LDS feeds
  // 2 * kFPB FMAs and the frame samples are wave-wide broadcasts
  for (int k = tid; k < nbins; k += 256) {
    float re[kFPB], im[kFPB];
#pragma unroll
    for (int f = 0; f < kFPB; ++f) re[f] = im[f] = 0.f;
    int t = 0;
    for (int n = 0; n < n_fft; ++n) {
      const float c = tw_c[t], sn = tw_s[t];
#pragma unroll
      for (int f = 0; f < kFPB; ++f) {
        const float v = frame[f][n];
        re[f] += v * c;
        im[f] -= v * sn;
      }
      t += k;
      if (t >= n_fft) t -= n_fft;
    }
#pragma unroll
    for (int f = 0; f < kFPB; ++f) power[f][k] = re[f] * re[f] + im[f] * im[f];
  }
  __syncthreads();
  float mx = -INFINITY;
  for (int pr = tid; pr < kFPB * n_mels; pr += 256) {
    const int f = pr / n_mels, m = pr - f * n_mels;
    if (f0 + f >= F) continue;
    const float* w = mel + (long)m * nbins;
    float e = 0.f;
    for (int k = 0; k < nbins; ++k) e += w[k] * power[f][k];
    const float l = log10f(fmaxf(e, 1e-10f));
    out[((long)b * F + f0 + f) * n_mels + m] = l;
    mx = fmaxf(mx, l);
  }
  mx = wave_max(mx);
  if ((tid & 63) == 0) red[tid >> 6] = mx;
  __syncthreads();
  if (tid == 0) {
    const float m = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
    atomicMax(gmax + b, float_order_key(m));
  }
}

// dst rows per clip = rows (>= F + pad + pad_end); frame t of clip b -> row b*rows + pad + t
__global__ void logmel_finalize_kernel(const float* __restrict__ logmel, const int* __restrict__ gmax,
                                       bf16_t* __restrict__ dst, int B, int F, int n_mels, int rows,
                                       int pad, int ld) {
  const long total = (long)B * rows * n_mels;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int m = i % n_mels;
    const long r = i / n_mels;
    const int b = r / rows, row = r - (long)b * rows;
    const int t = row - pad;
    float y = 0.f;
    if (t >= 0 && t < F) {
      const float mx = float_from_key(gmax[b]);
      y = (fmaxf(logmel[((long)b * F + t) * n_mels + m], mx - 8.f) + 4.f) * 0.25f;
    }
    dst[((long)b * rows + row) * ld + m] = f2bf(y);
  }
}

}  // namespace aiko

extern "C" int aiko_logmel(const float* audio, int B, int N, const float* mel, int n_mels,
                           int n_fft, int hop, int F, float* logmel, int* gmax, void* dst, int rows,
                           int pad, int ld, hipStream_t stream) {
  if (n_fft > aiko::kMaxFFT || n_fft % 2) return -1;
  hipMemsetAsync(gmax, 0x80, sizeof(int) * B, stream);  // 0x80808080: below every key
  dim3 grid((F + aiko::kFPB - 1) / aiko::kFPB, B);
  aiko::logmel_kernel<<<grid, 256, 0, stream>>>(audio, N, mel, n_mels, n_fft, hop, F, logmel, gmax);
  const long total = (long)B * rows * n_mels;
  long g = (total + 255) / 256;
  if (g > 4096) g = 4096;
  aiko::logmel_finalize_kernel<<<(int)g, 256, 0, stream>>>(logmel, gmax, static_cast<aiko::bf16_t*>(dst),
                                                          B, F, n_mels, rows, pad, ld);
  return (int)hipGetLastError();
}
