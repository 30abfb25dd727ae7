// Probe: how v_mfma_scale_f32_16x16x128_f8f6f4 maps per-lane A scales onto (row, k-block).
// A = 1.0 everywhere except one k-block per experiment; B = 1.0.  Lane l's A scale = 2^(l % 8)
// ... printed outputs reveal which lane's scale applies to which rows / k ranges.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef __attribute__((ext_vector_type(8))) int i32x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;

__global__ void probe(float* out, int kb_only) {
  const int lane = threadIdx.x;
  // e4m3 1.0 = 0x38; zero = 0x00.  lane holds row lane%16, k = 32*(lane/16) .. +31
  const int g = lane >> 4;
  const int v = (kb_only < 0 || g == kb_only) ? 0x38383838 : 0;
  i32x8 a = {v, v, v, v, v, v, v, v};
  i32x8 b = {0x38383838, 0x38383838, 0x38383838, 0x38383838, 0x38383838, 0x38383838, 0x38383838, 0x38383838};
  const int sa = 127 + (lane & 15) % 4 + 4 * g;     // distinct per (row%4, g)
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  acc = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, acc, 0, 0, 0, sa, 0, 127);
  for (int e = 0; e < 4; ++e) out[lane * 4 + e] = acc[e];
}

int main() {
  float* d;
  hipMalloc(&d, 256 * 4);
  float h[256];
  for (int kb = -1; kb < 4; ++kb) {
    probe<<<1, 64>>>(d, kb);
    hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    printf("A nonzero only in lane-group k-block %d:\n", kb);
    // output layout: lane l, element e -> row 4*(l/16)+e, col l%16
    for (int r = 0; r < 16; ++r) {
      const int l = (r / 4) * 16 + 0, e = r % 4;
      printf("  row %2d col 0: %g\n", r, h[l * 4 + e]);
    }
  }
  return 0;
}
