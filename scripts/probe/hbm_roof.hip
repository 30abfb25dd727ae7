// HBM roof probe (MI355X / gfx950): streaming read-only, write-only, copy and 2:1 read:write
// bandwidth with a working set far above the 256 MB MALL (default 4 GiB per buffer set), on one
// stream and on two concurrent streams (the two-frame-lane case).  Every kernel is a grid-stride
// loop of 16-byte vector accesses, UNROLL independent accesses in flight per lane; the grid is
// swept over workgroups-per-CU so the table shows the occupancy at which the roof is reached.
//
// Output: one line per (pattern, streams, grid, unroll) with bytes moved / time in TB/s (1e12).
// Build: hipcc --offload-arch=gfx950 -O3 -o hbm_roof hbm_roof.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>

typedef __attribute__((ext_vector_type(4))) unsigned u32x4;

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1); } } while (0)

// read-only: XOR-fold into a register, one predicated store per thread keeps the loads live
template <int U>
__global__ __launch_bounds__(256) void k_read(const u32x4* __restrict__ a, size_t n, unsigned* sink) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  u32x4 acc = {0u, 0u, 0u, 0u};
  for (; i + (U - 1) * stride < n; i += U * stride) {
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = __builtin_nontemporal_load(a + i + u * stride);
#pragma unroll
    for (int u = 0; u < U; ++u) acc ^= v[u];
  }
  for (; i < n; i += stride) acc ^= a[i];
  if ((acc[0] ^ acc[1] ^ acc[2] ^ acc[3]) == 0x9e3779b9u) sink[threadIdx.x] = acc[0];
}

template <int U>
__global__ __launch_bounds__(256) void k_write(u32x4* __restrict__ c, size_t n, unsigned seed) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const u32x4 v = {seed, seed + 1u, seed + 2u, seed + 3u};
  for (; i + (U - 1) * stride < n; i += U * stride) {
#pragma unroll
    for (int u = 0; u < U; ++u) __builtin_nontemporal_store(v, c + i + u * stride);
  }
  for (; i < n; i += stride) c[i] = v;
}

template <int U>
__global__ __launch_bounds__(256) void k_copy(const u32x4* __restrict__ a, u32x4* __restrict__ c, size_t n) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i + (U - 1) * stride < n; i += U * stride) {
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = __builtin_nontemporal_load(a + i + u * stride);
#pragma unroll
    for (int u = 0; u < U; ++u) __builtin_nontemporal_store(v[u], c + i + u * stride);
  }
  for (; i < n; i += stride) c[i] = a[i];
}

// 2:1 read:write (c = a ^ b), the shape of a conv with a residual input
template <int U>
__global__ __launch_bounds__(256) void k_r2w1(const u32x4* __restrict__ a, const u32x4* __restrict__ b,
                                              u32x4* __restrict__ c, size_t n) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i + (U - 1) * stride < n; i += U * stride) {
    u32x4 v[U], w[U];
#pragma unroll
    for (int u = 0; u < U; ++u) { v[u] = __builtin_nontemporal_load(a + i + u * stride);
                                  w[u] = __builtin_nontemporal_load(b + i + u * stride); }
#pragma unroll
    for (int u = 0; u < U; ++u) __builtin_nontemporal_store(v[u] ^ w[u], c + i + u * stride);
  }
  for (; i < n; i += stride) c[i] = a[i] ^ b[i];
}

struct Set { u32x4 *a, *b, *c; unsigned* sink; size_t n; hipStream_t s; };

static void launch(int pat, int unroll, int grid, Set& st) {
#define L(U) \
  switch (pat) { \
    case 0: hipLaunchKernelGGL(k_read<U>, dim3(grid), dim3(256), 0, st.s, st.a, st.n, st.sink); break; \
    case 1: hipLaunchKernelGGL(k_write<U>, dim3(grid), dim3(256), 0, st.s, st.c, st.n, 7u); break; \
    case 2: hipLaunchKernelGGL(k_copy<U>, dim3(grid), dim3(256), 0, st.s, st.a, st.c, st.n); break; \
    default: hipLaunchKernelGGL(k_r2w1<U>, dim3(grid), dim3(256), 0, st.s, st.a, st.b, st.c, st.n); }
  if (unroll == 1) { L(1) } else if (unroll == 2) { L(2) } else if (unroll == 4) { L(4) } else { L(8) }
#undef L
}

static double bytes_of(int pat, size_t n) {
  const double v = (double)n * 16.0;
  return pat == 0 ? v : pat == 1 ? v : pat == 2 ? 2 * v : 3 * v;
}

int main(int argc, char** argv) {
  // per-set working set in GiB (each of a, b, c is this size; default 4 GiB each)
  const double gib = argc > 1 ? atof(argv[1]) : 4.0;
  const int reps = argc > 2 ? atoi(argv[2]) : 5;
  hipDeviceProp_t prop;
  CHECK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  printf("# device %s, %d CUs, working set %.1f GiB per buffer (3 buffers per stream set)\n",
         prop.gcnArchName, cus, gib);
  const size_t n = (size_t)(gib * (1ull << 30)) / 16;
  Set sets[2];
  for (int k = 0; k < 2; ++k) {
    CHECK(hipMalloc(&sets[k].a, n * 16));
    CHECK(hipMalloc(&sets[k].b, n * 16));
    CHECK(hipMalloc(&sets[k].c, n * 16));
    CHECK(hipMalloc(&sets[k].sink, 4096));
    CHECK(hipMemset(sets[k].a, 1, n * 16));
    CHECK(hipMemset(sets[k].b, 2, n * 16));
    CHECK(hipMemset(sets[k].c, 3, n * 16));
    sets[k].n = n;
    CHECK(hipStreamCreateWithFlags(&sets[k].s, hipStreamNonBlocking));
  }
  CHECK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  const char* names[4] = {"read", "write", "copy", "r2w1"};
  const int wpc[4] = {2, 4, 8, 16};  // 256-thread workgroups per CU
  const int unrolls[3] = {1, 4, 8};
  double best[4][2] = {{0}};
  printf("%-6s %-7s %-6s %-6s %-9s\n", "pat", "streams", "wg/CU", "unroll", "TB/s");
  for (int pat = 0; pat < 4; ++pat) {
    for (int ns = 1; ns <= 2; ++ns) {
      for (int w : wpc) {
        for (int u : unrolls) {
          const int grid = cus * w / ns;  // the streams share the chip: same total grid
          for (int k = 0; k < ns; ++k) launch(pat, u, grid, sets[k]);
          CHECK(hipDeviceSynchronize());
          CHECK(hipEventRecord(e0, 0));
          for (int r = 0; r < reps; ++r) {
            // fork: the side streams wait on the start event; the null stream joins them at the end
            for (int k = 0; k < ns; ++k) {
              CHECK(hipStreamWaitEvent(sets[k].s, e0, 0));
              launch(pat, u, grid, sets[k]);
            }
          }
          for (int k = 0; k < ns; ++k) {
            hipEvent_t j;
            CHECK(hipEventCreateWithFlags(&j, hipEventDisableTiming));
            CHECK(hipEventRecord(j, sets[k].s));
            CHECK(hipStreamWaitEvent(0, j, 0));
            CHECK(hipEventDestroy(j));
          }
          CHECK(hipEventRecord(e1, 0));
          CHECK(hipEventSynchronize(e1));
          float ms = 0.f;
          CHECK(hipEventElapsedTime(&ms, e0, e1));
          const double tbs = bytes_of(pat, n) * ns * reps / (ms * 1e-3) / 1e12;
          printf("%-6s %-7d %-6d %-6d %-9.3f\n", names[pat], ns, w, u, tbs);
          fflush(stdout);
          if (tbs > best[pat][ns - 1]) best[pat][ns - 1] = tbs;
        }
      }
    }
  }
  printf("# best TB/s: pattern  1-stream  2-streams\n");
  for (int pat = 0; pat < 4; ++pat) printf("# %-6s %.3f %.3f\n", names[pat], best[pat][0], best[pat][1]);
  // torch-independent sanity: hipMemcpy D2D of the same working set
  CHECK(hipEventRecord(e0, 0));
  for (int r = 0; r < reps; ++r) CHECK(hipMemcpyAsync(sets[0].c, sets[0].a, n * 16, hipMemcpyDeviceToDevice, 0));
  CHECK(hipEventRecord(e1, 0));
  CHECK(hipEventSynchronize(e1));
  float ms = 0.f;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  printf("# hipMemcpyAsync D2D: %.3f TB/s (read+write bytes)\n", 2.0 * n * 16 * reps / (ms * 1e-3) / 1e12);
  for (int k = 0; k < 2; ++k) {
    hipFree(sets[k].a); hipFree(sets[k].b); hipFree(sets[k].c); hipFree(sets[k].sink);
    hipStreamDestroy(sets[k].s);
  }
  return 0;
}
