// mb_mfma64.hip -- FP64 issue-rate microbenchmark (dev tool, run on the GPU box; not part of the
// library): the peak the IPM's small dense blocks could reach on the vector ALUs and on the
// matrix cores of gfx950.
//
//   valu    : v_fma_f64, 16 independent chains per lane
//   mfma4   : v_mfma_f64_4x4x4f64 (four 4x4x4 blocks per instruction -- the shape of the 4x4
//             Riccati products of four egos), 8 independent accumulators per wave
//   mfma16  : v_mfma_f64_16x16x4f64, 8 independent accumulators per wave
//
// Every variant runs a grid of 2048 workgroups x 256 lanes (8 waves per CU on 256 CUs), times
// with HIP events, prints TFLOP/s (2 flops per FMA).
// build: hipcc --offload-arch=gfx950 -O3 -o tools/mb_mfma64 tools/mb_mfma64.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>

#define CK(x)                                                                        \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));      \
      exit(1);                                                                       \
    }                                                                                \
  } while (0)

typedef double d4 __attribute__((ext_vector_type(4)));

constexpr int kBlocks = 2048, kThreads = 256;

__global__ __launch_bounds__(256) void k_valu(double* out, int iters, double a) {
  double c[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) c[i] = threadIdx.x * 1e-9 + i;
  for (int it = 0; it < iters; ++it)
#pragma unroll
    for (int i = 0; i < 16; ++i) c[i] = fma(c[i], a, 1e-7);
  double s = 0;
#pragma unroll
  for (int i = 0; i < 16; ++i) s += c[i];
  if (s == 1.2345) out[blockIdx.x] = s;   // keep the chains alive
}

__global__ __launch_bounds__(256) void k_mfma4(double* out, int iters, double a) {
  double c[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) c[i] = threadIdx.x * 1e-9 + i;
  const double b = a * 0.5;
  for (int it = 0; it < iters; ++it)
#pragma unroll
    for (int i = 0; i < 8; ++i) c[i] = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c[i], 0, 0, 0);
  double s = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) s += c[i];
  if (s == 1.2345) out[blockIdx.x] = s;
}

__global__ __launch_bounds__(256) void k_mfma16(double* out, int iters, double a) {
  d4 c[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) c[i] = d4{threadIdx.x * 1e-9, 1.0 * i, 0.5, 0.25};
  const double b = a * 0.5;
  for (int it = 0; it < iters; ++it)
#pragma unroll
    for (int i = 0; i < 8; ++i) c[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c[i], 0, 0, 0);
  double s = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) s += c[i].x + c[i].y + c[i].z + c[i].w;
  if (s == 1.2345) out[blockIdx.x] = s;
}

static float time_kernel(void (*launch)(int), int iters) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  launch(iters / 10 + 1);   // warm
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(e0));
  launch(iters);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  return ms;
}

static double* g_out;

int main(int argc, char** argv) {
  const char* mode = argc > 1 ? argv[1] : "all";
  CK(hipMalloc(&g_out, 1 << 20));
  const int iters = 20000;
  const double waves = (double)kBlocks * kThreads / 64;
  auto run = [&](const char* name, void (*launch)(int), double flop_per_wave_iter) {
    const float ms = time_kernel(launch, iters);
    const double tf = flop_per_wave_iter * waves * iters / (ms * 1e-3) / 1e12;
    printf("%-8s %8.3f ms  %7.2f TFLOP/s (fp64)\n", name, ms, tf);
  };
  if (!strcmp(mode, "all") || !strcmp(mode, "peak")) {
    run("valu", [](int it) { k_valu<<<kBlocks, kThreads>>>(g_out, it, 0.999); }, 64.0 * 16 * 2);
    run("mfma4", [](int it) { k_mfma4<<<kBlocks, kThreads>>>(g_out, it, 0.999); }, 4.0 * 4 * 4 * 4 * 2 * 8);
    run("mfma16", [](int it) { k_mfma16<<<kBlocks, kThreads>>>(g_out, it, 0.999); }, 16.0 * 16 * 4 * 2 * 8);
  }
  return 0;
}
