// mb_calib.hip -- calibration microbenchmarks for the measurement of the IPM kernels (dev tool,
// run on the GPU box; not part of the library).
//
//  mode "fetch8" / "fetch16": stream-read a 1 GiB buffer with 8 / 16 B per lane (the IPM kernels'
//      vector passes issue 8 B per lane: global_load_dwordx2), so that rocprofv3's FETCH_SIZE can be
//      compared with the known byte count (MI355X_MICROARCH.md: FETCH_SIZE reports 1/2 of a
//      16 B/lane streaming read on gfx950; other widths uncalibrated);
//  mode "write8" / "write16": the same for stores (WRITE_SIZE);
//  mode "scratch": a kernel whose callee saves / restores 48 VGPRs per call (the AMDGPU calling
//      convention's callee-saved stripes), to price a call's scratch traffic;
//  mode "launch": a chain of dependent launches of an almost empty 4096-workgroup kernel
//      (one 64-lane wave per workgroup, the solver kernels' grid) -- stream launches and one
//      hipGraph replay -- to price a kernel boundary of a phase-per-kernel IPM.
//
// build: hipcc --offload-arch=gfx950 -O3 -o tools/mb_calib tools/mb_calib.hip
#include <hip/hip_runtime.h>

#include <chrono>
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

__global__ void k_fetch8(const double* __restrict__ a, size_t n, double* out) {
  double s = 0.0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) s += a[i];
  if (s == 1.2345) out[0] = s;   // never true: keeps the loads
}
__global__ void k_fetch16(const double2* __restrict__ a, size_t n2, double* out) {
  double s = 0.0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n2; i += (size_t)gridDim.x * blockDim.x) {
    const double2 v = a[i];
    s += v.x + v.y;
  }
  if (s == 1.2345) out[0] = s;
}
__global__ void k_write8(double* __restrict__ a, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    a[i] = (double)i;
}
__global__ void k_write16(double2* __restrict__ a, size_t n2) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n2; i += (size_t)gridDim.x * blockDim.x)
    a[i] = make_double2((double)i, 1.0);
}

// a callee that needs many VGPRs (v40+ stripes are callee-saved: its prologue / epilogue save
// and restore the ones it uses)
__device__ __attribute__((noinline)) double heavy(const double* p, int k) {
  double v[48];
#pragma unroll
  for (int i = 0; i < 48; ++i) v[i] = p[(k + i * 64) & 4095];
  double s = 0.0;
#pragma unroll
  for (int i = 0; i < 48; ++i) s = fma(s, 1.0000001, v[i] * v[(i + 7) % 48]);
  return s;
}
__global__ __launch_bounds__(64) void k_scratch(const double* __restrict__ p, int calls, double* out) {
  double s = 0.0;
  for (int c = 0; c < calls; ++c) s += heavy(p, threadIdx.x + c);
  if (s == 1.2345) out[blockIdx.x] = s;
}

__global__ __launch_bounds__(64) void k_empty(int* flag) {
  if (flag[blockIdx.x] == 12345) flag[blockIdx.x] = 0;   // one load per workgroup, like a done-flag check
}

int main(int argc, char** argv) {
  const char* mode = argc > 1 ? argv[1] : "fetch8";
  const size_t bytes = (size_t)1 << 30;
  double *a = nullptr, *out = nullptr;
  CK(hipMalloc(&out, 1 << 20));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  float ms = 0.f;
  if (!strcmp(mode, "launch")) {
    const int nwg = argc > 2 ? atoi(argv[2]) : 4096, chain = 1000;
    int* flag;
    CK(hipMalloc(&flag, sizeof(int) * nwg));
    CK(hipMemset(flag, 0, sizeof(int) * nwg));
    hipStream_t st;
    CK(hipStreamCreate(&st));
    for (int w = 0; w < 50; ++w) hipLaunchKernelGGL(k_empty, dim3(nwg), dim3(64), 0, st, flag);
    CK(hipStreamSynchronize(st));
    CK(hipEventRecord(e0, st));
    for (int i = 0; i < chain; ++i) hipLaunchKernelGGL(k_empty, dim3(nwg), dim3(64), 0, st, flag);
    CK(hipEventRecord(e1, st));
    CK(hipEventSynchronize(e1));
    CK(hipEventElapsedTime(&ms, e0, e1));
    printf("launch stream: %d dependent launches of %d workgroups: %.3f ms, %.2f us per launch\n", chain, nwg, ms,
           1e3 * ms / chain);
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(st, hipStreamCaptureModeGlobal));
    for (int i = 0; i < 100; ++i) hipLaunchKernelGGL(k_empty, dim3(nwg), dim3(64), 0, st, flag);
    CK(hipStreamEndCapture(st, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    CK(hipGraphLaunch(ge, st));
    CK(hipStreamSynchronize(st));
    CK(hipEventRecord(e0, st));
    for (int r = 0; r < 10; ++r) CK(hipGraphLaunch(ge, st));
    CK(hipEventRecord(e1, st));
    CK(hipEventSynchronize(e1));
    CK(hipEventElapsedTime(&ms, e0, e1));
    printf("launch graph: %d dependent kernel nodes of %d workgroups: %.3f ms, %.2f us per node\n", 1000, nwg, ms,
           1e3 * ms / 1000);
    // host cost of issuing the launches (the CPU side of a phase-per-kernel solve)
    auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < chain; ++i) hipLaunchKernelGGL(k_empty, dim3(nwg), dim3(64), 0, st, flag);
    auto t1 = std::chrono::steady_clock::now();
    CK(hipStreamSynchronize(st));
    printf("launch host: %.2f us per hipLaunchKernelGGL call\n",
           std::chrono::duration<double, std::micro>(t1 - t0).count() / chain);
    return 0;
  }
  if (!strcmp(mode, "scratch")) {
    const int nwg = 4096, calls = 100;
    double* p;
    CK(hipMalloc(&p, 4096 * sizeof(double)));
    CK(hipMemset(p, 0, 4096 * sizeof(double)));
    hipLaunchKernelGGL(k_scratch, dim3(nwg), dim3(64), 0, 0, p, calls, out);
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    hipLaunchKernelGGL(k_scratch, dim3(nwg), dim3(64), 0, 0, p, calls, out);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    CK(hipEventElapsedTime(&ms, e0, e1));
    printf("scratch: %d workgroups x %d calls: %.3f ms\n", nwg, calls, ms);
    return 0;
  }
  CK(hipMalloc(&a, bytes));
  CK(hipMemset(a, 0, bytes));
  const size_t n = bytes / sizeof(double);
  for (int rep = 0; rep < 3; ++rep) {
    CK(hipEventRecord(e0));
    if (!strcmp(mode, "fetch8")) hipLaunchKernelGGL(k_fetch8, dim3(4096), dim3(256), 0, 0, a, n, out);
    else if (!strcmp(mode, "fetch16")) hipLaunchKernelGGL(k_fetch16, dim3(4096), dim3(256), 0, 0, (double2*)a, n / 2, out);
    else if (!strcmp(mode, "write8")) hipLaunchKernelGGL(k_write8, dim3(4096), dim3(256), 0, 0, a, n);
    else hipLaunchKernelGGL(k_write16, dim3(4096), dim3(256), 0, 0, (double2*)a, n / 2);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    CK(hipEventElapsedTime(&ms, e0, e1));
    printf("%s: %zu bytes in %.3f ms = %.1f GB/s\n", mode, bytes, ms, bytes / (ms * 1e6));
  }
  return 0;
}
