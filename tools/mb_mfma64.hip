// mb_mfma64.hip -- FP64 issue-rate microbenchmark (dev tool, run on the GPU box; not part of the
// library): the peak the IPM's small dense blocks could reach on the vector ALUs and on the
// matrix cores of gfx950.
//
//   valu    : v_fma_f64, 8 independent chains per lane
//   mfma4   : v_mfma_f64_4x4x4f64 (four 4x4x4 blocks per instruction -- the shape of the 4x4
//             Riccati products of four egos), 4 independent accumulators per wave
//   mfma16  : v_mfma_f64_16x16x4f64, 4 independent accumulators per wave
//   ric     : the Riccati node product Pn = A' P A of 16 egos per wave in one MFMA form (two
//             4x4x4 products per block, 4 blocks per instruction) against the same product on
//             the vector ALUs (lane = ego x row, row gathers through ds_bpermute), checked
//             against each other; time per 4096 egos x 64 nodes
//
// Every variant runs a grid of 2048 workgroups x 256 lanes (8 waves per CU on 256 CUs), times
// with HIP events, prints TFLOP/s (2 flops per FMA).
// build: hipcc --offload-arch=gfx950 -O3 -o tools/mb_mfma64 tools/mb_mfma64.hip
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

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
  double c[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) c[i] = threadIdx.x * 1e-9 + i;
  for (int it = 0; it < iters; ++it)
#pragma unroll
    for (int i = 0; i < 8; ++i) c[i] = fma(c[i], a, 1e-7);
  double s = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) s += c[i];
  if (s == 1.2345) out[blockIdx.x] = s;   // keep the chains alive
}

__global__ __launch_bounds__(256) void k_mfma4(double* out, int iters, double a) {
  double c[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) c[i] = threadIdx.x * 1e-9 + i;
  const double b = a * 0.5;
  for (int it = 0; it < iters; ++it)
#pragma unroll
    for (int i = 0; i < 4; ++i) c[i] = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c[i], 0, 0, 0);
  double s = c[0] + c[1] + c[2] + c[3];
  if (s == 1.2345) out[blockIdx.x] = s;
}

__global__ __launch_bounds__(256) void k_mfma16(double* out, int iters, double a) {
  d4 c[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) c[i] = d4{threadIdx.x * 1e-9, 1.0 * i, 0.5, 0.25};
  const double b = a * 0.5;
  for (int it = 0; it < iters; ++it)
#pragma unroll
    for (int i = 0; i < 4; ++i) c[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c[i], 0, 0, 0);
  double s = 0;
#pragma unroll
  for (int i = 0; i < 4; ++i) s += c[i].x + c[i].y + c[i].z + c[i].w;
  if (s == 1.2345) out[blockIdx.x] = s;
}

// ---- Riccati-shaped product Pn = A' (P A) for 16 egos per wave ---------------------------------
// data: per ego e and node k, A[4][4] and P[4][4] (row-major), interleaved 16 egos per group:
// X[((g * nodes + k) * 16 + entry) * 16 + e16], so one load of 64 lanes reads 4 entries of 16 egos.
// VALU form: lane (e16 = lane / 4, i = lane % 4) owns row i of its ego; rows of the other matrices
// come from the lanes of the ego's quad (ds_bpermute).
__device__ __forceinline__ double quad_get(double v, int src_lane) {
  const int lo = __builtin_amdgcn_ds_bpermute(src_lane << 2, __double2loint(v));
  const int hi = __builtin_amdgcn_ds_bpermute(src_lane << 2, __double2hiint(v));
  return __hiloint2double(hi, lo);
}

__global__ __launch_bounds__(64) void k_ric_valu(const double* __restrict__ A, const double* __restrict__ P,
                                                 double* __restrict__ O, int nodes) {
  const int g = blockIdx.x, lane = threadIdx.x, e16 = lane >> 2, i = lane & 3, q0 = lane & ~3;
  for (int k = 0; k < nodes; ++k) {
    const size_t base = (size_t)(g * nodes + k) * 256;
    double ar[4], pr[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      ar[j] = A[base + (i * 4 + j) * 16 + e16];
      pr[j] = P[base + (i * 4 + j) * 16 + e16];
    }
    // M = P A (own row i): M[i][j] = sum_r P[i][r] A[r][j]; A's rows from the quad
    double m[4] = {0, 0, 0, 0};
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int j = 0; j < 4; ++j) m[j] += pr[r] * quad_get(ar[j], q0 + r);
    // Pn = A' M (own row i): Pn[i][j] = sum_r A[r][i] M[r][j]
    double o[4] = {0, 0, 0, 0};
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      double ari = 0.0;
#pragma unroll
      for (int c = 0; c < 4; ++c) ari = c == i ? quad_get(ar[c], q0 + r) : ari;   // A[r][i]
#pragma unroll
      for (int j = 0; j < 4; ++j) o[j] += ari * quad_get(m[j], q0 + r);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) O[base + (i * 4 + j) * 16 + e16] = o[j];
  }
}

// MFMA form: v_mfma_f64_4x4x4f64 multiplies four independent 4x4 blocks per instruction; the 16
// egos of the group are 4 instructions.  Operand layout: see the layout probe in main (the block
// of lane l is l / 16; the probe fixes the (row, k) and (k, col) of each lane).
__global__ __launch_bounds__(64) void k_ric_mfma(const double* __restrict__ A, const double* __restrict__ P,
                                                 double* __restrict__ O, int nodes, const int* __restrict__ lay) {
  const int g = blockIdx.x, lane = threadIdx.x;
  // lay[0..63]: A-operand (row, k) of each lane as row*4+k; lay[64..127]: B-operand (k, col) as
  // k*4+col; lay[128..191]: D element (row, col) as row*4+col
  const int ao = lay[lane], bo = lay[64 + lane], dop = lay[128 + lane];
  const int blk = lane >> 4;
  for (int k = 0; k < nodes; ++k) {
    const size_t base = (size_t)(g * nodes + k) * 256;
#pragma unroll
    for (int h = 0; h < 4; ++h) {   // egos 4h .. 4h + 3, one per block
      const int e = h * 4 + blk;
      // M = P A: A-operand P[row][k], B-operand A[k][col]
      const double pa = P[base + ao * 16 + e], ab = A[base + bo * 16 + e];
      const double m = __builtin_amdgcn_mfma_f64_4x4x4f64(pa, ab, 0.0, 0, 0, 0);
      // Pn = A' M: A-operand A'[row][k] = A[k][row], B-operand M[k][col] (D layout -> B layout)
      const int ar = ao >> 2, ak = ao & 3;
      const double at = A[base + (ak * 4 + ar) * 16 + e];
      // M's element (k, col) for this lane's B slot lives in the lane whose D slot is (k, col)
      int src = 0;
      for (int l = 0; l < 16; ++l) src = lay[128 + (blk << 4) + l] == bo ? (blk << 4) + l : src;
      const double mb = quad_get(m, src);
      const double o = __builtin_amdgcn_mfma_f64_4x4x4f64(at, mb, 0.0, 0, 0, 0);
      O[base + dop * 16 + e] = o;
    }
  }
}

// layout probes of v_mfma_f64_4x4x4f64 (block 0 = lanes 0..15; the other blocks repeat it):
//   out[l]            D of A = 2^l, B = 1      -> the A lanes of each output's row
//   out[64 + l]       D of A = 1, B = 2^l      -> the B lanes of each output's column
//   out[128 + 64b + l] D of A = 2^l, B = [l == b] -> the A lanes paired (same k) with B lane b
__global__ void k_probe(double* out) {
  const int lane = threadIdx.x;
  const double bit = 1.0 * (1 << (lane & 15));
  out[lane] = __builtin_amdgcn_mfma_f64_4x4x4f64(bit, 1.0, 0.0, 0, 0, 0);
  out[64 + lane] = __builtin_amdgcn_mfma_f64_4x4x4f64(1.0, bit, 0.0, 0, 0, 0);
  for (int b = 0; b < 16; ++b)
    out[128 + 64 * b + lane] = __builtin_amdgcn_mfma_f64_4x4x4f64(bit, (lane & 15) == b ? 1.0 : 0.0, 0.0, 0, 0, 0);
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
    run("valu", [](int it) { k_valu<<<kBlocks, kThreads>>>(g_out, it, 0.999); }, 64.0 * 8 * 2);
    run("mfma4", [](int it) { k_mfma4<<<kBlocks, kThreads>>>(g_out, it, 0.999); }, 4.0 * 4 * 4 * 4 * 2 * 4);
    run("mfma16", [](int it) { k_mfma16<<<kBlocks, kThreads>>>(g_out, it, 0.999); }, 16.0 * 16 * 4 * 2 * 4);
  }
  if (!strcmp(mode, "all") || !strcmp(mode, "ric")) {
    // operand layout of v_mfma_f64_4x4x4f64 from the probes
    std::vector<double> h(128 + 64 * 16);
    k_probe<<<1, 64>>>(g_out);
    CK(hipMemcpy(h.data(), g_out, h.size() * 8, hipMemcpyDeviceToHost));
    std::vector<int> lay(192, -1);
    auto label = [](std::vector<long long>& sets, long long v) {
      for (size_t i = 0; i < sets.size(); ++i)
        if (sets[i] == v) return (int)i;
      sets.push_back(v);
      return (int)sets.size() - 1;
    };
    std::vector<long long> rows, cols, ks;
    int rowof[16], colof[16], arow[16], bcol[16], kA[16], kB[16];
    for (int o = 0; o < 16; ++o) {
      rowof[o] = label(rows, std::llround(h[o]));
      colof[o] = label(cols, std::llround(h[64 + o]));
    }
    for (int l = 0; l < 16; ++l)
      for (int r = 0; r < (int)rows.size(); ++r) {
        if (rows[r] >> l & 1) arow[l] = r;
        if (r < (int)cols.size() && cols[r] >> l & 1) bcol[l] = r;
      }
    for (int b = 0; b < 16; ++b) {   // A lanes paired with B lane b: the nonzero outputs' bits
      long long set = 0;
      for (int o = 0; o < 16; ++o) set |= std::llround(h[128 + 64 * b + o]);
      kB[b] = label(ks, set);
      for (int l = 0; l < 16; ++l)
        if (set >> l & 1) kA[l] = kB[b];
    }
    for (int l = 0; l < 16; ++l) {
      lay[l] = arow[l] * 4 + kA[l];
      lay[64 + l] = kB[l] * 4 + bcol[l];
      lay[128 + l] = rowof[l] * 4 + colof[l];
    }
    for (int l = 16; l < 64; ++l)
      for (int t = 0; t < 3; ++t) lay[t * 64 + l] = lay[t * 64 + (l & 15)];
    printf("mfma_f64_4x4x4 layout (block 0): A (row,k) / B (k,col) / D (row,col) per lane:\n");
    for (int l = 0; l < 16; ++l)
      printf("  lane %2d: A(%d,%d) B(%d,%d) D(%d,%d)\n", l, lay[l] >> 2, lay[l] & 3, lay[64 + l] >> 2, lay[64 + l] & 3,
             lay[128 + l] >> 2, lay[128 + l] & 3);
    const int egos = 4096, nodes = 64, groups = egos / 16;
    const size_t n = (size_t)groups * nodes * 256;
    std::vector<double> hA(n), hP(n);
    srand(7);
    for (size_t i = 0; i < n; ++i) hA[i] = rand() / (double)RAND_MAX - 0.5, hP[i] = rand() / (double)RAND_MAX;
    double *dA, *dP, *dO1, *dO2;
    int* dl;
    CK(hipMalloc(&dA, n * 8));
    CK(hipMalloc(&dP, n * 8));
    CK(hipMalloc(&dO1, n * 8));
    CK(hipMalloc(&dO2, n * 8));
    CK(hipMalloc(&dl, 192 * 4));
    CK(hipMemcpy(dA, hA.data(), n * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(dP, hP.data(), n * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(dl, lay.data(), 192 * 4, hipMemcpyHostToDevice));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    float tv = 1e9, tm = 1e9;
    for (int rep = 0; rep < 5; ++rep) {
      float ms;
      CK(hipEventRecord(e0));
      k_ric_valu<<<groups, 64>>>(dA, dP, dO1, nodes);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      CK(hipEventElapsedTime(&ms, e0, e1));
      tv = ms < tv ? ms : tv;
      CK(hipEventRecord(e0));
      k_ric_mfma<<<groups, 64>>>(dA, dP, dO2, nodes, dl);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      CK(hipEventElapsedTime(&ms, e0, e1));
      tm = ms < tm ? ms : tm;
    }
    std::vector<double> o1(n), o2(n);
    CK(hipMemcpy(o1.data(), dO1, n * 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(o2.data(), dO2, n * 8, hipMemcpyDeviceToHost));
    // host check of one group / node
    double md = 0, mh = 0;
    for (size_t i = 0; i < n; ++i) md = fmax(md, fabs(o1[i] - o2[i]));
    for (int e = 0; e < 16; ++e)
      for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) {
          double s = 0;
          for (int r = 0; r < 4; ++r)
            for (int c = 0; c < 4; ++c) s += hA[(r * 4 + i) * 16 + e] * hP[(r * 4 + c) * 16 + e] * hA[(c * 4 + j) * 16 + e];
          mh = fmax(mh, fabs(s - o1[(i * 4 + j) * 16 + e]));
        }
    const double gb = 3.0 * n * 8 / 1e9;
    printf("ric A'PA, 4096 egos x 64 nodes: valu %.3f ms (%.0f GB/s), mfma %.3f ms (%.0f GB/s); "
           "max |valu - mfma| %.2e, max |valu - host| %.2e\n", tv, gb / (tv * 1e-3), tm, gb / (tm * 1e-3), md, mh);
  }
  return 0;
}
