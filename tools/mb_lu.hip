// mb_lu.hip -- microbenchmark of the coupling LU and its substitutions as the small-batch kernel runs
// them (one 256-lane workgroup, the n x n system in LDS), per variant and per part (dev tool, run on
// the GPU box; not part of the library).  Cycles are s_memtime ticks of lane 0 (the phase
// profiler's clock), averaged over R factorisations of the same matrix.
//
//   block   : small_lu's structure on 4 waves (pivot by two LDS reductions, workgroup barriers)
//   wred    : one wave, pivot by two DPP wave reductions, fences between the steps
//   wscan   : one wave, lane k+1 scans column k+1 during the update (no reductions)
//   wnoupd  : wred without the trailing update (the per-pivot overhead)
//   wupd    : the trailing update alone (pivot k, no search, no swap)
//   solve_lds / solve_reg : the permutation + L + U substitutions on one wave, b in LDS / registers
//
// build: hipcc --offload-arch=gfx950 -O3 -o tools/mb_lu tools/mb_lu.hip
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

typedef __attribute__((address_space(3))) double ldouble;

__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}
template <int CTRL>
__device__ __forceinline__ double dpp_d(double v) {
  const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), CTRL, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), CTRL, 0xF, 0xF, false);
  return __hiloint2double(hi, lo);
}
template <int OP>
__device__ __forceinline__ double red_op(double a, double b) { return OP == 1 ? fmax(a, b) : fmin(a, b); }
template <int O, int OP>
__device__ __forceinline__ double xor_level(double v) {
  if constexpr (O == 32 || O == 16) {
    const unsigned lo = __double2loint(v), hi = __double2hiint(v);
    const auto a = O == 32 ? __builtin_amdgcn_permlane32_swap(lo, lo, false, false)
                           : __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
    const auto b = O == 32 ? __builtin_amdgcn_permlane32_swap(hi, hi, false, false)
                           : __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
    const double x = __hiloint2double(b[0], a[0]), y = __hiloint2double(b[1], a[1]);
    return (__lane_id() & O) == 0 ? red_op<OP>(x, y) : red_op<OP>(y, x);
  } else if constexpr (O == 8) {
    return red_op<OP>(v, dpp_d<0x128>(v));
  } else if constexpr (O == 4) {
    const double up = dpp_d<0x114>(v), dn = dpp_d<0x104>(v);
    return red_op<OP>(v, (__lane_id() & 4) ? up : dn);
  } else if constexpr (O == 2) {
    return red_op<OP>(v, dpp_d<0x4E>(v));
  } else {
    return red_op<OP>(v, dpp_d<0xB1>(v));
  }
}
template <int OP>
__device__ __forceinline__ double wave_reduce(double v) {
  v = xor_level<32, OP>(v);
  v = xor_level<16, OP>(v);
  v = xor_level<8, OP>(v);
  v = xor_level<4, OP>(v);
  v = xor_level<2, OP>(v);
  return xor_level<1, OP>(v);
}
__device__ __forceinline__ double bcast(double v, int l) {
  return __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(v), l),
                          __builtin_amdgcn_readlane(__double2loint(v), l));
}

// block reduction over 4 waves (one barrier, two buffers in turn)
__device__ double block_red(int OP, double v, ldouble* red, int& turn) {
  v = OP == 1 ? wave_reduce<1>(v) : wave_reduce<2>(v);
  const int wv = threadIdx.x >> 6;
  ldouble* buf = red + (turn ? 4 : 0);
  if ((threadIdx.x & 63) == 0) buf[wv] = v;
  turn ^= 1;
  __syncthreads();
  double a = buf[0];
  for (int w = 1; w < 4; ++w) a = OP == 1 ? fmax(a, buf[w]) : fmin(a, buf[w]);
  return a;
}

__device__ void lu_block(ldouble* M, ldouble* piv, int n, ldouble* red, int& turn) {
  const int lane = threadIdx.x, nl = blockDim.x;
  for (int k = 0; k < n; ++k) {
    double best = -1.0, bi = 1e300;
    for (int i = k + lane; i < n; i += nl) {
      const double a = fabs(M[i * n + k]);
      if (a > best || (a == best && i < bi)) best = a, bi = (double)i;
    }
    const double amax = block_red(1, best, red, turn);
    const int p = (int)block_red(2, best == amax ? bi : 1e300, red, turn);
    __syncthreads();
    if (p != k)
      for (int j = lane; j < n; j += nl) {
        const double t = M[k * n + j];
        M[k * n + j] = M[p * n + j];
        M[p * n + j] = t;
      }
    if (lane == 0) piv[k] = p;
    __syncthreads();
    const double d = M[k * n + k];
    for (int i = k + 1 + lane; i < n; i += nl) M[i * n + k] = M[i * n + k] / d;
    __syncthreads();
    const int m = n - k - 1;
    for (int t = lane; t < m * m; t += nl) {
      const int i = k + 1 + t / m, j = k + 1 + t % m;
      M[i * n + j] = M[i * n + j] - M[i * n + k] * M[k * n + j];
    }
    __syncthreads();
  }
}

template <bool SEARCH, bool UPDATE>
__device__ void lu_wred(int j, ldouble* M, ldouble* piv, int n) {
  for (int k = 0; k < n; ++k) {
    int p = k;
    if constexpr (SEARCH) {
      const bool live = j >= k && j < n;
      const double best = live ? fabs(M[j * n + k]) : -1.0;
      const double amax = wave_reduce<1>(best);
      p = (int)wave_reduce<2>(live && best == amax ? (double)j : 1e300);
      if (p != k && j < n) {
        const double t = M[k * n + j];
        M[k * n + j] = M[p * n + j];
        M[p * n + j] = t;
      }
      if (j == 0) piv[k] = p;
      wave_sync();
      const double d = M[k * n + k];
      if (j > k && j < n) M[j * n + k] = M[j * n + k] / d;
      wave_sync();
    }
    if constexpr (UPDATE) {
      if (j > k && j < n) {
        const double mk = M[k * n + j];
        for (int i0 = k + 1; i0 < n; i0 += 8) {
          double l[8], a[8];
#pragma unroll
          for (int u = 0; u < 8; ++u) {
            const int i = i0 + u < n ? i0 + u : i0;
            l[u] = M[i * n + k];
            a[u] = M[i * n + j];
          }
#pragma unroll
          for (int u = 0; u < 8; ++u)
            if (i0 + u < n) M[(i0 + u) * n + j] = a[u] - l[u] * mk;
        }
      }
      wave_sync();
    }
  }
}

__device__ void lu_wscan(int j, ldouble* M, ldouble* piv, int n) {
  const bool col = j < n;
  double best = -1.0, bi = 0.0, sv = 0.0;
  if (j == 0)
    for (int i = 0; i < n; ++i) {
      const double v = M[i * n], a = fabs(v);
      if (a > best) best = a, bi = (double)i, sv = v;
    }
  for (int k = 0; k < n; ++k) {
    const double d = bcast(sv, k);
    const int p = __builtin_amdgcn_readfirstlane((int)bcast(bi, k));
    if (col) {
      if (p != k && j != k) {
        const double t = M[k * n + j];
        M[k * n + j] = M[p * n + j];
        M[p * n + j] = t;
      }
      if (j > k) {
        if (j == p) {
          const double v = M[k * n + k];
          M[k * n + k] = d;
          M[p * n + k] = v / d;
        } else {
          M[j * n + k] = M[j * n + k] / d;
        }
      }
    }
    if (j == 0) piv[k] = p;
    wave_sync();
    if (col && j > k) {
      const double mk = M[k * n + j];
      best = -1.0;
      for (int i0 = k + 1; i0 < n; i0 += 8) {
        double l[8], a[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const int i = i0 + u < n ? i0 + u : i0;
          l[u] = M[i * n + k];
          a[u] = M[i * n + j];
        }
#pragma unroll
        for (int u = 0; u < 8; ++u)
          if (i0 + u < n) {
            const double v = a[u] - l[u] * mk;
            M[(i0 + u) * n + j] = v;
            const double av = fabs(v);
            if (av > best) best = av, bi = (double)(i0 + u), sv = v;
          }
      }
    }
    wave_sync();
  }
}

// trailing updates alone (pivot k), variants: UB rows per batch on one wave; or NWV waves with
// rows dealt round-robin over the waves (a workgroup barrier per step)
template <int UB, int NWV>
__device__ void upd_only(int lane, ldouble* M, int n) {
  const int j = lane & 63, w = lane >> 6;
  for (int k = 0; k < n; ++k) {
    if (w < NWV && j > k && j < n) {
      const double mk = M[k * n + j];
      for (int i0 = k + 1 + w * UB; i0 < n; i0 += UB * NWV) {
        double l[UB], a[UB];
#pragma unroll
        for (int u = 0; u < UB; ++u) {
          const int i = i0 + u < n ? i0 + u : i0;
          l[u] = M[i * n + k];
          a[u] = M[i * n + j];
        }
#pragma unroll
        for (int u = 0; u < UB; ++u)
          if (i0 + u < n) M[(i0 + u) * n + j] = a[u] - l[u] * mk;
      }
    }
    if (NWV > 1) __syncthreads(); else wave_sync();
  }
}
// the same with a lane per (row, column) entry over all 256 lanes: rows i = k+1+t/m without a
// division (t walks a 2-D lane grid: row group = lane / 64 step 4, column = lane % 64)
// 4 waves: the trailing update with rows dealt over the waves (UB-row batches, a lane per
// column), each wave's lane k+1 scanning its rows of column k+1 for the next pivot; the four
// partial pivots through LDS (the update's barrier), the row swap and column k's division on
// wave 0 (one pass), a barrier -- two barriers a pivot, no reductions
template <int UB>
__device__ void lu_h4(int lane, ldouble* M, ldouble* piv, int n, ldouble* cand) {
  const int j = lane & 63, w = lane >> 6;
  double best = -1.0, bi = 0.0, sv = 0.0;
  if (lane == 0) {
    for (int i = 0; i < n; ++i) {
      const double v = M[i * n], a = fabs(v);
      if (a > best) best = a, bi = (double)i, sv = v;
    }
    cand[0] = best, cand[4] = bi, cand[8] = sv;
    cand[1] = cand[2] = cand[3] = -1.0;
  }
  __syncthreads();
  for (int k = 0; k < n; ++k) {
    // the pivot: the largest |a| of the four waves' candidates, the smallest row among equal
    double amax = cand[0], pr = cand[4], d = cand[8];
#pragma unroll
    for (int q = 1; q < 4; ++q) {
      const double a = cand[q], r = cand[4 + q];
      if (a > amax || (a == amax && r < pr)) amax = a, pr = r, d = cand[8 + q];
    }
    const int p = __builtin_amdgcn_readfirstlane((int)pr);
    if (!(amax > 0.0)) return;
    if (w == 0 && j < n) {
      if (p != k && j != k) {
        const double t = M[k * n + j];
        M[k * n + j] = M[p * n + j];
        M[p * n + j] = t;
      }
      if (j > k) {
        if (j == p) {
          const double v = M[k * n + k];
          M[k * n + k] = d;
          M[p * n + k] = v / d;
        } else {
          M[j * n + k] = M[j * n + k] / d;
        }
      }
      if (j == 0) piv[k] = p;
    }
    __syncthreads();
    best = -1.0, bi = 0.0, sv = 0.0;
    if (j > k && j < n) {
      const double mk = M[k * n + j];
      for (int i0 = k + 1 + w * UB; i0 < n; i0 += UB * 4) {
        double l[UB], a[UB];
#pragma unroll
        for (int u = 0; u < UB; ++u) {
          const int i = i0 + u < n ? i0 + u : i0;
          l[u] = M[i * n + k];
          a[u] = M[i * n + j];
        }
#pragma unroll
        for (int u = 0; u < UB; ++u)
          if (i0 + u < n) {
            const double v = a[u] - l[u] * mk;
            M[(i0 + u) * n + j] = v;
            const double av = fabs(v);
            if (av > best) best = av, bi = (double)(i0 + u), sv = v;
          }
      }
    }
    if (j == k + 1) cand[w] = best, cand[4 + w] = bi, cand[8 + w] = sv;
    __syncthreads();
  }
}

// one wave, the trailing update over the rows whose multiplier is non-zero only (a ballot of
// column k after the division; a row with l_i = 0 would get a_ij - 0 * m_kj = a_ij), the pivot by
// one DPP max and a ballot (the smallest row attaining it)
__device__ bool lu_wsparse(int j, ldouble* M, ldouble* piv, int n) {
  for (int k = 0; k < n; ++k) {
    const bool live = j >= k && j < n;
    const double best = live ? fabs(M[j * n + k]) : -1.0;
    const double amax = wave_reduce<1>(best);
    const unsigned long long at = __ballot(live && best == amax);
    const int p = at ? (int)__builtin_ctzll(at) : k;
    if (!(amax > 0.0)) return false;
    if (p != k && j < n) {
      const double t = M[k * n + j];
      M[k * n + j] = M[p * n + j];
      M[p * n + j] = t;
    }
    if (j == 0) piv[k] = p;
    wave_sync();
    const double d = M[k * n + k];
    double lj = 0.0;
    if (j > k && j < n) {
      lj = M[j * n + k] / d;
      M[j * n + k] = lj;
    }
    unsigned long long nz = __ballot(j > k && j < n && lj != 0.0);
    wave_sync();
    if (nz) {
      const double mk = j > k && j < n ? (double)M[k * n + j] : 0.0;
      while (nz) {
        int r[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          r[u] = nz ? (int)__builtin_ctzll(nz) : -1;
          nz &= nz ? nz - 1 : 0ull;
        }
        double l[8], a[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const int i = r[u] >= 0 ? r[u] : r[0];
          l[u] = M[i * n + k];
          a[u] = M[i * n + (j < n ? j : 0)];
        }
        if (j > k && j < n)
#pragma unroll
          for (int u = 0; u < 8; ++u)
            if (r[u] >= 0) M[r[u] * n + j] = a[u] - l[u] * mk;
      }
    }
    wave_sync();
  }
  return true;
}

// permutation + L + U substitutions, b in LDS (lane 0 permutes; rows on lanes, fences)
__device__ void solve_lds(int j, const ldouble* M, const ldouble* piv, ldouble* b, int n) {
  if (j == 0)
    for (int k = 0; k < n; ++k) {
      const int p = (int)piv[k];
      if (p != k) {
        const double t = b[k];
        b[k] = b[p];
        b[p] = t;
      }
    }
  wave_sync();
  const bool row = j < n;
  const int rj = (row ? j : 0) * n;
  for (int i0 = 0; i0 < n; i0 += 8) {
    double mc[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) mc[u] = M[rj + (i0 + u < n ? i0 + u : 0)];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int i = i0 + u;
      if (i < n) {
        const double bi = b[i];
        if (row && j > i) b[j] -= mc[u] * bi;
        wave_sync();
      }
    }
  }
  for (int i1 = n - 1; i1 >= 0; i1 -= 8) {
    double mc[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) mc[u] = M[rj + (i1 - u >= 0 ? i1 - u : 0)];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int i = i1 - u;
      if (i >= 0) {
        if (j == i) b[i] = b[i] / mc[u];
        wave_sync();
        const double bi = b[i];
        if (row && j < i) b[j] -= mc[u] * bi;
        wave_sync();
      }
    }
  }
}

__device__ void solve_reg(int j, const ldouble* M, const ldouble* piv, ldouble* b, int n) {
  const bool row = j < n;
  const int rj = (row ? j : 0) * n;
  double bj = row ? (double)b[j] : 0.0;
  for (int k0 = 0; k0 < n; k0 += 8) {
    double pv[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) pv[u] = piv[k0 + u < n ? k0 + u : k0];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int k = k0 + u;
      if (k < n) {
        const int p = __builtin_amdgcn_readfirstlane((int)pv[u]);
        if (p != k) {
          const double vk = bcast(bj, k), vp = bcast(bj, p);
          if (j == k) bj = vp;
          if (j == p) bj = vk;
        }
      }
    }
  }
  for (int i0 = 0; i0 < n; i0 += 8) {
    double mc[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) mc[u] = M[rj + (i0 + u < n ? i0 + u : 0)];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int i = i0 + u;
      if (i < n) {
        const double bi = bcast(bj, i);
        if (row && j > i) bj -= mc[u] * bi;
      }
    }
  }
  for (int i1 = n - 1; i1 >= 0; i1 -= 8) {
    double mc[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) mc[u] = M[rj + (i1 - u >= 0 ? i1 - u : 0)];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int i = i1 - u;
      if (i >= 0) {
        if (j == i) bj = bj / mc[u];
        const double bi = bcast(bj, i);
        if (row && j < i) bj -= mc[u] * bi;
      }
    }
  }
  if (row) b[j] = bj;
  wave_sync();
}

// V: 0 block, 1 wred, 2 wscan, 3 wnoupd, 4 wupd, 5 solve_lds, 6 solve_reg
template <int V>
__global__ void __launch_bounds__(256) k_lu(const double* A, const double* rhs, int n, int R, double* out,
                                            double* cyc) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  ldouble* M = (ldouble*)smem;
  ldouble* piv = M + 64 * 64;
  ldouble* b = piv + 64;
  ldouble* red = b + 64;   // 16 doubles
  int turn = 0;
  const int lane = threadIdx.x;
  double tot = 0.0;
  for (int r = 0; r < R; ++r) {
    for (int i = lane; i < n * n; i += blockDim.x) M[i] = A[i];
    if (V == 5 || V == 6) {
      // factor once with the block LU for the substitution variants
      if (r == 0) {
        __syncthreads();
        lu_block(M, piv, n, red, turn);
      }
      for (int i = lane; i < n; i += blockDim.x) b[i] = rhs[i];
    }
    __syncthreads();
    const long long t0 = __builtin_amdgcn_s_memtime();
    if constexpr (V == 0) lu_block(M, piv, n, red, turn);
    if constexpr (V == 1 || V == 3 || V == 4) {
      if (lane < 64) lu_wred<V != 4, V != 3>(lane, M, piv, n);
    }
    if constexpr (V == 2) {
      if (lane < 64) lu_wscan(lane, M, piv, n);
    }
    if constexpr (V == 15) {
      if (lane < 64) lu_wsparse(lane, M, piv, n);
    }
    if constexpr (V == 13) lu_h4<2>(lane, M, piv, n, red);
    if constexpr (V == 14) lu_h4<4>(lane, M, piv, n, red);
    if constexpr (V == 7) upd_only<8, 1>(lane, M, n);
    if constexpr (V == 8) upd_only<16, 1>(lane, M, n);
    if constexpr (V == 9) upd_only<4, 1>(lane, M, n);
    if constexpr (V == 10) upd_only<8, 4>(lane, M, n);
    if constexpr (V == 11) upd_only<4, 4>(lane, M, n);
    if constexpr (V == 12) upd_only<2, 4>(lane, M, n);
    if constexpr (V == 5) {
      if (lane < 64) solve_lds(lane, M, piv, b, n);
    }
    if constexpr (V == 6) {
      if (lane < 64) solve_reg(lane, M, piv, b, n);
    }
    __syncthreads();
    const long long t1 = __builtin_amdgcn_s_memtime();
    tot += (double)(t1 - t0);
    if (V == 5 || V == 6) {
      // the factor must survive: skip the M reload next round
      break;
    }
  }
  if (lane == 0) cyc[blockIdx.x] = tot / (V == 5 || V == 6 ? 1 : R);
  __syncthreads();
  for (int i = lane; i < n * n; i += blockDim.x) out[i] = M[i];
  for (int i = lane; i < n; i += blockDim.x) out[n * n + i] = (V == 5 || V == 6) ? (double)b[i] : (double)piv[i];
}

template <int V>
static void run(const char* name, int n, int R, const std::vector<double>& A, const std::vector<double>& rhs,
                std::vector<double>& res, bool print) {
  double *dA, *dr, *dout, *dc;
  CK(hipMalloc(&dA, 64 * 64 * 8));
  CK(hipMalloc(&dr, 64 * 8));
  CK(hipMalloc(&dout, (64 * 64 + 64) * 8));
  CK(hipMalloc(&dc, 8));
  CK(hipMemcpy(dA, A.data(), n * n * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(dr, rhs.data(), n * 8, hipMemcpyHostToDevice));
  const size_t lds = (64 * 64 + 64 + 64 + 16) * 8;
  CK(hipFuncSetAttribute((const void*)k_lu<V>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  k_lu<V><<<1, 256, lds>>>(dA, dr, n, R, dout, dc);
  CK(hipEventRecord(e0));
  k_lu<V><<<1, 256, lds>>>(dA, dr, n, R, dout, dc);
  CK(hipEventRecord(e1));
  CK(hipDeviceSynchronize());
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  double cyc = 0;
  CK(hipMemcpy(&cyc, dc, 8, hipMemcpyDeviceToHost));
  res.resize(n * n + n);
  CK(hipMemcpy(res.data(), dout, (n * n + n) * 8, hipMemcpyDeviceToHost));
  if (print)
    printf("%-10s n=%2d  %9.0f ticks per call  (%6.0f per pivot)  kernel %.3f ms\n", name, n, cyc, cyc / n, ms);
  CK(hipFree(dA));
  CK(hipFree(dr));
  CK(hipFree(dout));
  CK(hipFree(dc));
}

int main(int argc, char** argv) {
  const int R = argc > 1 ? atoi(argv[1]) : 20;
  for (int n : {13, 46, 48, 64}) {
    std::vector<double> A(n * n), rhs(n);
    srand(7);
    for (int i = 0; i < n * n; ++i) A[i] = (double)rand() / RAND_MAX - 0.5;
    for (int i = 0; i < n; ++i) A[i * n + i] += (i % 3 == 0 ? 0.1 : 2.0), rhs[i] = (double)rand() / RAND_MAX;
    std::vector<double> r0, r1, r2, r3, r4, r5, r6;
    run<0>("block", n, R, A, rhs, r0, true);
    run<1>("wred", n, R, A, rhs, r1, true);
    run<2>("wscan", n, R, A, rhs, r2, true);
    run<3>("wnoupd", n, R, A, rhs, r3, true);
    run<4>("wupd", n, R, A, rhs, r4, true);
    std::vector<double> h2, h4;
    run<13>("h4x2", n, R, A, rhs, h2, true);
    run<14>("h4x4", n, R, A, rhs, h4, true);
    printf("  h4x2 == block: %d  h4x4 == block: %d\n", (int)(h2 == r0), (int)(h4 == r0));
    std::vector<double> u7, u8, u9, u10, u11, u12;
    run<7>("upd8x1", n, R, A, rhs, u7, true);
    run<8>("upd16x1", n, R, A, rhs, u8, true);
    run<9>("upd4x1", n, R, A, rhs, u9, true);
    run<10>("upd8x4w", n, R, A, rhs, u10, true);
    run<11>("upd4x4w", n, R, A, rhs, u11, true);
    run<12>("upd2x4w", n, R, A, rhs, u12, true);
    printf("  upd variants equal: %d %d %d %d %d\n", (int)(u7 == u8), (int)(u7 == u9), (int)(u7 == u10), (int)(u7 == u11),
           (int)(u7 == u12));
    run<5>("solve_lds", n, 1, A, rhs, r5, true);
    run<6>("solve_reg", n, 1, A, rhs, r6, true);
    printf("  n=%d  wred == block: %d  wscan == block: %d  solve_reg == solve_lds: %d\n", n,
           (int)(memcmp(r0.data(), r1.data(), r0.size() * 8) == 0), (int)(memcmp(r0.data(), r2.data(), r0.size() * 8) == 0),
           (int)(memcmp(r5.data(), r6.data(), r5.size() * 8) == 0));
  }
  // the coupling system's structure (N=8 NB=2: bd = 4 parent branches, m = 3, 13 cones; N=20 NB=1:
  // bd = 1, 4 cones): globals rho | sigma | mu+ | mu- | J with a diagonal for rho and mu, the CVaR
  // rows coupling rho_b, sigma_b and mu-_b., the cone block dense, each cone on 3-4 globals
  for (int cfg = 0; cfg < 2; ++cfg) {
    const int bd = cfg == 0 ? 4 : 1, m = 3, nc = cfg == 0 ? 13 : 4;
    const int ng = bd * (2 * m + 2) + 1, n = ng + bd + nc;
    std::vector<double> A(n * n, 0.0), rhs(n);
    srand(11);
    auto rnd = [] { return (double)rand() / RAND_MAX - 0.5; };
    for (int b = 0; b < bd; ++b) A[b * n + b] = 50.0 + 100.0 * rnd();
    for (int q = 0; q < 2 * bd * m; ++q) A[(2 * bd + q) * n + 2 * bd + q] = 30.0 + 40.0 * rnd();
    for (int b = 0; b < bd; ++b) {
      const int row = ng + b;
      A[row * n + b] = A[b * n + row] = 1.0;
      A[row * n + bd + b] = A[(bd + b) * n + row] = 1.0;
      for (int i = 0; i < m; ++i) {
        const int gi = 2 * bd + bd * m + b * m + i;
        A[row * n + gi] = A[gi * n + row] = -0.3 + 0.1 * rnd();
      }
    }
    for (int k = 0; k < nc; ++k) {
      const int ck = ng + bd + k;
      for (int j2 = 0; j2 < nc; ++j2) A[ck * n + ng + bd + j2] = (k == j2 ? 1.0 : 0.0) + 0.2 * rnd();
      const int b = k == nc - 1 ? 0 : k / m % bd, i = k % m;
      const int gl[4] = {bd + b, 2 * bd + b * m + i, 2 * bd + bd * m + b * m + i, k == nc - 1 ? ng - 1 : b};
      for (int q = 0; q < 4; ++q) {
        const double gv = rnd();
        A[gl[q] * n + ck] = gv;
        A[ck * n + gl[q]] = -2.0 * gv;
      }
    }
    for (int i = 0; i < n; ++i) rhs[i] = rnd();
    std::vector<double> s0, s1, s2;
    printf("structured n=%d\n", n);
    run<0>("block", n, R, A, rhs, s0, true);
    run<1>("wred", n, R, A, rhs, s1, true);
    run<15>("wsparse", n, R, A, rhs, s2, true);
    printf("  wred == block: %d  wsparse == block: %d\n", (int)(s0 == s1), (int)(s0 == s2));
  }
  // ticks vs wall clock: one long block-LU kernel
  std::vector<double> A(46 * 46), rhs(46), r;
  for (int i = 0; i < 46 * 46; ++i) A[i] = (double)rand() / RAND_MAX - 0.5;
  for (int i = 0; i < 46; ++i) A[i * 46 + i] += 2.0;
  run<0>("clock", 46, 400, A, rhs, r, true);
  return 0;
}
