// bmpc_dev.h -- the solver kernels of libbmpc.so (gfx950) and their launchers.
//
// Mapping: one 64-lane wavefront (one 64-thread workgroup) per ego.  k_tree rebuilds the ego's
// scenario tree (warm start, rollouts, linearisation, collision rows); k_ipm / k_qp run the
// structured interior-point solve and unpack the solution.  All per-ego state lives in one
// contiguous slab of HBM (Layout), so every strided lane loop reads and writes contiguous
// 512-byte segments.  Each predictive model's kernels are instantiated in a translation unit of
// their own (bmpc_k_*.hip, compiled in parallel); bmpc_hip.hip holds the C ABI.
#pragma once

#include <hip/hip_runtime.h>

#include <type_traits>

#include "bmpc_env.h"
#include "bmpc_hmm.h"
#include "bmpc_plan.h"
#include "bmpc_qp.h"
#include "bmpc_qpplan.h"
#include "bmpc_solve.h"

namespace bmpc {
namespace dev {

#ifndef BMPC_WPE
#define BMPC_WPE 4   // waves per SIMD the IPM kernel is register-limited to (4 = all 4096 egos resident)
#endif


#ifndef BMPC_DPP_REDUCE
// wave butterflies on DPP / permlane swaps instead of __shfl_xor (ds_bpermute): 1 in the multi-wave
// small-batch executor (latency-bound: one ego N=20 NB=1 10.11 -> 9.44 ms, N=8 NB=2 19.00 -> 18.78,
// bit-identical), 0 in the one-wave k_ipm (bandwidth-bound: +1.3% time and +1.2% bytes at 4,096
// headline egos from the extra registers, +0.3% on config 3; profiles/r06/r06d_*); 2 both, 0 neither
#define BMPC_DPP_REDUCE 1
#endif
constexpr bool kDppWave = BMPC_DPP_REDUCE == 2;                              // DevExecT (k_ipm, k_qp, k_tree)
constexpr bool kDppBlock = BMPC_DPP_REDUCE == 1 || BMPC_DPP_REDUCE == 2;     // DevBlockExecT (k_solve_blk)

template <bool TR, bool TL = true>
struct DevExecT {
  static constexpr bool kTransform = TR;   // per-ego S / bx constants in LDS (merge plans)
  // LDS-rich launch (TL): topology tables copied to LDS and the coupling system in LDS;
  // lean launch: tables read from the plan's blob, coupling system in the slab
  static constexpr bool kCoupLds = TL;
  using tab_ptr = typename std::conditional<TL, lint*, gint*>::type;
  int lane;
  ldouble* lds;  // this wave's LDS scratch (Plan::nlds doubles; k_ipm / k_qp only)
  tab_ptr tab;   // topology tables (k_ipm / k_qp only)
  ldouble* eco;  // per-ego constants of the solve (ECO_*; kTransform only)
  static constexpr int nlanes = 64;
  // one wave runs a band QP: blocked factorisation and sweeps on wave broadcasts (bmpc_bandqp.h)
  static constexpr bool kBqpWave = true;
  static constexpr bool kInlineG = true;    // apply_G inline (bmpc_ipm.h)
  // small dense systems with a lane per row (bmpc_ipm.h, small_lu_solve_rows)
  static constexpr bool kRowLanes = true;
  // lane l's v, wave-uniform (l uniform)
  __device__ double rlane(double v, int l) const {
    return __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(v), l),
                            __builtin_amdgcn_readlane(__double2loint(v), l));
  }
  // task groups of 4 lanes (one DPP quad) for the tree sweeps
  static constexpr int kTaskLanes = 4;
  // cone rows per lane the fused IPM passes hold in registers (bmpc_ipm.h, cone_regs)
  static constexpr int kConeRegRows = 8;
  __device__ double tsum(double v) const {
    v += dpp_d<0xB1>(v);   // quad_perm [1,0,3,2]
    v += dpp_d<0x4E>(v);   // quad_perm [2,3,0,1]
    return v;
  }
  template <int S>
  __device__ double tget(double v) const { return dpp_d<S | (S << 2) | (S << 4) | (S << 6)>(v); }
  // sum over aligned groups of g lanes (g a power of two)
  __device__ double gsum(double v, int g) const { return group_reduce<0, kDppWave>(v, g); }
  __device__ double gmax(double v, int g) const { return group_reduce<1, kDppWave>(v, g); }
  __device__ double gmin(double v, int g) const { return group_reduce<2, kDppWave>(v, g); }
  __device__ void sync() const { __syncthreads(); }
  // a wave-uniform flag as a scalar: branches on it (and the calls they guard) run with the
  // full exec mask instead of an exec mask derived from a VGPR the compiler cannot prove uniform
  __device__ bool uniform(bool b) const { return __builtin_amdgcn_readfirstlane((int)b) != 0; }
  __device__ double sum(double v) const { return wave_reduce<0, kDppWave>(v); }
  __device__ double max(double v) const { return wave_reduce<1, kDppWave>(v); }
  __device__ double min(double v) const { return wave_reduce<2, kDppWave>(v); }
  // K sums / minima at once (in place)
  template <int K>
  __device__ void sum_n(double* v) const {
#pragma unroll
    for (int k = 0; k < K; ++k) v[k] = sum(v[k]);
  }
  template <int K>
  __device__ void min_n(double* v) const {
#pragma unroll
    for (int k = 0; k < K; ++k) v[k] = min(v[k]);
  }
};

using DevExec = DevExecT<false>;

#ifndef BMPC_BLK_RED2
#define BMPC_BLK_RED2 1   // whole-executor reductions with one barrier (two buffers in turn)
#endif
// Multi-wave executor: one ego on NW waves of one workgroup (batch-1 / small-batch callers --
// main_branch's one solve per step): the same phase templates with 64*NW lanes, so the tree
// solve's tasks, the cone groups and every lane loop spread over NW waves.  Wave-level
// operations (DPP quads, cone-group shuffles) are unchanged; whole-executor reductions go
// through LDS (`red`: K*NW doubles of one of two buffers) and one barrier.
template <bool TR, bool TL, int NW>
struct DevBlockExecT {
  static constexpr bool kTransform = TR;
  static constexpr bool kCoupLds = TL;
  using tab_ptr = typename std::conditional<TL, lint*, gint*>::type;
  int lane;
  ldouble* lds;
  tab_ptr tab;
  ldouble* eco;
  ldouble* red;   // reduction scratch: 2 * kRedMax * NW doubles, then NW turn slots
  static constexpr int nlanes = 64 * NW;
  static constexpr int kBatchDiv = NW;   // lane batches NW times narrower (bmpc_core.h, lane_batch)
  static constexpr bool kRowLanes = true;
  static constexpr int kTaskLanes = 4;
  // wider cone groups than one wave's (exec_cgrp): fewer rows per lane in the fused cone passes
  // and the cone groups' strided loops (4 waves: a 122-row cone on 64 lanes holds 2 rows a lane)
  static constexpr int kConeRegRows = NW == 4 ? 4 : 8;
  static constexpr int kConeBatch = NW == 4 ? 2 : 4;
  static constexpr int kRedMax = 16;
  __device__ double tsum(double v) const {
    v += dpp_d<0xB1>(v);
    v += dpp_d<0x4E>(v);
    return v;
  }
  template <int S>
  __device__ double tget(double v) const { return dpp_d<S | (S << 2) | (S << 4) | (S << 6)>(v); }
  __device__ double gsum(double v, int g) const { return group_reduce<0, kDppBlock>(v, g); }
  __device__ double gmax(double v, int g) const { return group_reduce<1, kDppBlock>(v, g); }
  __device__ double gmin(double v, int g) const { return group_reduce<2, kDppBlock>(v, g); }
  __device__ void sync() const { __syncthreads(); }
  __device__ bool uniform(bool b) const { return __builtin_amdgcn_readfirstlane((int)b) != 0; }
  // OP 0 sum, 1 max, 2 min of K values per lane over all lanes (in place)
  template <int OP, int K>
  __device__ void reduce(double* v) const {
    static_assert(K <= kRedMax, "reduction scratch");
#pragma unroll
    for (int k = 0; k < K; ++k) v[k] = wave_reduce<OP, kDppBlock>(v[k]);
    const int wv = lane >> 6;
#if BMPC_BLK_RED2
    // two buffers used in turn (each wave's turn kept in its LDS slot: every wave runs the same
    // reductions in the same order): a wave writing reduction r + 2 into the buffer of r has
    // passed r + 1's barrier, which every wave reaches only after reading r -- one barrier each
    ldouble* turn = red + 2 * kRedMax * NW + wv;
    const int odd = __builtin_amdgcn_readfirstlane((int)*turn);
    ldouble* buf = red + (odd ? kRedMax * NW : 0);
    if ((lane & 63) == 0) {
#pragma unroll
      for (int k = 0; k < K; ++k) buf[k * NW + wv] = v[k];
      *turn = odd ? 0.0 : 1.0;
    }
#else
    ldouble* buf = red;
    __syncthreads();   // the previous reduction's readers are done with red
    if ((lane & 63) == 0)
#pragma unroll
      for (int k = 0; k < K; ++k) red[k * NW + wv] = v[k];
#endif
    __syncthreads();
#pragma unroll
    for (int k = 0; k < K; ++k) {
      double a = buf[k * NW];
#pragma unroll
      for (int w = 1; w < NW; ++w) {
        const double b = buf[k * NW + w];
        a = OP == 0 ? a + b : OP == 1 ? fmax(a, b) : fmin(a, b);
      }
      v[k] = a;
    }
  }
  __device__ double sum(double v) const { reduce<0, 1>(&v); return v; }
  __device__ double max(double v) const { reduce<1, 1>(&v); return v; }
  __device__ double min(double v) const { reduce<2, 1>(&v); return v; }
  template <int K>
  __device__ void sum_n(double* v) const { reduce<0, K>(v); }
  template <int K>
  __device__ void min_n(double* v) const { reduce<2, K>(v); }
};

#if defined(BMPC_WITH_PHASED)
constexpr int kMaxSub = 8;   // sub-batch streams of the phase-per-kernel IPM (experimental/)
#endif

struct Bundle {
  Plan P;
  Layout L;
};

// Dynamic LDS of the solver kernels: Plan::nlds doubles of scratch, then a copy of the
// topology tables (Plan::ntab int32).  The copy is one batched pass at kernel start; every
// later tree / cone / node-index lookup of the solve is an LDS read.
// Dynamic LDS of the solver kernels: Plan::nlds doubles of scratch, then a copy of the
// topology tables (Plan::ntab int32), then (transform-capable models) ECO_COUNT doubles of
// per-ego constants.  The table copy is one batched pass at kernel start; every later tree /
// cone / node-index lookup of the solve is an LDS read.
__host__ __device__ inline size_t solver_lds_bytes(const Plan& P, bool transform, bool rich) {
  const size_t tab = rich ? (sizeof(int32_t) * (size_t)P.ntab + 7) & ~(size_t)7 : 0;
  return sizeof(double) * (size_t)(rich ? P.nlds : P.nlds_lean) + tab + (transform ? sizeof(double) * ECO_COUNT : 0);
}
template <bool TR, bool TL>
__device__ __forceinline__ DevExecT<TR, TL> solver_exec(const Plan& P, double* lds_dyn) {
  const int32_t* gtab = (const int32_t*)P.t.br_depth;   // blob base (the first table)
  double* eco = lds_dyn + (solver_lds_bytes(P, false, TL) / sizeof(double));
  // W1 | Wu | Fx | Fu for the IPM passes' per-lane row lookups
  for (int i = threadIdx.x; i < P.nconst; i += 64) lds_dyn[P.lds_w + i] = plan_const(P, i);
  if constexpr (TL) {
    int32_t* tabl = reinterpret_cast<int32_t*>(lds_dyn + P.nlds);
    for (int i = threadIdx.x; i < P.ntab; i += 64) tabl[i] = gtab[i];
    __syncthreads();
    return DevExecT<TR, TL>{(int)threadIdx.x, (ldouble*)lds_dyn, (lint*)tabl, (ldouble*)eco};
  } else {
    __syncthreads();
    return DevExecT<TR, TL>{(int)threadIdx.x, (ldouble*)lds_dyn, (gint*)gtab, (ldouble*)eco};
  }
}

// waves per ego of the small-batch solver kernel (k_solve_blk): 4, or 8 for trees of at least
// BMPC_BLK_WIDE_T state nodes (measured at one ego, profiles/r03/r03x_blk_waves.log: N=8 NB=2
// 22 ms on 4 waves, 24 on 8, 38 on 16, 30 on one; N=20 NB=1 12-14 / 14-17 / 20-22 / 14-16;
// N=30 NB=2 48-54 / 44-49 / 62-65 / 61-65)
#ifndef BMPC_BLK_WIDE_T
#define BMPC_BLK_WIDE_T 256
#endif
#define BMPC_BLK_WAVES_MAX 8

// LDS of a multi-wave solver launch: the wave launch's, then the reduction scratch
__host__ __device__ inline size_t solver_lds_bytes_blk(const Plan& P, bool transform, int nw) {
  return ((solver_lds_bytes(P, transform, true) + 7) & ~(size_t)7) + sizeof(double) * (2 * 16 + 1) * (size_t)nw;
}
template <bool TR, int NW>
__device__ __forceinline__ DevBlockExecT<TR, true, NW> solver_exec_blk(const Plan& P, double* lds_dyn) {
  const int t = threadIdx.x, nt = 64 * NW;
  for (int i = t; i < P.nconst; i += nt) lds_dyn[P.lds_w + i] = plan_const(P, i);
  const int32_t* gtab = (const int32_t*)P.t.br_depth;
  int32_t* tabl = reinterpret_cast<int32_t*>(lds_dyn + P.nlds);
  for (int i = t; i < P.ntab; i += nt) tabl[i] = gtab[i];
  double* eco = lds_dyn + (solver_lds_bytes(P, false, true) / sizeof(double));
  double* red = lds_dyn + ((solver_lds_bytes(P, TR, true) + 7) & ~(size_t)7) / sizeof(double);
  if (t < NW) red[2 * 16 * NW + t] = 0.0;   // each wave's reduction turn (BMPC_BLK_RED2)
  __syncthreads();
  return DevBlockExecT<TR, true, NW>{t, (ldouble*)lds_dyn, (lint*)tabl, (ldouble*)eco, (ldouble*)red};
}

// One ego per workgroup of NW waves (small batches: every wave of the chip on few egos);
// QP: the OSQP-class controllers' k_qp path, else the CVaR IPM.
//
// LDS-resident arrays (lay != NULL; translation units with BMPC_FLAT_SLAB only): lay[e] is ego e's
// copy of the layout in which spans of the IPM's own arrays (written before they are read within a
// solve: the NT scaling, the node factors and tree-solve vectors, z / s / lambda) are offset from
// the ego's slab to this workgroup's LDS at hot_off doubles (flat addresses: LDS aperture + offset,
// bmpc_hip.hip blk_layouts); the tree's linearisation (A, B and dh, written by k_tree) is copied
// in when its span is relocated.  A layout that does not land in this workgroup's LDS fails the
// solve with EXIT_GUARD.
template <class M, bool QP, int NW>
__global__ __launch_bounds__(64 * NW) void k_solve_blk(const Bundle* __restrict__ B, double* __restrict__ ws,
                                                      const bmpc_policy* __restrict__ pol, double* upred,
                                                      double* xpred, double* bw, double* J, int32_t* status,
                                                      int32_t* iters, int batch, const Layout* __restrict__ lay,
                                                      size_t hot_off) {
  const int e = blockIdx.x;
  if (e >= batch) return;
  const Plan& P = B->P;
  const Layout& L0 = B->L;
  const Layout& L = lay ? lay[e] : L0;
  constexpr bool TR = QP ? false : M::kTransform;
  extern __shared__ double lds_dyn[];
  const auto ex = solver_exec_blk<TR, NW>(P, lds_dyn);
  using X = DevBlockExecT<TR, true, NW>;
#if defined(BMPC_FLAT_SLAB)
  // the slab pointer through readfirstlane: the compiler cannot infer from the kernel argument
  // that the arrays behind it are global memory, so every slab access is a flat access (LDS or
  // global by address)
  EgoView E{uniform_ptr(ws + L0.stride * (size_t)e), pol + (size_t)e * P.m};
#else
  EgoView E{ws + L0.stride * (size_t)e, pol + (size_t)e * P.m};
#endif
  IpmResult r;
#if defined(BMPC_FLAT_SLAB)
  if (lay) {
    const int t = threadIdx.x, nt = 64 * NW;
    double* w = E.ws;
    if ((uintptr_t)(w + L.dl) != (uintptr_t)(lds_dyn + hot_off)) {   // the first relocated span
      if (t == 0) {
        if (status) status[e] = EXIT_GUARD;
        if (iters) iters[e] = 0;
      }
      return;
    }
    if (L.Ad != L0.Ad)
      for (size_t i = t; i < L0.Cd - L0.Ad; i += nt) w[L.Ad + i] = w[L0.Ad + i];
    if (L.dh != L0.dh)
      for (size_t i = t; i < L0.h0 - L0.dh; i += nt) w[L.dh + i] = w[L0.dh + i];
    __syncthreads();
  }
#endif
  if constexpr (QP) r = solve_ego_qp<X, M>(ex, P, L, E);
  else r = solve_ego_ipm<X, M>(ex, P, L, E);
  const double* w = E.ws;
  const int lane = threadIdx.x, nt = 64 * NW;
  if (upred)
    for (int i = lane; i < P.U * P.d; i += nt) upred[(size_t)e * P.U * P.d + i] = w[L.upred + i];
  if (xpred)
    for (int i = lane; i < P.T * P.n; i += nt) xpred[(size_t)e * P.T * P.n + i] = w[L.xpred + i];
  if (bw)
    for (int i = lane; i < P.nbranch - 1; i += nt) bw[(size_t)e * (P.nbranch - 1) + i] = w[L.w + 1 + i];
  if (lane == 0) {
    if (J) J[e] = QP ? r.pcost : w[L.sol + P.oJ];
    if (status) status[e] = r.exit_flag;
    if (iters) iters[e] = r.iters;
  }
}

#if defined(BMPC_BLK2)
// Tools-only A/B (-DBMPC_BLK2, BMPC_IPM_W2=1): the large-batch CVaR IPM with one ego on TWO waves
// (the small-batch kernel's executor at 128 lanes, slab arrays in global memory, the register
// budget of k_ipm) -- 8 egos per CU instead of 16, each on twice the lanes.
template <class M>
__global__ __launch_bounds__(128) __attribute__((amdgpu_waves_per_eu(BMPC_WPE))) void k_ipm_w2(
    const Bundle* __restrict__ B, double* __restrict__ ws, const bmpc_policy* __restrict__ pol, double* upred,
    double* xpred, double* bw, double* J, int32_t* status, int32_t* iters, int batch) {
  const int e = blockIdx.x;
  if (e >= batch) return;
  const Plan& P = B->P;
  const Layout& L = B->L;
  extern __shared__ double lds_dyn[];
  const auto ex = solver_exec_blk<M::kTransform, 2>(P, lds_dyn);
  EgoView E{ws + L.stride * (size_t)e, pol + (size_t)e * P.m};
  IpmResult r = solve_ego_ipm<DevBlockExecT<M::kTransform, true, 2>, M>(ex, P, L, E);
  const double* w = E.ws;
  const int lane = threadIdx.x;
  if (upred)
    for (int i = lane; i < P.U * P.d; i += 128) upred[(size_t)e * P.U * P.d + i] = w[L.upred + i];
  if (xpred)
    for (int i = lane; i < P.T * P.n; i += 128) xpred[(size_t)e * P.T * P.n + i] = w[L.xpred + i];
  if (bw)
    for (int i = lane; i < P.nbranch - 1; i += 128) bw[(size_t)e * (P.nbranch - 1) + i] = w[L.w + 1 + i];
  if (lane == 0) {
    if (J) J[e] = w[L.sol + P.oJ];
    if (status) status[e] = r.exit_flag;
    if (iters) iters[e] = r.iters;
  }
}
#endif

#ifndef BMPC_TREE_WPE
#define BMPC_TREE_WPE 4   // k_tree's register budget in batches beyond 2 waves per SIMD (r05ad: 1.23 -> 0.99 ms at 4,096 egos; 3: 1.30)
#endif
// WPE: waves per SIMD the register budget allows (1: 2 waves, the compiler's own choice of 220 VGPRs).  The
// budget pays where the batch has more egos than 2 waves per SIMD hold (launch_tree); a one-ego
// launch is faster without its spills.
template <class M, int WPE>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(WPE > 1 ? WPE : 2))) void k_tree(const Bundle* __restrict__ B, double* __restrict__ ws,
                                             const bmpc_policy* __restrict__ pol,
                                             const double* __restrict__ x, const double* __restrict__ z,
                                             const double* __restrict__ xref, int batch) {
  const int e = blockIdx.x;
  if (e >= batch) return;
  const Plan& P = B->P;
  const Layout& L = B->L;
  DevExec ex{(int)threadIdx.x, nullptr, nullptr, nullptr};
  EgoView E{ws + L.stride * (size_t)e, pol + (size_t)e * P.m};
  BMPC_PROF(E.ws, L, PROF_TREE);
  tree_step<DevExec, M>(ex, P, L, E, x + e * P.n, z + e * P.n, xref + e * P.n);
}

template <class M, bool TL>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(BMPC_WPE))) void k_ipm(const Bundle* __restrict__ B, double* __restrict__ ws,
                                            const bmpc_policy* __restrict__ pol, double* upred,
                                            double* xpred, double* bw, double* J, int32_t* status,
                                            int32_t* iters, int batch) {
  const int e = blockIdx.x;
  if (e >= batch) return;
  const Plan& P = B->P;
  const Layout& L = B->L;
  extern __shared__ double lds_dyn[];
  const auto ex = solver_exec<M::kTransform, TL>(P, lds_dyn);
  EgoView E{ws + L.stride * (size_t)e, pol + (size_t)e * P.m};
  IpmResult r = solve_ego_ipm<DevExecT<M::kTransform, TL>, M>(ex, P, L, E);
  const double* w = E.ws;
  const int lane = threadIdx.x;
  if (upred)
    for (int i = lane; i < P.U * P.d; i += 64) upred[(size_t)e * P.U * P.d + i] = w[L.upred + i];
  if (xpred)
    for (int i = lane; i < P.T * P.n; i += 64) xpred[(size_t)e * P.T * P.n + i] = w[L.xpred + i];
  if (bw)
    for (int i = lane; i < P.nbranch - 1; i += 64) bw[(size_t)e * (P.nbranch - 1) + i] = w[L.w + 1 + i];
  if (lane == 0) {
    if (J) J[e] = w[L.sol + P.oJ];
    if (status) status[e] = r.exit_flag;
    if (iters) iters[e] = r.iters;
  }
}

template <class M, bool TL>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(BMPC_WPE))) void k_qp(
    const Bundle* __restrict__ B, double* __restrict__ ws, const bmpc_policy* __restrict__ pol, double* upred,
    double* xpred, double* bw, double* J, int32_t* status, int32_t* iters, int batch) {
  const int e = blockIdx.x;
  if (e >= batch) return;
  const Plan& P = B->P;
  const Layout& L = B->L;
  extern __shared__ double lds_dyn[];
  const auto ex = solver_exec<false, TL>(P, lds_dyn);
  EgoView E{ws + L.stride * (size_t)e, pol + (size_t)e * P.m};
  IpmResult r = solve_ego_qp<DevExecT<false, TL>, M>(ex, P, L, E);
  const double* w = E.ws;
  const int lane = threadIdx.x;
  if (upred)
    for (int i = lane; i < P.U * P.d; i += 64) upred[(size_t)e * P.U * P.d + i] = w[L.upred + i];
  if (xpred)
    for (int i = lane; i < P.T * P.n; i += 64) xpred[(size_t)e * P.T * P.n + i] = w[L.xpred + i];
  if (bw)
    for (int i = lane; i < P.nbranch - 1; i += 64) bw[(size_t)e * (P.nbranch - 1) + i] = w[L.w + 1 + i];
  if (lane == 0) {
    if (J) J[e] = r.pcost;
    if (status) status[e] = r.exit_flag;
    if (iters) iters[e] = r.iters;
  }
}

// The three parts of a k_loop step as calls of their own: each gets its registers allocated
// apart from the others' (the scene step's and the tree step's private arrays and live values
// stay out of the IPM loop's 128-VGPR budget).
template <class X, class M>
__device__ __attribute__((noinline)) void loop_tree_step(const X ex, const Plan& P, const Layout& L, EgoView E,
                                                          const double* x, const double* z, const double* xref) {
  tree_step<X, M>(ex, P, L, E, x, z, xref);
}
template <class X, class M>
__device__ __attribute__((noinline)) IpmResult loop_ipm(const X ex, const Plan& P, const Layout& L, EgoView E) {
  return solve_ego_ipm<X, M>(ex, P, L, E);
}
__device__ __attribute__((noinline)) void loop_env_step(const bmpc_env_desc& env, double dt, int N, int m, int t,
                                                        double* st, bmpc_policy* pol, const double* up, double* x,
                                                        double* z, double* xr, double Jv, int status, int iters,
                                                        double* stats) {
  if (t > 0 && stats) env_accumulate(st, Jv, status, iters, true, stats);
  env_step_ego(env, dt, N, m, t, st, pol, up, x, z, xr);
}

// nsteps closed-loop steps of one ego per wave (bmpc_loop_device): k_env's scene step (lane 0),
// k_tree's tree step and k_ipm's solve + unpack, in that order, per step -- the same per-ego
// functions the three launches run, so the same bits -- with no device-wide boundary between
// the steps: the egos' loops are independent, and a wave whose ego needs few IPM iterations in
// one step starts its next step instead of idling until the slowest ego of the batch finishes.
template <class M, bool TL>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(BMPC_WPE))) void k_loop(
    const Bundle* __restrict__ B, double* __restrict__ ws, bmpc_policy* __restrict__ pol, bmpc_env_desc env, int t0,
    int nsteps, double* scene, double* upred, double* xs, double* zs, double* xrefs, double* J, int32_t* status,
    int32_t* iters, double* stats, int batch) {
  const int e = blockIdx.x;
  if (e >= batch) return;
  const Plan& P = B->P;
  const Layout& L = B->L;
  extern __shared__ double lds_dyn[];
  const auto ex = solver_exec<M::kTransform, TL>(P, lds_dyn);
  bmpc_policy* pe = pol + (size_t)e * P.m;
  EgoView E{ws + L.stride * (size_t)e, pe};
  double* st = scene + (size_t)e * ENV_STRIDE;
  double* up = upred + (size_t)e * P.U * P.d;
  double* x = xs + (size_t)e * P.n;
  double* z = zs + (size_t)e * P.n;
  double* xr = xrefs + (size_t)e * P.n;
  const int lane = threadIdx.x;
  for (int s = 0; s < nsteps; ++s) {
    const int t = t0 + s;
    if (lane == 0)   // k_env
      loop_env_step(env, P.desc.dt, P.N, P.m, t, st, pe, up, x, z, xr, J[e], status[e], iters[e],
                    stats ? stats + (size_t)e * ENVS_STRIDE : nullptr);
    __syncthreads();
    loop_tree_step<DevExecT<M::kTransform, TL>, M>(ex, P, L, E, x, z, xr);   // k_tree
    const IpmResult r = loop_ipm<DevExecT<M::kTransform, TL>, M>(ex, P, L, E);   // k_ipm
    const double* w = E.ws;
    for (int i = lane; i < P.U * P.d; i += 64) up[i] = w[L.upred + i];
    if (lane == 0) {
      J[e] = w[L.sol + P.oJ];
      status[e] = r.exit_flag;
      iters[e] = r.iters;
    }
    __syncthreads();
  }
}

// one solve launch of a plan (device pointers; the timing events are recorded by the caller
// between the two launches)
struct SolveLaunch {
  const Bundle* bundle;
  double* ws;
  const bmpc_policy* pol;
  const double *x, *z, *xref;
  double *upred, *xpred, *bw, *J;
  int32_t *status, *iters;
  int batch;
  size_t lds_bytes;   // dynamic LDS of the solver kernel (solver_lds_bytes)
  bool rich;          // LDS-rich solver launch (choose_lds_rich)
  bool qp;            // OSQP-class controller (k_qp) instead of the CVaR IPM (k_ipm)
  hipStream_t stream;
  int nw = 4;        // small-batch launch: waves per ego (4 or 8)
  const Layout* blk_lay = nullptr;   // ... per-ego layouts with LDS-resident spans (or NULL)
  int cus = 256;                     // compute units of the device (k_tree's register budget)
  const Plan* hplan = nullptr;       // the plan on the host (launch sizes)
  size_t blk_hot_off = 0;            // ... their LDS offset (doubles)
#if defined(BMPC_WITH_PHASED)
  // phase-per-kernel IPM (experimental/bmpc_dev_ph.h, tools-only builds): per-iteration "egos
  // going on" counters, their pinned read-back slot, the iteration limit, the sub-batch streams
  int32_t* d_count = nullptr;
  int32_t* h_count = nullptr;
  int maxit = 0;
  int ph_mode = 1;   // 1: one kernel per phase, 2: one kernel calling grouped out-of-line phases
  int nsub = 1;                   // mode 1: sub-batches, one stream each
  hipStream_t* sub = nullptr;     // their streams [kMaxSub]
  hipEvent_t* sub_ev = nullptr;   // [kMaxSub + 1] fork / join events
#endif
};

template <class M>
hipError_t launch_tree(const SolveLaunch& a) {
  if (BMPC_TREE_WPE > 1 && a.batch > 2 * 4 * a.cus)
    hipLaunchKernelGGL((k_tree<M, (BMPC_TREE_WPE > 1 ? BMPC_TREE_WPE : 1)>), dim3(a.batch), dim3(64), 0, a.stream,
                       a.bundle, a.ws, a.pol, a.x, a.z, a.xref, a.batch);
  else
    hipLaunchKernelGGL((k_tree<M, 1>), dim3(a.batch), dim3(64), 0, a.stream, a.bundle, a.ws, a.pol, a.x, a.z, a.xref,
                     a.batch);
  return hipGetLastError();
}

template <class K>
hipError_t launch_solver_kernel(K kernel, const SolveLaunch& a) {
  if (a.lds_bytes > 64 * 1024) {   // dynamic LDS above 64 KB needs the per-kernel opt-in
    const hipError_t e =
        hipFuncSetAttribute((const void*)kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)a.lds_bytes);
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL(kernel, dim3(a.batch), dim3(64), a.lds_bytes, a.stream, a.bundle, a.ws, a.pol, a.upred,
                     a.xpred, a.bw, a.J, a.status, a.iters, a.batch);
  return hipGetLastError();
}

// WITH_QP: the model also serves the OSQP-class controllers (Prox, BranchMPC, robustMPC)
template <class M, bool WITH_QP>
hipError_t launch_solver(const SolveLaunch& a) {
  if constexpr (WITH_QP) {
    if (a.qp) return a.rich ? launch_solver_kernel(k_qp<M, true>, a) : launch_solver_kernel(k_qp<M, false>, a);
  }
#if defined(BMPC_BLK2)
  if (const char* e = getenv("BMPC_IPM_W2")) {
    if (atoi(e) == 1) {
      const size_t lds = solver_lds_bytes_blk(*a.hplan, M::kTransform, 2);
      if (lds > 64 * 1024) {
        const hipError_t he = hipFuncSetAttribute((const void*)k_ipm_w2<M>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (he != hipSuccess) return he;
      }
      hipLaunchKernelGGL(k_ipm_w2<M>, dim3(a.batch), dim3(128), lds, a.stream, a.bundle, a.ws, a.pol, a.upred,
                         a.xpred, a.bw, a.J, a.status, a.iters, a.batch);
      return hipGetLastError();
    }
  }
#endif
  return a.rich ? launch_solver_kernel(k_ipm<M, true>, a) : launch_solver_kernel(k_ipm<M, false>, a);
}

// the fused closed loop (k_loop): the one-wave IPM's LDS and register budget
template <class M>
hipError_t launch_loop(const SolveLaunch& a, const bmpc_env_desc& env, int t0, int nsteps, double* scene,
                       double* stats) {
  void (*k)(const Bundle*, double*, bmpc_policy*, bmpc_env_desc, int, int, double*, double*, double*, double*,
            double*, double*, int32_t*, int32_t*, double*, int) = a.rich ? k_loop<M, true> : k_loop<M, false>;
  if (a.lds_bytes > 64 * 1024) {
    const hipError_t e = hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)a.lds_bytes);
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL(k, dim3(a.batch), dim3(64), a.lds_bytes, a.stream, a.bundle, a.ws, const_cast<bmpc_policy*>(a.pol),
                     env, t0, nsteps, scene, a.upred, const_cast<double*>(a.x), const_cast<double*>(a.z),
                     const_cast<double*>(a.xref), a.J, a.status, a.iters, stats, a.batch);
  return hipGetLastError();
}

// the small-batch launch: one ego per NW-wave workgroup (solver_lds_bytes_blk of LDS)
template <class M, bool QP, int NW>
hipError_t launch_blk_kernel(const SolveLaunch& a) {
  // the opt-in is a driver call of its own (~1.5 ms per one-ego solve when made on every launch):
  // made once per device and size
  static size_t opted[16] = {};
  int dev = 0;
  if (a.lds_bytes > 64 * 1024 && hipGetDevice(&dev) == hipSuccess && a.lds_bytes > opted[dev & 15]) {
    const hipError_t e = hipFuncSetAttribute((const void*)k_solve_blk<M, QP, NW>,
                                             hipFuncAttributeMaxDynamicSharedMemorySize, (int)a.lds_bytes);
    if (e != hipSuccess) return e;
    opted[dev & 15] = a.lds_bytes;
  }
  hipLaunchKernelGGL((k_solve_blk<M, QP, NW>), dim3(a.batch), dim3(64 * NW), a.lds_bytes, a.stream, a.bundle, a.ws,
                     a.pol, a.upred, a.xpred, a.bw, a.J, a.status, a.iters, a.batch, a.blk_lay, a.blk_hot_off);
  return hipGetLastError();
}
// (the OSQP-class controllers never take this path: bmpc_hip.hip chooses it for the CVaR IPM only)
template <class M, bool WITH_QP>
hipError_t launch_solver_blk(const SolveLaunch& a) {
  if (a.qp) return hipErrorInvalidValue;
#if defined(BMPC_BLK_ALLOW2)   // tools-only A/B: two waves per ego (BMPC_BLOCK_WAVES=2)
  if (a.nw == 2) return launch_blk_kernel<M, false, 2>(a);
#endif
  return a.nw == 8 ? launch_blk_kernel<M, false, 8>(a) : launch_blk_kernel<M, false, 4>(a);
}

// the per-model launchers (bmpc_k_highway.hip, bmpc_k_highway_t.hip, bmpc_k_merge.hip,
// bmpc_k_quadruped.hip)
hipError_t launch_tree_highway(const SolveLaunch& a);
hipError_t launch_solver_highway(const SolveLaunch& a);
hipError_t launch_tree_highway_t(const SolveLaunch& a);
hipError_t launch_solver_highway_t(const SolveLaunch& a);
hipError_t launch_tree_merge(const SolveLaunch& a);
hipError_t launch_solver_merge(const SolveLaunch& a);
hipError_t launch_tree_quadruped(const SolveLaunch& a);
hipError_t launch_solver_quadruped(const SolveLaunch& a);
hipError_t launch_solver_blk_highway(const SolveLaunch& a);
hipError_t launch_solver_blk_highway_t(const SolveLaunch& a);
hipError_t launch_solver_blk_merge(const SolveLaunch& a);
hipError_t launch_solver_blk_quadruped(const SolveLaunch& a);
hipError_t launch_loop_highway(const SolveLaunch& a, const bmpc_env_desc& env, int t0, int nsteps, double* scene,
                               double* stats);
#if defined(BMPC_WITH_PHASED)
// the phase-per-kernel CVaR IPM (experimental/bmpc_kp_*.hip; tools-only builds with -DBMPC_WITH_PHASED)
hipError_t launch_ipm_phased_highway(const SolveLaunch& a);
hipError_t launch_ipm_phased_highway_t(const SolveLaunch& a);
hipError_t launch_ipm_phased_merge(const SolveLaunch& a);
#endif

}  // namespace dev
}  // namespace bmpc
