// bmpc_core.h -- shared definitions of the batched branch-MPC solver.
//
// Everything under csrc/ is written once as "wave-cooperative" C++: each solver phase is a
// loop strided over the lanes of one executor `X` (one 64-lane wavefront per ego on the GPU),
// with X::sync() between phases and X::sum/max() for reductions.  The HIP kernels
// instantiate the templates with the device executor (bmpc_hip.hip); tests/hostsim
// instantiates them with a 1-lane host executor to check the algorithm on CPU.
#pragma once

#include <stddef.h>
#include <stdint.h>

#include "bmpc.h"

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define BMPC_HD __host__ __device__ __forceinline__
#else
#define BMPC_HD inline
#endif

#include <math.h>

namespace bmpc {

// ------------------------------------------------------------------------------------
// Plan: per-plan constants and topology tables (shared by every ego of the batch).
// ------------------------------------------------------------------------------------
struct Topo {
  // per branch (BFS order of MPC_branch.inittree)
  const int32_t* br_depth;
  const int32_t* br_len;
  const int32_t* br_ndx;
  const int32_t* br_ndu;
  const int32_t* br_child0;   // first child (children are contiguous), -1 for leaves
  // per x node
  const int32_t* x_u;         // u node of x node (-1 for leaf terminal nodes)
  const int32_t* x_srcu;      // u node whose (A,B,C) defines this node (-1 for root)
  const int32_t* x_srcx;      // x node of that source
  const int32_t* x_cone;      // cone whose middle rows contain x (-1 none)
  const int32_t* x_conepos;   // position j of the node inside the cone's branch
  const int32_t* x_branch;
  const int32_t* succ_off;    // CSR successors of each x node: nodes defined by its (A,B,C)
  const int32_t* succ;
  const int32_t* lvl_off;     // x nodes grouped by tree level (root = level 0)
  const int32_t* lvl_nodes;
  // per u node
  const int32_t* u_x;
  const int32_t* u_cone;
  // per cone
  const int32_t* cone_b;      // parent non-leaf branch index (-1 = root cone)
  const int32_t* cone_i;      // child slot i
  const int32_t* cone_c;      // child branch (-1 = root cone)
  const int32_t* cone_q;      // cone dimension
  const int32_t* cone_off;    // first row of the cone in the conic row vector
};

struct Plan {
  bmpc_plan_desc desc;
  int n, d, N, NB, m, nFx, nFu, Nc;
  int T, U, nbranch, bdim, ncones, nlevels;
  // primal vector layout (reference sol['x'] layout, MPC_branch.py:2100-2102)
  int oX, oU, oRho, oSig, oMup, oMum, oS, oJ, nv;
  // equality rows: T*n dynamics rows then bdim CVaR rows (MPC_branch.py:1752-1804)
  int neq;
  // conic rows: Fx|Fu|risk|positivity LP rows then SOC rows (MPC_branch.py:1869-1990)
  int rFx, rFu, rRisk, rPos, nlp, nrows;
  int ng;     // number of "global" variables (rho, sigma, mu+, mu-, J)
  int nsm;    // dense coupling system size
  double W1[BMPC_MAX_N * BMPC_MAX_N];   // sqrtm(Q) / chol(Q)'  (MPC_branch.py:1628-1631)
  double Wu[BMPC_MAX_D * BMPC_MAX_D];   // chol(R)'             (:1633-1636)
  double QQ[BMPC_MAX_N * BMPC_MAX_N];   // W1'W1
  double RR[BMPC_MAX_D * BMPC_MAX_D];   // Wu'Wu
  Topo t;
};

// ------------------------------------------------------------------------------------
// Per-ego workspace layout (offsets in doubles inside one ego's slab)
// ------------------------------------------------------------------------------------
struct Layout {
  // persistent state (survives between solves)
  size_t uLin, pprev, misc, xpred, upred, sol;
  // tree of the current solve
  size_t xbar, zbar, ubar, Ad, Bd, Cd, dh, h0, w, p, boost, xref;
  // IPM vectors
  size_t x, y, z, s, lam, x1, y1, z1, x2, y2, z2, dz, ds, rx, ry, rz, hvec, bvec;
  size_t ta, ya, ra, rb, rc, bestx;
  // KKT-solve scratch
  size_t k_r0, k_nv0, k_e1, k_e2, k_e3, k_t3, k_cx, k_cy, k_cz, k_nv1;
  // scaling
  size_t dl, eta, wbar, vnt;
  // KKT
  size_t hx, hu, sd, P, Kg, Luu, kff, lvec, gk, colk, colnu, Msm, piv, smrhs;
  size_t stride;  // doubles per ego
};

// misc slots
enum { MISC_INIT = 0, MISC_JCONS = 1, MISC_OLDU = 2 /* d values */ };

// ------------------------------------------------------------------------------------
// small dense helpers (row-major, compile-time sizes)
// ------------------------------------------------------------------------------------
template <int R, int C>
BMPC_HD void mat_load(double (&M)[R][C], const double* p) {
#pragma unroll
  for (int i = 0; i < R; ++i)
#pragma unroll
    for (int j = 0; j < C; ++j) M[i][j] = p[i * C + j];
}

template <int R, int C>
BMPC_HD void mat_store(const double (&M)[R][C], double* p) {
#pragma unroll
  for (int i = 0; i < R; ++i)
#pragma unroll
    for (int j = 0; j < C; ++j) p[i * C + j] = M[i][j];
}

// in-place Cholesky of an SPD D x D matrix (lower factor in L); returns false on failure
template <int D>
BMPC_HD bool chol(double (&L)[D][D]) {
#pragma unroll
  for (int j = 0; j < D; ++j) {
    double s = L[j][j];
#pragma unroll
    for (int k = 0; k < j; ++k) s -= L[j][k] * L[j][k];
    if (!(s > 0.0)) return false;
    const double r = sqrt(s);
    L[j][j] = r;
#pragma unroll
    for (int i = j + 1; i < D; ++i) {
      double t = L[i][j];
#pragma unroll
      for (int k = 0; k < j; ++k) t -= L[i][k] * L[j][k];
      L[i][j] = t / r;
    }
#pragma unroll
    for (int i = 0; i < j; ++i) L[i][j] = 0.0;
  }
  return true;
}

// solve L L' x = b in place
template <int D>
BMPC_HD void chol_solve(const double (&L)[D][D], double (&b)[D]) {
#pragma unroll
  for (int i = 0; i < D; ++i) {
    double t = b[i];
#pragma unroll
    for (int k = 0; k < i; ++k) t -= L[i][k] * b[k];
    b[i] = t / L[i][i];
  }
#pragma unroll
  for (int i = D - 1; i >= 0; --i) {
    double t = b[i];
#pragma unroll
    for (int k = i + 1; k < D; ++k) t -= L[k][i] * b[k];
    b[i] = t / L[i][i];
  }
}

// v0^2 - ||v1||^2 as (v0-|v_k|)(v0+|v_k|) - sum_{i != k} v_i^2 (k = argmax |v_i|)
BMPC_HD double cone_res_parts(double v0, double vk_abs, double sumsq_rest) {
  return (v0 - vk_abs) * (v0 + vk_abs) - sumsq_rest;
}

}  // namespace bmpc
