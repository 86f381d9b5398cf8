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
// phase-sized functions stay out of line: the IPM kernel calls them from many sites and
// inlining them all blows the kernel past the instruction cache
#if defined(BMPC_INLINE_ALL)
#define BMPC_FN __host__ __device__ __forceinline__
#else
#define BMPC_FN __host__ __device__ __attribute__((noinline))
#endif
#else
#define BMPC_HD inline
#define BMPC_FN inline
#endif

#include <math.h>

namespace bmpc {

// ------------------------------------------------------------------------------------
// Address spaces.  Arguments of an out-of-line device function arrive as generic,
// lane-varying pointers: every load through them is a flat_load (counted by both vmcnt and
// lgkmcnt, so a wait for LDS or scalar data also waits for HBM) and every Plan field is a
// vector load queued behind the wave's HBM misses.  The device code therefore types its
// pointers: the ego workspace and the plan's topology tables are global memory (gdouble,
// gint), the Plan / Layout are constant memory read with wave-uniform addresses (s_load
// through the scalar cache), the per-wave scratch is LDS (ldouble).  On the host build the
// qualifiers vanish.
// ------------------------------------------------------------------------------------
// The small-batch kernel's translation units (bmpc_kb_*.hip) define BMPC_FLAT_SLAB: their slab
// pointers are generic (flat loads and stores), so that a per-ego layout can place the IPM's
// most-visited arrays in the workgroup's LDS (bmpc_dev.h, k_solve_blk).
#if defined(__HIP_DEVICE_COMPILE__)
#if defined(BMPC_FLAT_SLAB)
#define BMPC_AS_GLOBAL
#else
#define BMPC_AS_GLOBAL __attribute__((address_space(1)))
#endif
#define BMPC_AS_LDS __attribute__((address_space(3)))
#define BMPC_AS_CONST __attribute__((address_space(4)))
#else
#define BMPC_AS_GLOBAL
#define BMPC_AS_LDS
#define BMPC_AS_CONST
#endif
typedef BMPC_AS_GLOBAL double gdouble;
typedef BMPC_AS_LDS double ldouble;
typedef const BMPC_AS_GLOBAL int32_t gint;

// the value of a wave-uniform pointer held in a VGPR, moved to SGPRs
template <class T>
BMPC_HD T* uniform_ptr(T* p) {
#if defined(__HIP_DEVICE_COMPILE__)
  const uint64_t v = reinterpret_cast<uint64_t>(p);
  const uint32_t lo = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(v));
  const uint32_t hi = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(v >> 32));
  return reinterpret_cast<T*>((static_cast<uint64_t>(hi) << 32) | lo);
#else
  return p;
#endif
}

// ------------------------------------------------------------------------------------
// Plan: per-plan constants and topology tables (shared by every ego of the batch).
// ------------------------------------------------------------------------------------
// The tables (one concatenated int32 blob, see HostPlan): per branch in BFS order of
// MPC_branch.inittree -- depth, length, first x / u node, first child (children are
// contiguous; -1 for leaves); per x node -- its u node (-1 for leaf terminal nodes), the
// u node whose (A,B,C) defines it and that node's x (-1 for the root), the cone whose middle
// rows contain it (-1 none) and its position in that cone's branch, its branch, CSR
// successors (nodes defined by its (A,B,C)), the nodes grouped by tree level; per u node --
// its x node and cone; per cone -- parent non-leaf branch (-1 = root cone), child slot,
// child branch (-1 = root cone), dimension and first row in the conic row vector.
#define BMPC_TOPO_FIELDS(F)                                                                  \
  F(br_depth) F(br_len) F(br_ndx) F(br_ndu) F(br_child0) F(x_u) F(x_srcu) F(x_srcx) F(x_cone) \
  F(x_conepos) F(x_branch) F(succ_off) F(succ) F(lvl_off) F(lvl_nodes) F(u_x) F(u_cone)       \
  F(cone_b) F(cone_i) F(cone_c) F(cone_q) F(cone_off)
#define BMPC_TOPO_COUNT_(n) +1
enum { BMPC_TOPO_N = 0 BMPC_TOPO_FIELDS(BMPC_TOPO_COUNT_) };
#define BMPC_TOPO_MEMBER_(n) IP n;
template <class IP>
struct TopoT {
  BMPC_TOPO_FIELDS(BMPC_TOPO_MEMBER_)
};
// the tables in global memory (k_tree) and the per-wave LDS copy (k_ipm / k_qp: every
// topology lookup on the solver's dependent chains is an LDS read, not a memory round trip)
typedef const BMPC_AS_LDS int32_t lint;
typedef TopoT<gint*> Topo;
typedef TopoT<lint*> TopoL;

// transform slots (Layout::xform): S row-major, the current bx (solve's bx argument), "S is
// not None", "bx was set", the current Fx (solve's Fx argument), "Fx was set", and the state
// rows / bound the solves use -- written on the first solve and on solves with S on, kept
// otherwise (buildIneqConstr :1894-1901 vs updateIneqConstr :2016-2036) -- and "rows written"
// (an ego resumed through the warm-start ABI has none yet: its next solve writes them)
enum { XF_S = 0, XF_BX = BMPC_MAX_N * BMPC_MAX_N, XF_SON = XF_BX + BMPC_MAX_FX, XF_BXSET = XF_SON + 1,
       XF_FX = XF_BXSET + 1, XF_FXSET = XF_FX + BMPC_MAX_FX * BMPC_MAX_N, XF_ROWS = XF_FXSET + 1,
       XF_BROWS = XF_ROWS + BMPC_MAX_FX * BMPC_MAX_N, XF_ROWSET = XF_BROWS + BMPC_MAX_FX,
       XF_COUNT = XF_ROWSET + 1 };

// Per-ego constants of a transform-capable solve (X::kTransform), formed once per solve in
// the wave's LDS: Fx S, W1 S, (W1 S)'(W1 S) and bx (MPC_branch.py:1894-1901,1935-1937);
// without S (or for the other models) the plan's Fx, W1, QQ, bx are read directly.
enum { ECO_FX = 0, ECO_W1 = BMPC_MAX_FX * BMPC_MAX_N, ECO_QQ = ECO_W1 + BMPC_MAX_N * BMPC_MAX_N,
       ECO_BX = ECO_QQ + BMPC_MAX_N * BMPC_MAX_N, ECO_COUNT = ECO_BX + BMPC_MAX_FX };

struct Plan {
  bmpc_plan_desc desc;
  int n, d, N, NB, m, nFx, nFu, Nc;
  // collision rows per state node (robustMPC: one per obstacle prediction of the node's time
  // slot, padded to m^NB; the others 1) and the obstacle tree depth (robustMPC's QP is a
  // chain, NB = 0, over a scenario tree of obstacle predictions of depth zNB)
  int Ncol, zNB;
  int T, U, nbranch, bdim, ncones, nlevels;
  // primal vector layout (reference sol['x'] layout, MPC_branch.py:2100-2102)
  int oX, oU, oRho, oSig, oMup, oMum, oS, oJ, nv;
  // equality rows: T*n dynamics rows then bdim CVaR rows (MPC_branch.py:1752-1804)
  int neq;
  // conic rows: Fx|Fu|risk|positivity LP rows then SOC rows (MPC_branch.py:1869-1990)
  int rFx, rFu, rRisk, rPos, nlp, nrows;
  int ng;     // number of "global" variables (rho, sigma, mu+, mu-, J)
  int nsm;    // dense coupling system size
  // per-wave LDS scratch (doubles): coupling matrix, pivots, rhs, reduction slots
  int lds_M, lds_piv, lds_rhs, lds_rhs2, lds_red, nlds;   // lds_rhs2: the second rhs of a paired back half
  // plan-constant matrices in LDS, read with lane-varying rows (a lane-varying index into the
  // constant buffer is a vector memory round trip): W1 (n x n), Wu (d x d), Fx (nFx x n), Fu (nFu x d)
  int lds_w, lds_wu, lds_fx, lds_fu, nconst;
  int nlds_lean;            // LDS doubles when the coupling system lives in the slab (Layout::coup)
  int lds_scr, nscr;       // tree-solve LDS scratch (slack terms of the pre-pass; 0 = none)
  int cgrp;   // lanes per cone group (power of two, cgrp * ceil(ncones / ngrp) covers all cones)
  int maxq;   // largest cone dimension (fused cone passes hold a cone's rows in registers when
              // maxq <= X::kConeRegRows * cgrp)
  double W1[BMPC_MAX_N * BMPC_MAX_N];   // sqrtm(Q) / chol(Q)'  (MPC_branch.py:1628-1631)
  double Wu[BMPC_MAX_D * BMPC_MAX_D];   // chol(R)'             (:1633-1636)
  double QQ[BMPC_MAX_N * BMPC_MAX_N];   // W1'W1
  double RR[BMPC_MAX_D * BMPC_MAX_D];   // Wu'Wu
  Topo t;
  int toff[BMPC_TOPO_N];   // offset of each table in the blob (int32 units)
  int ntab;                // blob length (int32 units); its LDS copy follows the nlds doubles
  // lane reference of the *_PSIREF policies (bmpc_set_lane_ref): grid then values, nlref
  // points each (device copy in the plan's Bundle; 0 = none)
  const double* lref;
  int nlref;
};

template <class X>
BMPC_HD double fxv(const BMPC_AS_CONST Plan& P, const X& ex, int r, int j) {
  if constexpr (X::kTransform) return ex.eco[ECO_FX + r * P.n + j];
  else return ex.lds[P.lds_fx + r * P.n + j];
}
template <class X>
BMPC_HD double fuv(const BMPC_AS_CONST Plan& P, const X& ex, int r, int j) {
  return ex.lds[P.lds_fu + r * P.d + j];
}
template <class X>
BMPC_HD double w1v(const BMPC_AS_CONST Plan& P, const X& ex, int r, int j) {
  if constexpr (X::kTransform) return ex.eco[ECO_W1 + r * P.n + j];
  else return P.W1[r * P.n + j];
}
template <class X>
BMPC_HD double qqv(const BMPC_AS_CONST Plan& P, const X& ex, int i, int j) {
  if constexpr (X::kTransform) return ex.eco[ECO_QQ + i * P.n + j];
  else return P.QQ[i * P.n + j];
}
template <class X>
BMPC_HD double bxv(const BMPC_AS_CONST Plan& P, const X& ex, int r) {
  if constexpr (X::kTransform) return ex.eco[ECO_BX + r];
  else return P.desc.bx[r];
}

// entry i of the plan-constant LDS area (Plan::lds_w .. + nconst): W1 | Wu | Fx | Fu
BMPC_HD double plan_const(const Plan& P, int i) {
  if (i < P.lds_wu) return P.W1[i - P.lds_w];
  if (i < P.lds_fx) return P.Wu[i - P.lds_wu];
  if (i < P.lds_fu) return P.desc.Fx[i - P.lds_fx];
  return P.desc.Fu[i - P.lds_fu];
}

// view of the topology tables through ex.tab: the wave's LDS copy of the blob, or the blob in
// global memory when the copy would cost resident waves (bmpc_hip.hip, choose_topo_lds)
#define BMPC_TOPO_SET_(n) v.n = ex.tab + P.toff[i++];
template <class X>
BMPC_HD TopoT<typename X::tab_ptr> topo_view(const BMPC_AS_CONST Plan& P, const X& ex) {
  TopoT<typename X::tab_ptr> v;
  int i = 0;
  BMPC_TOPO_FIELDS(BMPC_TOPO_SET_)
  return v;
}

// ------------------------------------------------------------------------------------
// Per-ego workspace layout (offsets in doubles inside one ego's slab)
// ------------------------------------------------------------------------------------
struct Layout {
  // persistent state (survives between solves)
  size_t uLin, pprev, misc, xpred, upred, sol;
  // tree of the current solve
  size_t xbar, zbar, ubar, Ad, Bd, Cd, dh, h0, w, p, dp, boost, xref;
  // IPM vectors
  size_t x, y, z, s, lam, x1, y1, z1, x2, y2, z2, dz, ds, rx, ry, rz, hvec, bvec;
  size_t ta, ta2, ya, ra, rb, rc, bestx;
  // ECOS's equilibration of this solve (bmpc_ipm.h equilibrate): column factors (nv), A row factors
  // (neq), G row factors (nrows; one value per second-order cone)
  size_t xeq, aeq, geq;
  // KKT-solve scratch
  size_t k_r0, k_nv0, k_e1, k_e2, k_e3, k_t3, k_t3b, k_cx, k_cy, k_cz, k_nv1, zeros;
  // scaling
  size_t dl, dli, eta, wbar, vnt;   // NT scaling: LP d and 1/d, cone eta, wbar, v
  // KKT
  size_t hx, hu, sd, P, Kg, Luu, kff, lvec, qx0, gk, colk, colnu;
  size_t coup;    // coupling matrix | pivots | rhs when they are not in LDS (lean-LDS launches; the
                  // phase-per-kernel IPM keeps the factored matrix and pivots here between kernels)
  size_t ist;     // the phase-per-kernel IPM's per-ego state (IS_* slots, bmpc_ipm_ph.h)
  size_t prof;    // PROF_COUNT phase cycle counters (BMPC_PROFILE builds)
  // BranchMPCProx QP: u-rate couplings, linear cost, augmented Riccati P~, [Kx Kv], l~
  size_t qo, qq, Pa, Ka, la;
  // robustMPC: carried linearisation trajectory, obstacle predictions [time][Ncol][n]
  size_t xlin, zrob;
  // merge scene (HIGHWAY_MERGE plans): per-ego S [n*n], bx [BMPC_MAX_FX], flags (XF_*)
  size_t xform;
  size_t stride;  // doubles per ego
};

typedef const BMPC_AS_CONST Plan CPlan;
typedef const BMPC_AS_CONST Layout CLayout;

// misc slots
enum { MISC_INIT = 0, MISC_JCONS = 1, MISC_OLDU = 2 /* d values */, MISC_BEST = 6 /* best score, its tau (IPM guard) */,
       MISC_X0 = 8 /* n values (robustMPC) */ };



// ------------------------------------------------------------------------------------
// phase cycle counters: built with -DBMPC_PROFILE the device code accumulates s_memtime
// cycles of each phase per ego (lane 0) into Layout::prof; otherwise the scopes vanish.
// ------------------------------------------------------------------------------------
enum {
  PROF_TREE = 0, PROF_RESID, PROF_SCALING, PROF_FACTOR, PROF_COUPLING, PROF_KKT, PROF_TREESOLVE,
  PROF_REFINE, PROF_STEP, PROF_INIT, PROF_TOTAL, PROF_NSOLVE, PROF_APPLYW, PROF_APPLYG, PROF_APPLYGT,
  PROF_NTREE, PROF_G_LP, PROF_G_CONE, PROF_NAPPLYG, PROF_X1, PROF_X2, PROF_X3, PROF_X4,
#if defined(BMPC_PROFILE)
  // profile builds only (the product's slab keeps 24): the coupling's parts
  PROF_RIC = 23, PROF_CTS, PROF_CDOT, PROF_LU, PROF_LUS, PROF_BACK, PROF_RIC_LD, PROF_RIC_A, PROF_RIC_B, PROF_COUNT = 32
#else
  PROF_COUNT = 24
#endif
};
#if defined(BMPC_PROFILE) && defined(__HIP_DEVICE_COMPILE__)
struct ProfScope {
  gdouble* slot;
  long long t0;
  template <class PT>
  __device__ ProfScope(PT ws, size_t base, int id) : slot((gdouble*)(ws + base + id)), t0(__builtin_amdgcn_s_memtime()) {}
  __device__ ~ProfScope() {
    const long long t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) *slot += (double)(t1 - t0);
  }
};
#define BMPC_PROF(ws, L, id) ProfScope _prof_##id((ws), (L).prof, id)
#define BMPC_TIC(v) const long long v = __builtin_amdgcn_s_memtime()
#define BMPC_TOC(ws, L, id, v) \
  if (threadIdx.x == 0) (ws)[(L).prof + (id)] += (double)(__builtin_amdgcn_s_memtime() - (v))
#define BMPC_COUNT(ws, L, id) \
  if (threadIdx.x == 0) (ws)[(L).prof + (id)] += 1.0
// a phase boundary inside a dependent chain: wait for every outstanding load first (profile builds)
#define BMPC_TOC_WAIT(ws, L, id, v) \
  __builtin_amdgcn_s_waitcnt(0);      \
  BMPC_TOC(ws, L, id, v)
#else
#define BMPC_PROF(ws, L, id) ((void)0)
#define BMPC_TIC(v) ((void)0)
#define BMPC_TOC(ws, L, id, v) ((void)0)
#define BMPC_COUNT(ws, L, id) ((void)0)
#define BMPC_TOC_WAIT(ws, L, id, v) ((void)0)
#endif

// ------------------------------------------------------------------------------------
// iteration trace of the IPMs (diagnostics builds only): -DBMPC_HOST_DEBUG on the host build,
// -DBMPC_DEV_DEBUG on the device (lane 0 of workgroup 0 -- trace a one-ego batch), the same
// format on both so tools/trace_diff.py can line them up
// ------------------------------------------------------------------------------------
#if defined(BMPC_HOST_DEBUG) && !defined(__HIP_DEVICE_COMPILE__)
#define BMPC_TRACING 1
#define BMPC_TRACE(...) printf(__VA_ARGS__)
#elif defined(BMPC_DEV_DEBUG) && defined(__HIP_DEVICE_COMPILE__)
#define BMPC_TRACING 1
#define BMPC_TRACE(...) \
  do { if (blockIdx.x == 0 && threadIdx.x == 0) printf(__VA_ARGS__); } while (0)
#else
#define BMPC_TRACING 0
#define BMPC_TRACE(...) ((void)0)
#endif

// ------------------------------------------------------------------------------------
// batched lane loops: every lane first evaluates ld(i) for up to UN of its indices -- all
// loads of the batch are in flight together instead of one memory round trip per element
// -- then commits them with st(i, v).  ld must not read what st of the same batch writes.
// ------------------------------------------------------------------------------------
// The loads are unconditional (an index past hi is clamped to b, which is valid): a load
// under a per-lane guard would sit in its own exec-masked block with its own wait, i.e. one
// memory round trip per element instead of one per batch.
#ifndef BMPC_TAIL_BATCH
#define BMPC_TAIL_BATCH 0   // 1: full batches, then halving ones (no clamped loads): headline -1.4%, 1,024 egos +8% (r05aa), off
#endif
template <int UN = 8, class Ld, class St>
BMPC_HD void strided_batch(int first, int stride, int hi, Ld ld, St st) {
#if BMPC_TAIL_BATCH
  // full batches of UN while all of a lane's UN slots are in range, the rest in halving
  // batches (16 + 4 slots for 20 elements instead of 32): no clamped duplicate loads; a lane
  // still visits its indices in increasing order
  int b = first;
  for (; b + (UN - 1) * stride < hi; b += UN * stride) {
    decltype(ld(b)) v[UN];
#pragma unroll
    for (int u = 0; u < UN; ++u) v[u] = ld(b + u * stride);
#pragma unroll
    for (int u = 0; u < UN; ++u) st(b + u * stride, v[u]);
  }
  if constexpr (UN > 1) strided_batch<UN / 2>(b, stride, hi, ld, st);
  else if (b < hi) st(b, ld(b));
  return;
#endif
  for (int b = first; b < hi; b += UN * stride) {
    decltype(ld(b)) v[UN];
#pragma unroll
    for (int u = 0; u < UN; ++u) {
      const int i = b + u * stride;
      v[u] = ld(i < hi ? i : b);
    }
#pragma unroll
    for (int u = 0; u < UN; ++u) {
      const int i = b + u * stride;
      if (i < hi) st(i, v[u]);
    }
  }
}

// Executors that spread one ego over several waves (the small-batch kernel's DevBlockExecT:
// kBatchDiv = its waves) give each lane that many times fewer elements of a pass: their batches
// shrink by the same factor, so a pass issues its loads for the elements a lane has instead of
// UN clamped slots (per lane the stores still come in index order: the same values, the same
// order of any accumulation in st).
template <class X, class = void>
struct BatchDiv {
  static constexpr int v = 1;
};
template <class X>
struct BatchDiv<X, decltype((void)X::kBatchDiv)> {
  static constexpr int v = X::kBatchDiv;
};

template <int UN, class X>
struct Narrow {
  static constexpr int v = UN / BatchDiv<X>::v > 0 ? UN / BatchDiv<X>::v : 1;
};
// the batch width of a cone group's strided loops (4; the small-batch kernel's executor may
// set kConeBatch for its wider cone groups)
template <class X, class = void>
struct ConeBatch {
  static constexpr int v = 4;
};
template <class X>
struct ConeBatch<X, decltype((void)X::kConeBatch)> {
  static constexpr int v = X::kConeBatch;
};

template <int UN = 8, class X, class Ld, class St>
BMPC_HD void lane_batch(const X& ex, int lo, int hi, Ld ld, St st) {
  strided_batch<Narrow<UN, X>::v>(lo + ex.lane, ex.nlanes, hi, ld, st);
}

// per-lane partial reduction of f(i) over first, first+stride, ... < hi with UN
// independent accumulators (op: 0 sum, 1 max, 2 min).  The slots past hi are masked by
// arithmetic, not by a select on f's value: the compiler turns a select whose operand is a
// load (or a division) into a branch around it, i.e. one memory round trip per element.
// For finite values the result is bit-identical (x + 0*v == x; fmax / fmin ignore the NaN of
// v + (-inf) or v + inf).
template <int UN = 8, int OP = 0, class F>
BMPC_HD double strided_partial(int first, int stride, int hi, F f) {
  const double init = OP == 0 ? 0.0 : OP == 1 ? -1e300 : 1e300;
  double acc[UN];
#pragma unroll
  for (int u = 0; u < UN; ++u) acc[u] = init;
  for (int b = first; b < hi; b += UN * stride) {
#pragma unroll
    for (int u = 0; u < UN; ++u) {
      const int i = b + u * stride;
      const bool in = i < hi;
      const double v = f(in ? i : b);   // unconditional (see strided_batch)
      if constexpr (OP == 0) acc[u] += (in ? 1.0 : 0.0) * v;
      else if constexpr (OP == 1) acc[u] = fmax(acc[u], v + (in ? 0.0 : -INFINITY));
      else acc[u] = fmin(acc[u], v + (in ? 0.0 : INFINITY));
    }
  }
  double s = init;
#pragma unroll
  for (int u = 0; u < UN; ++u) s = OP == 0 ? s + acc[u] : OP == 1 ? fmax(s, acc[u]) : fmin(s, acc[u]);
  return s;
}

template <int UN = 8, class X, class F>
BMPC_HD double lane_partial(const X& ex, int lo, int hi, F f) {
  return strided_partial<Narrow<UN, X>::v, 0>(lo + ex.lane, ex.nlanes, hi, f);
}

// this lane's max (OP 1) / min (OP 2) of f(i) over its indices of [lo, hi)
template <int UN, int OP, class X, class F>
BMPC_HD double lane_extreme(const X& ex, int lo, int hi, F f) {
  return strided_partial<Narrow<UN, X>::v, OP>(lo + ex.lane, ex.nlanes, hi, f);
}

// sum over the lanes of f(i), i in [lo, hi)
template <int UN = 8, class X, class F>
BMPC_HD double lane_sum(const X& ex, int lo, int hi, F f) {
  return ex.sum(strided_partial<Narrow<UN, X>::v, 0>(lo + ex.lane, ex.nlanes, hi, f));
}

// Cone groups: the lanes split into groups of cg lanes (a power of two); group g handles
// cones g, g + ngrp, ... in lock-step rounds so that group reductions stay convergent.
// f(k, gl, cg) is called once per round with k = -1 for an idle group.
struct ConeGroups {
  int cg, ngrp, g, gl, rounds;
};
// lanes per cone group of an executor: 1 on the host, the plan's cgrp on one wave (cgrp *
// ncones <= 64), and on a multi-wave executor the largest power of two <= 64 that still gives
// every cone a group of its own
template <class X>
BMPC_HD int exec_cgrp(const X& ex, int cgrp, int ncones) {
  if (ex.nlanes == 1) return 1;
  if (ex.nlanes <= 64) return cgrp;
  int cg = 64;
  while (cg > 1 && cg * ncones > ex.nlanes) cg >>= 1;
  return cg;
}
template <class X>
BMPC_HD ConeGroups cone_groups(const X& ex, int cgrp, int ncones) {
  ConeGroups G;
  G.cg = exec_cgrp(ex, cgrp, ncones);
  G.ngrp = ex.nlanes / G.cg;
  G.g = ex.lane / G.cg;
  G.gl = ex.lane % G.cg;
  G.rounds = (ncones + G.ngrp - 1) / G.ngrp;
  return G;
}

// ------------------------------------------------------------------------------------
// small dense helpers (row-major, compile-time sizes)
// ------------------------------------------------------------------------------------
template <int R, int C, class PT>
BMPC_HD void mat_load(double (&M)[R][C], PT p) {
#pragma unroll
  for (int i = 0; i < R; ++i)
#pragma unroll
    for (int j = 0; j < C; ++j) M[i][j] = p[i * C + j];
}

template <int R, int C, class PT>
BMPC_HD void mat_store(const double (&M)[R][C], PT p) {
#pragma unroll
  for (int i = 0; i < R; ++i)
#pragma unroll
    for (int j = 0; j < C; ++j) p[i * C + j] = M[i][j];
}

template <int R, int C>
BMPC_HD void mat_copy(const double (&S)[R][C], double (&D)[R][C]) {
#pragma unroll
  for (int i = 0; i < R; ++i)
#pragma unroll
    for (int j = 0; j < C; ++j) D[i][j] = S[i][j];
}

template <int R, int C>
BMPC_HD void mat_zero(double (&D)[R][C]) {
#pragma unroll
  for (int i = 0; i < R; ++i)
#pragma unroll
    for (int j = 0; j < C; ++j) D[i][j] = 0.0;
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

// x / y given r = 1 / y (correctly rounded): q0 = x r, then one FMA for the remainder and one
// for the correction give the correctly rounded quotient (Markstein's theorem; no overflow or
// underflow in range), so the quotients of a shared divisor cost one division and three
// operations each instead of a division sequence each -- the same bits as x / y
// (tools/markstein_check.c: 2e8 random pairs).  The host build divides.
BMPC_HD double div_rcp(double x, double y, double r) {
#if defined(__HIP_DEVICE_COMPILE__)
  const double q0 = x * r;
  return fma(fma(-q0, y, x), r, q0);
#else
  (void)r;
  return x / y;
#endif
}
// chol_solve with the reciprocals of L's diagonal given (div_rcp): the same bits
template <int D>
BMPC_HD void chol_solve_r(const double (&L)[D][D], const double (&ri)[D], double (&b)[D]) {
#pragma unroll
  for (int i = 0; i < D; ++i) {
    double t = b[i];
#pragma unroll
    for (int k = 0; k < i; ++k) t -= L[i][k] * b[k];
    b[i] = div_rcp(t, L[i][i], ri[i]);
  }
#pragma unroll
  for (int i = D - 1; i >= 0; --i) {
    double t = b[i];
#pragma unroll
    for (int k = i + 1; k < D; ++k) t -= L[k][i] * b[k];
    b[i] = div_rcp(t, L[i][i], ri[i]);
  }
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
