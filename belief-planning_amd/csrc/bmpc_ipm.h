// bmpc_ipm.h -- structured interior-point solve of the scenario-tree CVaR SOCP of one ego.
//
// Problem (exactly what BranchMPC_CVaR hands to ecos.solve, MPC_branch.py:2043-2092):
//   min c'z  s.t.  A z = b  (dynamics + CVaR dual rows, :1752-1804)
//                  G z + s = h, s in R+^l x Q^{q1} x ... (LP + rotated SOC rows, :1869-1990)
// Algorithm: ECOS' homogeneous self-dual embedding with Nesterov-Todd scaling and
// Mehrotra predictor-corrector (same as oracle/ecos_ipm.py), but the KKT system is never
// assembled.  With dz eliminated the reduced Hessian is
//   G'W^-2 G = sum_LP (z/s) a a'  +  sum_cones (1/eta^2) (F2'F2 + 2 g g'),  g = G'(J wbar)
// (each rotated cone has first row f and last row -f, so its NT term is block-diagonal plus
// ONE rank-1 term).  The block-diagonal part lives on the tree nodes and is factored by a
// tree Riccati recursion (children merge into their parent's cost-to-go); the rank-1 cone
// terms and the few "global" CVaR variables (rho, sigma, mu+-, J) form a small dense
// coupling system (Woodbury / Schur), solved by LU with partial pivoting.
#pragma once

#include <type_traits>

#include "bmpc_tree.h"
#include "bmpc_wave.h"

#ifndef BMPC_EQUIL
#define BMPC_EQUIL 1         // 0: no equilibration (the unscaled IPM of rounds 1-4)
#endif
#ifndef BMPC_EQUIL_ITERS
#define BMPC_EQUIL_ITERS 3   // ECOS glblopts.h EQUIL_ITERS
#endif
// right-hand sides from which the coupling tree solve takes the post-pass that loads a node's
// data once per four right-hand sides (tree_solve<..., RB=true>); a separate instantiation
// with the same arithmetic per right-hand side (tests/test_kernel_host.py compares the two)
#ifndef BMPC_TS_POST_RB_MIN
#define BMPC_TS_POST_RB_MIN 8
#endif
#ifndef BMPC_TS_POST_RB
#define BMPC_TS_POST_RB 4    // right-hand sides per pass of that post-pass
#endif
#ifndef BMPC_PAIR_REFINE
#define BMPC_PAIR_REFINE 1   // the pair's refinement rounds share their correction tree solves
#endif
#ifndef BMPC_BLK_WAVE_SUBST
#define BMPC_BLK_WAVE_SUBST 1   // multi-wave executors: the coupling substitutions on one wave
#endif
#ifndef BMPC_BLK_PAIR_DOTS
#define BMPC_BLK_PAIR_DOTS 1    // multi-wave executors: the cone-cone coupling block with a lane per (k, j) entry
#endif
#ifndef BMPC_WAVE_LU
#define BMPC_WAVE_LU 1          // device executors: the coupling LU on one wave over its non-zero rows (small_lu_wave)
#endif
#ifndef BMPC_WAVE_LU_MIN1
#define BMPC_WAVE_LU_MIN1 32    // ... in the one-wave executor from this order on (config 3: 50; multi-wave: always)
#endif
#ifndef BMPC_SUBST_REG
#define BMPC_SUBST_REG 1        // the one-wave coupling substitutions with the right-hand side in registers
#endif
#ifndef BMPC_REFINE_CALLS
#define BMPC_REFINE_CALLS 1  // 1: kkt_refine_pair's correction back halves are calls of their own
#endif
#ifndef BMPC_FLAT_PAIR
#define BMPC_FLAT_PAIR 1     // 1: the IPM loop calls the pair's coupling solve and refinement directly
#endif
#ifndef BMPC_PAIR_BACK
#define BMPC_PAIR_BACK 1     // kkt_solve_pair's two back halves in one pass over the Woodbury data
#endif
#ifndef BMPC_TS_UN
#define BMPC_TS_UN 2         // elements per lane batch in the tree solve's slack pre- / post-passes (2: -1.1% k_ipm vs 4, 8: +15%)
#endif
#ifndef BMPC_TS_UN_AV
#define BMPC_TS_UN_AV 8      // ... and in the pre-pass's slack-term pass
#endif
#ifndef BMPC_NITREF
#define BMPC_NITREF 1        // refinement rounds per KKT solve (oracle: 3; 1 keeps parity)
#endif
#ifndef BMPC_NITREF_INIT
#define BMPC_NITREF_INIT 0   // refinement rounds of the two initial-point solves (far from the tolerances)
#endif
#ifndef BMPC_REFSCORE
#define BMPC_REFSCORE 1e-3   // refine only when max(pres, dres, relgap) of the iterate < this (1e-4 flips replay exit codes)
#endif
#ifndef BMPC_REFSCORE2
#define BMPC_REFSCORE2 1e-6  // ... and BMPC_NITREF2 rounds in the end game (score below this)
#endif
#ifndef BMPC_NITREF2
#define BMPC_NITREF2 2
#endif
#ifndef BMPC_REFTOL
#define BMPC_REFTOL 1e-14    // refinement stop: scaled residual <= tol * max(1, |rhs|) (oracle: 1e-14)
#endif
#ifndef BMPC_REF_STALL
#define BMPC_REF_STALL 0     // > 0: ECOS's refinement stop (IRERRFACT): a round that cuts the residual by less than
                             // this factor ends the refinement, one that grows it is undone
#endif

// per-phase inlining overrides (experiments: -DBMPC_FN_APPLY_G=BMPC_HD ...)
#ifndef BMPC_FN_APPLY_G
#define BMPC_FN_APPLY_G BMPC_FN
#endif
#ifndef BMPC_FN_APPLY_GT
#define BMPC_FN_APPLY_GT BMPC_FN
#endif
#ifndef BMPC_FN_SCALING
#define BMPC_FN_SCALING BMPC_FN
#endif
#ifndef BMPC_FN_MAX_STEP
#define BMPC_FN_MAX_STEP BMPC_FN
#endif
#ifndef BMPC_FN_TREE_SOLVE
#define BMPC_FN_TREE_SOLVE BMPC_FN
#endif
#ifndef BMPC_FN_FUSED
#define BMPC_FN_FUSED BMPC_FN   // the fused cone passes (out of line: -0.8% k_ipm vs inlined, A/B at 4096 egos)
#endif

namespace bmpc {

enum {
  EXIT_OPTIMAL = 0, EXIT_PINF = 1, EXIT_DINF = 2, EXIT_INACC = 10,
  EXIT_MAXIT = -1, EXIT_NUMERICS = -2,
  EXIT_GUARD = -9   // internal consistency guard tripped (never expected; tests assert status >= 0)
};

// ------------------------------------------------------------------------------------
// context bundling the per-ego pointers
// ------------------------------------------------------------------------------------
struct Ctx {
  CPlan* P;
  CLayout* L;
  gdouble* ws;
  BMPC_HD gdouble* at(size_t off) const { return ws + off; }
  // the same context with its pointers in SGPRs (first statement of every out-of-line phase)
  BMPC_HD Ctx uniform() const { return Ctx{uniform_ptr(P), uniform_ptr(L), uniform_ptr(ws)}; }
};

// xRef' Q (the cone rows' linear cost term, MPC_branch.py:1927-1940); xref is written by the
// tree kernel, Q is plan constant
template <int NX>
BMPC_HD void ctx_qx(const Ctx& C, double (&qx)[NX]) {
  const gdouble* xref = C.at(C.L->xref);
  double xr[NX];
#pragma unroll
  for (int r = 0; r < NX; ++r) xr[r] = xref[r];
#pragma unroll
  for (int c = 0; c < NX; ++c) {
    double v = 0.0;
#pragma unroll
    for (int r = 0; r < NX; ++r) v += xr[r] * C.P->desc.Q[r * NX + c];
    qx[c] = v;
  }
}

// cone-group rounds (see ConeGroups): G, and per round k / off / q of the owned cone
#define BMPC_CONE_ROUNDS(ex, P, G)                                \
  const auto G##_t = topo_view((P), ex);                         \
  const ConeGroups G = cone_groups(ex, (P).cgrp, (P).ncones);     \
  for (int rnd_ = 0; rnd_ < G.rounds; ++rnd_)
#define BMPC_CONE_K(P, G, k, off, q)                              \
  const int k = rnd_ * G.ngrp + G.g < (P).ncones ? rnd_ * G.ngrp + G.g : -1; \
  const int off = k >= 0 ? G##_t.cone_off[k] : 0;                 \
  const int q = k >= 0 ? G##_t.cone_q[k] : 0

// multi-wave executors (the small-batch kernel's DevBlockExecT: one ego on several waves)
template <class X>
struct MultiWave : std::integral_constant<bool, (BatchDiv<X>::v > 1)> {};

// e^-beta_k of cone k: the multi-wave executor (one ego, issue-bound) reads the value k_tree stored
// after the boosts; the batch kernels (HBM-bound: a dependent load costs more than the exp there,
// headline -2% measured) recompute it -- the same value either way
template <class X, class PB>
BMPC_HD double ebeta(const PB* boost, int nc, int k) {
  if constexpr (MultiWave<X>::value) return boost[nc + k];
  return exp(-boost[k]);
}

// ------------------------------------------------------------------------------------
// block of dot products in one pass: acc[a][b] = sum_i A_a[i] B_b[i] over the tree-variable
// ranges [lo1, hi1) and [lo2, hi2), rows A_a = A + a*astr (a < na <= 4), B_b = B + b*bstr
// (b < nb <= 4); every load of a lane's step is issued together (one round trip per pass
// instead of one per dot product), then each entry is reduced over the wave.
// ------------------------------------------------------------------------------------
// NBR: the B vectors the caller reads (1 or 2: the back halves' g_k' dx), so that the
// multi-wave executor forms and reduces only those 4 * NBR sums (each sum's reduction is
// independent of the others: the same bits); the batch kernels keep the sixteen (the trimmed
// pass cost the headline k_ipm 3.6% -- its register allocation, profiles/r06/r06ad_*)
template <int NBR0 = 4, class X>
BMPC_HD void block_dots(const X ex, const gdouble* A, size_t astr, int na, const gdouble* B, size_t bstr, int nb,
                        int lo1, int hi1, int lo2, int hi2, double (&acc)[4][4]) {
  constexpr int NBR = MultiWave<X>::value ? NBR0 : 4;
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[a][b] = 0.0;
  const int n1 = hi1 - lo1, ntot = n1 + (hi2 - lo2);
  auto idx = [&](int t) { return t < n1 ? lo1 + t : lo2 + (t - n1); };
#pragma unroll 2
  for (int t = ex.lane; t < ntot; t += ex.nlanes) {
    const int i = idx(t);
    double av[4], bv[4];
#pragma unroll
    for (int a = 0; a < 4; ++a) av[a] = a < na ? A[a * astr + i] : 0.0;
#pragma unroll
    for (int b = 0; b < 4; ++b) bv[b] = b < nb ? B[b * bstr + i] : 0.0;
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int b = 0; b < (NBR < 4 ? NBR : 4); ++b) acc[a][b] += av[a] * bv[b];
  }
  if constexpr (NBR >= 4) {
    ex.template sum_n<16>(&acc[0][0]);   // all sixteen in one reduction (one barrier on a multi-wave executor)
  } else {
    double v[4 * NBR];
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int b = 0; b < NBR; ++b) v[a * NBR + b] = acc[a][b];
    ex.template sum_n<4 * NBR>(v);
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int b = 0; b < NBR; ++b) acc[a][b] = v[a * NBR + b];
  }
}

// ------------------------------------------------------------------------------------
// Cone k's rank-1 vector g_k = G_k'(J wbar) is zero outside its support among the tree
// variables: the x / u / S entries of its child branch's N nodes (the root cone: the root
// node's u and S).  Plans with many cones (NB = 2: 13, each supported on 1/13 of the tree) form
// the coupling products over the support only; the N = 20 NB = 1 plan's 4 cones cover a third
// each, and there one pass over all tree variables is faster (block_dots).
// ------------------------------------------------------------------------------------
template <class T>
BMPC_HD int cone_supp_len(CPlan& P, const T& t, int k) {
  return t.cone_c[k] >= 0 ? P.N * (P.n + P.d + P.Nc) : P.d + P.Nc;
}
// index (into the primal vector) of entry e of cone k's support
template <class T>
BMPC_HD int cone_supp_idx(CPlan& P, const T& t, int k, int e) {
  const int c = t.cone_c[k];
  if (c < 0) return e < P.d ? P.oU + e : P.oS + (e - P.d);
  const int xn = P.N * P.n, un = P.N * P.d;
  if (e < xn) return P.oX + t.br_ndx[c] * P.n + e;
  if (e < xn + un) return P.oU + t.br_ndu[c] * P.d + (e - xn);
  return P.oS + t.br_ndx[c] * P.Nc + (e - xn - un);
}
BMPC_HD bool coup_supp_dots(CPlan& P) { return P.ncones > 4; }

// acc[j] = g_k' v_{j0 + j} over cone k's support (j < 16, j0 + j < nvec; v_j = v0 + j * vstr)
template <class X, class T>
BMPC_HD void cone_supp_dots(const X& ex, CPlan& P, const T& t, const gdouble* gk, int k, const gdouble* v0,
                            size_t vstr, int j0, int nvec, double (&acc)[16]) {
#pragma unroll
  for (int j = 0; j < 16; ++j) acc[j] = 0.0;
  const int tot = cone_supp_len(P, t, k);
  for (int e = ex.lane; e < tot; e += ex.nlanes) {
    const int i = cone_supp_idx(P, t, k, e);
    const double g = gk[i];
    double v[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) v[j] = v0[(size_t)(j0 + j < nvec ? j0 + j : j0) * vstr + i];
#pragma unroll
    for (int j = 0; j < 16; ++j) acc[j] += (j0 + j < nvec ? g : 0.0) * v[j];
  }
  ex.template sum_n<16>(acc);
}

// acc[k] = g_k' dx over each cone's support, all cones in one batched pass (k < 16 per call:
// cones k0 .. k0 + 15)
template <class X, class T>
BMPC_HD void cone_supp_gdx(const X& ex, CPlan& P, const T& t, const gdouble* g0, size_t gstr, const gdouble* dx, int k0,
                           double (&acc)[16]) {
#pragma unroll
  for (int j = 0; j < 16; ++j) acc[j] = 0.0;
  const int nc = P.ncones;
  const int kn = nc - k0 < 16 ? nc - k0 : 16;
  const int full = P.N * (P.n + P.d + P.Nc);   // support length of every non-root cone
  // flattened (cone, entry) index: cones k0.. in order, the root cone (last) shorter
  int tot = 0;
  for (int j = 0; j < kn; ++j) tot += cone_supp_len(P, t, k0 + j);
  constexpr int UN = 8;
  for (int b = ex.lane; b < tot; b += UN * ex.nlanes) {
    double gv[UN], xv[UN];
    int kk[UN];
#pragma unroll
    for (int u = 0; u < UN; ++u) {
      const int f = b + u * ex.nlanes < tot ? b + u * ex.nlanes : b;
      const int j = f / full < kn ? f / full : kn - 1;
      const int e = f - j * full;
      const int i = cone_supp_idx(P, t, k0 + j, e);
      kk[u] = b + u * ex.nlanes < tot ? j : -1;
      gv[u] = g0[(size_t)(k0 + j) * gstr + i];
      xv[u] = dx[i];
    }
#pragma unroll
    for (int u = 0; u < UN; ++u)
#pragma unroll
      for (int j = 0; j < 16; ++j) acc[j] += (kk[u] == j ? gv[u] : 0.0) * xv[u];
  }
  ex.template sum_n<16>(acc);
}

// cone_supp_gdx for two vectors at once (each g_k entry loaded once for both); per vector the
// same products and sums as cone_supp_gdx
template <class X, class T>
BMPC_HD void cone_supp_gdx2(const X& ex, CPlan& P, const T& t, const gdouble* g0, size_t gstr, const gdouble* dx1,
                            const gdouble* dx2, int k0, double (&acc1)[16], double (&acc2)[16]) {
#pragma unroll
  for (int j = 0; j < 16; ++j) acc1[j] = 0.0, acc2[j] = 0.0;
  const int nc = P.ncones;
  const int kn = nc - k0 < 16 ? nc - k0 : 16;
  const int full = P.N * (P.n + P.d + P.Nc);
  int tot = 0;
  for (int j = 0; j < kn; ++j) tot += cone_supp_len(P, t, k0 + j);
  constexpr int UN = 4;
  for (int b = ex.lane; b < tot; b += UN * ex.nlanes) {
    double gv[UN], xv1[UN], xv2[UN];
    int kk[UN];
#pragma unroll
    for (int u = 0; u < UN; ++u) {
      const int f = b + u * ex.nlanes < tot ? b + u * ex.nlanes : b;
      const int j = f / full < kn ? f / full : kn - 1;
      const int e = f - j * full;
      const int i = cone_supp_idx(P, t, k0 + j, e);
      kk[u] = b + u * ex.nlanes < tot ? j : -1;
      gv[u] = g0[(size_t)(k0 + j) * gstr + i];
      xv1[u] = dx1[i];
      xv2[u] = dx2[i];
    }
#pragma unroll
    for (int u = 0; u < UN; ++u)
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        const double g = kk[u] == j ? gv[u] : 0.0;
        acc1[j] += g * xv1[u];
        acc2[j] += g * xv2[u];
      }
  }
  ex.template sum_n<16>(acc1);
  ex.template sum_n<16>(acc2);
}

// ------------------------------------------------------------------------------------
// reductions over one cone's rows, by the cone group G that owns the cone (k >= 0) or as an
// idle member (k < 0, q = 0): every lane of the wave must make the same calls.
// ------------------------------------------------------------------------------------
template <class X>
BMPC_HD double cone_dot(const X ex, const ConeGroups& G, const gdouble* a, const gdouble* b, int off, int q) {
  return ex.gsum(strided_partial<ConeBatch<X>::v>(G.gl, G.cg, q, [&](int i) { return a[off + i] * b[off + i]; }), G.cg);
}

// v0^2 - ||v1||^2 without squaring the dominant entry (see oracle.ecos_ipm.cone_res)
template <class X>
BMPC_HD double cone_res(const X ex, const ConeGroups& G, const gdouble* v, int off, int q) {
  // a lane's largest |v_i| (first index on ties) over batches of 8 loads in flight together
  constexpr int UN = 8;
  double amax = 0.0, aidx = 1e300;
  for (int b = 1 + G.gl; b < q; b += UN * G.cg) {
    double a[UN];
#pragma unroll
    for (int u = 0; u < UN; ++u) {
      const int i = b + u * G.cg;
      a[u] = fabs(v[off + (i < q ? i : b)]);
    }
#pragma unroll
    for (int u = 0; u < UN; ++u) {
      const int i = b + u * G.cg;
      const bool take = i < q && a[u] > amax;
      amax = take ? a[u] : amax;
      aidx = take ? (double)i : aidx;
    }
  }
  const double gm = ex.gmax(amax, G.cg);
  const double kd = ex.gmin(amax == gm && aidx < 1e300 ? aidx : 1e300, G.cg);
  const int kidx = kd < 1e300 ? (int)kd : -1;
  const double ss = ex.gsum(strided_partial<ConeBatch<X>::v>(1 + G.gl, G.cg, q, [&](int i) {
    const double t = v[off + i];
    return (i == kidx ? 0.0 : 1.0) * (t * t);
  }), G.cg);
  return q > 0 ? cone_res_parts(v[off], gm, ss) : 1.0;
}

// ------------------------------------------------------------------------------------
// structured operators
// ------------------------------------------------------------------------------------
// x-coefficients of LP row c of state node k: c = 0 -> -dh_k, c >= 1 -> Fx[c-1]
template <class X>
BMPC_HD double fx_coef(const Ctx& C, const X& ex, int k, int c, int j) {
  CPlan& P = *C.P;
  if (c == 0) return -C.ws[C.L->dh + k * P.n + j];
  return fxv(P, ex, c - 1, j);
}

template <class X>
BMPC_HD void apply_W(const X ex, const Ctx& C, int mode, const gdouble* in, gdouble* out, double sw = 1.0,
                     const gdouble* add = nullptr, double sa = 0.0);

// Fused cone passes: a chain of whole-vector passes whose intermediate vectors were written
// to the slab and read straight back becomes one pass that keeps each cone's rows in
// registers (lane gl of the cone's group owns rows gl + uu*cg, uu < X::kConeRegRows).
// Plans whose largest cone does not fit (P.maxq > kConeRegRows * cg) run the unfused chain.
template <class X>
BMPC_HD bool cone_regs(const X& ex, CPlan& P) {
  return P.maxq <= X::kConeRegRows * exec_cgrp(ex, P.cgrp, P.ncones);
}

// y = sc (2 a (a'v) - J v) over one cone's register rows (rows past q hold a = v = 0);
// v0 = row 0 of v, known on every lane of the group
template <int UC, class X>
BMPC_HD void cone_W_regs(const X& ex, const ConeGroups& G, const double (&a)[UC], const double (&v)[UC], double v0,
                         double sc, double (&y)[UC]) {
  double part = 0.0;
#pragma unroll
  for (int uu = 0; uu < UC; ++uu) part += a[uu] * v[uu];
  const double dot = ex.gsum(part, G.cg);
#pragma unroll
  for (int uu = 0; uu < UC; ++uu) {
    const int i = G.gl + uu * G.cg;
    y[uu] = sc * (2.0 * a[uu] * dot - (i == 0 ? v0 : -v[uu]));
  }
}

// the NT vector of a cone in register rows: v (W, W^2 use v / wbar) or J v (inverses)
template <int UC, class X>
BMPC_HD void cone_a_regs(const ConeGroups& G, const gdouble* a, bool jconj, int off, int q, double (&av)[UC]) {
#pragma unroll
  for (int uu = 0; uu < UC; ++uu) {   // masked by arithmetic (a select on t would branch around its load)
    const int i = G.gl + uu * G.cg;
    const double t = a[off + (i < q ? i : 0)];
    av[uu] = (i < q ? ((jconj && i > 0) ? -1.0 : 1.0) : 0.0) * t;
  }
}

// row 0 of a register-held cone vector, broadcast to the group (lane gl = 0 owns it)
template <int UC, class X>
BMPC_HD double cone_row0(const X& ex, const ConeGroups& G, const double (&v)[UC]) {
  return ex.gsum(G.gl == 0 ? v[0] : 0.0, G.cg);
}

// out(rows) = G zv, cone rows boosted.  WM = 1: out = W^-1 (G zv) - r3h, WM = 2: out =
// W^-1 (W^-1 (G zv) - r3h), WM = 3: out = W^-1 (G zv) -- the tail of kkt_solve_once without the
// G dx vector in the slab (tr: scratch of the unfused chain).
//
// Executors with kInlineG (the one-wave kernels) take it inline: its callers already hold the
// registers an out-of-line apply_G saves and restores on every call (-3% bytes, -1% k_ipm at
// 4,096 egos, profiles/r04/r04y_inline_apply_g_*.log); the multi-wave kernel calls it out of line
// (one-ego latency +2-3% inline).
template <class X, class = void>
struct inline_g { static constexpr bool value = false; };
template <class X>
struct inline_g<X, decltype((void)X::kInlineG)> { static constexpr bool value = X::kInlineG; };
template <class X, int NX, int NU, int WM = 0>
BMPC_HD void apply_G(const X ex, const Ctx& C, const gdouble* zv, gdouble* out, const gdouble* r3h = nullptr,
                     gdouble* tr = nullptr);
template <class X, int NX, int NU, int WM>
BMPC_HD void apply_G_body(const X ex, const Ctx Cin, const gdouble* zv, gdouble* out, const gdouble* r3h,
                          gdouble* tr) {
  const Ctx C = Cin.uniform();
  CPlan& P = *C.P;
  if constexpr (WM > 0) {
    r3h = uniform_ptr(r3h);
    if (!cone_regs(ex, P)) {
      apply_G<X, NX, NU, 0>(ex, C, zv, tr);
      if (WM == 3) apply_W(ex, C, 1, tr, out);
      else apply_W(ex, C, 1, tr, out, 1.0, r3h, -1.0);
      if (WM == 2) apply_W(ex, C, 1, out, out);
      return;
    }
  }
  constexpr int UC = X::kConeRegRows;
  double qx[NX];
  ctx_qx<NX>(C, qx);
  BMPC_PROF(C.ws, *C.L, PROF_APPLYG);
  BMPC_COUNT(C.ws, *C.L, PROF_NAPPLYG);
  BMPC_TIC(t_glp);
  const auto t = topo_view(P, ex);
  const int Nc = P.Nc;
  const gdouble* dh = C.at(C.L->dh);
  const gdouble* dli = C.at(C.L->dli);
  // LP rows: W^-1 = diag(1/d)
  auto lp = [&](int row, double g) {
    if constexpr (WM == 0) {
      return g;
    } else {
      const double w = dli[row];
      if (WM == 3) return w * g;
      const double h = w * g - r3h[row];
      return WM == 2 ? w * h : h;
    }
  };
  // Fx rows + positivity rows
  struct Two { double a, b; };
  // branch-free bodies: every load of a batch is issued before the first wait (a branch on
  // a loaded topology index would serialise the batch into one round trip per element)
  lane_batch<4>(ex, 0, P.T * Nc, [&](int it) {
    const int k = it / Nc, c = it % Nc;
    const double S = zv[P.oS + it];
    const double on = t.x_u[k] >= 0 ? 1.0 : 0.0;
    const int cr = c > 0 ? c - 1 : 0;
    const double m0 = c == 0 ? 1.0 : 0.0;
    double v = -S;
#pragma unroll
    for (int j = 0; j < NX; ++j) {
      const double fd = dh[k * NX + j], fx = fxv(P, ex, cr, j);
      v += (on * (m0 * (-fd) + (1.0 - m0) * fx)) * zv[P.oX + k * NX + j];   // -fd for c == 0, fx otherwise (exact)
    }
    return Two{lp(P.rFx + it, v), lp(P.rPos + it, -S)};
  }, [&](int it, Two r) { out[P.rFx + it] = r.a; out[P.rPos + it] = r.b; });
  // Fu rows
  lane_batch(ex, 0, P.U * P.nFu, [&](int it) {
    const int u = it / P.nFu, r = it % P.nFu;
    double v = 0.0;
#pragma unroll
    for (int j = 0; j < NU; ++j) v += fuv(P, ex, r, j) * zv[P.oU + u * NU + j];
    return lp(P.rFu + it, v);
  }, [&](int it, double v) { out[P.rFu + it] = v; });
  // risk rows: -rho, -mu+, -mu-
  lane_batch(ex, 0, P.bdim * (2 * P.m + 1), [&](int it) {
    return lp(P.rRisk + it, it < P.bdim ? -zv[P.oRho + it] : -zv[P.oMup + (it - P.bdim)]);
  }, [&](int it, double v) { out[P.rRisk + it] = v; });
  const gdouble* boost = C.at(C.L->boost);
  const gdouble* vn = C.at(C.L->vnt);
  const gdouble* eta = C.at(C.L->eta);
  const double Qs = P.desc.Qslack[1];
  BMPC_TOC(C.ws, *C.L, PROF_G_LP, t_glp);
  BMPC_TIC(t_gcone);
  BMPC_CONE_ROUNDS(ex, P, G) {
    BMPC_CONE_K(P, G, k, off, q);
    // topology of the cone, loaded together (clamped indices, no branch on loaded values)
    const int kk = k >= 0 ? k : 0;
    const int c = k >= 0 ? t.cone_c[kk] : -1;
    const int cb = t.cone_b[kk], ci = t.cone_i[kk];
    const double ebst = ebeta<X>(boost, P.ncones, kk);
    const int c0 = c >= 0 ? c : 0;
    const int ndx = t.br_ndx[c0], ndu = t.br_ndu[c0];
    const bool hasch = t.br_child0[c0] >= 0;
    // first/last rows: +-e^-beta (F1 . zv), F1 spread over the group's lanes by node
    double f;
    {
      // the root cone (c < 0) holds the root node's slacks only (ndx = br_ndx[0] = 0)
      const int nn = c >= 0 ? P.N : (k >= 0 ? 1 : 0);
      const double xon = c >= 0 ? -2.0 : 0.0;
      const int Nc = P.Nc;
      // branch-free: a node's x and slack loads are issued together (the slack loop runs to the
      // compile-time bound with clamped indices; rows past Nc are multiplied by 0)
      double part = strided_partial<2>(G.gl, G.cg, nn, [&](int j) {
        const int xb = P.oX + (ndx + j) * NX, sb = P.oS + (ndx + j) * Nc;
        double xs[NX], ss[BMPC_MAX_FX + 1];
#pragma unroll
        for (int r2 = 0; r2 < NX; ++r2) xs[r2] = zv[xb + r2];
#pragma unroll
        for (int cc = 0; cc <= BMPC_MAX_FX; ++cc) ss[cc] = zv[sb + (cc < Nc ? cc : 0)];
        double a = 0.0;
#pragma unroll
        for (int r2 = 0; r2 < NX; ++r2) a += xon * qx[r2] * xs[r2];
#pragma unroll
        for (int cc = 0; cc <= BMPC_MAX_FX; ++cc) a += (cc < Nc ? Qs : 0.0) * ss[cc];
        return a;
      });
      // risk-variable terms, loaded before the reduction and added after it
      double tail = 0.0;
      if (k >= 0 && G.gl == 0) {
        if (c >= 0) {
          tail = zv[P.oSig + cb] + zv[P.oMup + cb + ci] - zv[P.oMum + cb + ci];
        } else {
          tail = -zv[P.oJ] + zv[P.oRho + 0];
        }
      }
      const double rho_c = (k >= 0 && G.gl == 0 && c >= 0 && hasch) ? zv[P.oRho + c] : 0.0;
      double acc = ex.gsum(part, G.cg);
      acc += tail;
      if (c >= 0 && hasch) acc += rho_c;
      f = acc * ebst;   // exact on the group's lane 0
    }
    // middle rows: rows are contiguous after each cone's first: N x-rows blocks (-2 W1 x_j),
    // then N (root cone: 1) u-row blocks (-2 Wu u_j).  Branch-free: every row loads NX
    // entries from its node's block (u rows read past their NU entries into valid slab memory
    // and weight them 0), and the weight row comes from register copies of W1 / Wu, so all
    // loads of a batch of rows are in flight together.
    const int nxn = c >= 0 ? P.N * NX : 0;
    const int nmid = k < 0 ? 0 : c >= 0 ? P.N * (NX + NU) : NU;
    // the weight rows come from LDS (a lane-varying row index into registers would become an
    // indexed private array, i.e. scratch memory): W1 S of this ego or the plan's W1, and Wu
    const ldouble* W1l = X::kTransform ? ex.eco + ECO_W1 : ex.lds + P.lds_w;
    const ldouble* Wul = ex.lds + P.lds_wu;
    auto mid_base = [&](int it) {
      const bool isx = it < nxn;
      const int iu = isx ? 0 : it - nxn;
      return isx ? P.oX + (ndx + it / NX) * NX : P.oU + (c >= 0 ? ndu + iu / NU : 0) * NU;
    };
    auto mid_val = [&](int it, const double (&zs)[NX]) {
      const bool isx = it < nxn;
      const int r = isx ? it % NX : (it - nxn) % NU;
      const int rx = isx ? r : 0, ru = isx ? 0 : r;
      double vx = 0.0, vu = 0.0;
#pragma unroll
      for (int s2 = 0; s2 < NX; ++s2) vx += -2.0 * W1l[rx * NX + s2] * zs[s2];
#pragma unroll
      for (int s2 = 0; s2 < NU; ++s2) vu += -2.0 * Wul[ru * NU + s2] * zs[s2];
      return isx ? vx : vu;
    };
    auto mid = [&](int it) {
      const int b = mid_base(it);
      double zs[NX];
#pragma unroll
      for (int s2 = 0; s2 < NX; ++s2) zs[s2] = zv[b + s2];
      return mid_val(it, zs);
    };
    if constexpr (WM == 0) {
      if (k >= 0 && G.gl == 0) {
        out[off] = f;
        out[off + q - 1] = -f;
      }
      strided_batch<ConeBatch<X>::v>(G.gl, G.cg, nmid, mid, [&](int it, double v) { out[off + 1 + it] = v; });
    } else {
      // the cone's rows of G zv in registers (q = nmid + 2), then W^-1 (and again for WM = 2)
      const double f0 = ex.gsum(G.gl == 0 ? f : 0.0, G.cg);
      double v[UC], a[UC], y[UC];
      // the rows' loads in two batches of UC/2 rows (all of a batch in flight together)
#pragma unroll
      for (int h = 0; h < UC; h += UC / 2) {
        double zs[UC / 2][NX];
#pragma unroll
        for (int u2 = 0; u2 < UC / 2; ++u2) {
          const int i = G.gl + (h + u2) * G.cg;
          const int b = mid_base(i >= 1 && i <= nmid ? i - 1 : 0);
#pragma unroll
          for (int s2 = 0; s2 < NX; ++s2) zs[u2][s2] = zv[b + s2];
        }
#pragma unroll
        for (int u2 = 0; u2 < UC / 2; ++u2) {
          const int i = G.gl + (h + u2) * G.cg;
          const double m = mid_val(i >= 1 && i <= nmid ? i - 1 : 0, zs[u2]);
          v[h + u2] = i >= q ? 0.0 : i == 0 ? f0 : i == q - 1 ? -f0 : m;
        }
      }
      cone_a_regs<UC, X>(G, vn, true, off, q, a);
      const double sc = 1.0 / (k >= 0 ? eta[kk] : 1.0);
      cone_W_regs<UC>(ex, G, a, v, f0, sc, y);
#pragma unroll
      for (int uu = 0; uu < UC; ++uu) {
        const int i = G.gl + uu * G.cg;
        if (WM != 3) y[uu] = (i < q ? 1.0 : 0.0) * (y[uu] - r3h[off + (i < q ? i : 0)]);
      }
      if constexpr (WM == 2) {
        const double y0 = cone_row0<UC>(ex, G, y);
        cone_W_regs<UC>(ex, G, a, y, y0, sc, v);
#pragma unroll
        for (int uu = 0; uu < UC; ++uu) {
          const int i = G.gl + uu * G.cg;
          if (i < q) out[off + i] = v[uu];
        }
      } else {
#pragma unroll
        for (int uu = 0; uu < UC; ++uu) {
          const int i = G.gl + uu * G.cg;
          if (i < q) out[off + i] = y[uu];
        }
      }
    }
  }
  BMPC_TOC(C.ws, *C.L, PROF_G_CONE, t_gcone);
  ex.sync();
}
template <class X, int NX, int NU, int WM>
BMPC_FN_APPLY_G void apply_G_call(const X ex, const Ctx Cin, const gdouble* zv, gdouble* out, const gdouble* r3h,
                                  gdouble* tr) {
  apply_G_body<X, NX, NU, WM>(ex, Cin, zv, out, r3h, tr);
}
template <class X, int NX, int NU, int WM>
BMPC_HD void apply_G(const X ex, const Ctx& C, const gdouble* zv, gdouble* out, const gdouble* r3h, gdouble* tr) {
  if constexpr (inline_g<X>::value) apply_G_body<X, NX, NU, WM>(ex, C, zv, out, r3h, tr);
  else apply_G_call<X, NX, NU, WM>(ex, C, zv, out, r3h, tr);
}

// out(nv) = G' r (+ add, when add is not NULL)
template <class X, int NX, int NU>
BMPC_FN_APPLY_GT void apply_GT(const X ex, const Ctx Cin, const gdouble* r, gdouble* out, const gdouble* add = nullptr) {
  const Ctx C = Cin.uniform();
  add = uniform_ptr(add);
  const double sa = add ? 1.0 : 0.0;
  const gdouble* ad = add ? add : r;   // read and scaled by 0 without an addend
  double qx[NX];
  ctx_qx<NX>(C, qx);
  CPlan& P = *C.P;
  BMPC_PROF(C.ws, *C.L, PROF_APPLYGT);
  const auto t = topo_view(P, ex);
  const int Nc = P.Nc;
  const gdouble* boost = C.at(C.L->boost);
  const gdouble* dh = C.at(C.L->dh);
  const double Qs = P.desc.Qslack[1];
  // state nodes: x and S parts (all loads of a node first, stores after)
  for (int k = ex.lane; k < P.T; k += ex.nlanes) {
    double ax[NX], cx[NX], os[BMPC_MAX_FX + 1];
#pragma unroll
    for (int j = 0; j < NX; ++j) ax[j] = 0.0, cx[j] = 0.0;
    const bool term = t.x_u[k] < 0;
    double fS = 0.0;
    const int kc = t.x_cone[k];
    if (kc >= 0) {
      const int off = t.cone_off[kc], q = t.cone_q[kc], j = t.x_conepos[k];
      const double f = (r[off] - r[off + q - 1]) * ebeta<X>(boost, P.ncones, kc);
#pragma unroll
      for (int s2 = 0; s2 < NX; ++s2) {
        double v = 0.0;
#pragma unroll
        for (int rr = 0; rr < NX; ++rr) v += -2.0 * w1v(P, ex, rr, s2) * r[off + 1 + j * NX + rr];
        cx[s2] = v - 2.0 * qx[s2] * f;
      }
      fS = Qs * f;
    } else if (k == 0) {  // root slack in the root cone
      const int kr = P.ncones - 1;
      const int off = t.cone_off[kr], q = t.cone_q[kr];
      fS = Qs * (r[off] - r[off + q - 1]) * ebeta<X>(boost, P.ncones, kr);
    }
    double dhk[NX];
#pragma unroll
    for (int j = 0; j < NX; ++j) dhk[j] = dh[k * NX + j];
    for (int c = 0; c < Nc; ++c) {
      const double rv = r[P.rFx + k * Nc + c];
      if (!term)
#pragma unroll
        for (int j = 0; j < NX; ++j) ax[j] += (c == 0 ? -dhk[j] : fxv(P, ex, c - 1, j)) * rv;
      os[c] = -rv - r[P.rPos + k * Nc + c] + fS;
    }
    for (int c = 0; c < Nc; ++c) out[P.oS + k * Nc + c] = os[c] + sa * ad[P.oS + k * Nc + c];
#pragma unroll
    for (int j = 0; j < NX; ++j) out[P.oX + k * NX + j] = (kc >= 0 ? ax[j] + cx[j] : ax[j]) + sa * ad[P.oX + k * NX + j];
  }
  // input nodes
  for (int u = ex.lane; u < P.U; u += ex.nlanes) {
    double au[NU];
#pragma unroll
    for (int j = 0; j < NU; ++j) au[j] = 0.0;
    for (int rr = 0; rr < P.nFu; ++rr) {
      const double rv = r[P.rFu + u * P.nFu + rr];
#pragma unroll
      for (int j = 0; j < NU; ++j) au[j] += P.desc.Fu[rr * NU + j] * rv;
    }
    const int kc = t.u_cone[u];
    if (kc >= 0) {
      const int off = t.cone_off[kc];
      const int c = t.cone_c[kc];
      const int base = c >= 0 ? 1 + P.N * NX + (u - t.br_ndu[c]) * NU : 1;
#pragma unroll
      for (int s2 = 0; s2 < NU; ++s2) {
        double v = 0.0;
#pragma unroll
        for (int rr = 0; rr < NU; ++rr) v += -2.0 * P.Wu[rr * NU + s2] * r[off + base + rr];
        au[s2] += v;
      }
    }
#pragma unroll
    for (int j = 0; j < NU; ++j) out[P.oU + u * NU + j] = au[j] + sa * ad[P.oU + u * NU + j];
  }
  // globals: one lane per global variable, gathering its cone and risk-row terms
  for (int i = ex.lane; i < P.ng; i += ex.nlanes) {
    double v = 0.0;
    const int gi = i == P.ng - 1 ? P.oJ : P.oRho + i;
    if (gi < P.oSig) v = -r[P.rRisk + (gi - P.oRho)];                     // rho
    else if (gi >= P.oMup && gi < P.oS) v = -r[P.rRisk + P.bdim + (gi - P.oMup)];   // mu+, mu-
    for (int k = 0; k < P.ncones; ++k) {
      const int off = t.cone_off[k], q = t.cone_q[k], c = t.cone_c[k];
      double w = 0.0;
      if (c >= 0) {
        const int b = t.cone_b[k], ii = t.cone_i[k];
        if (gi == P.oSig + b) w += 1.0;
        if (gi == P.oMup + b + ii) w += 1.0;
        if (gi == P.oMum + b + ii) w -= 1.0;
        if (t.br_child0[c] >= 0 && gi == P.oRho + c) w += 1.0;
      } else {
        if (gi == P.oJ) w -= 1.0;
        if (gi == P.oRho) w += 1.0;
      }
      if (w != 0.0) v += w * (r[off] - r[off + q - 1]) * ebeta<X>(boost, P.ncones, k);
    }
    out[gi] = v + sa * ad[gi];
  }
  ex.sync();
}

// out(neq) = A zv
template <class X, int NX, int NU>
BMPC_HD void apply_A(const X ex, const Ctx& C, const gdouble* zv, gdouble* out) {
  CPlan& P = *C.P;
  const auto t = topo_view(P, ex);
  const gdouble* Ad = C.at(C.L->Ad);
  const gdouble* Bd = C.at(C.L->Bd);
  struct V4 { double v[NX]; };
  lane_batch<2>(ex, 0, P.T, [&](int k) {
    const int su = t.x_srcu[k], sx = t.x_srcx[k];
    V4 o;
#pragma unroll
    for (int r = 0; r < NX; ++r) o.v[r] = zv[P.oX + k * NX + r];
    if (su >= 0) {
      double xs[NX], us[NU];
#pragma unroll
      for (int s2 = 0; s2 < NX; ++s2) xs[s2] = zv[P.oX + sx * NX + s2];
#pragma unroll
      for (int s2 = 0; s2 < NU; ++s2) us[s2] = zv[P.oU + su * NU + s2];
#pragma unroll
      for (int r = 0; r < NX; ++r) {
#pragma unroll
        for (int s2 = 0; s2 < NX; ++s2) o.v[r] -= Ad[su * NX * NX + r * NX + s2] * xs[s2];
#pragma unroll
        for (int s2 = 0; s2 < NU; ++s2) o.v[r] -= Bd[su * NX * NU + r * NU + s2] * us[s2];
      }
    }
    return o;
  }, [&](int k, const V4& o) {
#pragma unroll
    for (int r = 0; r < NX; ++r) out[k * NX + r] = o.v[r];
  });
  const gdouble* p = C.at(C.L->p);
  for (int b = ex.lane; b < P.bdim; b += ex.nlanes) {
    double v = zv[P.oRho + b] + zv[P.oSig + b];
    for (int i = 0; i < P.m; ++i) v -= p[b * P.m + i] / P.desc.ralpha * zv[P.oMum + b * P.m + i];
    out[P.T * NX + b] = v;
  }
  ex.sync();
}

// out(nv) = A' y
template <class X, int NX, int NU>
BMPC_HD void apply_AT(const X ex, const Ctx& C, const gdouble* y, gdouble* out) {
  CPlan& P = *C.P;
  const auto t = topo_view(P, ex);
  const gdouble* Ad = C.at(C.L->Ad);
  const gdouble* Bd = C.at(C.L->Bd);
  for (int k = ex.lane; k < P.T; k += ex.nlanes) {
    double ax[NX], au[NU];
#pragma unroll
    for (int r = 0; r < NX; ++r) ax[r] = y[k * NX + r];
#pragma unroll
    for (int r = 0; r < NU; ++r) au[r] = 0.0;
    const int u = t.x_u[k];
    if (u >= 0) {
      double ys[NX];
#pragma unroll
      for (int r = 0; r < NX; ++r) ys[r] = 0.0;
      for (int e = t.succ_off[k]; e < t.succ_off[k + 1]; ++e) {
        const int c = t.succ[e];
#pragma unroll
        for (int r = 0; r < NX; ++r) ys[r] += y[c * NX + r];
      }
#pragma unroll
      for (int s2 = 0; s2 < NX; ++s2) {
        double v = 0.0;
#pragma unroll
        for (int r = 0; r < NX; ++r) v += Ad[u * NX * NX + r * NX + s2] * ys[r];
        ax[s2] -= v;
      }
#pragma unroll
      for (int s2 = 0; s2 < NU; ++s2) {
        double v = 0.0;
#pragma unroll
        for (int r = 0; r < NX; ++r) v += Bd[u * NX * NU + r * NU + s2] * ys[r];
        au[s2] -= v;
      }
#pragma unroll
      for (int s2 = 0; s2 < NU; ++s2) out[P.oU + u * NU + s2] = au[s2];
    }
#pragma unroll
    for (int r = 0; r < NX; ++r) out[P.oX + k * NX + r] = ax[r];
  }
  lane_batch(ex, P.oS, P.oJ, [&](int) { return 0.0; }, [&](int i, double v) { out[i] = v; });
  const gdouble* p = C.at(C.L->p);
  for (int i = ex.lane; i < P.ng; i += ex.nlanes) {
    const int gi = i == P.ng - 1 ? P.oJ : P.oRho + i;
    double v = 0.0;
    if (gi < P.oSig) v = y[P.T * NX + (gi - P.oRho)];
    else if (gi < P.oMup) v = y[P.T * NX + (gi - P.oSig)];
    else if (gi >= P.oMum && gi < P.oS) {
      const int j = gi - P.oMum, b = j / P.m, ii = j % P.m;
      v = -p[b * P.m + ii] / P.desc.ralpha * y[P.T * NX + b];
    }
    out[gi] = v;
  }
  ex.sync();
}

// h (rows) and b (eq) of this solve
template <class X, int NX, int NU>
BMPC_HD void build_hb(const X ex, const Ctx& C, gdouble* h, gdouble* bv) {
  CPlan& P = *C.P;
  const auto t = topo_view(P, ex);
  const int Nc = P.Nc;
  const gdouble* h0 = C.at(C.L->h0);
  for (int it = ex.lane; it < P.T * Nc; it += ex.nlanes) {
    const int k = it / Nc, c = it % Nc;
    double v = 0.0;
    if (t.x_u[k] >= 0) v = c == 0 ? h0[k] : bxv(P, ex, c - 1);
    h[P.rFx + it] = v;
    h[P.rPos + it] = 0.0;
  }
  for (int it = ex.lane; it < P.U * P.nFu; it += ex.nlanes) h[P.rFu + it] = P.desc.bu[it % P.nFu];
  for (int it = ex.lane; it < P.bdim * (2 * P.m + 1); it += ex.nlanes) h[P.rRisk + it] = 0.0;
  const gdouble* boost = C.at(C.L->boost);
  for (int k = 0; k < P.ncones; ++k) {
    const int off = t.cone_off[k], q = t.cone_q[k];
    for (int i = ex.lane; i < q; i += ex.nlanes) h[off + i] = 0.0;
  }
  ex.sync();
  for (int k = ex.lane; k < P.ncones; k += ex.nlanes) {
    const int off = t.cone_off[k], q = t.cone_q[k];
    const double a = t.cone_c[k] >= 0 ? C.ws[C.L->misc + MISC_JCONS] * P.N : 0.0;
    const double h0v = 1.0 - a, hlv = 1.0 + a;
    const double ch = cosh(boost[k]), sh = sinh(boost[k]);
    h[off] = ch * h0v + sh * hlv;
    h[off + q - 1] = sh * h0v + ch * hlv;
  }
  const gdouble* Cd = C.at(C.L->Cd);
  const gdouble* xbar = C.at(C.L->xbar);
  for (int k = ex.lane; k < P.T; k += ex.nlanes) {
    const int su = t.x_srcu[k];
    for (int r = 0; r < NX; ++r) bv[k * NX + r] = su >= 0 ? Cd[su * NX + r] : xbar[r];
  }
  for (int b = ex.lane; b < P.bdim; b += ex.nlanes) bv[P.T * NX + b] = 0.0;
  ex.sync();
}

// ------------------------------------------------------------------------------------
// Nesterov-Todd scaling and the cone algebra (ECOS; oracle/ecos_ipm.py)
// ------------------------------------------------------------------------------------
// returns false when an iterate left its cone
template <class X>
BMPC_FN_SCALING bool compute_scaling(const X ex, const Ctx Cin, const gdouble* s, const gdouble* z) {
  const Ctx C = Cin.uniform();
  BMPC_PROF(C.ws, *C.L, PROF_SCALING);
  CPlan& P = *C.P;
  gdouble* dl = C.at(C.L->dl);
  gdouble* lam = C.at(C.L->lam);
  gdouble* eta = C.at(C.L->eta);
  gdouble* wb = C.at(C.L->wbar);
  gdouble* vn = C.at(C.L->vnt);
  struct DL { double d, l; };
  double bad = lane_extreme<8, 1>(ex, 0, P.nlp, [&](int i) {
    const double si = s[i], zi = z[i];   // both loaded: no short-circuit branch around z's load
    return ((si > 0.0) & (zi > 0.0)) ? 0.0 : 1.0;
  });
  gdouble* dli = C.at(C.L->dli);
  struct DLI { double d, di, l; };
  lane_batch(ex, 0, P.nlp, [&](int i) {
    const double d = sqrt(s[i] / z[i]);
    return DLI{d, 1.0 / d, sqrt(s[i] * z[i])};
  }, [&](int i, DLI v) { dl[i] = v.d; dli[i] = v.di; lam[i] = v.l; });
  BMPC_CONE_ROUNDS(ex, P, G) {
    BMPC_CONE_K(P, G, k, off, q);
    const double sres = cone_res(ex, G, s, off, q);
    const double zres = cone_res(ex, G, z, off, q);
    if (!(sres > 0.0 && zres > 0.0)) bad = 1.0;
    const double sn = sqrt(sres), zn = sqrt(zres);
    const double sz = cone_dot(ex, G, s, z, off, q) / (sn * zn);
    const double gam = sqrt((1.0 + sz) / 2.0);
    // wbar = (s/sn + J z/zn) / (2 gam);  v = (wbar + e0) / sqrt(2 (wbar0 + 1))
    const double w0 = q > 0 ? (s[off] / sn + z[off] / zn) / (2.0 * gam) : 0.0;
    const double nrm = sqrt(2.0 * (w0 + 1.0));
    const double e = sqrt(sn / zn);
    // v'z without storing v first: v_i = (wbar_i + [i==0]) / nrm
    const double vz = ex.gsum(strided_partial<ConeBatch<X>::v>(G.gl, G.cg, q, [&](int i) {
      const double zi = z[off + i];
      const double jz = i == 0 ? zi : -zi;
      const double w = (s[off + i] / sn + jz / zn) / (2.0 * gam);
      return (w + (i == 0 ? 1.0 : 0.0)) / nrm * z[off + i];
    }), G.cg);
    struct WV { double w, v, l; };
    strided_batch<ConeBatch<X>::v>(G.gl, G.cg, q, [&](int i) {
      const double zi = z[off + i];
      const double jz = i == 0 ? zi : -zi;
      const double w = (s[off + i] / sn + jz / zn) / (2.0 * gam);
      const double v = (w + (i == 0 ? 1.0 : 0.0)) / nrm;
      return WV{w, v, e * (2.0 * v * vz - jz)};
    }, [&](int i, WV r) { wb[off + i] = r.w; vn[off + i] = r.v; lam[off + i] = r.l; });
    if (k >= 0 && G.gl == 0) eta[k] = e;
  }
  bad = ex.max(bad);
  ex.sync();
  return bad == 0.0;
}

// identity scaling for the initial point: W = I of ECOS's equilibrated variables, i.e. W = diag(ge)
// here (LP rows d = ge; a cone's eta = its ge, wbar = v = e0); ge = 1 without equilibration
template <class X>
BMPC_HD void identity_scaling(const X ex, const Ctx& C) {
  CPlan& P = *C.P;
  gdouble* dl = C.at(C.L->dl);
  gdouble* wb = C.at(C.L->wbar);
  gdouble* vn = C.at(C.L->vnt);
  gdouble* dli = C.at(C.L->dli);
  const gdouble* ge = C.at(C.L->geq);
  struct DD { double d, di; };
  lane_batch(ex, 0, P.nlp, [&](int i) {
    const double g = BMPC_EQUIL ? ge[i] : 1.0;
    return DD{g, 1.0 / g};
  }, [&](int i, DD v) { dl[i] = v.d; dli[i] = v.di; });
  const int c0 = P.nlp;
  lane_batch(ex, c0, P.nrows, [&](int) { return 0.0; }, [&](int i, double v) { wb[i] = v; vn[i] = v; });
  ex.sync();
  for (int k = ex.lane; k < P.ncones; k += ex.nlanes) {
    const int off = topo_view(P, ex).cone_off[k];
    wb[off] = 1.0;
    vn[off] = 1.0;
    C.ws[C.L->eta + k] = BMPC_EQUIL ? ge[off] : 1.0;
  }
  ex.sync();
}

// out = sw * W_mode in + sa * add   (add may be NULL; in == out allowed: every output row
// depends on its own input row and its cone's dot product, read before any write)
// mode 0: W v, 1: W^-1 v, 2: W^2 v, 3: W^-2 v   (W symmetric NT scaling)
template <class X>
BMPC_HD void apply_W(const X ex, const Ctx& C, int mode, const gdouble* in, gdouble* out, double sw,
                     const gdouble* add, double sa) {
  CPlan& P = *C.P;
  BMPC_PROF(C.ws, *C.L, PROF_APPLYW);
  const gdouble* dl = C.at((mode == 0 || mode == 2) ? C.L->dl : C.L->dli);   // d or 1/d
  const gdouble* ad = add ? add : in;   // read and scaled by 0 without an addend
  if (!add) sa = 0.0;
  const bool sq = mode >= 2;
  lane_batch<16>(ex, 0, P.nlp, [&](int i) {
    const double w = dl[i];
    return sw * ((sq ? w * w : w) * in[i]) + sa * ad[i];
  }, [&](int i, double v) { out[i] = v; });
  const gdouble* eta = C.at(C.L->eta);
  // W = e (2 v v' - J); W^-1 = (2 Jv Jv' - J)/e; W^2 = e^2 (2 wb wb' - J); W^-2 = (2 Jwb Jwb' - J)/e^2
  const gdouble* a = C.at((mode == 0 || mode == 1) ? C.L->vnt : C.L->wbar);
  const bool jconj = (mode == 1 || mode == 3);
  constexpr int UC = 8;   // cone rows per lane held in registers between the two passes
  BMPC_CONE_ROUNDS(ex, P, G) {
    BMPC_CONE_K(P, G, k, off, q);
    const double e = k >= 0 ? eta[k] : 1.0;
    const double sc = sw * (mode == 0 ? e : mode == 1 ? 1.0 / e : mode == 2 ? e * e : 1.0 / (e * e));
    const double in0 = q > 0 ? in[off] : 0.0;
    if (q <= UC * G.cg) {   // one pass: the cone's rows stay in registers
      double av[UC], iv[UC];
      double part = 0.0;
#pragma unroll
      for (int uu = 0; uu < UC; ++uu) {
        const int i = G.gl + uu * G.cg;
        const int ic = off + (i < q ? i : 0);
        const double m = i < q ? 1.0 : 0.0;
        av[uu] = (jconj && i > 0 ? -m : m) * a[ic];
        iv[uu] = m * in[ic];
        part += av[uu] * iv[uu];
      }
      const double dot = ex.gsum(part, G.cg);
      double adv[UC];
#pragma unroll
      for (int uu = 0; uu < UC; ++uu) {
        const int i = G.gl + uu * G.cg;
        adv[uu] = (i < q ? 1.0 : 0.0) * ad[off + (i < q ? i : 0)];
      }
#pragma unroll
      for (int uu = 0; uu < UC; ++uu) {
        const int i = G.gl + uu * G.cg;
        if (i < q) out[off + i] = sc * (2.0 * av[uu] * dot - (i == 0 ? in0 : -iv[uu])) + sa * adv[uu];
      }
    } else {                // long cones: dot pass, then write pass
      const double dot = ex.gsum(strided_partial<ConeBatch<X>::v>(G.gl, G.cg, q, [&](int i) {
        const double ai = (jconj && i > 0) ? -a[off + i] : a[off + i];
        return ai * in[off + i];
      }), G.cg);
      strided_batch<ConeBatch<X>::v>(G.gl, G.cg, q, [&](int i) {
        const double ai = (jconj && i > 0) ? -a[off + i] : a[off + i];
        const double jv = i == 0 ? in0 : -in[off + i];
        return sc * (2.0 * ai * dot - jv) + sa * ad[off + i];
      }, [&](int i, double v) { out[off + i] = v; });
    }
  }
  ex.sync();
}

// Jordan product out = u o v
template <class X>
BMPC_HD void jprod(const X ex, const Ctx& C, const gdouble* u, const gdouble* v, gdouble* out) {
  CPlan& P = *C.P;
  lane_batch(ex, 0, P.nlp, [&](int i) { return u[i] * v[i]; }, [&](int i, double r) { out[i] = r; });
  BMPC_CONE_ROUNDS(ex, P, G) {
    BMPC_CONE_K(P, G, k, off, q);
    const double dot = cone_dot(ex, G, u, v, off, q);
    const double u0 = q > 0 ? u[off] : 0.0, v0 = q > 0 ? v[off] : 0.0;
    strided_batch<ConeBatch<X>::v>(G.gl, G.cg, q, [&](int i) {
      const double m0 = i == 0 ? 1.0 : 0.0;   // blend, not a select around the loads
      return m0 * dot + (1.0 - m0) * (u0 * v[off + i] + v0 * u[off + i]);
    }, [&](int i, double r) { out[off + i] = r; });
  }
  ex.sync();
}

// out = lam \ v  (lam o out = v)
template <class X>
BMPC_HD void jdiv(const X ex, const Ctx& C, const gdouble* lam, const gdouble* v, gdouble* out) {
  CPlan& P = *C.P;
  lane_batch(ex, 0, P.nlp, [&](int i) { return v[i] / lam[i]; }, [&](int i, double r) { out[i] = r; });
  BMPC_CONE_ROUNDS(ex, P, G) {
    BMPC_CONE_K(P, G, k, off, q);
    const double rho = cone_res(ex, G, lam, off, q);
    const double lv = ex.gsum(strided_partial<ConeBatch<X>::v>(1 + G.gl, G.cg, q, [&](int i) { return lam[off + i] * v[off + i]; }),
                              G.cg);
    const double l0 = q > 0 ? lam[off] : 1.0;
    const double x0 = q > 0 ? (l0 * v[off] - lv) / rho : 0.0;
    strided_batch<ConeBatch<X>::v>(G.gl, G.cg, q, [&](int i) {
      const double m0 = i == 0 ? 1.0 : 0.0;
      return m0 * x0 + (1.0 - m0) * ((v[off + i] - x0 * lam[off + i]) / l0);
    }, [&](int i, double r) { out[off + i] = r; });
  }
  ex.sync();
}

// largest alpha with lam + alpha d in the cone (ECOS lineSearch for one direction)
template <class X>
BMPC_FN_MAX_STEP double max_step(const X ex, const Ctx Cin, const gdouble* lam, const gdouble* d) {
  const Ctx C = Cin.uniform();
  CPlan& P = *C.P;
  // -lam / min(d, -0): the ratio where d < 0, +inf elsewhere (no branch around the division)
  double a = lane_extreme<8, 2>(ex, 0, P.nlp, [&](int i) { return -lam[i] / fmin(d[i], -0.0); });
  double bad = 0.0;
  BMPC_CONE_ROUNDS(ex, P, G) {
    BMPC_CONE_K(P, G, k, off, q);
    const double ln2 = cone_res(ex, G, lam, off, q);
    if (!(ln2 > 0.0)) bad = 1.0;
    const double ln = sqrt(ln2);
    const double ld = ex.gsum(strided_partial<ConeBatch<X>::v>(1 + G.gl, G.cg, q, [&](int i) { return lam[off + i] * d[off + i]; }),
                              G.cg);
    const double lb0 = q > 0 ? lam[off] / ln : 0.0;
    const double rho0 = q > 0 ? (lam[off] * d[off] - ld) / ln : 0.0;
    const double fac = q > 0 ? (rho0 + d[off]) / (lb0 + 1.0) : 0.0;
    const double ss = ex.gsum(strided_partial<ConeBatch<X>::v>(1 + G.gl, G.cg, q, [&](int i) {
      const double r1 = d[off + i] - fac * lam[off + i] / ln;
      return r1 * r1;
    }), G.cg);
    const double tt = sqrt(ss) - rho0;
    if (k >= 0 && tt > 0.0) a = fmin(a, ln / tt);
  }
  a = ex.min(a);
  return ex.max(bad) > 0.0 ? 0.0 : a;
}

// both step lengths of an IPM step in one pass over lam: min(max_step(lam, d1), max_step(lam, d2))
template <class X>
BMPC_FN_MAX_STEP double max_step2(const X ex, const Ctx Cin, const gdouble* lam, const gdouble* d1, const gdouble* d2) {
  const Ctx C = Cin.uniform();
  CPlan& P = *C.P;
  struct A2 { double a, b; };
  double a1 = 1e300, a2 = 1e300;
  lane_batch<8>(ex, 0, P.nlp, [&](int i) {
    const double l = lam[i], u = d1[i], v = d2[i];
    return A2{-l / fmin(u, -0.0), -l / fmin(v, -0.0)};   // +inf where the direction is >= 0
  }, [&](int, A2 r) { a1 = fmin(a1, r.a); a2 = fmin(a2, r.b); });
  double bad = 0.0;
  BMPC_CONE_ROUNDS(ex, P, G) {
    BMPC_CONE_K(P, G, k, off, q);
    const double ln2 = cone_res(ex, G, lam, off, q);
    if (!(ln2 > 0.0)) bad = 1.0;
    const double ln = sqrt(ln2);
    const double lb0 = q > 0 ? lam[off] / ln : 0.0;
    auto one = [&](const gdouble* d, double& a) {
      const double ld = ex.gsum(strided_partial<ConeBatch<X>::v>(1 + G.gl, G.cg, q, [&](int i) { return lam[off + i] * d[off + i]; }),
                                G.cg);
      const double rho0 = q > 0 ? (lam[off] * d[off] - ld) / ln : 0.0;
      const double fac = q > 0 ? (rho0 + d[off]) / (lb0 + 1.0) : 0.0;
      const double ss = ex.gsum(strided_partial<ConeBatch<X>::v>(1 + G.gl, G.cg, q, [&](int i) {
        const double r1 = d[off + i] - fac * lam[off + i] / ln;
        return r1 * r1;
      }), G.cg);
      const double tt = sqrt(ss) - rho0;
      if (k >= 0 && tt > 0.0) a = fmin(a, ln / tt);
    };
    one(d1, a1);
    one(d2, a2);
  }
  double mm[3] = {a1, a2, -bad};   // both minima and the max of bad in one reduction
  ex.template min_n<3>(mm);
  const double a = fmin(mm[0], mm[1]);
  return -mm[2] > 0.0 ? 0.0 : a;
}

// out1 = W^-1 in and out2 = W^-1 out1 in one pass (kkt_solve: r3h and the G' operand of
// kkt_solve_once)
template <class X>
BMPC_FN_FUSED void apply_Winv2(const X ex, const Ctx Cin, const gdouble* in, gdouble* out1, gdouble* out2) {
  const Ctx C = Cin.uniform();
  in = uniform_ptr(in), out1 = uniform_ptr(out1), out2 = uniform_ptr(out2);
  CPlan& P = *C.P;
  if (!cone_regs(ex, P)) {
    apply_W(ex, C, 1, in, out1);
    apply_W(ex, C, 1, out1, out2);
    return;
  }
  BMPC_PROF(C.ws, *C.L, PROF_APPLYW);
  constexpr int UC = X::kConeRegRows;
  const gdouble* dli = C.at(C.L->dli);
  struct Two { double a, b; };
  lane_batch<8>(ex, 0, P.nlp, [&](int i) {
    const double w = dli[i];
    const double a = w * in[i];
    return Two{a, w * a};
  }, [&](int i, Two v) { out1[i] = v.a; out2[i] = v.b; });
  const gdouble* vn = C.at(C.L->vnt);
  const gdouble* eta = C.at(C.L->eta);
  BMPC_CONE_ROUNDS(ex, P, G) {
    BMPC_CONE_K(P, G, k, off, q);
    double a[UC], v[UC], y[UC];
    cone_a_regs<UC, X>(G, vn, true, off, q, a);
#pragma unroll
    for (int uu = 0; uu < UC; ++uu) {
      const int i = G.gl + uu * G.cg;
      const double t = in[off + (i < q ? i : 0)];
      v[uu] = i < q ? t : 0.0;
    }
    const double v0 = q > 0 ? in[off] : 0.0;
    const double sc = 1.0 / (k >= 0 ? eta[k] : 1.0);
    cone_W_regs<UC>(ex, G, a, v, v0, sc, y);
#pragma unroll
    for (int uu = 0; uu < UC; ++uu) {
      const int i = G.gl + uu * G.cg;
      if (i < q) out1[off + i] = y[uu];
    }
    cone_W_regs<UC>(ex, G, a, y, cone_row0<UC>(ex, G, y), sc, v);
#pragma unroll
    for (int uu = 0; uu < UC; ++uu) {
      const int i = G.gl + uu * G.cg;
      if (i < q) out2[off + i] = v[uu];
    }
  }
  ex.sync();
}

// the affine step's directions in one pass: dz = z2 + t z1, rb = W dz, ds = -lam - rb
template <class X>
BMPC_FN_FUSED void affine_dirs(const X ex, const Ctx Cin, const gdouble* z2, const gdouble* z1, double t,
                               const gdouble* lam, gdouble* rb, gdouble* ds) {
  const Ctx C = Cin.uniform();
  z2 = uniform_ptr(z2), z1 = uniform_ptr(z1), lam = uniform_ptr(lam), rb = uniform_ptr(rb), ds = uniform_ptr(ds);
  CPlan& P = *C.P;
  if (!cone_regs(ex, P)) {
    gdouble* dz = C.at(C.L->dz);
    lane_batch<8>(ex, 0, P.nrows, [&](int i) { return z2[i] + t * z1[i]; }, [&](int i, double v) { dz[i] = v; });
    ex.sync();
    apply_W(ex, C, 0, dz, rb);
    lane_batch<8>(ex, 0, P.nrows, [&](int i) { return -lam[i] - rb[i]; }, [&](int i, double v) { ds[i] = v; });
    ex.sync();
    return;
  }
  BMPC_PROF(C.ws, *C.L, PROF_APPLYW);
  constexpr int UC = X::kConeRegRows;
  const gdouble* dl = C.at(C.L->dl);
  struct Two { double a, b; };
  lane_batch<8>(ex, 0, P.nlp, [&](int i) {
    const double r = dl[i] * (z2[i] + t * z1[i]);
    return Two{r, -lam[i] - r};
  }, [&](int i, Two v) { rb[i] = v.a; ds[i] = v.b; });
  const gdouble* vn = C.at(C.L->vnt);
  const gdouble* eta = C.at(C.L->eta);
  BMPC_CONE_ROUNDS(ex, P, G) {
    BMPC_CONE_K(P, G, k, off, q);
    double a[UC], v[UC], y[UC], l[UC];
    cone_a_regs<UC, X>(G, vn, false, off, q, a);
#pragma unroll
    for (int uu = 0; uu < UC; ++uu) {
      const int i = G.gl + uu * G.cg;
      const int ic = off + (i < q ? i : 0);
      const double d = z2[ic] + t * z1[ic];
      l[uu] = lam[ic];
      v[uu] = i < q ? d : 0.0;
    }
    const double v0 = q > 0 ? z2[off] + t * z1[off] : 0.0;
    const double sc = k >= 0 ? eta[k] : 1.0;
    cone_W_regs<UC>(ex, G, a, v, v0, sc, y);
#pragma unroll
    for (int uu = 0; uu < UC; ++uu) {
      const int i = G.gl + uu * G.cg;
      if (i < q) {
        rb[off + i] = y[uu];
        ds[off + i] = -l[uu] - y[uu];
      }
    }
  }
  ex.sync();
}

// the combined step's directions in one pass: z2 += t z1 (dz), rb = W dz, ds -= rb (dsW) and
// rc = W dsW (the s update)
template <class X>
BMPC_FN_FUSED void combined_dirs(const X ex, const Ctx Cin, gdouble* z2, const gdouble* z1, double t, gdouble* ds,
                                 gdouble* rb, gdouble* rc) {
  const Ctx C = Cin.uniform();
  z2 = uniform_ptr(z2), z1 = uniform_ptr(z1), ds = uniform_ptr(ds), rb = uniform_ptr(rb), rc = uniform_ptr(rc);
  CPlan& P = *C.P;
  if (!cone_regs(ex, P)) {
    lane_batch<8>(ex, 0, P.nrows, [&](int i) { return z2[i] + t * z1[i]; }, [&](int i, double v) { z2[i] = v; });
    ex.sync();
    apply_W(ex, C, 0, z2, rb);
    lane_batch<8>(ex, 0, P.nrows, [&](int i) { return ds[i] - rb[i]; }, [&](int i, double v) { ds[i] = v; });
    ex.sync();
    apply_W(ex, C, 0, ds, rc);
    return;
  }
  BMPC_PROF(C.ws, *C.L, PROF_APPLYW);
  constexpr int UC = X::kConeRegRows;
  const gdouble* dl = C.at(C.L->dl);
  struct Four { double z, r, d, c; };
  lane_batch<4>(ex, 0, P.nlp, [&](int i) {
    const double w = dl[i];
    const double z = z2[i] + t * z1[i];
    const double r = w * z;
    const double d = ds[i] - r;
    return Four{z, r, d, w * d};
  }, [&](int i, Four v) { z2[i] = v.z; rb[i] = v.r; ds[i] = v.d; rc[i] = v.c; });
  const gdouble* vn = C.at(C.L->vnt);
  const gdouble* eta = C.at(C.L->eta);
  BMPC_CONE_ROUNDS(ex, P, G) {
    BMPC_CONE_K(P, G, k, off, q);
    double a[UC], v[UC], y[UC], d[UC];
    cone_a_regs<UC, X>(G, vn, false, off, q, a);
#pragma unroll
    for (int uu = 0; uu < UC; ++uu) {
      const int i = G.gl + uu * G.cg;
      const int ic = off + (i < q ? i : 0);
      const double z = z2[ic] + t * z1[ic];
      d[uu] = ds[ic];
      v[uu] = i < q ? z : 0.0;
    }
    const double v0 = q > 0 ? z2[off] + t * z1[off] : 0.0;
    const double sc = k >= 0 ? eta[k] : 1.0;
    cone_W_regs<UC>(ex, G, a, v, v0, sc, y);
#pragma unroll
    for (int uu = 0; uu < UC; ++uu) {
      const int i = G.gl + uu * G.cg;
      d[uu] = i < q ? d[uu] - y[uu] : 0.0;
      if (i < q) {
        z2[off + i] = v[uu];
        rb[off + i] = y[uu];
        ds[off + i] = d[uu];
      }
    }
    cone_W_regs<UC>(ex, G, a, d, cone_row0<UC>(ex, G, d), sc, v);
#pragma unroll
    for (int uu = 0; uu < UC; ++uu) {
      const int i = G.gl + uu * G.cg;
      if (i < q) rc[off + i] = v[uu];
    }
  }
  ex.sync();
}

// the combined step's right-hand side in one pass (ECOS, oracle/ecos_ipm.py): with
// ds = dsW_aff and rb = W dz_aff on entry,
//   r = -lam o lam - dsW_aff o W dz_aff + smu e,  ds <- xi = lam \ r,  rb <- eta1 rz - W xi
template <class X>
BMPC_FN_FUSED void combined_rhs(const X ex, const Ctx Cin, const gdouble* lam, gdouble* ds, gdouble* rb,
                                const gdouble* rz, double smu, double eta1) {
  const Ctx C = Cin.uniform();
  lam = uniform_ptr(lam), ds = uniform_ptr(ds), rb = uniform_ptr(rb), rz = uniform_ptr(rz);
  CPlan& P = *C.P;
  if (!cone_regs(ex, P)) {
    gdouble* ra = C.at(C.L->ra);
    gdouble* rc = C.at(C.L->rc);
    jprod(ex, C, lam, lam, ra);
    jprod(ex, C, ds, rb, rc);
    lane_batch<8>(ex, 0, P.nrows, [&](int i) {
      const double v = -ra[i] - rc[i];
      return i < P.nlp ? v + smu : v;   // + sigma mu e on the LP rows
    }, [&](int i, double v) { ra[i] = v; });
    ex.sync();
    for (int k = ex.lane; k < P.ncones; k += ex.nlanes) ra[topo_view(P, ex).cone_off[k]] += smu;   // ... and cone heads
    ex.sync();
    jdiv(ex, C, lam, ra, ds);                                // xi (kept in ds)
    apply_W(ex, C, 0, ds, rb, -1.0, rz, eta1);               // eta1 rz - W xi
    return;
  }
  BMPC_PROF(C.ws, *C.L, PROF_APPLYW);
  constexpr int UC = X::kConeRegRows;
  const gdouble* dl = C.at(C.L->dl);
  struct Two { double a, b; };
  lane_batch<8>(ex, 0, P.nlp, [&](int i) {
    const double l = lam[i];
    const double xi = (-(l * l) - ds[i] * rb[i] + smu) / l;
    return Two{xi, -(dl[i] * xi) + eta1 * rz[i]};
  }, [&](int i, Two v) { ds[i] = v.a; rb[i] = v.b; });
  const gdouble* vn = C.at(C.L->vnt);
  const gdouble* eta = C.at(C.L->eta);
  BMPC_CONE_ROUNDS(ex, P, G) {
    BMPC_CONE_K(P, G, k, off, q);
    double l[UC], bw[UC], r[UC], rzv[UC];
    double pll = 0.0, pdr = 0.0;
#pragma unroll
    for (int uu = 0; uu < UC; ++uu) {   // loads unconditional, masked by arithmetic
      const int i = G.gl + uu * G.cg;
      const int ic = off + (i < q ? i : 0);
      const double m = i < q ? 1.0 : 0.0;
      const double lv = lam[ic], dv = ds[ic], bv = rb[ic];
      rzv[uu] = rz[ic];
      l[uu] = m * lv;
      bw[uu] = m * bv;
      r[uu] = m * dv;
      pll += l[uu] * l[uu];
      pdr += r[uu] * bw[uu];
    }
    const double l0 = q > 0 ? lam[off] : 1.0;
    const double d0 = q > 0 ? ds[off] : 0.0, b0 = q > 0 ? rb[off] : 0.0;
    const double dll = ex.gsum(pll, G.cg), ddr = ex.gsum(pdr, G.cg);
    // r_i = -(lam o lam)_i - (dsW o W dz)_i for i > 0 (row 0 below)
#pragma unroll
    for (int uu = 0; uu < UC; ++uu) r[uu] = -(l0 * l[uu] + l0 * l[uu]) - (d0 * bw[uu] + b0 * r[uu]);
    const double r0 = -dll - ddr + smu;
    // xi = lam \ r: rho = lam0^2 - |lam1|^2 (cone_res), x0 = (l0 r0 - lam1'r1) / rho
    double amax = 0.0, aidx = 1e300, plr = 0.0;
#pragma unroll
    for (int uu = 0; uu < UC; ++uu) {
      const int i = G.gl + uu * G.cg;
      const double a = fabs(l[uu]);
      if (i >= 1 && i < q && a > amax) amax = a, aidx = (double)i;
      if (i >= 1) plr += l[uu] * r[uu];
    }
    const double gm = ex.gmax(amax, G.cg);
    const double kd = ex.gmin(amax == gm && aidx < 1e300 ? aidx : 1e300, G.cg);
    const int kidx = kd < 1e300 ? (int)kd : -1;
    double pss = 0.0;
#pragma unroll
    for (int uu = 0; uu < UC; ++uu) {
      const int i = G.gl + uu * G.cg;
      if (i >= 1 && i != kidx) pss += l[uu] * l[uu];
    }
    const double ss = ex.gsum(pss, G.cg), lr = ex.gsum(plr, G.cg);
    const double rho = q > 0 ? cone_res_parts(l0, gm, ss) : 1.0;
    const double x0 = q > 0 ? (l0 * r0 - lr) / rho : 0.0;
    double a[UC];
    cone_a_regs<UC, X>(G, vn, false, off, q, a);
#pragma unroll
    for (int uu = 0; uu < UC; ++uu) {
      const int i = G.gl + uu * G.cg;
      r[uu] = i >= q ? 0.0 : i == 0 ? x0 : (r[uu] - x0 * l[uu]) / l0;
    }
    const double sc = -(k >= 0 ? eta[k] : 1.0);
    cone_W_regs<UC>(ex, G, a, r, x0, sc, l);
#pragma unroll
    for (int uu = 0; uu < UC; ++uu) {
      const int i = G.gl + uu * G.cg;
      if (i < q) {
        ds[off + i] = r[uu];
        rb[off + i] = l[uu] + eta1 * rzv[uu];
      }
    }
  }
  ex.sync();
}

// branches of depth dep are contiguous in BFS order: sum_{i<dep} m^i .. + m^dep
BMPC_HD int branch_count(CPlan& P, int dep) {
  int c = 1;
  for (int i = 0; i < dep; ++i) c *= P.m;
  return c;
}
BMPC_HD int branch_start(CPlan& P, int dep) {
  int s = 0, c = 1;
  for (int i = 0; i < dep; ++i) s += c, c *= P.m;
  return s;
}

// one Riccati step at a node with input: P = hx + A'Pb A - Qux' Quu^-1 Qux,
// Quu = hu + B'Pb B (its inverse stored), K = -Quu^-1 Qux (stored).  Pout receives P.
// The node's data arrive in registers (hx, hu, A, B loaded together by the caller: one memory
// round trip per node instead of one per operand).
template <int NX, int NU>
BMPC_HD bool riccati_step(const double (&Hx)[NX][NX], const double (&Hu)[NU][NU], const double (&A)[NX][NX],
                          const double (&B)[NX][NU], const double (&Pb)[NX][NX], double (&Pk)[NX][NX],
                          gdouble* Luu_out, gdouble* K_out) {
  double M[NX][NX];
  mat_copy(Hx, Pk);
#pragma unroll
  for (int i = 0; i < NX; ++i)
#pragma unroll
    for (int j = 0; j < NX; ++j) {
      double v = 0.0;
#pragma unroll
      for (int r = 0; r < NX; ++r) v += Pb[i][r] * A[r][j];
      M[i][j] = v;
    }
  double Qux[NU][NX], Quu[NU][NU];
#pragma unroll
  for (int i = 0; i < NX; ++i)
#pragma unroll
    for (int j = 0; j < NX; ++j) {
      double v = 0.0;
#pragma unroll
      for (int r = 0; r < NX; ++r) v += A[r][i] * M[r][j];
      Pk[i][j] += v;
    }
#pragma unroll
  for (int i = 0; i < NU; ++i)
#pragma unroll
    for (int j = 0; j < NX; ++j) {
      double v = 0.0;
#pragma unroll
      for (int r = 0; r < NX; ++r) v += B[r][i] * M[r][j];
      Qux[i][j] = v;
    }
  mat_copy(Hu, Quu);
#pragma unroll
  for (int i = 0; i < NU; ++i)
#pragma unroll
    for (int j = 0; j < NU; ++j) {
      double v = 0.0;
#pragma unroll
      for (int r = 0; r < NX; ++r) {
        double pb = 0.0;
#pragma unroll
        for (int c = 0; c < NX; ++c) pb += Pb[r][c] * B[c][j];
        v += B[r][i] * pb;
      }
      Quu[i][j] += v;
    }
  const bool ok = chol<NU>(Quu);
  double Qi[NU][NU];   // Quu^-1 (the tree sweeps multiply by it: no divisions on their chains)
#pragma unroll
  for (int j = 0; j < NU; ++j) {
    double col[NU];
#pragma unroll
    for (int i = 0; i < NU; ++i) col[i] = i == j ? 1.0 : 0.0;
    chol_solve<NU>(Quu, col);
#pragma unroll
    for (int i = 0; i < NU; ++i) Qi[i][j] = col[i];
  }
  mat_store(Qi, Luu_out);
  double K[NU][NX];
#pragma unroll
  for (int j = 0; j < NX; ++j) {
    double col[NU];
#pragma unroll
    for (int i = 0; i < NU; ++i) col[i] = -Qux[i][j];
    chol_solve<NU>(Quu, col);
#pragma unroll
    for (int i = 0; i < NU; ++i) K[i][j] = col[i];
  }
  mat_store(K, K_out);
#pragma unroll
  for (int i = 0; i < NX; ++i)
#pragma unroll
    for (int j = 0; j < NX; ++j) {
      double v = 0.0;
#pragma unroll
      for (int r = 0; r < NU; ++r) v += Qux[r][i] * K[r][j];
      Pk[i][j] += v;
    }
#pragma unroll
  for (int i = 0; i < NX; ++i)
#pragma unroll
    for (int j = i + 1; j < NX; ++j) {
      const double a = 0.5 * (Pk[i][j] + Pk[j][i]);
      Pk[i][j] = a;
      Pk[j][i] = a;
    }
  return ok;
}

// all NX entries of a row-distributed vector (lane gl holds rows gl*RX .. gl*RX+RX-1)
template <int NX, int RX, int W, class X, int S = 0>
BMPC_HD void task_gather(const X& ex, const double (&mine)[RX], double (&full)[NX]) {
  if constexpr (S < W) {
#pragma unroll
    for (int r = 0; r < RX; ++r)
      if (S * RX + r < NX) full[S * RX + r] = ex.template tget<S>(mine[r]);
    task_gather<NX, RX, W, X, S + 1>(ex, mine, full);
  }
}

// ------------------------------------------------------------------------------------
// KKT factorisation
// ------------------------------------------------------------------------------------
template <class X, int NX, int NU>
BMPC_FN bool kkt_factor(const X ex, const Ctx Cin, bool zero_g) {
  const Ctx C = Cin.uniform();
  double qx[NX];
  ctx_qx<NX>(C, qx);
  CPlan& P = *C.P;
  CLayout& L = *C.L;
  BMPC_PROF(C.ws, L, PROF_FACTOR);
  const auto t = topo_view(P, ex);
  const int Nc = P.Nc;
  gdouble* ws = C.ws;
  const gdouble* dl = ws + L.dl;
  const gdouble* eta = ws + L.eta;
  const gdouble* wb = ws + L.wbar;
  const gdouble* boost = ws + L.boost;
  const double Qs = P.desc.Qslack[1];
  // ---- node Hessian blocks (LP rows with slack elimination + cone F2'F2/eta^2) ----------
  for (int k = ex.lane; k < P.T; k += ex.nlanes) {
    double H[NX][NX];
    for (int i = 0; i < NX; ++i)
      for (int j = 0; j < NX; ++j) H[i][j] = 0.0;
    const bool term = t.x_u[k] < 0;
    for (int c = 0; c < Nc; ++c) {
      const double wf = dl[P.rFx + k * Nc + c], wp = dl[P.rPos + k * Nc + c];
      const double df = 1.0 / (wf * wf), dp = 1.0 / (wp * wp);
      ws[L.sd + (k * Nc + c) * 2 + 0] = df + dp;
      ws[L.sd + (k * Nc + c) * 2 + 1] = df;
      if (!term) {
        const double om = df * dp / (df + dp);
        double f[NX];
        for (int j = 0; j < NX; ++j) f[j] = fx_coef(C, ex, k, c, j);
        for (int i = 0; i < NX; ++i)
          for (int j = 0; j < NX; ++j) H[i][j] += om * f[i] * f[j];
      }
    }
    const int kc = t.x_cone[k];
    if (kc >= 0) {
      const double sc = 4.0 / (eta[kc] * eta[kc]);
      for (int i = 0; i < NX; ++i)
        for (int j = 0; j < NX; ++j) H[i][j] += sc * qqv(P, ex, i, j);
    }
    mat_store(H, ws + L.hx + k * NX * NX);
  }
  for (int u = ex.lane; u < P.U; u += ex.nlanes) {
    double H[NU][NU];
    for (int i = 0; i < NU; ++i)
      for (int j = 0; j < NU; ++j) H[i][j] = 0.0;
    for (int r = 0; r < P.nFu; ++r) {
      const double w = dl[P.rFu + u * P.nFu + r];
      const double dr = 1.0 / (w * w);
      for (int i = 0; i < NU; ++i)
        for (int j = 0; j < NU; ++j) H[i][j] += dr * P.desc.Fu[r * NU + i] * P.desc.Fu[r * NU + j];
    }
    const int kc = t.u_cone[u];
    if (kc >= 0) {
      const double sc = 4.0 / (eta[kc] * eta[kc]);
      for (int i = 0; i < NU; ++i)
        for (int j = 0; j < NU; ++j) H[i][j] += sc * P.RR[i * NU + j];
    }
    mat_store(H, ws + L.hu + u * NU * NU);
  }
  // ---- rank-1 cone vectors g_k = G_k'(J wbar) (boosted rows) ----------------------------
  // the support of each g_k is fixed by the plan: zeroed once per solve (the first
  // factorisation), afterwards only the support is rewritten
  if (zero_g) {
    for (int k = 0; k < P.ncones; ++k) {
      gdouble* g = ws + L.gk + (size_t)k * P.nv;
      for (int i = ex.lane; i < P.nv; i += ex.nlanes) g[i] = 0.0;
    }
    ex.sync();
  }
  for (int k = 0; k < P.ncones; ++k) {
    gdouble* g = ws + L.gk + (size_t)k * P.nv;
    const int off = t.cone_off[k], q = t.cone_q[k], c = t.cone_c[k];
    const double kap = (wb[off] + wb[off + q - 1]) * ebeta<X>(boost, P.ncones, k);
    if (c >= 0) {
      for (int it = ex.lane; it < P.N; it += ex.nlanes) {
        const int xk = t.br_ndx[c] + it, uk = t.br_ndu[c] + it;
        const gdouble* wx = wb + off + 1 + it * NX;
        const gdouble* wu = wb + off + 1 + P.N * NX + it * NU;
        for (int s = 0; s < NX; ++s) {
          double v = 0.0;
          for (int r = 0; r < NX; ++r) v += w1v(P, ex, r, s) * wx[r];
          g[P.oX + xk * NX + s] = kap * (-2.0 * qx[s]) + 2.0 * v;
        }
        for (int s = 0; s < NU; ++s) {
          double v = 0.0;
          for (int r = 0; r < NU; ++r) v += P.Wu[r * NU + s] * wu[r];
          g[P.oU + uk * NU + s] = 2.0 * v;
        }
        for (int cc = 0; cc < Nc; ++cc) g[P.oS + xk * Nc + cc] = kap * Qs;
      }
      if (ex.lane == 0) {
        const int b = t.cone_b[k], i = t.cone_i[k];
        g[P.oSig + b] = kap;      // one term per entry of g_k: stored, not accumulated
        g[P.oMup + b + i] = kap;
        g[P.oMum + b + i] = -kap;
        if (t.br_child0[c] >= 0) g[P.oRho + c] = kap;
      }
    } else if (ex.lane == 0) {
      g[P.oJ] = -kap;
      g[P.oRho + 0] = kap;
      for (int cc = 0; cc < Nc; ++cc) g[P.oS + cc] = kap * Qs;
      for (int s = 0; s < NU; ++s) {
        double v = 0.0;
        for (int r = 0; r < NU; ++r) v += P.Wu[r * NU + s] * wb[off + 1 + r];
        g[P.oU + s] = 2.0 * v;
      }
    }
  }
  ex.sync();
  BMPC_TIC(t_ric);
  // ---- tree Riccati factorisation (leaves -> root), one task group per branch ----------------
  // A group of W = X::kTaskLanes lanes (a DPP quad) runs a branch; lane gl owns rows
  // gl*RX .. of the node matrices, carries its rows of the cost-to-go P backward along the
  // branch, and gathers the full A, B, M = Pb A, Pb B and P rows it needs from the group by DPP
  // broadcasts -- every sum is the one riccati_step forms, term for term (bit-identical), but a
  // lane holds a quarter of the node data (one lane per branch spilled the Riccati state to
  // scratch on every node).  Only at a branch end are the children's first-node P rows read back.
  const gdouble* Ad = ws + L.Ad;
  const gdouble* Bd = ws + L.Bd;
  constexpr int W = X::kTaskLanes;
  constexpr int RX = (NX + W - 1) / W;
  const int gl = ex.lane % W, grp = ex.lane / W, ngrp = ex.nlanes / W;
  double bad = 0.0;
  // the full NX x NC matrix of row-distributed rows (lane gl: rows gl*RX + q)
  auto gather_rows = [&](const auto& mine, auto& full) {
    constexpr int NC = sizeof(full[0]) / sizeof(double);
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      double col[RX], fc[NX];
#pragma unroll
      for (int q = 0; q < RX; ++q) col[q] = mine[q][c];
      task_gather<NX, RX, W>(ex, col, fc);
#pragma unroll
      for (int r = 0; r < NX; ++r) full[r][c] = fc[r];
    }
  };
  // Lane-varying picks (row gi's column of a matrix every lane holds) are taken while the
  // values are formed, as selects between fresh values: a select chain over a register array's
  // elements would be folded into a runtime index, i.e. the array moved to scratch memory.
  for (int dep = P.NB; dep >= 0; --dep) {
    const int b0 = branch_start(P, dep), nbd = branch_count(P, dep);
    const int rounds = (nbd + ngrp - 1) / ngrp;
    for (int rd = 0; rd < rounds; ++rd) {
      const int bi = rd * ngrp + grp;
      if (bi >= nbd) continue;   // whole group idle together
      const int b = b0 + bi;
      const int ndx = t.br_ndx[b], ndu = t.br_ndu[b], len = t.br_len[b];
      const bool leaf = dep == P.NB;
      double Pn[RX][NX];   // this lane's rows of the cost-to-go after the current node
      if (leaf) {   // terminal node: P = hx
#pragma unroll
        for (int q = 0; q < RX; ++q) {
          const int i = gl * RX + q < NX ? gl * RX + q : NX - 1;
#pragma unroll
          for (int j = 0; j < NX; ++j) Pn[q][j] = ws[L.hx + (ndx + len) * NX * NX + i * NX + j];
          if (gl * RX + q < NX)
#pragma unroll
            for (int j = 0; j < NX; ++j) ws[L.P + (ndx + len) * NX * NX + i * NX + j] = Pn[q][j];
        }
      }
      for (int jn = len - 1; jn >= 0; --jn) {
        const int k = ndx + jn, u = ndu + jn;
        BMPC_TIC(t_rn);
        // this lane's rows of the node's data (independent of the recursion)
        double Hx[RX][NX], Ar[RX][NX], Ac[RX][NX], Br[RX][NU], Hu[NU][NU];
#pragma unroll
        for (int q = 0; q < RX; ++q) {
          const int i = gl * RX + q < NX ? gl * RX + q : NX - 1;
#pragma unroll
          for (int j = 0; j < NX; ++j) Hx[q][j] = ws[L.hx + k * NX * NX + i * NX + j];
#pragma unroll
          for (int j = 0; j < NX; ++j) Ar[q][j] = Ad[u * NX * NX + i * NX + j];
#pragma unroll
          for (int j = 0; j < NX; ++j) Ac[q][j] = Ad[u * NX * NX + j * NX + i];   // column i
#pragma unroll
          for (int m = 0; m < NU; ++m) Br[q][m] = Bd[u * NX * NU + i * NU + m];
        }
        mat_load(Hu, ws + L.hu + u * NU * NU);
        double Pb[RX][NX];
        if (jn < len - 1 || leaf) {
#pragma unroll
          for (int q = 0; q < RX; ++q)
#pragma unroll
            for (int c = 0; c < NX; ++c) Pb[q][c] = Pn[q][c];
        } else {
          // the children's first-node P rows (written by the previous depth phase), in the
          // order riccati_step's caller sums them (pairs, the odd one padded with weight 0)
#pragma unroll
          for (int q = 0; q < RX; ++q)
#pragma unroll
            for (int c = 0; c < NX; ++c) Pb[q][c] = 0.0;
          const int c0 = t.br_child0[b];
          for (int i0 = 0; i0 < P.m; i0 += 2) {
            double Pc[2][RX][NX];
#pragma unroll
            for (int h = 0; h < 2; ++h) {
              const int ch = i0 + h < P.m ? i0 + h : i0;
#pragma unroll
              for (int q = 0; q < RX; ++q) {
                const int i = gl * RX + q < NX ? gl * RX + q : NX - 1;
#pragma unroll
                for (int c = 0; c < NX; ++c) Pc[h][q][c] = ws[L.P + t.br_ndx[c0 + ch] * NX * NX + i * NX + c];
              }
            }
#pragma unroll
            for (int h = 0; h < 2; ++h) {
              const double w = i0 + h < P.m ? 1.0 : 0.0;
#pragma unroll
              for (int q = 0; q < RX; ++q)
#pragma unroll
                for (int c = 0; c < NX; ++c) Pb[q][c] += w * Pc[h][q][c];
            }
          }
        }
        BMPC_TOC_WAIT(C.ws, L, PROF_RIC_LD, t_rn);
        BMPC_TIC(t_ra);
        // full A and B (every lane)
        double Af[NX][NX], Bf[NX][NU];
        gather_rows(Ar, Af);
        gather_rows(Br, Bf);
        // M = Pb A (own rows), then the full M
        double Mr[RX][NX], Mf[NX][NX];
#pragma unroll
        for (int q = 0; q < RX; ++q)
#pragma unroll
          for (int j = 0; j < NX; ++j) {
            double v = 0.0;
#pragma unroll
            for (int r = 0; r < NX; ++r) v += Pb[q][r] * Af[r][j];
            Mr[q][j] = v;
          }
        gather_rows(Mr, Mf);
        // Pk = Hx + A'M (own rows)
        double Pk[RX][NX];
#pragma unroll
        for (int q = 0; q < RX; ++q)
#pragma unroll
          for (int j = 0; j < NX; ++j) {
            double v = 0.0;
#pragma unroll
            for (int r = 0; r < NX; ++r) v += Ac[q][r] * Mf[r][j];
            Pk[q][j] = Hx[q][j] + v;
          }
        // Qux = B'M and Quu = Hu + B'(Pb B) (full, every lane)
        double Qux[NU][NX], Quu[NU][NU], qc[RX][NU];   // qc: column gl*RX+q of Qux
#pragma unroll
        for (int i = 0; i < NU; ++i)
#pragma unroll
          for (int j = 0; j < NX; ++j) {
            double v = 0.0;
#pragma unroll
            for (int r = 0; r < NX; ++r) v += Bf[r][i] * Mf[r][j];
            Qux[i][j] = v;
#pragma unroll
            for (int q = 0; q < RX; ++q) qc[q][i] = (j == gl * RX + q || j == 0) ? v : qc[q][i];
          }
        double PBr[RX][NU], PBf[NX][NU];   // Pb B
#pragma unroll
        for (int q = 0; q < RX; ++q)
#pragma unroll
          for (int j = 0; j < NU; ++j) {
            double pb = 0.0;
#pragma unroll
            for (int c = 0; c < NX; ++c) pb += Pb[q][c] * Bf[c][j];
            PBr[q][j] = pb;
          }
        gather_rows(PBr, PBf);
        mat_copy(Hu, Quu);
#pragma unroll
        for (int i = 0; i < NU; ++i)
#pragma unroll
          for (int j = 0; j < NU; ++j) {
            double v = 0.0;
#pragma unroll
            for (int r = 0; r < NX; ++r) v += Bf[r][i] * PBf[r][j];
            Quu[i][j] += v;
          }
        BMPC_TOC_WAIT(C.ws, L, PROF_RIC_A, t_ra);
        BMPC_TIC(t_rb);
        if (!chol<NU>(Quu)) bad = 1.0;
        // the NU + NX column solves share the factor's diagonal: its reciprocals once (div_rcp)
        double ri[NU];
#pragma unroll
        for (int i = 0; i < NU; ++i) ri[i] = 1.0 / Quu[i][i];
        double Qi[NU][NU];   // Quu^-1 (the tree sweeps multiply by it)
#pragma unroll
        for (int j = 0; j < NU; ++j) {
          double col[NU];
#pragma unroll
          for (int i = 0; i < NU; ++i) col[i] = i == j ? 1.0 : 0.0;
          chol_solve_r<NU>(Quu, ri, col);
#pragma unroll
          for (int i = 0; i < NU; ++i) Qi[i][j] = col[i];
        }
        double K[NU][NX], kc[RX][NU];   // kc: column gl*RX+q of K
#pragma unroll
        for (int j = 0; j < NX; ++j) {
          double col[NU];
#pragma unroll
          for (int i = 0; i < NU; ++i) col[i] = -Qux[i][j];
          chol_solve_r<NU>(Quu, ri, col);
#pragma unroll
          for (int i = 0; i < NU; ++i) {
            K[i][j] = col[i];
#pragma unroll
            for (int q = 0; q < RX; ++q) kc[q][i] = (j == gl * RX + q || j == 0) ? col[i] : kc[q][i];
          }
        }
        // Pk += Qux' K (own rows), then symmetrise: P[i][j] = P[j][i] = (P[lo][hi] + P[hi][lo]) / 2
#pragma unroll
        for (int q = 0; q < RX; ++q)
#pragma unroll
          for (int j = 0; j < NX; ++j) {
            double v = 0.0;
#pragma unroll
            for (int r = 0; r < NU; ++r) v += qc[q][r] * K[r][j];
            Pk[q][j] += v;
          }
        // column gl*RX+q of the full Pk, gathered column by column
        double pcol[RX][NX];
#pragma unroll
        for (int c = 0; c < NX; ++c) {
          double cm[RX], fc[NX];
#pragma unroll
          for (int q = 0; q < RX; ++q) cm[q] = Pk[q][c];
          task_gather<NX, RX, W>(ex, cm, fc);
#pragma unroll
          for (int q = 0; q < RX; ++q)
#pragma unroll
            for (int r = 0; r < NX; ++r) pcol[q][r] = (c == gl * RX + q || c == 0) ? fc[r] : pcol[q][r];
        }
#pragma unroll
        for (int q = 0; q < RX; ++q) {
          const int i = gl * RX + q < NX ? gl * RX + q : NX - 1;
#pragma unroll
          for (int j = 0; j < NX; ++j) {
            const double pij = Pk[q][j], pji = pcol[q][j];   // own row entry, column entry
            Pn[q][j] = i == j ? pij : i < j ? 0.5 * (pij + pji) : 0.5 * (pji + pij);
          }
        }
        // stores: P rows, K columns (lane gl: entries j = gl*RX + q), Quu^-1 (lane gl 0)
#pragma unroll
        for (int q = 0; q < RX; ++q) {
          const int i = gl * RX + q;
          if (i < NX) {
#pragma unroll
            for (int j = 0; j < NX; ++j) ws[L.P + k * NX * NX + i * NX + j] = Pn[q][j];
#pragma unroll
            for (int m = 0; m < NU; ++m) ws[L.Kg + u * NU * NX + m * NX + i] = kc[q][m];
          }
        }
        if (gl == 0) mat_store(Qi, ws + L.Luu + u * NU * NU);
        BMPC_TOC_WAIT(C.ws, L, PROF_RIC_B, t_rb);
      }
    }
    ex.sync();
  }
  BMPC_TOC(C.ws, L, 23, t_ric);   // PROF_RIC
  return ex.max(bad) == 0.0;
}

// one backward Riccati-sweep node of a task: g (successor terms, own rows) -> l, kf
template <class X, int NX, int NU, int RX, int W>
BMPC_HD void bw_node(const X& ex, int gl, const double (&qx)[RX], const double (&Acol)[RX][NX],
                     const double (&Brow)[RX][NU], const double (&Kcol)[RX][NU], const double (&Lu)[NU][NU],
                     const double (&ru)[NU], double (&g)[RX], double (&l)[RX], double (&kfv)[NU]) {
#pragma unroll
  for (int q = 0; q < RX; ++q)
    if (gl * RX + q >= NX) g[q] = 0.0;
  double gfull[NX];
  task_gather<NX, RX, W>(ex, g, gfull);
  // qu = -ru + B'g ;  kf = -Quu^-1 qu ;  l = qx0 + A'g + K'qu
  double qu[NU];
#pragma unroll
  for (int m = 0; m < NU; ++m) {
    double v = 0.0;
#pragma unroll
    for (int q = 0; q < RX; ++q) v += Brow[q][m] * g[q];
    qu[m] = -ru[m] + ex.tsum(v);
  }
#pragma unroll
  for (int m = 0; m < NU; ++m) {   // kf = -Quu^-1 qu  (Lu holds Quu^-1)
    double v = 0.0;
#pragma unroll
    for (int c = 0; c < NU; ++c) v -= Lu[m][c] * qu[c];
    kfv[m] = v;
  }
#pragma unroll
  for (int q = 0; q < RX; ++q) {
    double v = qx[q];
#pragma unroll
    for (int j = 0; j < NX; ++j) v += Acol[q][j] * gfull[j];
#pragma unroll
    for (int m = 0; m < NU; ++m) v += Kcol[q][m] * qu[m];
    l[q] = v;
  }
}

// Tree solve of  [H_t A_dyn'; A_dyn 0] [v; nu] = [r; e]  for nr right-hand sides.
// rhs i: r_i = r0 + i*rs lives in z-space (x, u, S parts at P.oX/oU/oS), e_i = e0 + i*es in
// eq-space (first T*n rows; Layout::zeros with es = 0 for none).  Solutions go to
// o0 + i*os (z-space tree parts) and n0 + i*ns (eq-space multipliers; n0 = NULL skips).
// Every vector lives in the ego's slab.
// Structure: the two sequential sweeps, one task per (branch, rhs) run by a group of
// W = X::kTaskLanes lanes (a DPP quad on the GPU; lane gl owns state rows gl*RX..), carrying
// the affine term l / the state x in registers along the branch.  Each node's slack
// elimination (the x right-hand side qx0 = -r_x - sum_c f_c df r_S / sd) comes from a
// lane-parallel pre-pass or, for plans whose staging does not fit LDS, is formed inside the
// backward sweep from loads that do not depend on the recursion; a lane-parallel post-pass
// forms the multipliers nu and recovers the slacks.
// The first ncw right-hand sides are Woodbury cone columns (kkt_coupling): column k is
// supported on cone k's child branch only, so its backward sweep runs only on that branch and
// its ancestors (elsewhere l and kf are exactly zero and are not stored or read).
// RB: the post-pass takes four right-hand sides per pass (a separate instantiation, called by
// kkt_coupling for the many right-hand sides of NB=2 plans, so that the other solves' code is
// unchanged; each value formed as the one-rhs pass forms it).
template <class X, int NX, int NU, bool RB = false>
BMPC_FN_TREE_SOLVE void tree_solve(const X ex, const Ctx Cin, int nr, const gdouble* r0, size_t rs, const gdouble* e0,
                        size_t es, gdouble* o0, size_t os, gdouble* n0, size_t ns, int ncw = 0) {
  const Ctx C = Cin.uniform();
  r0 = uniform_ptr(r0);
  e0 = uniform_ptr(e0);
  o0 = uniform_ptr(o0);
  n0 = uniform_ptr(n0);
  constexpr int W = X::kTaskLanes;
  constexpr int RX = (NX + W - 1) / W;
  constexpr int NCM = BMPC_MAX_FX + 1;   // LP rows per state node, compile-time bound
  (void)NCM;
  CPlan& P = *C.P;
  CLayout& L = *C.L;
  BMPC_PROF(C.ws, L, PROF_TREESOLVE);
  BMPC_COUNT(C.ws, L, PROF_NTREE);
  const auto t = topo_view(P, ex);
  const int Nc = P.Nc;
  gdouble* ws = C.ws;
  gdouble* lv_ = ws + L.lvec;   // [nr][T][NX]
  gdouble* kf_ = ws + L.kff;    // [nr][U][NU]
  const size_t lstr = (size_t)P.T * NX, kstr = (size_t)P.U * NU;
  const gdouble* dh = ws + L.dh;
  const gdouble* sdv = ws + L.sd;
  const int gl = ex.lane % W, grp = ex.lane / W, ngrp = ex.nlanes / W;
  // rhs ri needs the backward sweep on branch b (see above)
  auto needed = [&](int b, int ri) {
    if (ri >= ncw) return true;
    int c = t.cone_c[ri];
    if (c < 0) return b == 0;   // the root cone: the root node
    while (c > b) c = (c - 1) / P.m;
    return c == b;
  };
  // the x right-hand side of row i of node k after slack elimination (qx0), all loads issued
  // together: -r_x + dh a_0 - sum_{c>=1} Fx[c-1] a_c, a_c = [k non-terminal] df_c r_S,c / sd_c
  auto qx0 = [&](const gdouble* rr, int k, int i) {
    double rS[NCM], s0[NCM], s1[NCM];
#pragma unroll
    for (int c = 0; c < NCM; ++c) {
      const int kc = k * Nc + (c < Nc ? c : 0);
      rS[c] = rr[P.oS + kc];
      s0[c] = sdv[kc * 2];
      s1[c] = sdv[kc * 2 + 1];
    }
    const double on = t.x_u[k] >= 0 ? 1.0 : 0.0;   // terminal nodes add 0
    double v = -rr[P.oX + k * NX + i] + dh[k * NX + i] * (on * s1[0] * rS[0] / s0[0]);
#pragma unroll
    for (int c = 1; c < NCM; ++c)
      if (c < Nc) v -= fxv(P, ex, c - 1, i) * (on * s1[c] * rS[c] / s0[c]);
    return v;
  };
  // plans whose slack terms fit the LDS staging area (Plan::nscr) form the x right-hand sides
  // in a lane-parallel pre-pass (two flat passes per rhs: the slack terms a_kc into LDS, then
  // the node sums); the others form them inside the backward sweep (qx0 above) -- measured:
  // the N=20 NB=1 plan is 2% faster with the pre-pass, N=8 NB=2 5% faster without
  const bool pre = ex.uniform(P.nscr >= P.T * Nc);
  gdouble* q0_ = ws + L.qx0;    // [nr][T][NX] (pre-pass plans)
  if (pre) {
    BMPC_TIC(t_pre);
    ldouble* av = ex.lds + P.lds_scr;
    for (int ri = 0; ri < nr; ++ri) {
      const gdouble* rr = r0 + ri * rs;
      gdouble* q0 = q0_ + ri * lstr;
      // the nodes whose q0 the backward sweep reads: all of them, or for a Woodbury column only
      // the nodes of its cone's root path (up to four branches, s_h / l_h: first node / count)
      int s0 = 0, l0 = P.T, s1 = 0, l1 = 0, s2 = 0, l2 = 0, s3 = 0, l3 = 0;
      if (ri < ncw) {
        int c = t.cone_c[ri] < 0 ? 0 : t.cone_c[ri];
        int st[4] = {0, 0, 0, 0}, ln[4] = {0, 0, 0, 0};
        bool deeper = true;   // (deeper trees keep the whole range)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          if (deeper) {
            st[q] = t.br_ndx[c];
            ln[q] = t.br_len[c] + (t.br_child0[c] < 0 ? 1 : 0);   // a leaf's terminal node
            if (c == 0) deeper = false;
            else c = (c - 1) / P.m;
          }
        }
        if (!deeper) s0 = st[0], l0 = ln[0], s1 = st[1], l1 = ln[1], s2 = st[2], l2 = ln[2], s3 = st[3], l3 = ln[3];
      }
      const int nn = l0 + l1 + l2 + l3;
      auto node = [&](int f) {   // the f-th node of the ranges (branch-free)
        const int f1 = f - l0, f2 = f1 - l1, f3 = f2 - l2;
        return f < l0 ? s0 + f : f1 < l1 ? s1 + f1 : f2 < l2 ? s2 + f2 : s3 + f3;
      };
      lane_batch<BMPC_TS_UN_AV>(ex, 0, nn * Nc, [&](int f) {
        const int k = node(f / Nc), it = k * Nc + f % Nc;
        const double on = t.x_u[k] >= 0 ? 1.0 : 0.0;   // terminal nodes add 0
        return on * sdv[it * 2 + 1] * rr[P.oS + it] / sdv[it * 2];
      }, [&](int f, double v) { av[node(f / Nc) * Nc + f % Nc] = v; });
      ex.sync();
      lane_batch<BMPC_TS_UN>(ex, 0, nn * NX, [&](int f) {
        const int k = node(f / NX), j = f % NX, it = k * NX + j;
        double v = -rr[P.oX + it] + dh[it] * av[k * Nc];
        for (int c = 1; c < Nc; ++c) v -= fxv(P, ex, c - 1, j) * av[k * Nc + c];
        return v;
      }, [&](int f, double v) { q0[node(f / NX) * NX + f % NX] = v; });
      ex.sync();
    }
    BMPC_TOC(C.ws, L, PROF_X1, t_pre);
  }

  BMPC_TIC(t_bw);
  // ---- backward sweep (leaves -> root) -------------------------------------------------------
  // The per-node loads do not depend on the recursion: one memory round trip per node.
  for (int dep = P.NB; dep >= 0; --dep) {
    const int b0 = branch_start(P, dep), nbd = branch_count(P, dep);
    // the needed tasks of this depth, in order: first the (branch, rhs >= ncw) pairs, then for
    // every cone column the branch of its root path at this depth
    const int nfull = nbd * (nr - ncw);
    int ncol = 0;
    for (int ri = 0; ri < ncw; ++ri) {
      const int c = t.cone_c[ri];
      ncol += (c < 0 ? 0 : t.br_depth[c]) >= dep ? 1 : 0;
    }
    const int ntask = nfull + ncol;
    const int rounds = (ntask + ngrp - 1) / ngrp;
    const bool leaf = dep == P.NB;
    for (int rd = 0; rd < rounds; ++rd) {
      const int task = rd * ngrp + grp;
      if (task >= ntask) continue;       // whole group idle together
      int b, ri;
      if (task < nfull) {
        b = b0 + task / (nr - ncw);
        ri = ncw + task % (nr - ncw);
      } else {
        int want = task - nfull;
        ri = 0;
        for (int r2 = 0; r2 < ncw; ++r2) {
          const int c = t.cone_c[r2];
          if ((c < 0 ? 0 : t.br_depth[c]) >= dep) {
            if (want == 0) {
              ri = r2;
              break;
            }
            --want;
          }
        }
        int c = t.cone_c[ri];
        if (c < 0) c = 0;
        while (t.br_depth[c] > dep) c = (c - 1) / P.m;
        b = c;
      }
      const gdouble* rr = r0 + ri * rs;
      const gdouble* ee = e0 + ri * es;
      const gdouble* q0 = q0_ + ri * lstr;
      gdouble* lvec = lv_ + ri * lstr;
      gdouble* kf = kf_ + ri * kstr;
      const int ndx = t.br_ndx[b], ndu = t.br_ndu[b], len = t.br_len[b];
      const int c0 = t.br_child0[b];
      double l[RX];
      if (leaf) {   // terminal node: l = -r_x (= qx0 there)
        const int tn = ndx + len;
#pragma unroll
        for (int q = 0; q < RX; ++q) {
          const int i = gl * RX + q;
          l[q] = i < NX ? (pre ? q0[tn * NX + i] : qx0(rr, tn, i)) : 0.0;
          if (i < NX) lvec[tn * NX + i] = l[q];
        }
      }
      for (int jn = len - 1; jn >= 0; --jn) {
        const int k = ndx + jn, u = ndu + jn;
        double qx[RX], Acol[RX][NX], Brow[RX][NU], Kcol[RX][NU], Lu[NU][NU], ru[NU];
#pragma unroll
        for (int q = 0; q < RX; ++q) {
          const int i = gl * RX + q < NX ? gl * RX + q : NX - 1;
          qx[q] = pre ? q0[k * NX + i] : qx0(rr, k, i);
#pragma unroll
          for (int j = 0; j < NX; ++j) Acol[q][j] = ws[L.Ad + u * NX * NX + j * NX + i];
#pragma unroll
          for (int m = 0; m < NU; ++m) Brow[q][m] = ws[L.Bd + u * NX * NU + i * NU + m];
#pragma unroll
          for (int m = 0; m < NU; ++m) Kcol[q][m] = ws[L.Kg + u * NU * NX + m * NX + i];
        }
        mat_load(Lu, ws + L.Luu + u * NU * NU);
#pragma unroll
        for (int m = 0; m < NU; ++m) ru[m] = rr[P.oU + u * NU + m];
        double g[RX];
        if (jn < len - 1 || leaf) {
          double ec[NX];
#pragma unroll
          for (int j = 0; j < NX; ++j) ec[j] = ee[(k + 1) * NX + j];
#pragma unroll
          for (int q = 0; q < RX; ++q) {
            const int i = gl * RX + q < NX ? gl * RX + q : NX - 1;
            double v = l[q];
#pragma unroll
            for (int j = 0; j < NX; ++j) v += ws[L.P + (k + 1) * NX * NX + i * NX + j] * ec[j];
            g[q] = v;
          }
        } else {
#pragma unroll
          for (int q = 0; q < RX; ++q) g[q] = 0.0;
          for (int ci = 0; ci < P.m; ++ci) {
            if (!needed(c0 + ci, ri)) continue;   // l = 0 and e = 0 there: adds exactly 0
            const int c = t.br_ndx[c0 + ci];
            double ec[NX];
#pragma unroll
            for (int j = 0; j < NX; ++j) ec[j] = ee[c * NX + j];
#pragma unroll
            for (int q = 0; q < RX; ++q) {
              const int i = gl * RX + q < NX ? gl * RX + q : NX - 1;
              double v = lvec[c * NX + i];
#pragma unroll
              for (int j = 0; j < NX; ++j) v += ws[L.P + c * NX * NX + i * NX + j] * ec[j];
              g[q] += v;
            }
          }
        }
        double kfv[NU];
        bw_node<X, NX, NU, RX, W>(ex, gl, qx, Acol, Brow, Kcol, Lu, ru, g, l, kfv);
#pragma unroll
        for (int q = 0; q < RX; ++q) {
          const int i = gl * RX + q;
          if (i < NX) lvec[k * NX + i] = l[q];
        }
        if (gl == 0)
#pragma unroll
          for (int m = 0; m < NU; ++m) kf[u * NU + m] = kfv[m];
      }
    }
    ex.sync();
  }
  BMPC_TOC(C.ws, L, PROF_X2, t_bw);
  BMPC_TIC(t_fw);
  // ---- forward sweep (root -> leaves): x, u, and each node's multipliers and slacks ----------
  for (int it = ex.lane; it < nr * NX; it += ex.nlanes) {
    const int ri = it / NX, j = it % NX;
    o0[ri * os + P.oX + j] = e0[ri * es + j];
  }
  ex.sync();
  for (int dep = 0; dep <= P.NB; ++dep) {
    const int b0 = branch_start(P, dep), nbd = branch_count(P, dep);
    const int ntask = nbd * nr;
    const int rounds = (ntask + ngrp - 1) / ngrp;
    const bool leaf = dep == P.NB;
    for (int rd = 0; rd < rounds; ++rd) {
      const int task = rd * ngrp + grp;
      if (task >= ntask) continue;
      const int b = b0 + task / nr, ri = task % nr;
      gdouble* o = o0 + ri * os;
      const gdouble* ee = e0 + ri * es;
      const gdouble* kf = kf_ + ri * kstr;
      const bool kfon = needed(b, ri);   // kf = 0 where the backward sweep was skipped
      const int ndx = t.br_ndx[b], ndu = t.br_ndu[b], len = t.br_len[b];
      const int c0 = t.br_child0[b];
      double xk[NX];      // full state (every lane of the group holds all of it)
#pragma unroll
      for (int j = 0; j < NX; ++j) xk[j] = o[P.oX + ndx * NX + j];   // written by the parent group
      for (int jn = 0; jn < len; ++jn) {
        const int k = ndx + jn, u = ndu + jn;
        // ---- loads ----
        double Arow[RX][NX], Brow[RX][NU], Kcol[RX][NU], kfu[NU], en[RX];
        const int kn = (jn < len - 1 || leaf) ? k + 1 : t.br_ndx[c0 >= 0 ? c0 : 0];
#pragma unroll
        for (int q = 0; q < RX; ++q) {
          const int i = gl * RX + q < NX ? gl * RX + q : NX - 1;
#pragma unroll
          for (int j = 0; j < NX; ++j) Arow[q][j] = ws[L.Ad + u * NX * NX + i * NX + j];
#pragma unroll
          for (int m = 0; m < NU; ++m) Brow[q][m] = ws[L.Bd + u * NX * NU + i * NU + m];
#pragma unroll
          for (int m = 0; m < NU; ++m) Kcol[q][m] = ws[L.Kg + u * NU * NX + m * NX + i];
          en[q] = ee[kn * NX + i];
        }
#pragma unroll
        for (int m = 0; m < NU; ++m) kfu[m] = kfon ? kf[u * NU + m] : 0.0;
        // ---- u = kf + K x ----
        double uk[NU];
#pragma unroll
        for (int m = 0; m < NU; ++m) {
          double v = 0.0;
#pragma unroll
          for (int q = 0; q < RX; ++q) v += gl * RX + q < NX ? Kcol[q][m] * xk[gl * RX + q < NX ? gl * RX + q : 0] : 0.0;
          uk[m] = kfu[m] + ex.tsum(v);
        }
        if (gl == 0)
#pragma unroll
          for (int m = 0; m < NU; ++m) o[P.oU + u * NU + m] = uk[m];
        // ---- x_next = A x + B u (+ e), own rows, then gather ----
        double xn[RX];
#pragma unroll
        for (int q = 0; q < RX; ++q) {
          double v = 0.0;
#pragma unroll
          for (int j = 0; j < NX; ++j) v += Arow[q][j] * xk[j];
#pragma unroll
          for (int m = 0; m < NU; ++m) v += Brow[q][m] * uk[m];
          xn[q] = v;
        }
        if (jn < len - 1 || leaf) {
#pragma unroll
          for (int q = 0; q < RX; ++q) {
            const int i = gl * RX + q;
            xn[q] += en[q];
            if (i < NX) o[P.oX + (k + 1) * NX + i] = xn[q];
          }
          task_gather<NX, RX, W>(ex, xn, xk);
        } else {
          for (int ci = 0; ci < P.m; ++ci) {
            const int c = t.br_ndx[c0 + ci];
#pragma unroll
            for (int q = 0; q < RX; ++q) {
              const int i = gl * RX + q;
              if (i < NX) o[P.oX + c * NX + i] = xn[q] + ee[c * NX + i];
            }
          }
        }
      }
    }
    ex.sync();
  }
  BMPC_TOC(C.ws, L, PROF_X3, t_fw);
  BMPC_TIC(t_post);
  // ---- post-pass: nu_k = -(l_k + P_k x_k), slack recovery -----------------------------------
  if constexpr (RB) {   // BMPC_TS_POST_RB (4) right-hand sides per pass: a node's P row, dh / Fx blend and slack weights loaded once
    constexpr int NB4 = BMPC_TS_POST_RB;
    struct VR { double v[NB4]; };
    for (int rb = 0; rb < nr; rb += NB4) {
      const int rn = nr - rb < NB4 ? nr - rb : NB4;
      if (n0) {
        lane_batch<BMPC_TS_UN>(ex, 0, P.T * NX, [&](int it) {
          const int k = it / NX, i = it % NX;
          double pr[NX];
#pragma unroll
          for (int j = 0; j < NX; ++j) pr[j] = ws[L.P + k * NX * NX + i * NX + j];
          VR out;
#pragma unroll
          for (int a = 0; a < NB4; ++a) {
            const int ri = rb + (a < rn ? a : 0);
            const gdouble* o = o0 + ri * os;
            double v = (ri >= ncw || needed(t.x_branch[k], ri)) ? lv_[ri * lstr + it] : 0.0;
#pragma unroll
            for (int j = 0; j < NX; ++j) v += pr[j] * o[P.oX + k * NX + j];
            out.v[a] = -v;
          }
          return out;
        }, [&](int it, const VR& r) {
#pragma unroll
          for (int a = 0; a < NB4; ++a)
            if (a < rn) n0[(rb + a) * ns + it] = r.v[a];
        });
      }
      lane_batch<BMPC_TS_UN>(ex, 0, P.T * Nc, [&](int it) {
        const int k = it / Nc, c = it % Nc;
        const double on = t.x_u[k] >= 0 ? 1.0 : 0.0;
        double cf[NX];
#pragma unroll
        for (int j = 0; j < NX; ++j) {
          const double dhv = dh[k * NX + j], fxj = fxv(P, ex, c > 0 ? c - 1 : 0, j), m0 = c == 0 ? 1.0 : 0.0;
          cf[j] = m0 * (-dhv) + (1.0 - m0) * fxj;
        }
        const double s0 = sdv[it * 2], s1 = sdv[it * 2 + 1];
        VR out;
#pragma unroll
        for (int a = 0; a < NB4; ++a) {
          const int ri = rb + (a < rn ? a : 0);
          const gdouble* o = o0 + ri * os;
          double fx = 0.0;
#pragma unroll
          for (int j = 0; j < NX; ++j) fx += cf[j] * o[P.oX + k * NX + j];
          out.v[a] = (r0[ri * rs + P.oS + it] + s1 * on * fx) / s0;
        }
        return out;
      }, [&](int it, const VR& r) {
#pragma unroll
        for (int a = 0; a < NB4; ++a)
          if (a < rn) o0[(rb + a) * os + P.oS + it] = r.v[a];
      });
    }
    ex.sync();
    BMPC_TOC(C.ws, L, PROF_X4, t_post);
    return;
  }
  for (int ri = 0; ri < nr; ++ri) {
    gdouble* o = o0 + ri * os;
    const gdouble* rr = r0 + ri * rs;
    const gdouble* lvec = lv_ + ri * lstr;
    if (n0) {
      gdouble* nn = n0 + ri * ns;
      const bool lon = ex.uniform(ri >= ncw);   // Woodbury columns: l = 0 off the column's root path
      lane_batch<BMPC_TS_UN>(ex, 0, P.T * NX, [&](int it) {
        const int k = it / NX, i = it % NX;
        double v = (lon || needed(t.x_branch[k], ri)) ? lvec[it] : 0.0;
#pragma unroll
        for (int j = 0; j < NX; ++j) v += ws[L.P + k * NX * NX + i * NX + j] * o[P.oX + k * NX + j];
        return -v;
      }, [&](int it, double v) { nn[it] = v; });
    }
    lane_batch<BMPC_TS_UN>(ex, 0, P.T * Nc, [&](int it) {
      const int k = it / Nc, c = it % Nc;
      const double on = t.x_u[k] >= 0 ? 1.0 : 0.0;   // branch-free: terminal nodes add 0
      double fx = 0.0;
#pragma unroll
      for (int j = 0; j < NX; ++j) {   // -dh for c == 0, Fx[c-1] otherwise (blend: no branch around the dh load)
        const double dhv = dh[k * NX + j], fxj = fxv(P, ex, c > 0 ? c - 1 : 0, j), m0 = c == 0 ? 1.0 : 0.0;
        fx += (m0 * (-dhv) + (1.0 - m0) * fxj) * o[P.oX + k * NX + j];
      }
      return (rr[P.oS + it] + sdv[it * 2 + 1] * on * fx) / sdv[it * 2];
    }, [&](int it, double v) { o[P.oS + it] = v; });
  }
  ex.sync();
  BMPC_TOC(C.ws, L, PROF_X4, t_post);
}

// dense LU with partial pivoting of the coupling system (row-major n x n, in LDS)
template <class X, class PM, class PP>
BMPC_FN bool small_lu(const X ex, PM* M, PP* piv, int n) {
  for (int k = 0; k < n; ++k) {
    double best = -1.0, bi = 1e300;
    for (int i = k + ex.lane; i < n; i += ex.nlanes) {
      const double a = fabs(M[i * n + k]);
      if (a > best || (a == best && i < bi)) best = a, bi = (double)i;
    }
    const double amax = ex.max(best);
    const int p = (int)ex.min(best == amax ? bi : 1e300);
    if (!(amax > 0.0)) return false;
    ex.sync();
    if (p != k)
      for (int j = ex.lane; j < n; j += ex.nlanes) {
        const double tmp = M[k * n + j];
        M[k * n + j] = M[p * n + j];
        M[p * n + j] = tmp;
      }
    if (ex.lane == 0) piv[k] = (double)p;
    ex.sync();
    const double d = M[k * n + k];
    for (int i = k + 1 + ex.lane; i < n; i += ex.nlanes) M[i * n + k] = M[i * n + k] / d;
    ex.sync();
    // trailing update: every entry (i, j) of rows and columns k+1.. dealt over the lanes with
    // eight entries' loads in flight per lane (a row per lane would chain its n - k - 1
    // read-modify-writes, a memory round trip each when the system lives in the slab); each
    // entry gets the same single update M_ij - l_i M_kj as before
    const int m = n - k - 1;
    lane_batch<8>(ex, 0, m * m, [&](int t) {
      const int i = k + 1 + t / m, j = k + 1 + t % m;
      return M[i * n + j] - M[i * n + k] * M[k * n + j];
    }, [&](int t, double v) { M[(k + 1 + t / m) * n + k + 1 + t % m] = v; });
    ex.sync();
  }
  return true;
}

// wave-scope ordering of LDS steps (one wave alone, no workgroup barrier)
BMPC_HD void wave_sync() {
#if defined(__HIP_DEVICE_COMPILE__)
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
#endif
}
// small_lu on one wave (n <= 64; the one-wave executors' own wave, or the first wave of a
// multi-wave executor): the pivot by one DPP max and a ballot (the smallest row attaining it: the
// same pivot as small_lu's max-then-min), the trailing update with a lane per column over the
// rows whose multiplier is non-zero only -- a ballot of column k after the division, since a row
// with l_i = 0 would get a_ij - 0 * m_kj = a_ij: the coupling system is sparse (a diagonal block of
// CVaR globals, 3-4 globals per cone), so most pivots update a few rows.  Steps ordered by
// workgroup-scope fences (the system lives in LDS, or in the slab for lean launches); the same
// pivots and the same operation per updated entry as small_lu.  Measured (tools/mb_lu.hip,
// profiles/r06/r06p_*): 2,090 vs 3,057 cycles per pivot on the N=8 NB=2 structure (n = 50),
// 1,826 vs 2,238 at N=20 NB=1 (n = 14), bit-identical.
BMPC_HD void lu_fence() {
#if defined(__HIP_DEVICE_COMPILE__)
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
  __builtin_amdgcn_wave_barrier();
#endif
}
template <class PM, class PP>
BMPC_HD bool small_lu_wave(int j, PM* M, PP* piv, int n) {
#if defined(__HIP_DEVICE_COMPILE__)
  for (int k = 0; k < n; ++k) {
    const bool live = j >= k && j < n;
    const double best = live ? fabs(M[j * n + k]) : -1.0;
    const double amax = dev::wave_reduce<1, true>(best);   // exact in any order
    const unsigned long long at = __ballot(live && best == amax);
    const int p = at ? (int)__builtin_ctzll(at) : k;
    if (!(amax > 0.0)) return false;
    if (p != k && j < n) {
      const double tmp = M[k * n + j];
      M[k * n + j] = M[p * n + j];
      M[p * n + j] = tmp;
    }
    if (j == 0) piv[k] = (double)p;
    lu_fence();
    const double d = M[k * n + k];
    double lj = 0.0;
    if (j > k && j < n) {
      lj = M[j * n + k] / d;
      M[j * n + k] = lj;
    }
    unsigned long long nz = __ballot(j > k && j < n && lj != 0.0);
    lu_fence();
    if (nz) {
      const bool upd = j > k && j < n;
      const double mk = upd ? (double)M[k * n + j] : 0.0;
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
          a[u] = M[i * n + (upd ? j : k)];
        }
        if (upd)
#pragma unroll
          for (int u = 0; u < 8; ++u)
            if (r[u] >= 0) M[r[u] * n + j] = a[u] - l[u] * mk;
      }
    }
    lu_fence();
  }
  return true;
#else
  return false;
#endif
}

// small_lu_solve on the first wave alone for K right-hand sides with b in registers (lane j: b_j):
// the row swaps and each substitution step's pivot entry by readlane -- no LDS round trip and no
// fence on the chain, and K chains interleaved; per right-hand side the same swaps and the same
// operations in the same order (small_lu_solve, small_lu_solve_rows)
template <int K, class PM, class PP, class PB>
BMPC_HD void small_lu_solve_wave(int j, const PM* M, const PP* piv, PB* const (&b)[K], int n) {
#if defined(__HIP_DEVICE_COMPILE__)
  auto bcast = [](double v, int l) {
    return __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(v), l),
                            __builtin_amdgcn_readlane(__double2loint(v), l));
  };
  const bool row = j < n;
  const size_t rj = (size_t)(row ? j : 0) * n;
  double bj[K];
#pragma unroll
  for (int r = 0; r < K; ++r) bj[r] = row ? (double)b[r][j] : 0.0;
  for (int k0 = 0; k0 < n; k0 += 8) {   // P
    double pv[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) pv[u] = piv[k0 + u < n ? k0 + u : k0];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int k = k0 + u;
      if (k < n) {
        const int p = __builtin_amdgcn_readfirstlane((int)pv[u]);
        if (p != k) {
#pragma unroll
          for (int r = 0; r < K; ++r) {
            const double vk = bcast(bj[r], k), vp = bcast(bj[r], p);
            if (j == k) bj[r] = vp;
            if (j == p) bj[r] = vk;
          }
        }
      }
    }
  }
  for (int i0 = 0; i0 < n; i0 += 8) {   // L (unit diagonal)
    double mc[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) mc[u] = M[rj + (i0 + u < n ? i0 + u : 0)];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int i = i0 + u;
      if (i < n) {
#pragma unroll
        for (int r = 0; r < K; ++r) {
          const double bi = bcast(bj[r], i);
          if (row && j > i) bj[r] -= mc[u] * bi;
        }
      }
    }
  }
  for (int i1 = n - 1; i1 >= 0; i1 -= 8) {   // U
    double mc[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) mc[u] = M[rj + (i1 - u >= 0 ? i1 - u : 0)];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int i = i1 - u;
      if (i >= 0) {
#pragma unroll
        for (int r = 0; r < K; ++r) {
          if (j == i) bj[r] = bj[r] / mc[u];
          const double bi = bcast(bj[r], i);
          if (row && j < i) bj[r] -= mc[u] * bi;
        }
      }
    }
  }
  if (row)
#pragma unroll
    for (int r = 0; r < K; ++r) b[r][j] = bj[r];
#endif
}

template <class X, class = void>
struct RowLanes : std::false_type {};
template <class X>
struct RowLanes<X, std::void_t<decltype(X::kRowLanes)>> : std::integral_constant<bool, X::kRowLanes> {};

// The substitutions with lane j owning row j (n <= lanes, device executors): each lane loads
// its row's next eight matrix entries in one batch, so the per-row chain waits on the LDS
// right-hand side only (the matrix is in the slab in lean launches: one dependent global load
// per row otherwise).  Same operations in the same order as the column loops below.
template <class X, class PM, class PB>
BMPC_HD void small_lu_solve_rows(const X ex, const PM* M, PB* b, int n) {
  const int j = ex.lane;
  const bool row = j < n;
  const size_t rj = (size_t)(row ? j : 0) * n;
  for (int i0 = 0; i0 < n; i0 += 8) {   // L (unit diagonal)
    double mc[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) mc[u] = M[rj + (i0 + u < n ? i0 + u : 0)];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int i = i0 + u;
      if (i < n) {   // uniform
        const double bi = b[i];
        if (row && j > i) b[j] -= mc[u] * bi;
        ex.sync();
      }
    }
  }
  for (int i1 = n - 1; i1 >= 0; i1 -= 8) {   // U: row i's lane divides by its diagonal first
    double mc[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) mc[u] = M[rj + (i1 - u >= 0 ? i1 - u : 0)];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int i = i1 - u;
      if (i >= 0) {   // uniform
        if (j == i) b[i] = b[i] / mc[u];
        ex.sync();
        const double bi = b[i];
        if (row && j < i) b[j] -= mc[u] * bi;
        ex.sync();
      }
    }
  }
}

// small_lu_solve_rows on the first wave of a multi-wave executor alone: its rows' steps ordered
// by wave-scope fences instead of one workgroup barrier each (3n barriers per solve; the other
// waves wait at the caller's one barrier).  Same operations in the same order.
template <class PM, class PB>
BMPC_HD void small_lu_solve_rows_wave(int j, const PM* M, PB* b, int n) {
  const bool row = j < n;
  const size_t rj = (size_t)(row ? j : 0) * n;
  for (int i0 = 0; i0 < n; i0 += 8) {   // L (unit diagonal)
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
  for (int i1 = n - 1; i1 >= 0; i1 -= 8) {   // U
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

// solve with the LU above; b in LDS, column-oriented substitution (one step per row)
template <class X, class PM, class PP, class PB>
BMPC_HD void small_lu_solve(const X ex, const PM* M, const PP* piv, PB* b, int n) {
#if BMPC_SUBST_REG
  if constexpr (MultiWave<X>::value) {
    if (n <= 64) {
      PB* const bs[1] = {b};
      if (ex.lane < 64) small_lu_solve_wave<1>(ex.lane, M, piv, bs, n);
      ex.sync();
      return;
    }
  }
#endif
  if (ex.lane == 0)
    for (int k = 0; k < n; ++k) {
      const int p = (int)piv[k];
      if (p != k) {
        const double tmp = b[k];
        b[k] = b[p];
        b[p] = tmp;
      }
    }
  ex.sync();
  if constexpr (RowLanes<X>::value) {
#if BMPC_BLK_WAVE_SUBST
    if constexpr (X::nlanes > 64) {
      if (n <= 64) {
        if (ex.lane < 64) small_lu_solve_rows_wave(ex.lane, M, b, n);
        ex.sync();
        return;
      }
    }
#endif
    if (n <= X::nlanes) {
      small_lu_solve_rows(ex, M, b, n);
      return;
    }
  }
  for (int i = 0; i < n; ++i) {          // L (unit diagonal)
    const double bi = b[i];
    for (int j = i + 1 + ex.lane; j < n; j += ex.nlanes) b[j] -= M[j * n + i] * bi;
    ex.sync();
  }
  for (int i = n - 1; i >= 0; --i) {     // U
    const double bi = b[i] / M[i * n + i];
    for (int j = ex.lane; j < i; j += ex.nlanes) b[j] -= M[j * n + i] * bi;
    ex.sync();
    if (ex.lane == 0) b[i] = bi;
    ex.sync();
  }
}

// the dense coupling system (matrix | pivots | rhs at the plan's lds_M / lds_piv / lds_rhs):
// in LDS, or in the ego's slab for lean-LDS launches (X::kCoupLds false)
template <class X>
BMPC_HD auto coup_mem(const X& ex, gdouble* ws, CLayout& L, CPlan& P, int off) {
  if constexpr (X::kCoupLds) return ex.lds + off;
  else return ws + L.coup + (off - P.lds_M);
}
// its pivots and right-hand side: LDS in every launch (Plan::lds_piv / lds_rhs precede lds_M)
template <class X>
BMPC_HD auto coup_vec(const X& ex, int off) { return ex.lds + off; }


// global variable index -> position in the primal vector
BMPC_HD int gvar(CPlan& P, int i) { return i == P.ng - 1 ? P.oJ : P.oRho + i; }

// Woodbury columns, coupling matrix and its LU; returns false on breakdown.  `extra` (0 or 2)
// more right-hand sides ride in the same tree solve: the z-space slots after the cone vectors
// (gk + nc nv: the c-direction and affine solves' G'W^-2 r3 + r1), the eq-space slots after the
// nc zero vectors (bvec, ry), solutions to the slots after the Woodbury columns (x1 / x2,
// y1 / y2) -- the Riccati data are read once for all of them (Layout, bmpc_plan.cpp).
template <class X, int NX, int NU>
BMPC_FN bool kkt_coupling(const X ex, const Ctx Cin, int extra) {
  const Ctx C = Cin.uniform();
  CPlan& P = *C.P;
  CLayout& L = *C.L;
  BMPC_PROF(C.ws, L, PROF_COUPLING);
  gdouble* ws = C.ws;
  const int nc = P.ncones;
  BMPC_TIC(t_cts);
  if (ex.uniform(nc + extra >= BMPC_TS_POST_RB_MIN))   // NB=2 plans (15 right-hand sides): the batched post-pass
    tree_solve<X, NX, NU, true>(ex, C, nc + extra, ws + L.gk, P.nv, ws + L.zeros, P.neq, ws + L.colk, P.nv,
                                ws + L.colnu, P.neq, nc);
  else
    tree_solve<X, NX, NU>(ex, C, nc + extra, ws + L.gk, P.nv, ws + L.zeros, P.neq, ws + L.colk, P.nv, ws + L.colnu,
                          P.neq, nc);
  BMPC_TOC(C.ws, L, PROF_CTS, t_cts);
  BMPC_TIC(t_cdot);
  const int ng = P.ng, nb = P.bdim, ns = P.nsm;
  auto* M = coup_mem(ex, ws, L, P, P.lds_M);
  const gdouble* eta = ws + L.eta;
  const gdouble* dl = ws + L.dl;
  const gdouble* p = ws + L.p;
  const int ntree = P.oRho;    // x and u parts are [0, oRho); S part [oS, oJ)
  for (int i = ex.lane; i < ns * ns; i += ex.nlanes) M[i] = 0.0;
  ex.sync();
  // cone-cone block: c_k (I/c_k + M) with M[k][j] = g_k' col_j over tree variables
  if (coup_supp_dots(P) && BMPC_BLK_PAIR_DOTS && MultiWave<X>::value) {
    // multi-wave executors (one ego, latency-bound): a lane per entry (k, j), the sum over g_k's
    // support in order (the host build's order), eight entries' loads in flight -- no reductions
    const auto t = topo_view(P, ex);
    for (int pr = ex.lane; pr < nc * nc; pr += ex.nlanes) {
      const int k = pr / nc, j = pr - (pr / nc) * nc;
      const gdouble* g = ws + L.gk + (size_t)k * P.nv;
      const gdouble* v = ws + L.colk + (size_t)j * P.nv;
      const int tot = cone_supp_len(P, t, k);
      double acc = 0.0;
      for (int e0 = 0; e0 < tot; e0 += 8) {
        double gv[8], vv[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const int i = cone_supp_idx(P, t, k, e0 + u < tot ? e0 + u : e0);
          gv[u] = g[i];
          vv[u] = v[i];
        }
#pragma unroll
        for (int u = 0; u < 8; ++u)
          if (e0 + u < tot) acc += gv[u] * vv[u];
      }
      const double ck = 2.0 / (eta[k] * eta[k]);
      M[(ng + nb + k) * ns + ng + nb + j] = ck * acc + (k == j ? 1.0 : 0.0);
    }
  } else if (coup_supp_dots(P)) {   // many cones: over each g_k's support, 16 columns per pass
    const auto t = topo_view(P, ex);
    for (int k = 0; k < nc; ++k)
      for (int j0 = 0; j0 < nc; j0 += 16) {
        double acc[16];
        cone_supp_dots(ex, P, t, ws + L.gk + (size_t)k * P.nv, k, ws + L.colk, P.nv, j0, nc, acc);
        if (ex.lane == 0) {
          const double ck = 2.0 / (eta[k] * eta[k]);
          for (int j = j0; j < nc && j < j0 + 16; ++j)
            M[(ng + nb + k) * ns + ng + nb + j] = ck * acc[j - j0] + (k == j ? 1.0 : 0.0);
        }
      }
  } else {   // 4 x 4 blocks of dot products per pass over all tree variables
    for (int k0 = 0; k0 < nc; k0 += 4)
      for (int j0 = 0; j0 < nc; j0 += 4) {
        const int na = nc - k0 < 4 ? nc - k0 : 4, nbk = nc - j0 < 4 ? nc - j0 : 4;
        double acc[4][4];
        block_dots(ex, ws + L.gk + (size_t)k0 * P.nv, P.nv, na, ws + L.colk + (size_t)j0 * P.nv, P.nv, nbk,
                   0, ntree, P.oS, P.oJ, acc);
        if (ex.lane == 0)
          for (int a = 0; a < na; ++a) {
            const int k = k0 + a;
            const double ck = 2.0 / (eta[k] * eta[k]);
            for (int b = 0; b < nbk; ++b) {
              const int j = j0 + b;
              M[(ng + nb + k) * ns + ng + nb + j] = ck * acc[a][b] + (k == j ? 1.0 : 0.0);
            }
          }
      }
  }
  // H_gg diagonal: LP rows -rho, -mu+, -mu-
  for (int b = ex.lane; b < nb; b += ex.nlanes) {
    const double w = dl[P.rRisk + b];
    M[b * ns + b] = 1.0 / (w * w);
  }
  for (int j = ex.lane; j < 2 * nb * P.m; j += ex.nlanes) {
    const double w = dl[P.rRisk + nb + j];
    const int gi = 2 * nb + j;
    M[gi * ns + gi] = 1.0 / (w * w);
  }
  // CVaR equality rows and their transpose
  for (int b = ex.lane; b < nb; b += ex.nlanes) {
    const int row = ng + b;
    M[row * ns + b] = 1.0;
    M[b * ns + row] = 1.0;
    M[row * ns + nb + b] = 1.0;
    M[(nb + b) * ns + row] = 1.0;
    for (int i = 0; i < P.m; ++i) {
      const int gi = 2 * nb + nb * P.m + b * P.m + i;
      const double a = -p[b * P.m + i] / P.desc.ralpha;
      M[row * ns + gi] = a;
      M[gi * ns + row] = a;
    }
  }
  // cone coupling with the globals
  for (int it = ex.lane; it < nc * ng; it += ex.nlanes) {
    const int k = it / ng, i = it % ng;
    const double gv = ws[L.gk + (size_t)k * P.nv + gvar(P, i)];
    const double ck = 2.0 / (eta[k] * eta[k]);
    M[i * ns + ng + nb + k] = gv;
    M[(ng + nb + k) * ns + i] = -ck * gv;
  }
  ex.sync();
  BMPC_TOC(C.ws, L, PROF_CDOT, t_cdot);
  BMPC_TIC(t_lu);
  bool ok;
  // device executors: the one-wave sparse LU -- the multi-wave executor always, the one-wave
  // executor in lean launches (config 3: n = 50, +2.5%) from BMPC_WAVE_LU_MIN1 on; the LDS-rich
  // one-wave k_ipm (the headline, n = 14) keeps small_lu's code (-0.2..-0.7% with the other)
  if constexpr (BMPC_WAVE_LU && RowLanes<X>::value && (MultiWave<X>::value || !X::kCoupLds)) {
    if (ns <= 64 && (MultiWave<X>::value || ns >= BMPC_WAVE_LU_MIN1)) {
      double bad = 0.0;
      if (ex.lane < 64) bad = small_lu_wave(ex.lane, M, coup_vec(ex, P.lds_piv), ns) ? 0.0 : 1.0;
      ok = ex.max(bad) == 0.0;   // a multi-wave executor's barrier also hands the factors to the other waves
    } else {
      ok = small_lu(ex, M, coup_vec(ex, P.lds_piv), ns);
    }
  } else {
    ok = small_lu(ex, M, coup_vec(ex, P.lds_piv), ns);
  }
  BMPC_TOC(C.ws, L, PROF_LU, t_lu);
  return ok;
}

template <class X, int NX, int NU, bool R3ZERO>
BMPC_HD void kkt_back(const X ex, const Ctx& C, const gdouble* tz, const gdouble* r2, const gdouble* r3h,
                      gdouble* dx, gdouble* dy, gdouble* dzh, bool fin);

// One pass of the W-scaled KKT system (oracle/ecos_ipm.py KKT)
//   [0 A' G'W^-1; A 0 0; W^-1 G 0 -I] [dx; dy; dzh] = [r1; r2; r3h],   dzh = W dz,
// by the reduced Hessian G'W^-2G (tree Riccati + Woodbury coupling).
// R3ZERO: r3h = 0 (refinement corrections): G'W^-1 r3h + r1 = r1 feeds the tree solve directly
template <class X, int NX, int NU, bool R3ZERO = false>
BMPC_HD void kkt_solve_once(const X ex, const Ctx Cin, const gdouble* r1, const gdouble* r2,
                            const gdouble* r3h, gdouble* dx, gdouble* dy, gdouble* dzh, bool tr_ready, bool fin) {
  const Ctx C = Cin.uniform();
  CPlan& P = *C.P;
  CLayout& L = *C.L;
  gdouble* ws = C.ws;
  gdouble* tr = ws + L.k_r0;
  gdouble* tz = ws + L.k_nv0;
  if constexpr (R3ZERO) {
    tz = const_cast<gdouble*>(r1);
  } else {
    if (!tr_ready) apply_W(ex, C, 1, r3h, tr);    // W^-1 r3h (kkt_solve forms it with r3h)
    apply_GT<X, NX, NU>(ex, C, tr, tz, r1);       // G' W^-1 r3h + r1
  }
  tree_solve<X, NX, NU>(ex, C, 1, tz, 0, r2, 0, dx, 0, dy, 0);
  kkt_back<X, NX, NU, R3ZERO>(ex, C, tz, r2, r3h, dx, dy, dzh, fin);
}

// The back half of a KKT solve: with the tree solution (dx, dy) of K [v; nu] = [tz; r2] in
// place, the Woodbury correction through the coupling system (globals and rank-1 cone terms),
// then dzh = W^-1 G dx - r3h, or (fin) dz = W^-1 dzh, in one pass.
template <class X, int NX, int NU, bool R3ZERO>
BMPC_HD void kkt_back(const X ex, const Ctx& C, const gdouble* tz, const gdouble* r2, const gdouble* r3h,
                      gdouble* dx, gdouble* dy, gdouble* dzh, bool fin) {
  CPlan& P = *C.P;
  CLayout& L = *C.L;
  BMPC_PROF(C.ws, L, PROF_BACK);
  gdouble* ws = C.ws;
  gdouble* tr = ws + L.k_r0;
  const int ng = P.ng, nb = P.bdim, nc = P.ncones, ns = P.nsm;
  auto* b = coup_vec(ex, P.lds_rhs);
  const gdouble* eta = ws + L.eta;
  if (coup_supp_dots(P)) {   // g_k' dx over each cone's support, sixteen cones per pass
    const auto t = topo_view(P, ex);
    for (int k0 = 0; k0 < nc; k0 += 16) {
      double acc[16];
      cone_supp_gdx(ex, P, t, ws + L.gk, P.nv, dx, k0, acc);
      if (ex.lane == 0)
        for (int a = 0; a < 16 && k0 + a < nc; ++a) b[ng + nb + k0 + a] = 2.0 / (eta[k0 + a] * eta[k0 + a]) * acc[a];
    }
  } else {
    for (int k0 = 0; k0 < nc; k0 += 4) {   // g_k' dx, four cones per pass
      const int na = nc - k0 < 4 ? nc - k0 : 4;
      double acc[4][4];
      block_dots<1>(ex, ws + L.gk + (size_t)k0 * P.nv, P.nv, na, dx, 0, 1, 0, P.oRho, P.oS, P.oJ, acc);
      if (ex.lane == 0)
        for (int a = 0; a < na; ++a) b[ng + nb + k0 + a] = 2.0 / (eta[k0 + a] * eta[k0 + a]) * acc[a][0];
    }
  }
  for (int i = ex.lane; i < ng + nb; i += ex.nlanes) b[i] = i < ng ? tz[gvar(P, i)] : r2[P.T * NX + i - ng];
  ex.sync();
  BMPC_TIC(t_lus);
  small_lu_solve(ex, coup_mem(ex, ws, L, P, P.lds_M), coup_vec(ex, P.lds_piv), b, ns);
  BMPC_TOC(C.ws, L, PROF_LUS, t_lus);
  const auto* bc = b + ng + nb;
  const gdouble* colk = ws + L.colk;
  const gdouble* colnu = ws + L.colnu;
  // dx (tree and slack parts) and dy in one pass; the columns are loaded four at a time so a
  // lane's loads are in flight together
  const int n1 = P.oRho, n2 = n1 + (P.oJ - P.oS), n3 = n2 + P.T * NX;
  auto row = [&](int t, int& i, bool& isx) {
    isx = t < n2;
    i = t < n1 ? t : t < n2 ? P.oS + (t - n1) : t - n2;
  };
  lane_batch(ex, 0, n3, [&](int t) {
    int i;
    bool isx;
    row(t, i, isx);
    const gdouble* col = isx ? colk : colnu;
    const size_t cs = isx ? (size_t)P.nv : (size_t)P.neq;
    const gdouble* src = isx ? dx : dy;   // one load through a selected pointer, not a select of two loads
    double v = src[i];
    for (int k0 = 0; k0 < nc; k0 += 4) {
      double c4[4], b4[4];
#pragma unroll
      for (int a = 0; a < 4; ++a) {
        c4[a] = col[(size_t)(k0 + a < nc ? k0 + a : nc - 1) * cs + i];
        b4[a] = k0 + a < nc ? bc[k0 + a] : 0.0;   // (LDS / uniform: a select here costs no round trip)
      }
#pragma unroll
      for (int a = 0; a < 4; ++a) v -= b4[a] * c4[a];
    }
    return v;
  }, [&](int t, double v) {
    int i;
    bool isx;
    row(t, i, isx);
    if (isx) dx[i] = v;
    else dy[i] = v;
  });
  for (int i = ex.lane; i < ng + nb; i += ex.nlanes) {
    if (i < ng) dx[gvar(P, i)] = b[i];
    else dy[P.T * NX + i - ng] = b[i];
  }
  ex.sync();
  // dzh = W^-1 G dx - r3h, or (fin) dz = W^-1 dzh, in one pass
  if constexpr (R3ZERO) apply_G<X, NX, NU, 3>(ex, C, dx, dzh, r3h, tr);
  else if (fin) apply_G<X, NX, NU, 2>(ex, C, dx, dzh, r3h, tr);
  else apply_G<X, NX, NU, 1>(ex, C, dx, dzh, r3h, tr);
}

// kkt_back for the pair's two directions (kkt_solve_pair: the c and affine solves) at once:
// each g_k and Woodbury column is loaded once for both; per direction every value is formed as
// kkt_back forms it (same products, same order).  The second right-hand side of the coupling
// solve sits at Plan::lds_rhs2.
template <class X, int NX, int NU, bool R3ZERO = false>
BMPC_HD void kkt_back_pair(const X ex, const Ctx& C, const gdouble* tz1, const gdouble* r21, const gdouble* r3h1,
                           gdouble* dx1, gdouble* dy1, gdouble* dzh1, const gdouble* tz2, const gdouble* r22,
                           const gdouble* r3h2, gdouble* dx2, gdouble* dy2, gdouble* dzh2, bool fin) {
  CPlan& P = *C.P;
  CLayout& L = *C.L;
  BMPC_PROF(C.ws, L, PROF_BACK);
  gdouble* ws = C.ws;
  gdouble* tr = ws + L.k_r0;
  const int ng = P.ng, nb = P.bdim, nc = P.ncones, ns = P.nsm;
  auto* b1 = coup_vec(ex, P.lds_rhs);
  auto* b2 = coup_vec(ex, P.lds_rhs2);
  const gdouble* eta = ws + L.eta;
  if (coup_supp_dots(P)) {   // g_k' dx over each cone's support, sixteen cones per pass
    const auto t = topo_view(P, ex);
    for (int k0 = 0; k0 < nc; k0 += 16) {
      double acc1[16], acc2[16];
      cone_supp_gdx2(ex, P, t, ws + L.gk, P.nv, dx1, dx2, k0, acc1, acc2);
      if (ex.lane == 0)
        for (int a = 0; a < 16 && k0 + a < nc; ++a) {
          b1[ng + nb + k0 + a] = 2.0 / (eta[k0 + a] * eta[k0 + a]) * acc1[a];
          b2[ng + nb + k0 + a] = 2.0 / (eta[k0 + a] * eta[k0 + a]) * acc2[a];
        }
    }
  } else {
    for (int k0 = 0; k0 < nc; k0 += 4) {   // g_k' dx1 and g_k' dx2, four cones per pass
      const int na = nc - k0 < 4 ? nc - k0 : 4;
      double acc[4][4];
      block_dots<2>(ex, ws + L.gk + (size_t)k0 * P.nv, P.nv, na, dx1, (size_t)(dx2 - dx1), 2, 0, P.oRho, P.oS, P.oJ,
                 acc);
      if (ex.lane == 0)
        for (int a = 0; a < na; ++a) {
          b1[ng + nb + k0 + a] = 2.0 / (eta[k0 + a] * eta[k0 + a]) * acc[a][0];
          b2[ng + nb + k0 + a] = 2.0 / (eta[k0 + a] * eta[k0 + a]) * acc[a][1];
        }
    }
  }
  for (int i = ex.lane; i < ng + nb; i += ex.nlanes) {
    b1[i] = i < ng ? tz1[gvar(P, i)] : r21[P.T * NX + i - ng];
    b2[i] = i < ng ? tz2[gvar(P, i)] : r22[P.T * NX + i - ng];
  }
  ex.sync();
  BMPC_TIC(t_lus);
  bool both = false;
#if BMPC_SUBST_REG
  if constexpr (MultiWave<X>::value) {   // both right-hand sides on one wave, their chains interleaved
    if (ns <= 64) {
      decltype(b1) const bs[2] = {b1, b2};
      if (ex.lane < 64) small_lu_solve_wave<2>(ex.lane, coup_mem(ex, ws, L, P, P.lds_M), coup_vec(ex, P.lds_piv), bs, ns);
      ex.sync();
      both = true;
    }
  }
#endif
  if (!both) {
    small_lu_solve(ex, coup_mem(ex, ws, L, P, P.lds_M), coup_vec(ex, P.lds_piv), b1, ns);
    small_lu_solve(ex, coup_mem(ex, ws, L, P, P.lds_M), coup_vec(ex, P.lds_piv), b2, ns);
  }
  BMPC_TOC(C.ws, L, PROF_LUS, t_lus);
  const auto* bc1 = b1 + ng + nb;
  const auto* bc2 = b2 + ng + nb;
  const gdouble* colk = ws + L.colk;
  const gdouble* colnu = ws + L.colnu;
  const int n1 = P.oRho, n2 = n1 + (P.oJ - P.oS), n3 = n2 + P.T * NX;
  auto row = [&](int t, int& i, bool& isx) {
    isx = t < n2;
    i = t < n1 ? t : t < n2 ? P.oS + (t - n1) : t - n2;
  };
  struct V2 { double a, b; };
  lane_batch<4>(ex, 0, n3, [&](int t) {
    int i;
    bool isx;
    row(t, i, isx);
    const gdouble* col = isx ? colk : colnu;
    const size_t cs = isx ? (size_t)P.nv : (size_t)P.neq;
    const gdouble* s1 = isx ? dx1 : dy1;
    const gdouble* s2 = isx ? dx2 : dy2;
    double v1 = s1[i], v2 = s2[i];
    for (int k0 = 0; k0 < nc; k0 += 4) {
      double c4[4], p4[4], q4[4];
#pragma unroll
      for (int a = 0; a < 4; ++a) {
        c4[a] = col[(size_t)(k0 + a < nc ? k0 + a : nc - 1) * cs + i];
        p4[a] = k0 + a < nc ? bc1[k0 + a] : 0.0;
        q4[a] = k0 + a < nc ? bc2[k0 + a] : 0.0;
      }
#pragma unroll
      for (int a = 0; a < 4; ++a) v1 -= p4[a] * c4[a];
#pragma unroll
      for (int a = 0; a < 4; ++a) v2 -= q4[a] * c4[a];
    }
    return V2{v1, v2};
  }, [&](int t, V2 v) {
    int i;
    bool isx;
    row(t, i, isx);
    if (isx) dx1[i] = v.a, dx2[i] = v.b;
    else dy1[i] = v.a, dy2[i] = v.b;
  });
  for (int i = ex.lane; i < ng + nb; i += ex.nlanes) {
    if (i < ng) dx1[gvar(P, i)] = b1[i], dx2[gvar(P, i)] = b2[i];
    else dy1[P.T * NX + i - ng] = b1[i], dy2[P.T * NX + i - ng] = b2[i];
  }
  ex.sync();
  if constexpr (R3ZERO) {
    apply_G<X, NX, NU, 3>(ex, C, dx1, dzh1, r3h1, tr);
    apply_G<X, NX, NU, 3>(ex, C, dx2, dzh2, r3h2, tr);
  } else if (fin) {
    apply_G<X, NX, NU, 2>(ex, C, dx1, dzh1, r3h1, tr);
    apply_G<X, NX, NU, 2>(ex, C, dx2, dzh2, r3h2, tr);
  } else {
    apply_G<X, NX, NU, 1>(ex, C, dx1, dzh1, r3h1, tr);
    apply_G<X, NX, NU, 1>(ex, C, dx2, dzh2, r3h2, tr);
  }
}

template <class X, int NX, int NU>
BMPC_HD void kkt_refine(const X ex, const Ctx& C, const gdouble* r1, const gdouble* r2, const gdouble* r3h,
                        gdouble* dx, gdouble* dy, gdouble* dz, int nitref);

// Solve [0 A' G'; A 0 0; G 0 -W^2] [dx; dy; dz] = [r1; r2; r3]: W-scaled solve with
// iterative refinement on the scaled residual (well conditioned, unlike the W^2 form whose
// residual is dominated by the rounding of W^2 dz near the boundary).
template <class X, int NX, int NU>
BMPC_FN void kkt_solve(const X ex, const Ctx Cin, const gdouble* r1, const gdouble* r2,
                       const gdouble* r3, gdouble* dx, gdouble* dy, gdouble* dz, int nitref) {
  const Ctx C = Cin.uniform();
  CPlan& P = *C.P;
  CLayout& L = *C.L;
  BMPC_PROF(C.ws, L, PROF_KKT);
  gdouble* ws = C.ws;
  gdouble* r3h = ws + L.k_t3;
  apply_Winv2(ex, C, r3, r3h, ws + L.k_r0);      // r3h = W^-1 r3 and kkt_solve_once's W^-1 r3h
  BMPC_COUNT(ws, L, PROF_NSOLVE);
  // without refinement the solve's tail applies the final W^-1 itself
  const bool fin = ex.uniform(nitref == 0);
  kkt_solve_once<X, NX, NU>(ex, C, r1, r2, r3h, dx, dy, dz, true, fin);   // dz holds dzh until the end
  if (fin) return;
  kkt_refine<X, NX, NU>(ex, C, r1, r2, r3h, dx, dy, dz, nitref);
}

// Iterative refinement of a W-scaled solve on its scaled residual (nitref > 0 rounds at most),
// then dz = W^-1 dzh in place (dz holds dzh on entry).
template <class X, int NX, int NU>
BMPC_HD void kkt_refine(const X ex, const Ctx& C, const gdouble* r1, const gdouble* r2, const gdouble* r3h,
                        gdouble* dx, gdouble* dy, gdouble* dz, int nitref) {
  CPlan& P = *C.P;
  CLayout& L = *C.L;
  gdouble* ws = C.ws;
  gdouble* e1 = ws + L.k_e1;
  gdouble* e2 = ws + L.k_e2;
  gdouble* e3 = ws + L.k_e3;
  gdouble* cx = ws + L.k_cx;
  gdouble* cy = ws + L.k_cy;
  gdouble* cz = ws + L.k_cz;
  gdouble* tv = ws + L.k_nv1;
  // the scale max(|r1|, |r2|, |r3h|) and the residual's max norm are taken in the passes that
  // read r1 / r2 and write e1 / e2 (max is exact: the same values as separate passes); the |r3h|
  // part before the first round
  double msc = nitref == 0 ? 0.0 : lane_extreme<8, 1>(ex, 0, P.nrows, [&](int i) { return fabs(r3h[i]); });
  double sc = 0.0, prev = 1e300;
  for (int itr = 0; itr < nitref; ++itr) {
#if defined(BMPC_PROFILE) && defined(__HIP_DEVICE_COMPILE__)
    ProfScope _pr(C.ws, L.prof, PROF_REFINE);
#endif
    double merr = -1e300;
    // e1 = r1 - A'dy - G'W^-1 dzh
    apply_W(ex, C, 1, dz, e3);
    apply_GT<X, NX, NU>(ex, C, e3, tv);
    apply_AT<X, NX, NU>(ex, C, dy, e1);
    lane_batch<16>(ex, 0, P.nv, [&](int i) { const double a = r1[i]; msc = fmax(msc, fabs(a)); return a - e1[i] - tv[i]; },
                   [&](int i, double v) { e1[i] = v; merr = fmax(merr, fabs(v)); });
    // e2 = r2 - A dx
    apply_A<X, NX, NU>(ex, C, dx, e2);
    lane_batch(ex, 0, P.neq, [&](int i) { const double a = r2[i]; msc = fmax(msc, fabs(a)); return a - e2[i]; },
               [&](int i, double v) { e2[i] = v; merr = fmax(merr, fabs(v)); });
    // e3 = r3h - W^-1 G dx + dzh is zero up to rounding: kkt_solve_once computed dzh as
    // W^-1 G dx - r3h from the final dx with the same operators (the correction solve takes
    // r3h = 0 without a vector)
    if (itr == 0) sc = ex.max(msc);
    const double err = ex.max(merr);
    ex.sync();
    BMPC_TRACE("   refine %d err %.3e sc %.3e\n", itr, err, sc);
    if (!(err > BMPC_REFTOL * fmax(sc, 1.0))) break;
    if (BMPC_REF_STALL > 0 && itr > 0) {
      if (ex.uniform(!(err < prev))) {   // the last correction made it worse: undo it (ECOS)
        lane_batch<16>(ex, 0, P.nv, [&](int i) { return dx[i] - cx[i]; }, [&](int i, double v) { dx[i] = v; });
        lane_batch(ex, 0, P.neq, [&](int i) { return dy[i] - cy[i]; }, [&](int i, double v) { dy[i] = v; });
        lane_batch<16>(ex, 0, P.nrows, [&](int i) { return dz[i] - cz[i]; }, [&](int i, double v) { dz[i] = v; });
        ex.sync();
        break;
      }
      if (ex.uniform(prev < BMPC_REF_STALL * err)) break;   // stalled: kept, no further round
    }
    prev = err;
    kkt_solve_once<X, NX, NU, true>(ex, C, e1, e2, nullptr, cx, cy, cz, false, false);
    lane_batch<16>(ex, 0, P.nv, [&](int i) { return dx[i] + cx[i]; }, [&](int i, double v) { dx[i] = v; });
    lane_batch(ex, 0, P.neq, [&](int i) { return dy[i] + cy[i]; }, [&](int i, double v) { dy[i] = v; });
    lane_batch<16>(ex, 0, P.nrows, [&](int i) { return dz[i] + cz[i]; }, [&](int i, double v) { dz[i] = v; });
    ex.sync();
  }
  // dz = W^-1 dzh (in place)
  apply_W(ex, C, 1, dz, dz);
}

// kkt_refine of the pair's two directions in lock step: while both refine, their correction
// solves share one tree solve (two right-hand sides) and one paired back half; a direction whose
// residual met the tolerance stops as kkt_refine stops it.  Each direction's operations are
// kkt_refine's, in the same order (its scratch: the second halves of k_e1 / k_e2 / k_cx /
// k_cy / k_cz).
#if BMPC_REFINE_CALLS
// kkt_refine_pair's correction back halves as calls of their own (a smaller refinement frame on
// the kernel's deepest call chain)
template <class X, int NX, int NU>
BMPC_FN void refine_back_pair(const X ex, const Ctx Cin) {
  const Ctx C = Cin.uniform();
  CPlan& P = *C.P;
  CLayout& L = *C.L;
  gdouble* ws = C.ws;
  const size_t nv = P.nv, neq = P.neq, nr = P.nrows;
  gdouble* cx = ws + L.k_cx;
  gdouble* cy = ws + L.k_cy;
  gdouble* cz = ws + L.k_cz;
  kkt_back_pair<X, NX, NU, true>(ex, C, ws + L.k_e1, ws + L.k_e2, nullptr, cx, cy, cz, ws + L.k_e1 + nv,
                                 ws + L.k_e2 + neq, nullptr, cx + nv, cy + neq, cz + nr, false);
}
template <class X, int NX, int NU>
BMPC_FN void refine_solve_one(const X ex, const Ctx Cin, int j) {
  const Ctx C = Cin.uniform();
  j = ex.uniform(j != 0) ? 1 : 0;
  CPlan& P = *C.P;
  CLayout& L = *C.L;
  gdouble* ws = C.ws;
  const size_t nv = P.nv, neq = P.neq, nr = P.nrows;
  kkt_solve_once<X, NX, NU, true>(ex, C, ws + L.k_e1 + j * nv, ws + L.k_e2 + j * neq, nullptr, ws + L.k_cx + j * nv,
                                  ws + L.k_cy + j * neq, ws + L.k_cz + j * nr, false, false);
}
#endif

template <class X, int NX, int NU>
BMPC_FN void kkt_refine_pair(const X ex, const Ctx Cin, const gdouble* r1a, const gdouble* r2a, const gdouble* r3ha,
                             gdouble* dxa, gdouble* dya, gdouble* dza, const gdouble* r1b, const gdouble* r2b,
                             const gdouble* r3hb, gdouble* dxb, gdouble* dyb, gdouble* dzb, int nitref) {
  const Ctx C = Cin.uniform();
  CPlan& P = *C.P;
  CLayout& L = *C.L;
  gdouble* ws = C.ws;
  const size_t nv = P.nv, neq = P.neq, nr = P.nrows;
  gdouble* e3 = ws + L.k_e3;
  gdouble* tv = ws + L.k_nv1;
  const gdouble* r1[2] = {r1a, r1b};
  const gdouble* r2[2] = {r2a, r2b};
  const gdouble* r3h[2] = {r3ha, r3hb};
  gdouble* dx[2] = {dxa, dxb};
  gdouble* dy[2] = {dya, dyb};
  gdouble* dz[2] = {dza, dzb};
  double sc[2] = {0.0, 0.0};
  double msc[2];
#pragma unroll
  for (int j = 0; j < 2; ++j)   // kkt_refine's scale and residual norms, per direction
    msc[j] = nitref == 0 ? 0.0 : lane_extreme<8, 1>(ex, 0, P.nrows, [&](int i) { return fabs(r3h[j][i]); });
  bool on[2] = {true, true};
  double prev[2] = {1e300, 1e300};
  for (int itr = 0; itr < nitref; ++itr) {
#if defined(BMPC_PROFILE) && defined(__HIP_DEVICE_COMPILE__)
    ProfScope _pr(C.ws, L.prof, PROF_REFINE);
#endif
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      if (!ex.uniform(on[j])) continue;
      gdouble* e1 = ws + L.k_e1 + j * nv;
      gdouble* e2 = ws + L.k_e2 + j * neq;
      double merr = -1e300;
      apply_W(ex, C, 1, dz[j], e3);
      apply_GT<X, NX, NU>(ex, C, e3, tv);
      apply_AT<X, NX, NU>(ex, C, dy[j], e1);
      lane_batch<16>(ex, 0, P.nv, [&](int i) { const double a = r1[j][i]; msc[j] = fmax(msc[j], fabs(a)); return a - e1[i] - tv[i]; },
                     [&](int i, double v) { e1[i] = v; merr = fmax(merr, fabs(v)); });
      apply_A<X, NX, NU>(ex, C, dx[j], e2);
      lane_batch(ex, 0, P.neq, [&](int i) { const double a = r2[j][i]; msc[j] = fmax(msc[j], fabs(a)); return a - e2[i]; },
                 [&](int i, double v) { e2[i] = v; merr = fmax(merr, fabs(v)); });
      if (itr == 0) sc[j] = ex.max(msc[j]);
      const double err = ex.max(merr);
      ex.sync();
      on[j] = ex.uniform(err > BMPC_REFTOL * fmax(sc[j], 1.0));
      BMPC_TRACE("   refine[%d] %d err %.3e sc %.3e\n", j, itr, err, sc[j]);
      if (BMPC_REF_STALL > 0 && itr > 0 && on[j]) {   // kkt_refine's stall rule, per direction
        if (ex.uniform(!(err < prev[j]))) {
          const gdouble* cxj = ws + L.k_cx + j * nv;
          const gdouble* cyj = ws + L.k_cy + j * neq;
          const gdouble* czj = ws + L.k_cz + j * nr;
          lane_batch<16>(ex, 0, P.nv, [&](int i) { return dx[j][i] - cxj[i]; }, [&](int i, double v) { dx[j][i] = v; });
          lane_batch(ex, 0, P.neq, [&](int i) { return dy[j][i] - cyj[i]; }, [&](int i, double v) { dy[j][i] = v; });
          lane_batch<16>(ex, 0, P.nrows, [&](int i) { return dz[j][i] - czj[i]; }, [&](int i, double v) { dz[j][i] = v; });
          ex.sync();
          on[j] = false;
        } else if (ex.uniform(prev[j] < BMPC_REF_STALL * err)) {
          on[j] = false;
        }
      }
      prev[j] = err;
    }
    if (!ex.uniform(on[0] || on[1])) break;
    gdouble* cx = ws + L.k_cx;
    gdouble* cy = ws + L.k_cy;
    gdouble* cz = ws + L.k_cz;
    if (ex.uniform(on[0] && on[1])) {   // both corrections: one tree solve, one back half
      tree_solve<X, NX, NU>(ex, C, 2, ws + L.k_e1, nv, ws + L.k_e2, neq, cx, nv, cy, neq);
#if BMPC_REFINE_CALLS
      refine_back_pair<X, NX, NU>(ex, C);
#else
      kkt_back_pair<X, NX, NU, true>(ex, C, ws + L.k_e1, ws + L.k_e2, nullptr, cx, cy, cz, ws + L.k_e1 + nv,
                                     ws + L.k_e2 + neq, nullptr, cx + nv, cy + neq, cz + nr, false);
#endif
    } else {
      const int j = on[0] ? 0 : 1;
#if BMPC_REFINE_CALLS
      refine_solve_one<X, NX, NU>(ex, C, j);
#else
      kkt_solve_once<X, NX, NU, true>(ex, C, ws + L.k_e1 + j * nv, ws + L.k_e2 + j * neq, nullptr, cx + j * nv,
                                      cy + j * neq, cz + j * nr, false, false);
#endif
    }
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      if (!ex.uniform(on[j])) continue;
      const gdouble* cxj = cx + j * nv;
      const gdouble* cyj = cy + j * neq;
      const gdouble* czj = cz + j * nr;
      lane_batch<16>(ex, 0, P.nv, [&](int i) { return dx[j][i] + cxj[i]; }, [&](int i, double v) { dx[j][i] = v; });
      lane_batch(ex, 0, P.neq, [&](int i) { return dy[j][i] + cyj[i]; }, [&](int i, double v) { dy[j][i] = v; });
      lane_batch<16>(ex, 0, P.nrows, [&](int i) { return dz[j][i] + czj[i]; }, [&](int i, double v) { dz[j][i] = v; });
      ex.sync();
    }
  }
  // dz = W^-1 dzh (in place)
  apply_W(ex, C, 1, dza, dza);
  apply_W(ex, C, 1, dzb, dzb);
}

// The two KKT solves of an IPM iteration that need only the factorisation -- the c direction
// [x1; y1; z1] = K^-1 [r1c; bvec; hvec] and the affine direction [x2; y2; z2] = K^-1 [r1a; ry; rb]
// -- together with the Woodbury columns, in ONE tree solve of nc + 2 right-hand sides
// (kkt_coupling).  Per right-hand side the arithmetic is that of kkt_solve.  Returns false
// when the coupling factorisation breaks down.
template <class X, int NX, int NU>
BMPC_FN bool kkt_solve_pair(const X ex, const Ctx Cin, const gdouble* r1c, const gdouble* r1a, const gdouble* r3a,
                            int nitref) {
  const Ctx C = Cin.uniform();
  r1c = uniform_ptr(r1c), r1a = uniform_ptr(r1a), r3a = uniform_ptr(r3a);
  CPlan& P = *C.P;
  CLayout& L = *C.L;
  BMPC_PROF(C.ws, L, PROF_KKT);
  gdouble* ws = C.ws;
  const size_t nv = P.nv, nc = P.ncones;
  gdouble* tzc = ws + L.gk + nc * nv;
  gdouble* tza = tzc + nv;
  gdouble* r3hc = ws + L.k_t3;
  gdouble* r3ha = ws + L.k_t3b;
  gdouble* tr = ws + L.k_r0;
  const gdouble* bv = ws + L.bvec;
  const gdouble* ry = ws + L.ry;
  apply_Winv2(ex, C, ws + L.hvec, r3hc, tr);
  apply_GT<X, NX, NU>(ex, C, tr, tzc, r1c);
  apply_Winv2(ex, C, r3a, r3ha, tr);
  apply_GT<X, NX, NU>(ex, C, tr, tza, r1a);
  BMPC_COUNT(ws, L, PROF_NSOLVE);
  BMPC_COUNT(ws, L, PROF_NSOLVE);
  if (!ex.uniform(kkt_coupling<X, NX, NU>(ex, C, 2))) return false;
  const bool fin = ex.uniform(nitref == 0);
  gdouble* x1 = ws + L.x1;
  gdouble* y1 = ws + L.y1;
  gdouble* z1 = ws + L.z1;
  gdouble* x2 = ws + L.x2;
  gdouble* y2 = ws + L.y2;
  gdouble* z2 = ws + L.z2;
#if BMPC_PAIR_BACK
  kkt_back_pair<X, NX, NU>(ex, C, tzc, bv, r3hc, x1, y1, z1, tza, ry, r3ha, x2, y2, z2, fin);
#else
  kkt_back<X, NX, NU, false>(ex, C, tzc, bv, r3hc, x1, y1, z1, fin);
  kkt_back<X, NX, NU, false>(ex, C, tza, ry, r3ha, x2, y2, z2, fin);
#endif
  if (fin) return true;
#if BMPC_PAIR_REFINE
  kkt_refine_pair<X, NX, NU>(ex, C, r1c, bv, r3hc, x1, y1, z1, r1a, ry, r3ha, x2, y2, z2, nitref);
#else
  kkt_refine<X, NX, NU>(ex, C, r1c, bv, r3hc, x1, y1, z1, nitref);
  kkt_refine<X, NX, NU>(ex, C, r1a, ry, r3ha, x2, y2, z2, nitref);
#endif
  return true;
}

#if BMPC_FLAT_PAIR
// kkt_solve_pair split so that the IPM loop calls the coupling solve and the pair's refinement
// itself (one call level less on the deepest call chain: the scratch stack is the sum of the
// frames along it): kkt_pair_rhs forms both right-hand sides' W^-1 / G' parts, kkt_pair_back the
// two back halves.  Same operations in the same order as kkt_solve_pair.
template <class X, int NX, int NU>
BMPC_FN void kkt_pair_rhs(const X ex, const Ctx Cin, const gdouble* r1c, const gdouble* r1a, const gdouble* r3a) {
  const Ctx C = Cin.uniform();
  r1c = uniform_ptr(r1c), r1a = uniform_ptr(r1a), r3a = uniform_ptr(r3a);
  CPlan& P = *C.P;
  CLayout& L = *C.L;
  BMPC_PROF(C.ws, L, PROF_KKT);
  gdouble* ws = C.ws;
  const size_t nv = P.nv, nc = P.ncones;
  gdouble* tzc = ws + L.gk + nc * nv;
  gdouble* tza = tzc + nv;
  gdouble* tr = ws + L.k_r0;
  apply_Winv2(ex, C, ws + L.hvec, ws + L.k_t3, tr);
  apply_GT<X, NX, NU>(ex, C, tr, tzc, r1c);
  apply_Winv2(ex, C, r3a, ws + L.k_t3b, tr);
  apply_GT<X, NX, NU>(ex, C, tr, tza, r1a);
  BMPC_COUNT(ws, L, PROF_NSOLVE);
  BMPC_COUNT(ws, L, PROF_NSOLVE);
}
template <class X, int NX, int NU>
BMPC_FN void kkt_pair_back(const X ex, const Ctx Cin, bool fin) {
  const Ctx C = Cin.uniform();
  fin = ex.uniform(fin);
  CPlan& P = *C.P;
  CLayout& L = *C.L;
  BMPC_PROF(C.ws, L, PROF_KKT);
  gdouble* ws = C.ws;
  const size_t nv = P.nv, nc = P.ncones;
  const gdouble* tzc = ws + L.gk + nc * nv;
  const gdouble* tza = tzc + nv;
#if BMPC_PAIR_BACK
  kkt_back_pair<X, NX, NU>(ex, C, tzc, ws + L.bvec, ws + L.k_t3, ws + L.x1, ws + L.y1, ws + L.z1, tza, ws + L.ry,
                           ws + L.k_t3b, ws + L.x2, ws + L.y2, ws + L.z2, fin);
#else
  kkt_back<X, NX, NU, false>(ex, C, tzc, ws + L.bvec, ws + L.k_t3, ws + L.x1, ws + L.y1, ws + L.z1, fin);
  kkt_back<X, NX, NU, false>(ex, C, tza, ws + L.ry, ws + L.k_t3b, ws + L.x2, ws + L.y2, ws + L.z2, fin);
#endif
}
#endif

// ECOS bring2cone: s = r + (1 + alpha) e
template <class X>
BMPC_HD void bring2cone(const X ex, const Ctx& C, const gdouble* r, gdouble* s) {
  CPlan& P = *C.P;
  double alpha = -0.99;
  const double mn = -ex.min(lane_extreme<8, 2>(ex, 0, P.nlp, [&](int i) { return r[i]; }));
  if (P.nlp > 0 && mn >= 0.0 && mn > alpha) alpha = mn;
  {
    double worst = -1e300;   // max over cones of -(r0 - ||r1||) where r0 - ||r1|| <= 0
    BMPC_CONE_ROUNDS(ex, P, G) {
      BMPC_CONE_K(P, G, k, off, q);
      const double ss = ex.gsum(strided_partial<ConeBatch<X>::v>(1 + G.gl, G.cg, q, [&](int i) { return r[off + i] * r[off + i]; }),
                                G.cg);
      const double cres = q > 0 ? r[off] - sqrt(ss) : 1.0;
      if (cres <= 0.0) worst = fmax(worst, -cres);
    }
    worst = ex.max(worst);
    if (worst > alpha) alpha = worst;
  }
  lane_batch<16>(ex, 0, P.nrows, [&](int i) { return r[i]; }, [&](int i, double v) { s[i] = i < P.nlp ? v + 1.0 + alpha : v; });
  ex.sync();
  for (int k = ex.lane; k < P.ncones; k += ex.nlanes) s[topo_view(P, ex).cone_off[k]] = r[topo_view(P, ex).cone_off[k]] + 1.0 + alpha;
  ex.sync();
}

template <class X>
BMPC_HD double vdot(const X ex, const gdouble* a, const gdouble* b, int n) {
  return lane_sum(ex, 0, n, [&](int i) { return a[i] * b[i]; });
}

// a1'b1 (n1 entries) + a2'b2 (n2 entries) in one pass
template <class X>
BMPC_HD double dot2(const X ex, const gdouble* a1, const gdouble* b1, int n1, const gdouble* a2, const gdouble* b2,
                    int n2) {
  return lane_sum(ex, 0, n1 + n2, [&](int i) {
    const bool f = i < n1;
    const int j = f ? i : i - n1;
    return (f ? a1 : a2)[j] * (f ? b1 : b2)[j];
  });
}

// ------------------------------------------------------------------------------------
// ECOS's equilibration (ECOS_setup -> set_equilibration, ECOS 2.0.x equil.c with RUIZ_EQUIL and
// EQUIL_ITERS = 3; restated in oracle/ecos_ipm.py:equilibration).  ECOS runs its IPM on
//   c / xe,  diag(1/ae) A diag(1/xe),  b / ae,  diag(1/ge) G diag(1/xe),  h / ge
// with xe, ae, ge the products over three rounds of sqrt(max-abs) of the current columns of
// [A; G], rows of A and rows of G (the rows of a second-order cone share the SUM of their row
// maxima; a maximum below 1e-6 gives 1).  The (unboosted) entries of A and G are enumerated
// here from the structured operators (apply_A / apply_G and their transposes).
//
// The IPM itself stays in the unscaled variables: with x~ = xe x, y~ = ae y, z~ = ge z, s~ = s / ge
// ECOS's Newton directions, step lengths and its NT scaling's lambda are those of the unscaled
// problem (ge is one value per cone, so the cone scalings commute), so the equilibration only
// enters where ECOS's iteration is not scale-invariant -- the initial point (W = I in the scaled
// variables is W = ge here; bring2cone acts on the scaled vectors) and the norms of the exit
// tests (ipm_solve below).
// ------------------------------------------------------------------------------------

template <class X, int NX, int NU>
BMPC_FN void equilibrate(const X ex, const Ctx Cin) {
  const Ctx C = Cin.uniform();
  CPlan& P = *C.P;
  CLayout& L = *C.L;
  gdouble* ws = C.ws;
  gdouble* xe = ws + L.xeq;
  gdouble* ae = ws + L.aeq;
  gdouble* ge = ws + L.geq;
  gdouble* cm = ws + L.k_nv0;   // this round's column / row maxima (KKT scratch, free before the first solve)
  gdouble* am = ws + L.k_e2;
  gdouble* gm = ws + L.k_r0;
  const auto t = topo_view(P, ex);
  const int Nc = P.Nc, nv = P.nv, neq = P.neq, nr = P.nrows, T = P.T;
  const gdouble* dh = ws + L.dh;
  const gdouble* Ad = ws + L.Ad;
  const gdouble* Bd = ws + L.Bd;
  const gdouble* p = ws + L.p;
  const double Qs = fabs(P.desc.Qslack[1]);
  double qx[NX];
  ctx_qx<NX>(C, qx);
  for (int i = ex.lane; i < nv; i += ex.nlanes) xe[i] = 1.0;
  for (int i = ex.lane; i < neq; i += ex.nlanes) ae[i] = 1.0;
  for (int i = ex.lane; i < nr; i += ex.nlanes) ge[i] = 1.0;
  ex.sync();
  // coefficient of x_{k,j} in Fx row c of state node k (non-terminal k)
  auto fcoef = [&](int k, int c, int j) { return c == 0 ? -dh[k * NX + j] : fxv(P, ex, c - 1, j); };
  // cone k's first-row (F1) variables: cb / ci / c / has children (tail terms of apply_G)
  for (int rnd = 0; rnd < BMPC_EQUIL_ITERS; ++rnd) {
    // ---- G: LP rows -------------------------------------------------------------------------
    for (int i = ex.lane; i < P.nlp; i += ex.nlanes) {
      const double rf = ge[i];
      double m = 0.0;
      if (i >= P.rFx && i < P.rFx + T * Nc) {
        const int it = i - P.rFx, k = it / Nc, c = it % Nc;
        m = 1.0 / (rf * xe[P.oS + it]);
        if (t.x_u[k] >= 0)
          for (int j = 0; j < NX; ++j) m = fmax(m, fabs(fcoef(k, c, j)) / (rf * xe[P.oX + k * NX + j]));
      } else if (i >= P.rPos && i < P.rPos + T * Nc) {
        m = 1.0 / (rf * xe[P.oS + (i - P.rPos)]);
      } else if (i >= P.rFu && i < P.rFu + P.U * P.nFu) {
        const int it = i - P.rFu, u = it / P.nFu, r = it % P.nFu;
        for (int j = 0; j < NU; ++j) m = fmax(m, fabs(fuv(P, ex, r, j)) / (rf * xe[P.oU + u * NU + j]));
      } else {   // risk rows: -rho_b, then -mu+ / -mu-
        const int it = i - P.rRisk;
        m = 1.0 / (rf * xe[it < P.bdim ? P.oRho + it : P.oMup + (it - P.bdim)]);
      }
      gm[i] = m;
    }
    // ---- G: cone rows (one lane per cone: the rows' maxima summed over the cone) --------------
    for (int k = ex.lane; k < P.ncones; k += ex.nlanes) {
      const int off = t.cone_off[k], q = t.cone_q[k], c = t.cone_c[k];
      const double rf = ge[off];   // one factor per cone
      double f1 = 0.0, mid = 0.0;
      if (c >= 0) {
        const int ndx = t.br_ndx[c], ndu = t.br_ndu[c];
        for (int j = 0; j < P.N; ++j) {
          const int xk = ndx + j, uk = ndu + j;
          for (int r = 0; r < NX; ++r) f1 = fmax(f1, 2.0 * fabs(qx[r]) / (rf * xe[P.oX + xk * NX + r]));
          for (int cc = 0; cc < Nc; ++cc) f1 = fmax(f1, Qs / (rf * xe[P.oS + xk * Nc + cc]));
          for (int rr = 0; rr < NX; ++rr) {
            double m = 0.0;
            for (int s2 = 0; s2 < NX; ++s2) m = fmax(m, 2.0 * fabs(w1v(P, ex, rr, s2)) / (rf * xe[P.oX + xk * NX + s2]));
            mid += m;
          }
          for (int rr = 0; rr < NU; ++rr) {
            double m = 0.0;
            for (int s2 = 0; s2 < NU; ++s2) m = fmax(m, 2.0 * fabs(P.Wu[rr * NU + s2]) / (rf * xe[P.oU + uk * NU + s2]));
            mid += m;
          }
        }
        const int cb = t.cone_b[k], ci = t.cone_i[k];
        f1 = fmax(f1, 1.0 / (rf * xe[P.oSig + cb]));
        f1 = fmax(f1, 1.0 / (rf * xe[P.oMup + cb + ci]));
        f1 = fmax(f1, 1.0 / (rf * xe[P.oMum + cb + ci]));
        if (t.br_child0[c] >= 0) f1 = fmax(f1, 1.0 / (rf * xe[P.oRho + c]));
      } else {   // the root cone: the root node's slacks, -J + rho_0, and the root input's Wu rows
        for (int cc = 0; cc < Nc; ++cc) f1 = fmax(f1, Qs / (rf * xe[P.oS + cc]));
        f1 = fmax(f1, 1.0 / (rf * xe[P.oJ]));
        f1 = fmax(f1, 1.0 / (rf * xe[P.oRho]));
        for (int rr = 0; rr < NU; ++rr) {
          double m = 0.0;
          for (int s2 = 0; s2 < NU; ++s2) m = fmax(m, 2.0 * fabs(P.Wu[rr * NU + s2]) / (rf * xe[P.oU + s2]));
          mid += m;
        }
      }
      const double tot = 2.0 * f1 + mid;   // first and last rows (+-F1) and the middle rows
      for (int i = 0; i < q; ++i) gm[off + i] = tot;
    }
    // ---- A rows: dynamics, then the CVaR rows --------------------------------------------------
    for (int i = ex.lane; i < neq; i += ex.nlanes) {
      const double rf = ae[i];
      double m = 0.0;
      if (i < T * NX) {
        const int k = i / NX, r = i % NX;
        m = 1.0 / (rf * xe[P.oX + i]);
        const int su = t.x_srcu[k], sx = t.x_srcx[k];
        if (su >= 0) {
          for (int s2 = 0; s2 < NX; ++s2) m = fmax(m, fabs(Ad[su * NX * NX + r * NX + s2]) / (rf * xe[P.oX + sx * NX + s2]));
          for (int s2 = 0; s2 < NU; ++s2) m = fmax(m, fabs(Bd[su * NX * NU + r * NU + s2]) / (rf * xe[P.oU + su * NU + s2]));
        }
      } else {
        const int b = i - T * NX;
        m = fmax(1.0 / (rf * xe[P.oRho + b]), 1.0 / (rf * xe[P.oSig + b]));
        for (int ii = 0; ii < P.m; ++ii)
          m = fmax(m, fabs(p[b * P.m + ii] / P.desc.ralpha) / (rf * xe[P.oMum + b * P.m + ii]));
      }
      am[i] = m;
    }
    // ---- columns ---------------------------------------------------------------------------------
    for (int col = ex.lane; col < nv; col += ex.nlanes) {
      const double cf = xe[col];
      double m = 0.0;
      if (col >= P.oX && col < P.oX + T * NX) {
        const int k = (col - P.oX) / NX, r = (col - P.oX) % NX;
        if (t.x_u[k] >= 0)
          for (int c = 0; c < Nc; ++c) m = fmax(m, fabs(fcoef(k, c, r)) / (ge[P.rFx + k * Nc + c] * cf));
        const int kc = t.x_cone[k];
        if (kc >= 0) {
          const double rf = ge[t.cone_off[kc]];
          m = fmax(m, 2.0 * fabs(qx[r]) / (rf * cf));
          for (int rr = 0; rr < NX; ++rr) m = fmax(m, 2.0 * fabs(w1v(P, ex, rr, r)) / (rf * cf));
        }
        m = fmax(m, 1.0 / (ae[k * NX + r] * cf));
        const int u = t.x_u[k];
        if (u >= 0)
          for (int e = t.succ_off[k]; e < t.succ_off[k + 1]; ++e) {
            const int kn = t.succ[e];
            for (int rr = 0; rr < NX; ++rr) m = fmax(m, fabs(Ad[u * NX * NX + rr * NX + r]) / (ae[kn * NX + rr] * cf));
          }
      } else if (col >= P.oU && col < P.oU + P.U * NU) {
        const int u = (col - P.oU) / NU, s2 = (col - P.oU) % NU;
        for (int r = 0; r < P.nFu; ++r) m = fmax(m, fabs(fuv(P, ex, r, s2)) / (ge[P.rFu + u * P.nFu + r] * cf));
        const int kc = t.u_cone[u];
        if (kc >= 0) {
          const double rf = ge[t.cone_off[kc]];
          for (int rr = 0; rr < NU; ++rr) m = fmax(m, 2.0 * fabs(P.Wu[rr * NU + s2]) / (rf * cf));
        }
        const int k = t.u_x[u];
        for (int e = t.succ_off[k]; e < t.succ_off[k + 1]; ++e) {
          const int kn = t.succ[e];
          for (int rr = 0; rr < NX; ++rr) m = fmax(m, fabs(Bd[u * NX * NU + rr * NU + s2]) / (ae[kn * NX + rr] * cf));
        }
      } else if (col >= P.oS && col < P.oS + T * Nc) {
        const int it = col - P.oS, k = it / Nc;
        m = fmax(1.0 / (ge[P.rFx + it] * cf), 1.0 / (ge[P.rPos + it] * cf));
        const int kc = t.x_cone[k] >= 0 ? t.x_cone[k] : (k == 0 ? P.ncones - 1 : -1);
        if (kc >= 0) m = fmax(m, Qs / (ge[t.cone_off[kc]] * cf));
      } else {   // the globals: risk row, the cones' first rows, the CVaR equality rows
        if (col < P.oSig) m = 1.0 / (ge[P.rRisk + (col - P.oRho)] * cf);
        else if (col >= P.oMup && col < P.oS) m = 1.0 / (ge[P.rRisk + P.bdim + (col - P.oMup)] * cf);
        for (int k = 0; k < P.ncones; ++k) {
          const int c = t.cone_c[k];
          bool on = false;
          if (c >= 0) {
            const int b = t.cone_b[k], ii = t.cone_i[k];
            on = col == P.oSig + b || col == P.oMup + b + ii || col == P.oMum + b + ii ||
                 (t.br_child0[c] >= 0 && col == P.oRho + c);
          } else {
            on = col == P.oJ || col == P.oRho;
          }
          if (on) m = fmax(m, 1.0 / (ge[t.cone_off[k]] * cf));
        }
        if (col < P.oMup) {   // rho_b, sigma_b: +1 in CVaR row b
          const int b = col < P.oSig ? col - P.oRho : col - P.oSig;
          m = fmax(m, 1.0 / (ae[T * NX + b] * cf));
        } else if (col >= P.oMum && col < P.oS) {
          const int j = col - P.oMum;
          m = fmax(m, fabs(p[j] / P.desc.ralpha) / (ae[T * NX + j / P.m] * cf));
        }
      }
      cm[col] = m;
    }
    ex.sync();
    auto fac = [](double v) { return fabs(v) < 1e-6 ? 1.0 : sqrt(v); };
    for (int i = ex.lane; i < nv; i += ex.nlanes) xe[i] *= fac(cm[i]);
    for (int i = ex.lane; i < neq; i += ex.nlanes) ae[i] *= fac(am[i]);
    for (int i = ex.lane; i < nr; i += ex.nlanes) ge[i] *= fac(gm[i]);
    ex.sync();
  }
}

struct IpmResult {
  int exit_flag;
  int iters;
  double pcost;
};

// ------------------------------------------------------------------------------------
// the HSDE interior-point loop (ECOS algorithm; oracle/ecos_ipm.py is its CPU restatement)
// ------------------------------------------------------------------------------------
template <class X, int NX, int NU>
BMPC_HD IpmResult ipm_solve(const X ex, const Ctx& C) {
  CPlan& P = *C.P;
  CLayout& L = *C.L;
  gdouble* ws = C.ws;
  const int nv = P.nv, neq = P.neq, nr = P.nrows;
  gdouble* x = ws + L.x;
  gdouble* y = ws + L.y;
  gdouble* z = ws + L.z;
  gdouble* s = ws + L.s;
  gdouble* lam = ws + L.lam;
  gdouble* x1 = ws + L.x1;
  gdouble* y1 = ws + L.y1;
  gdouble* z1 = ws + L.z1;
  gdouble* x2 = ws + L.x2;
  gdouble* y2 = ws + L.y2;
  gdouble* z2 = ws + L.z2;
  gdouble* dz = ws + L.dz;
  gdouble* ds = ws + L.ds;
  gdouble* rx = ws + L.rx;
  gdouble* ry = ws + L.ry;
  gdouble* rz = ws + L.rz;
  gdouble* hv = ws + L.hvec;
  gdouble* bv = ws + L.bvec;
  gdouble* tA = ws + L.ta;
  gdouble* tA2 = ws + L.ta2;
  gdouble* ya = ws + L.ya;
  gdouble* ra = ws + L.ra;
  gdouble* rb = ws + L.rb;
  gdouble* rc = ws + L.rc;
  const double feastol = P.desc.feastol, abstol = P.desc.abstol, reltol = P.desc.reltol;
  const double deg = (double)(P.nlp + P.ncones);
  IpmResult res{EXIT_MAXIT, 0, 0.0};
  BMPC_PROF(ws, L, PROF_TOTAL);
  BMPC_TIC(t_init);

  // ECOS's equilibration factors (all 1 without it): the exit tests' norms are those of the
  // equilibrated residuals and iterates -- ||r_x / xe||, ||r_y / ae||, ||r_z / ge||, ||xe x||, ||ae y||,
  // ||ge z||, ||s / ge|| -- and the initial point is ECOS's in the equilibrated variables
  const gdouble* xq = ws + L.xeq;
  const gdouble* aq = ws + L.aeq;
  const gdouble* gq = ws + L.geq;
  if (BMPC_EQUIL) equilibrate<X, NX, NU>(ex, C);
  build_hb<X, NX, NU>(ex, C, hv, bv);
  // ---- initial point with W = I (of the equilibrated variables) ----------------------------
  identity_scaling(ex, C);
  if (!kkt_factor<X, NX, NU>(ex, C, true) || !kkt_coupling<X, NX, NU>(ex, C, 0)) {
    res.exit_flag = EXIT_NUMERICS;
    return res;
  }
  lane_batch<16>(ex, 0, nv, [&](int i) { return 0.0; }, [&](int i, double v) { tA[i] = v; });
  ex.sync();
  kkt_solve<X, NX, NU>(ex, C, tA, bv, hv, x, y2, z2, BMPC_NITREF_INIT);
  // s = ge bring2cone(-ge z)  (ECOS: s~ = bring2cone(-z~), z~ = ge z, s = ge s~)
  lane_batch<16>(ex, 0, nr, [&](int i) { return -(BMPC_EQUIL ? gq[i] : 1.0) * z2[i]; }, [&](int i, double v) { ra[i] = v; });
  ex.sync();
  bring2cone(ex, C, ra, s);
  if (BMPC_EQUIL) {
    lane_batch<16>(ex, 0, nr, [&](int i) { return gq[i] * s[i]; }, [&](int i, double v) { s[i] = v; });
    ex.sync();
  }
  lane_batch<16>(ex, 0, nv, [&](int i) { return i == P.oJ ? -1.0 : 0.0; }, [&](int i, double v) { tA[i] = v; });
  lane_batch(ex, 0, neq, [&](int i) { return 0.0; }, [&](int i, double v) { ya[i] = v; });
  lane_batch<16>(ex, 0, nr, [&](int i) { return 0.0; }, [&](int i, double v) { ra[i] = v; });
  ex.sync();
  kkt_solve<X, NX, NU>(ex, C, tA, ya, ra, x2, y, z2, BMPC_NITREF_INIT);
  // z = bring2cone(ge z) / ge
  if (BMPC_EQUIL) {
    lane_batch<16>(ex, 0, nr, [&](int i) { return gq[i] * z2[i]; }, [&](int i, double v) { z2[i] = v; });
    ex.sync();
  }
  bring2cone(ex, C, z2, z);
  if (BMPC_EQUIL) {
    lane_batch<16>(ex, 0, nr, [&](int i) { return z[i] / gq[i]; }, [&](int i, double v) { z[i] = v; });
    ex.sync();
  }
  double tau = 1.0, kap = 1.0;
  // max(1, ||c~||), c~ = e_J / xe_J;  max(1, ||b / ae||);  max(1, ||h / ge||)
  const double resx0 = BMPC_EQUIL ? fmax(1.0, 1.0 / xq[P.oJ]) : 1.0;
  const double resy0 = fmax(1.0, sqrt(lane_sum(ex, 0, neq, [&](int i) {
    const double v = BMPC_EQUIL ? bv[i] / aq[i] : bv[i];
    return v * v;
  })));
  const double resz0 = fmax(1.0, sqrt(lane_sum(ex, 0, nr, [&](int i) {
    const double v = BMPC_EQUIL ? hv[i] / gq[i] : hv[i];
    return v * v;
  })));
  double best_score = 1e300, best_tau = 1.0;
  int best_it = 0;
  BMPC_TOC(ws, L, PROF_INIT, t_init);
  double bs_pres = 0, bs_dres = 0, bs_relgap = 0, bs_gap = 0, bs_pcost = 0;
  bool bs_ok_cx = false;

  for (int it = 0; it <= P.desc.maxit; ++it) {
#if defined(BMPC_PROFILE) && defined(__HIP_DEVICE_COMPILE__)
    {   // probe: latency of one dependent global load under the kernel's own load
      BMPC_TIC(t_lat);
      const double probe = *(volatile const gdouble*)(ws + L.bestx + ex.lane);
      if (probe == 1.2345e300) ws[L.prof + PROF_STEP] += 0.0;
      BMPC_TOC(ws, L, PROF_STEP, t_lat);
    }
#endif
    BMPC_TIC(t_res);
    // residuals
    apply_AT<X, NX, NU>(ex, C, y, rx);
    apply_GT<X, NX, NU>(ex, C, z, tA);
    // the norms and dot products are accumulated in the passes that produce rx, ry, rz
    double acx[2] = {0.0, 0.0}, acy[3] = {0.0, 0.0, 0.0}, acz[5] = {0.0, 0.0, 0.0, 0.0, 0.0};
    // each pass also forms its residual's and iterate's equilibrated norms (r / xe, xe x, ...)
    struct R2b { double v, rs, xs; };
    lane_batch<8>(ex, 0, nv, [&](int i) {
      const double xi = x[i], q = BMPC_EQUIL ? xq[i] : 1.0;
      const double v = rx[i] + (tA[i] + (i == P.oJ ? tau : 0.0));
      return R2b{v, v / q, q * xi};
    }, [&](int i, R2b r) { rx[i] = r.v; acx[0] += r.rs * r.rs; acx[1] += r.xs * r.xs; });
    apply_A<X, NX, NU>(ex, C, x, ry);
    struct R4 { double v, rs, a, ys; };
    lane_batch<8>(ex, 0, neq, [&](int i) {
      const double yi = y[i], bi = bv[i], q = BMPC_EQUIL ? aq[i] : 1.0;
      const double v = bi * tau - ry[i];
      return R4{v, v / q, bi * yi, q * yi};
    }, [&](int i, R4 r) { ry[i] = r.v; acy[0] += r.rs * r.rs; acy[1] += r.a; acy[2] += r.ys * r.ys; });
    apply_G<X, NX, NU>(ex, C, x, rz);
    struct R7 { double v, rs, a, zs, ss, sz; };
    lane_batch<4>(ex, 0, nr, [&](int i) {
      const double zi = z[i], si = s[i], hi = hv[i], q = BMPC_EQUIL ? gq[i] : 1.0;
      const double v = hi * tau - rz[i] - si;
      return R7{v, v / q, hi * zi, q * zi, si / q, si * zi};
    }, [&](int i, R7 r) { rz[i] = r.v; acz[0] += r.rs * r.rs; acz[1] += r.a; acz[2] += r.zs * r.zs; acz[3] += r.ss * r.ss; acz[4] += r.sz; });
    ex.sync();
    const double cx = x[P.oJ];
    // the ten sums in one reduction (one barrier pair on a multi-wave executor)
    double rsum[10] = {acy[1], acz[1], acx[1], acy[2], acz[2], acz[3], acz[4], acy[0], acz[0], acx[0]};
    ex.template sum_n<10>(rsum);
    const double by = rsum[0], hz = rsum[1];
    const double rt = kap + cx + by + hz;
    const double nx = sqrt(rsum[2]), ny = sqrt(rsum[3]);
    const double nz = sqrt(rsum[4]), ns = sqrt(rsum[5]);
    const double sz = rsum[6];
    const double mu = (sz + kap * tau) / (deg + 1.0);
    const double gap = sz / (tau * tau);
    const double pcost = cx / tau, dcost = -(hz + by) / tau;
    double relgap = -1.0;   // -1 = NaN
    if (pcost < 0.0) relgap = gap / (-pcost);
    else if (dcost > 0.0) relgap = gap / dcost;
    const double nry = neq ? sqrt(rsum[7]) / fmax(resy0 + nx, 1.0) : 0.0;
    const double nrz = sqrt(rsum[8]) / fmax(resz0 + nx + ns, 1.0);
    const double pres = fmax(nry, nrz) / tau;
    const double dres = sqrt(rsum[9]) / fmax(resx0 + ny + nz, 1.0) / tau;
    BMPC_TOC(ws, L, PROF_RESID, t_res);
    // infeasibility certificates (only evaluated when their preconditions hold)
    double pinfres = -1.0, dinfres = -1.0;
    if ((hz + by) / fmax(ny + nz, 1.0) < -reltol) {
      lane_batch<16>(ex, 0, nv, [&](int i) { return (rx[i] - (i == P.oJ ? tau : 0.0)) / (BMPC_EQUIL ? xq[i] : 1.0); },
                     [&](int i, double v) { ra[i] = v; });
      ex.sync();
      pinfres = sqrt(vdot(ex, ra, ra, nv)) / fmax(ny + nz, 1.0);
    }
    if (cx / fmax(nx, 1.0) < -reltol) {
      apply_A<X, NX, NU>(ex, C, x, rb);
      const double a1 = sqrt(lane_sum(ex, 0, neq, [&](int i) {
        const double v = rb[i] / (BMPC_EQUIL ? aq[i] : 1.0);
        return v * v;
      })) / fmax(nx, 1.0);
      apply_G<X, NX, NU>(ex, C, x, ra);
      lane_batch<16>(ex, 0, nr, [&](int i) { return (ra[i] + s[i]) / (BMPC_EQUIL ? gq[i] : 1.0); },
                     [&](int i, double v) { ra[i] = v; });
      ex.sync();
      const double a2 = sqrt(vdot(ex, ra, ra, nr)) / fmax(nx + ns, 1.0);
      dinfres = fmax(a1, a2);
    }
    auto check = [&](double ft, double at, double rtl) -> int {
      if (!(tau > 0.0 && kap >= 0.0)) return 99;
      if ((-cx > 0.0 || -by - hz >= -at) && pres < ft && dres < ft &&
          (gap < at || (relgap >= 0.0 && relgap < rtl)))
        return EXIT_OPTIMAL;
      if (dinfres >= 0.0 && dinfres < ft && tau < kap) return EXIT_DINF;
      if ((pinfres >= 0.0 && pinfres < ft && tau < kap) ||
          (tau < ft && kap < ft && pinfres >= 0.0 && pinfres < ft))
        return EXIT_PINF;
      return 99;
    };
    const double score = fmax(fmax(pres, dres), relgap >= 0.0 ? relgap : 1e300);
    if (score < best_score) {
      best_score = score;
      best_it = it;
      best_tau = tau;
      bs_pres = pres, bs_dres = dres, bs_relgap = relgap, bs_gap = gap, bs_pcost = pcost;
      bs_ok_cx = (-cx > 0.0 || -by - hz >= -5e-5);
      if (ex.lane == 0) {   // mirror for the guard below
        ws[L.misc + MISC_BEST] = best_score;
        ws[L.misc + MISC_BEST + 1] = best_tau;
      }
      lane_batch<16>(ex, 0, nv, [&](int i) { return x[i]; }, [&](int i, double v) { ws[L.bestx + i] = v; });
      ex.sync();
    }
    BMPC_TRACE("it %3d pcost %+.16e dcost %+.16e gap %.16e pres %.16e dres %.16e kap %.16e tau %.16e"
               " nx %.16e ny %.16e nz %.16e ns %.16e best %.3e\n",
               it, pcost, dcost, gap, pres, dres, kap, tau, nx, ny, nz, ns, best_score);
    int code = check(feastol, abstol, reltol);
    if (code == 99 && it == P.desc.maxit) {
      const int c2 = check(1e-4, 5e-5, 5e-5);
      code = c2 == 99 ? EXIT_MAXIT : c2 + EXIT_INACC;
    }
    if (code != 99) BMPC_TRACE("   code %d (it %d)\n", code, it);
    if (code != 99) {
      lane_batch<16>(ex, 0, nv, [&](int i) { return x[i] / tau; }, [&](int i, double v) { ws[L.sol + i] = v; });
      ex.sync();
      res.exit_flag = code;
      res.iters = it;
      res.pcost = pcost;
      return res;
    }
    // ---- Newton step ---------------------------------------------------------------------
    // the phase results are wave-uniform (each ends in a wave reduction); ex.uniform makes the
    // branches scalar, so no phase is ever called under a partial exec mask
    bool ok = ex.uniform(compute_scaling(ex, C, s, z));
    if (ok) ok = ex.uniform(kkt_factor<X, NX, NU>(ex, C, false));
    double alpha = 0.0, dtau = 0.0, dkap = 0.0;
    // refinement only once the iterate nears the tolerances: an unrefined direction is
    // accurate to ~1e-12 relative, far below what the early steps need
    const int nref = score < BMPC_REFSCORE2 ? BMPC_NITREF2 : score < BMPC_REFSCORE ? BMPC_NITREF : 0;
    if (ok) {
      // right-hand sides of the c direction (-c, bvec, hvec) and the affine direction
      // (-rx, ry, rb = rz - W xi = rz + W lam for xi = -lam), solved together with the
      // Woodbury columns (kkt_solve_pair)
      lane_batch<16>(ex, 0, nv, [&](int i) { return i == P.oJ ? -1.0 : 0.0; }, [&](int i, double v) { tA[i] = v; });
      lane_batch<16>(ex, 0, nv, [&](int i) { return -rx[i]; }, [&](int i, double v) { tA2[i] = v; });
      apply_W(ex, C, 0, lam, rb, 1.0, rz, 1.0);
#if BMPC_FLAT_PAIR
      kkt_pair_rhs<X, NX, NU>(ex, C, tA, tA2, rb);
      ok = ex.uniform(kkt_coupling<X, NX, NU>(ex, C, 2));
      if (ok) {
        kkt_pair_back<X, NX, NU>(ex, C, nref == 0);
        if (nref > 0) {
#if BMPC_PAIR_REFINE
          kkt_refine_pair<X, NX, NU>(ex, C, tA, bv, ws + L.k_t3, x1, y1, z1, tA2, ry, ws + L.k_t3b, x2, y2, z2, nref);
#else
          kkt_refine<X, NX, NU>(ex, C, tA, bv, ws + L.k_t3, x1, y1, z1, nref);
          kkt_refine<X, NX, NU>(ex, C, tA2, ry, ws + L.k_t3b, x2, y2, z2, nref);
#endif
        }
      }
#else
      ok = ex.uniform(kkt_solve_pair<X, NX, NU>(ex, C, tA, tA2, rb, nref));
#endif
    }
    if (ok) {
      const double den = kap / tau - (x1[P.oJ] + dot2(ex, bv, y1, neq, hv, z1, nr));
      const double dk_aff = -kap * tau;
      const double dtau_a = (rt + dk_aff / tau + x2[P.oJ] + dot2(ex, bv, y2, neq, hv, z2, nr)) / den;
      // dz_aff = z2 + dtau_a z1, rb = W dz_aff, ds = dsW_aff = xi - W dz_aff (one pass)
      affine_dirs(ex, C, z2, z1, dtau_a, lam, rb, ds);
      const double dkap_a = (dk_aff - kap * dtau_a) / tau;
      double a_aff = max_step2(ex, C, lam, ds, rb);
      if (dtau_a < 0.0) a_aff = fmin(a_aff, -tau / dtau_a);
      if (dkap_a < 0.0) a_aff = fmin(a_aff, -kap / dkap_a);
      a_aff = fmax(0.0, fmin(a_aff, 0.999));
      double sigma = (1.0 - a_aff) * (1.0 - a_aff) * (1.0 - a_aff);
      sigma = fmin(1.0, fmax(1e-4, sigma));
      const double eta1 = 1.0 - sigma;
      // combined: ds_comb = -lam o lam - dsW_a o Wdz_a + sigma mu e, xi = lam \ ds_comb (kept in
      // ds), rb = eta1 rz - W xi (one pass)
      combined_rhs(ex, C, lam, ds, rb, rz, sigma * mu, eta1);
      lane_batch<16>(ex, 0, nv, [&](int i) { return -eta1 * rx[i]; }, [&](int i, double v) { tA[i] = v; });
      lane_batch(ex, 0, neq, [&](int i) { return eta1 * ry[i]; }, [&](int i, double v) { ya[i] = v; });
      ex.sync();
      kkt_solve<X, NX, NU>(ex, C, tA, ya, rb, x2, y2, z2, nref);
      const double dk_c = -kap * tau - dtau_a * dkap_a + sigma * mu;
      dtau = (eta1 * rt + dk_c / tau + x2[P.oJ] + dot2(ex, bv, y2, neq, hv, z2, nr)) / den;
      double nonfinite = 0.0;   // the step's finiteness check, taken in the pass that forms dx
      lane_batch<8>(ex, 0, nv, [&](int i) { return x2[i] + (dtau * x1[i]); }, [&](int i, double v) {
        x2[i] = v;
        if (!isfinite(v)) nonfinite = 1.0;
      });
      lane_batch(ex, 0, neq, [&](int i) { return y2[i] + (dtau * y1[i]); }, [&](int i, double v) { y2[i] = v; });
      ex.sync();
      // dz = z2 + dtau z1, rb = W dz, ds = dsW = xi - W dz, rc = W dsW = ds (one pass)
      combined_dirs(ex, C, z2, z1, dtau, ds, rb, rc);
      dkap = (dk_c - kap * dtau) / tau;
      double a = max_step2(ex, C, lam, ds, rb);
      if (dtau < 0.0) a = fmin(a, -tau / dtau);
      if (dkap < 0.0) a = fmin(a, -kap / dkap);
      a = fmin(a, 0.999);
      alpha = a * 0.99;           // never step onto or past the cone / tau / kappa boundary
      const double fin = ex.max(nonfinite);
      ok = ex.uniform(fin == 0.0 && isfinite(dtau) && alpha > 1e-10);
      BMPC_TRACE("   step den %.16e dtau_a %.16e a_aff %.16e sigma %.16e dtau %.16e alpha %.16e nref %d ok %d\n",
                 den, dtau_a, a_aff, sigma, dtau, alpha, nref, (int)ok);
      if (ok) {
        lane_batch<8>(ex, 0, nv, [&](int i) { return x[i] + (alpha * x2[i]); }, [&](int i, double v) { x[i] = v; });
        lane_batch(ex, 0, neq, [&](int i) { return y[i] + (alpha * y2[i]); }, [&](int i, double v) { y[i] = v; });
        struct ZS { double z, s; };
        lane_batch<4>(ex, 0, nr, [&](int i) { return ZS{z[i] + alpha * z2[i], s[i] + alpha * rc[i]}; },
                   [&](int i, ZS v) { z[i] = v.z; s[i] = v.s; });
        tau += alpha * dtau;
        kap += alpha * dkap;
        ex.sync();
      }
    }
    if (!ok) {   // numerical failure: ECOS backtracks to the best iterate
      BMPC_TRACE("   backtrack (it %d) to the best iterate (it %d, score %.3e)\n", it, best_it, best_score);
      // guard: the best iterate's score and tau are held in registers across every phase call
      // of the loop; a build whose register allocation lost them is reported
      // as EXIT_GUARD instead of returning a wrong point
      if (best_score < 1e300 && (ws[L.misc + MISC_BEST] != best_score || ws[L.misc + MISC_BEST + 1] != best_tau)) {
        res.exit_flag = EXIT_GUARD;
        res.iters = it;
        return res;
      }
      const bool inacc = bs_ok_cx && bs_pres < 1e-4 && bs_dres < 1e-4 &&
                         (bs_gap < 5e-5 || (bs_relgap >= 0.0 && bs_relgap < 5e-5));
      lane_batch<16>(ex, 0, nv, [&](int i) { return ws[L.bestx + i] / best_tau; }, [&](int i, double v) { ws[L.sol + i] = v; });
      ex.sync();
      res.exit_flag = inacc ? EXIT_OPTIMAL + EXIT_INACC : EXIT_NUMERICS;
      res.iters = it;
      res.pcost = bs_pcost;
      (void)best_it;
      return res;
    }
  }
  return res;
}

}  // namespace bmpc
