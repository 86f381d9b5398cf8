// bmpc_solve.h -- one controller solve of one ego: tree update -> IPM -> unpack.
//
// BranchMPC_CVaR.solve (MPC_branch.py:2043-2092): xRef update, inittree/updatetree,
// (re)assembly, ecos.solve, unpackSolution (:2096-2106) with the "keep the previous
// solution when infeasible" rule, OldInput = uPred[0].
#pragma once

#include "bmpc_ipm.h"
#include "bmpc_qp.h"

namespace bmpc {

// once per solve, before the IPM: the first solve freezes Jcons = xRef Q xRef
// (MPC_branch.py:1939); transform plans write their state rows Fx S / bx (below)
template <class X, class M>
BMPC_HD void ipm_prelude(const X& ex, const Plan& P, const Layout& L, double* ws) {
  constexpr int NX = M::NX;
  const bool init = ws[L.misc + MISC_INIT] != 0.0;
  const double* xref = ws + L.xref;
  if (!init && ex.lane == 0) {
    double j = 0.0;
    for (int c = 0; c < NX; ++c) {
      double v = 0.0;
      for (int r = 0; r < NX; ++r) v += xref[r] * P.desc.Q[r * NX + c];
      j += v * xref[c];
    }
    ws[L.misc + MISC_JCONS] = j;
  }
  if constexpr (X::kTransform) {
    // State rows and their bound: Fx S / bx (Fx without S) from the current Fx and bx, written
    // by buildIneqConstr on the first solve (MPC_branch.py:1894-1901) and by updateIneqConstr
    // only while S is on (:2025-2036) -- with S off a later solve keeps the rows it finds
    // (:2016-2024 patch the collision row alone).
    double* xf = ws + L.xform;
    const bool son = xf[XF_SON] != 0.0, bxset = xf[XF_BXSET] != 0.0, fxset = xf[XF_FXSET] != 0.0;
    const bool rewrite = !init || son || xf[XF_ROWSET] == 0.0;
    const double* S = xf + XF_S;
    const int nF = P.nFx;
    if (rewrite) {
      for (int i = ex.lane; i < nF * NX + nF; i += ex.nlanes) {
        if (i < nF * NX) {
          const int r = i / NX, j = i % NX;
          const double* Fr = fxset ? xf + XF_FX + r * NX : P.desc.Fx + r * NX;
          double v = Fr[j];
          if (son) {
            v = 0.0;
            for (int k = 0; k < NX; ++k) v += Fr[k] * S[k * NX + j];
          }
          xf[XF_ROWS + i] = v;
        } else {
          const int r = i - nF * NX;
          xf[XF_BROWS + r] = bxset ? xf[XF_BX + r] : P.desc.bx[r];
        }
      }
      ex.sync();
      if (ex.lane == 0) xf[XF_ROWSET] = 1.0;
    }
  }
  ex.sync();
}

// per-ego constants of this solve in the wave's LDS (X::kTransform): the state rows written by
// ipm_prelude, W1 S (W1 without S) for the cone rows on every solve (:1935-1937, :1995-1998),
// (W1 S)'(W1 S) and bx.  Every kernel that runs a part of the IPM forms them on entry.
template <class X, class M>
BMPC_HD void ipm_eco(const X& ex, const Plan& P, const Layout& L, const double* ws) {
  constexpr int NX = M::NX;
  if constexpr (X::kTransform) {
    const double* xf = ws + L.xform;
    const bool son = xf[XF_SON] != 0.0;
    const double* S = xf + XF_S;
    const int nF = P.nFx;
    for (int i = ex.lane; i < nF * NX + 2 * NX * NX + nF; i += ex.nlanes) {
      double v;
      if (i < nF * NX) {
        ex.eco[ECO_FX + i] = xf[XF_ROWS + i];
      } else if (i < nF * NX + NX * NX) {
        const int q = i - nF * NX, r = q / NX, j = q % NX;
        v = P.W1[r * NX + j];
        if (son) {
          v = 0.0;
          for (int k = 0; k < NX; ++k) v += P.W1[r * NX + k] * S[k * NX + j];
        }
        ex.eco[ECO_W1 + q] = v;
      } else if (i < nF * NX + 2 * NX * NX) {
        const int q = i - nF * NX - NX * NX, a = q / NX, b = q % NX;
        v = P.QQ[a * NX + b];
        if (son) {
          v = 0.0;
          for (int r = 0; r < NX; ++r) {
            double wa = 0.0, wb = 0.0;
            for (int k = 0; k < NX; ++k) {
              wa += P.W1[r * NX + k] * S[k * NX + a];
              wb += P.W1[r * NX + k] * S[k * NX + b];
            }
            v += wa * wb;
          }
        }
        ex.eco[ECO_QQ + q] = v;
      } else {
        const int r = i - nF * NX - 2 * NX * NX;
        ex.eco[ECO_BX + r] = xf[XF_BROWS + r];
      }
    }
  }
  ex.sync();
}

// unpackSolution (MPC_branch.py:2096-2106) with the "keep the previous solution when
// infeasible" rule, OldInput = uPred[0]
template <class X, class M>
BMPC_HD void ipm_unpack(const X& ex, const Plan& P, const Layout& L, double* ws, const IpmResult& r) {
  constexpr int NX = M::NX, NU = M::NU;
  const double* sol = ws + L.sol;
  const bool feasible = r.exit_flag >= 0;
  if (feasible) {
    for (int i = ex.lane; i < P.U * NU; i += ex.nlanes) {
      const double v = sol[P.oU + i];
      ws[L.upred + i] = v;
      ws[L.uLin + i] = v;
    }
    for (int i = ex.lane; i < NU; i += ex.nlanes) ws[L.uLin + P.U * NU + i] = sol[P.oU + (P.U - 1) * NU + i];
    for (int i = ex.lane; i < P.T * NX; i += ex.nlanes) ws[L.xpred + i] = sol[P.oX + i];
  }
  for (int i = ex.lane; i < P.bdim * P.m; i += ex.nlanes) ws[L.pprev + i] = ws[L.p + i];
  ex.sync();
  if (ex.lane == 0) {
    ws[L.misc + MISC_INIT] = 1.0;
    for (int i = 0; i < NU; ++i) ws[L.misc + MISC_OLDU + i] = ws[L.upred + i];
  }
  ex.sync();
}

// phase 2: IPM + unpack (reads the tree written by tree_update; xref copied there)
template <class X, class M>
BMPC_HD IpmResult solve_ego_ipm(const X& ex, const Plan& P, const Layout& L, EgoView E) {
  constexpr int NX = M::NX, NU = M::NU;
  double* ws = E.ws;
  ipm_prelude<X, M>(ex, P, L, ws);
  ipm_eco<X, M>(ex, P, L, ws);
  Ctx C;
  C.P = (CPlan*)&P;
  C.L = (CLayout*)&L;
  C.ws = (gdouble*)ws;
  IpmResult r = ipm_solve<X, NX, NU>(ex, C);
  ipm_unpack<X, M>(ex, P, L, ws, r);
  return r;
}

template <class X, class M>
BMPC_HD IpmResult solve_ego(const X& ex, const Plan& P, const Layout& L, EgoView E,
                            const double* x, const double* z, const double* xref) {
  tree_step<X, M>(ex, P, L, E, x, z, xref);
  if (P.desc.controller != BMPC_CTRL_CVAR) return solve_ego_qp<X, M>(ex, P, L, E);
  return solve_ego_ipm<X, M>(ex, P, L, E);
}

// bmpc_model_eval for one point
template <class M>
BMPC_HD void model_eval_point(const bmpc_plan_desc& D, const bmpc_policy* pol, const double* x,
                              const double* u, const double* z, double* A, double* Bm, double* C,
                              double* xp, double* p, double* dp, double* zpred, double* h0,
                              double* dh, const LaneRef& R = LaneRef{}) {
  constexpr int NX = M::NX, NU = M::NU;
  double tA[NX * NX], tB[NX * NU], tC[NX], txp[NX];
  linearize<M>(D.dt, x, u, tA, tB, tC, txp);
  if (A)
    for (int i = 0; i < NX * NX; ++i) A[i] = tA[i];
  if (Bm)
    for (int i = 0; i < NX * NU; ++i) Bm[i] = tB[i];
  if (C)
    for (int i = 0; i < NX; ++i) C[i] = tC[i];
  if (xp)
    for (int i = 0; i < NX; ++i) xp[i] = txp[i];
  if (p) branch_eval<M>(D.mc, D.dt, D.N, D.m, pol, x, z, p, dp, R);
  if (zpred)
    for (int i = 0; i < D.m; ++i) rollout<M>(D.dt, D.N, pol[i], z, zpred + i * NX, D.m * NX, R);
  if (h0) col_eval<M>(D.mc, x, z, h0, dh);
}

}  // namespace bmpc
