// bmpc_tree.h -- scenario-tree update of one ego (warm start, rollouts, linearisation).
//
// Restates, per ego and lane-parallel over branches/nodes:
//   inittree   MPC_branch.py:1678-1747   (first solve: u = 0)
//   updatetree MPC_branch.py:1811-1858   (shift of uLin, argmax-p child, leaf repeat,
//                                         BFS rollout + linearisation)
//   col_eval rows of buildIneqConstr/updateIneqConstr (:1882-1892, :2016-2024)
// The per-node data (xbar, zbar, ubar, A/B/C, dh, h0, w, p) is what the reference keeps in
// BranchTree objects; here it is a flat array per ego.
#pragma once

#include "bmpc_model.h"

#ifndef BMPC_CONE_BOOST
#define BMPC_CONE_BOOST 1   // 0: boost 0 on every cone (A/B of the rotated-cone row boost)
#endif

namespace bmpc {

struct EgoView {
  double* ws;               // this ego's workspace slab
  const bmpc_policy* pol;   // this ego's m policies
};

template <class X, class M>
BMPC_HD void tree_update(const X& ex, const Plan& P, const Layout& L, EgoView E,
                         const double* x, const double* z, const double* xref) {
  const int n = P.n, d = P.d, N = P.N, m = P.m;
  double* ws = E.ws;
  double* xbar = ws + L.xbar;
  double* zbar = ws + L.zbar;
  double* ubar = ws + L.ubar;
  double* Ad = ws + L.Ad;
  double* Bd = ws + L.Bd;
  double* Cd = ws + L.Cd;
  double* w = ws + L.w;
  double* p = ws + L.p;
  const double* uLin = ws + L.uLin;
  const double* pprev = ws + L.pprev;
  const bool init = ws[L.misc + MISC_INIT] != 0.0;
  const double dt = P.desc.dt;
  const double* mc = P.desc.mc;
  const Topo& t = P.t;

  // ---- inputs of this solve ------------------------------------------------------------
  for (int i = ex.lane; i < n; i += ex.nlanes) {
    xbar[i] = x[i];
    zbar[i] = z[i];
    ws[L.xref + i] = xref[i];
  }
  // ---- warm start: updatetree's shift (:1813-1823), or zeros (inittree) -----------------
  for (int b = ex.lane; b < P.nbranch; b += ex.nlanes) {
    const int len = t.br_len[b], ndu = t.br_ndu[b];
    if (!init) {
      for (int j = 0; j < len * d; ++j) ubar[ndu * d + j] = 0.0;
      continue;
    }
    for (int j = 0; j < len - 1; ++j)
      for (int k = 0; k < d; ++k) ubar[(ndu + j) * d + k] = uLin[(ndu + j + 1) * d + k];
    int src;
    if (t.br_child0[b] >= 0) {
      int best = 0;
      for (int i = 1; i < m; ++i)
        if (pprev[b * m + i] > pprev[b * m + best]) best = i;   // np.argmax: first max
      src = t.br_ndu[t.br_child0[b] + best];
    } else {
      src = ndu + len - 1;     // utraj[-1] = utraj[-2] = uLin[ndu+len-1]
    }
    for (int k = 0; k < d; ++k) ubar[(ndu + len - 1) * d + k] = uLin[src * d + k];
  }
  ex.sync();
  // ---- root linearisation ---------------------------------------------------------------
  if (ex.lane == 0) {
    double xp[BMPC_MAX_N];
    linearize<M>(dt, xbar, ubar, Ad, Bd, Cd, xp);
    w[0] = 1.0;
  }
  ex.sync();
  // ---- BFS by depth ---------------------------------------------------------------------
  const LaneRef R{P.lref, P.lref + P.nlref, P.nlref};   // psiref policies' lane reference
  int b0 = 0, nb = 1;   // branches of the current depth: [b0, b0+nb)
  for (int D = 0; D < P.NB; ++D) {
    // (a) branch probabilities of each non-leaf branch at this depth, and zpred blocks
    for (int it = ex.lane; it < nb * (m + 1); it += ex.nlanes) {
      const int b = b0 + it / (m + 1), i = it % (m + 1) - 1;
      const int last = t.br_ndx[b] + t.br_len[b] - 1;
      if (i < 0) {
        branch_eval<M>(mc, dt, N, m, E.pol, xbar + last * n, zbar + last * n, p + b * m,
                       ws + L.dp + (size_t)b * m * n, R);   // BranchTree.dp (:1711, :1842)
      } else {
        const int c = t.br_child0[b] + i;
        rollout<M>(dt, N, E.pol[i], zbar + last * n, zbar + t.br_ndx[c] * n, n, R);
      }
    }
    ex.sync();
    // (b) child weights and rollouts of the linearisation trajectory (:1844-1856)
    for (int it = ex.lane; it < nb * m; it += ex.nlanes) {
      const int b = b0 + it / m, i = it % m;
      const int c = t.br_child0[b] + i;
      w[c] = w[b] * p[b * m + i];
      const int lastx = t.br_ndx[b] + t.br_len[b] - 1, lastu = t.br_ndu[b] + t.br_len[b] - 1;
      double xc[BMPC_MAX_N];
      step<M>(dt, xbar + lastx * n, ubar + lastu * d, xc);
      const int ndx = t.br_ndx[c], ndu = t.br_ndu[c];
      for (int j = 0; j < N; ++j) {
        double* xj = xbar + (ndx + j) * n;
        for (int k = 0; k < n; ++k) xj[k] = xc[k];
        const int u = ndu + j;
        linearize<M>(dt, xj, ubar + u * d, Ad + u * n * n, Bd + u * n * d, Cd + u * n, xc);
      }
      if (t.br_child0[c] < 0) {          // leaf terminal node: keep the one-step prediction
        for (int k = 0; k < n; ++k) {
          xbar[(ndx + N) * n + k] = xc[k];
          zbar[(ndx + N) * n + k] = zbar[(ndx + N - 1) * n + k];
        }
      }
    }
    ex.sync();
    b0 += nb;
    nb *= m;
  }
  // ---- collision linearisation of every non-terminal state node --------------------------
  double* dh = ws + L.dh;
  double* h0 = ws + L.h0;
  for (int k = ex.lane; k < P.T; k += ex.nlanes) {
    if (t.x_u[k] < 0) {
      h0[k] = 0.0;
      for (int j = 0; j < n; ++j) dh[k * n + j] = 0.0;
    } else {
      col_eval<M>(mc, xbar + k * n, zbar + k * n, h0 + k, dh + k * n);
      if constexpr (M::kTransform) {
        // updateIneqConstr with S (MPC_branch.py:2025-2036): dh[0] <- sign(dh0) max(0.1, |dh0|)
        // on every solve after the first; h0 keeps the unclipped dh (col_eval's h - dh.x)
        if (init && ws[L.xform + XF_SON] != 0.0) {
          const double a = dh[k * n];
          dh[k * n] = a > 0.0 ? fmax(0.1, a) : a < 0.0 ? -fmax(0.1, -a) : 0.0;
        }
      }
    }
  }
  // ---- per-cone Lorentz boost of the rotated-cone rows ("cone boost") ----
  double* boost = ws + L.boost;
  for (int k = ex.lane; k < P.ncones; k += ex.nlanes) {
    double est = 0.0;
    const int c = t.cone_c[k];
    const int nb_nodes = c >= 0 ? t.br_len[c] : 1;
    for (int j = 0; j < nb_nodes; ++j) {
      const int xk = c >= 0 ? t.br_ndx[c] + j : 0;
      const int uk = c >= 0 ? t.br_ndu[c] + j : 0;
      if (c >= 0) {
        const double* xv = xbar + xk * n;
        for (int r = 0; r < n; ++r) {
          double q = 0.0;
          for (int s = 0; s < n; ++s) q += P.desc.Q[r * n + s] * xv[s];
          est += xv[r] * q;
        }
      }
      const double* uv = ubar + uk * d;
      for (int r = 0; r < d; ++r) {
        double q = 0.0;
        for (int s = 0; s < d; ++s) q += P.desc.R[r * d + s] * uv[s];
        est += uv[r] * q;
      }
    }
    boost[k] = BMPC_CONE_BOOST ? 0.5 * log(est > 1.0 ? est : 1.0) : 0.0;
    boost[P.ncones + k] = exp(-boost[k]);   // e^-beta, read by the IPM's operators (the same value)
  }
  ex.sync();
}

// robustMPC (MPC_branch.py:1275-1443): the chain's linearisation trajectory -- the carried
// shifted prediction, or on the first solve the rollout of u = 0 from x (get_xLin :1326) --
// its dynamics (computeLTVdynamics :1438), the obstacle predictions of every time slot
// (inittree/updatetree :1336-1383: slot 0 the measured z, slot (D-1)N+i+1 the m^D
// predictions of depth D in BFS order) and one collision row per prediction
// (buildIneqConstr :1474-1483).  Rows past a slot's prediction count are padding: dh = 0 and
// h0 = 1, inactive at the optimum (their slack is 0, the row slack 1).
template <class X, class M>
BMPC_HD void tree_update_robust(const X& ex, const Plan& P, const Layout& L, EgoView E,
                                const double* x, const double* z, const double* xref) {
  constexpr int NX = M::NX, NU = M::NU;
  const int N = P.N, m = P.m, T = P.T, U = P.U, Ncol = P.Ncol;
  double* ws = E.ws;
  double* xbar = ws + L.xbar;
  double* ubar = ws + L.ubar;
  double* zr = ws + L.zrob;
  const bool init = ws[L.misc + MISC_INIT] != 0.0;
  const double dt = P.desc.dt;
  const double* mc = P.desc.mc;
  for (int i = ex.lane; i < NX; i += ex.nlanes) {
    ws[L.misc + MISC_X0 + i] = x[i];
    ws[L.xref + i] = xref[i];
    zr[i] = z[i];
  }
  if (ex.lane == 0) ws[L.w] = 1.0;
  if (init) {
    for (int i = ex.lane; i < T * NX; i += ex.nlanes) xbar[i] = ws[L.xlin + i];
    for (int i = ex.lane; i < U * NU; i += ex.nlanes) ubar[i] = ws[L.uLin + i];
  } else {
    for (int i = ex.lane; i < U * NU; i += ex.nlanes) ubar[i] = 0.0;
    if (ex.lane == 0) {
      double xc[NX], u0[NU];
      for (int k = 0; k < NU; ++k) u0[k] = 0.0;
      for (int k = 0; k < NX; ++k) xc[k] = xbar[k] = x[k];
      for (int i = 1; i < T; ++i) {
        step<M>(dt, xc, u0, xbar + i * NX);
        for (int k = 0; k < NX; ++k) xc[k] = xbar[i * NX + k];
      }
    }
  }
  ex.sync();
  for (int u = ex.lane; u < U; u += ex.nlanes) {
    double xp[NX];
    linearize<M>(dt, xbar + u * NX, ubar + u * NU, ws + L.Ad + u * NX * NX, ws + L.Bd + u * NX * NU,
                 ws + L.Cd + u * NX, xp);
  }
  // obstacle predictions, depth by depth: prediction j of depth D continues prediction j/m of
  // depth D-1 (its slot (D-1)N) under policy j%m
  int nd = 1;
  for (int D = 1; D <= P.zNB; ++D) {
    nd *= m;
    const int s0 = (D - 1) * N;
    for (int j = ex.lane; j < nd; j += ex.nlanes)
      rollout<M>(dt, N, E.pol[j % m], zr + ((size_t)s0 * Ncol + j / m) * NX, zr + ((size_t)(s0 + 1) * Ncol + j) * NX,
                 Ncol * NX);
    ex.sync();
  }
  double* dh = ws + L.dh;
  double* h0 = ws + L.h0;
  for (int it = ex.lane; it < T * Ncol; it += ex.nlanes) {
    const int k = it / Ncol, j = it % Ncol;
    int cnt = 0;
    if (k == 0) {
      cnt = 1;
    } else if (k < T - 1) {
      cnt = 1;
      for (int D = (k - 1) / N + 1; D > 0; --D) cnt *= m;
    }
    if (j < cnt) {
      col_eval<M>(mc, xbar + k * NX, zr + (size_t)it * NX, h0 + it, dh + (size_t)it * NX);
    } else {
      h0[it] = 1.0;
      for (int c = 0; c < NX; ++c) dh[(size_t)it * NX + c] = 0.0;
    }
  }
  ex.sync();
}

// the tree step of the plan's controller
template <class X, class M>
BMPC_HD void tree_step(const X& ex, const Plan& P, const Layout& L, EgoView E, const double* x, const double* z,
                       const double* xref) {
  if (P.desc.controller == BMPC_CTRL_ROBUST) tree_update_robust<X, M>(ex, P, L, E, x, z, xref);
  else tree_update<X, M>(ex, P, L, E, x, z, xref);
}

}  // namespace bmpc
