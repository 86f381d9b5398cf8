// bmpc_qp.h -- structured primal-dual interior point for the BranchMPCProx QP of one ego.
//
// Problem (what BranchMPCProx hands to OSQP, MPC_branch.py:265-487):
//   min 1/2 z'Pz + q'z   s.t.  E z = e (dynamics, :185-223),  G z <= g (:327-370)
//   z = [X(T n) | U(U d) | S(T Nc)],  P = 2 blockdiag(Hx, Hu, Qs0 I)   (buildCost :265-325)
// Quirks kept: the leaf's last Hu block is *assigned* w R (:303); Hu[0:d,0:d] += dR
// broadcasts the dR vector onto every row (:312) and OSQP reads the upper triangle only;
// qu[0:d] = -2 OldInput.dR is a scalar broadcast (:311); leaf-terminal rows are empty.
// Algorithm: Mehrotra predictor-corrector with the same steps as oracle/qp_ipm.py (the
// stand-in for OSQP + polish; OSQP itself is unpinned).  Hu couples consecutive
// inputs (rate cost dR), so the KKT is factored by a tree Riccati recursion over the
// augmented state s = [x_k; u_pred(k)] (n + d), one lane per branch.
#pragma once

#include "bmpc_ipm.h"

namespace bmpc {

struct QpCtx {
  CPlan* P;
  CLayout* L;
  gdouble* ws;
  BMPC_HD QpCtx uniform() const { return QpCtx{uniform_ptr(P), uniform_ptr(L), uniform_ptr(ws)}; }
};

// u node whose input created x node k's state (the rate-cost predecessor of x_u[k]); -1 root
template <class T>
BMPC_HD int qp_pred_u(const T& t, int u) { return t.x_srcu[t.u_x[u]]; }

// coefficient j of inequality row c of state node k: Ncol collision rows (-dh) then the Fx rows.
// Branch-free: both operands are read (clamped indices; Fx from the plan-constant LDS area) and
// blended exactly -- a select would become a branch around the dh load (one memory round trip
// per coefficient).
template <int NX, class X>
BMPC_HD double qp_row(CPlan& P, const X& ex, const gdouble* dh, int k, int c, int j) {
  const bool col = c < P.Ncol;
  const double d = dh[((size_t)k * P.Ncol + (col ? c : 0)) * NX + j];
  const double f = fxv(P, ex, col ? 0 : c - P.Ncol, j);
  const double m = col ? 1.0 : 0.0;
  return m * (-d) + (1.0 - m) * f;
}
// rows of state node k are live: every node with an input, and robustMPC's terminal node
// (its Fx rows carry slacks, MPC_branch.py:1470-1472); BranchMPC's leaf terminals are empty
template <class T>
BMPC_HD bool qp_rows_on(CPlan& P, const T& t, int k) { return t.x_u[k] >= 0 || P.desc.controller == BMPC_CTRL_ROBUST; }

// ---- cost, rhs (buildCost / buildIneqConstr / buildEqConstr of the current tree) ----------
template <class X, class M>
BMPC_FN void qp_build(const X ex, const QpCtx Cin, gdouble* hv, gdouble* bv) {
  const QpCtx C = Cin.uniform();
  constexpr int NX = M::NX, NU = M::NU;
  CPlan& P = *C.P;
  CLayout& L = *C.L;
  const auto t = topo_view(P, ex);
  gdouble* ws = C.ws;
  const int Nc = P.Nc;
  const gdouble* w = ws + L.w;
  const gdouble* xbar = ws + L.xbar;
  const gdouble* xref = ws + L.xref;
  const auto Q = P.desc.Q;
  const auto Qf = P.desc.Qf;
  double xq[NX], xqf[NX];
  for (int c = 0; c < NX; ++c) {
    double a = 0.0, b = 0.0;
    for (int r = 0; r < NX; ++r) a += xref[r] * Q[r * NX + c], b += xref[r] * Qf[r * NX + c];
    xq[c] = a;
    xqf[c] = b;
  }
  gdouble* q = ws + L.qq;
  // BranchMPCProx: dQ = 3Q (:270); BranchMPC: dQ = 0.5Q, leaf's last node tracks xRef with Qf
  // and the leaf terminal node has no linear term (:1068-1099)
  // robustMPC: unweighted Q (Qf on the terminal node) tracking xRef, no proximal term
  // (buildCost :1540-1569)
  const bool robust = P.desc.controller == BMPC_CTRL_ROBUST;
  const bool prox = P.desc.controller == BMPC_CTRL_PROX || robust;
  const double dq = robust ? 0.0 : P.desc.controller == BMPC_CTRL_PROX ? 3.0 : 0.5;
  // state nodes: Hx (doubled) and qx
  for (int k = ex.lane; k < P.T; k += ex.nlanes) {
    const int b = t.x_branch[k];
    const double wb = w[b];
    const bool term = t.x_u[k] < 0;
    const bool leaf_last = !term && t.br_child0[b] < 0 && k == t.br_ndx[b] + t.br_len[b] - 1;
    gdouble* H = ws + L.hx + k * NX * NX;
    for (int i = 0; i < NX * NX; ++i) H[i] = 2.0 * wb * (term ? Qf[i] : (dq + 1.0) * Q[i]);   // (dQ + Q) w
    for (int c = 0; c < NX; ++c) {
      double v;
      if (term) {
        v = prox ? -2.0 * wb * xqf[c] : 0.0;
      } else {
        double xd = 0.0;
        for (int r = 0; r < NX; ++r) xd += xbar[k * NX + r] * dq * Q[r * NX + c];
        v = -2.0 * wb * (((!prox && leaf_last) ? xqf[c] : xq[c]) + xd);
      }
      q[P.oX + k * NX + c] = v;
    }
    for (int c = 0; c < Nc; ++c) q[P.oS + k * Nc + c] = qp_rows_on(P, t, k) ? P.desc.Qslack[1] * wb : 0.0;
  }
  // input nodes: diagonal blocks (doubled), rate couplings with the predecessor, qu
  const auto R = P.desc.R;
  const auto dR = P.desc.dR;
  for (int u = ex.lane; u < P.U; u += ex.nlanes) {
    const int k = t.u_x[u], b = t.x_branch[k];
    const int j = k - t.br_ndx[b], len = t.br_len[b];
    const bool leaf = t.br_child0[b] < 0;
    const double wb = w[b];
    double D[NU][NU];
    for (int r = 0; r < NU; ++r)
      for (int c = 0; c < NU; ++c) D[r][c] = 0.0;
    if (robust) {   // R + 2 dR, the last input R + dR (:1545-1549)
      for (int r = 0; r < NU; ++r) {
        for (int c = 0; c < NU; ++c) D[r][c] = R[r * NU + c];
        D[r][r] += (u < P.U - 1 ? 2.0 : 1.0) * dR[r];
      }
    } else if ((leaf && j == len - 1) || !prox) {   // assigned w R (BranchMPC: every block, :1077-1090)
      for (int r = 0; r < NU; ++r)
        for (int c = 0; c < NU; ++c) D[r][c] = wb * R[r * NU + c];
    } else {
      for (int r = 0; r < NU; ++r) {
        for (int c = 0; c < NU; ++c) D[r][c] += wb * R[r * NU + c];
        D[r][r] += wb * dR[r];
        if (j >= 1 || b != 0) D[r][r] += wb * dR[r];
      }
    }
    if (u == 0 && prox && !robust)   // Hu[0:d,0:d] += dR (row broadcast), upper triangle read by OSQP
      for (int r = 0; r < NU; ++r)
        for (int c = 0; c < NU; ++c) D[r][c] += dR[r > c ? r : c];
    gdouble* Hu = ws + L.hu + u * NU * NU;
    gdouble* O = ws + L.qo + u * NU * NU;
    const int pu = qp_pred_u(t, u);
    for (int r = 0; r < NU; ++r)
      for (int c = 0; c < NU; ++c) {
        Hu[r * NU + c] = 2.0 * D[r][c];
        O[r * NU + c] = (prox && pu >= 0 && r == c) ? -2.0 * wb * dR[r] : 0.0;
      }
    double od = 0.0;
    if (u == 0)
      for (int r = 0; r < NU; ++r) od += ws[L.misc + MISC_OLDU + r] * dR[r];
    for (int c = 0; c < NU; ++c)   // robustMPC: -2 OldInput diag(dR), a vector (:1559)
      q[P.oU + u * NU + c] = u != 0 ? 0.0 : robust ? -2.0 * ws[L.misc + MISC_OLDU + c] * dR[c] : -2.0 * od;
  }
  // rhs of the inequalities: [h0 | bx] per non-terminal node, bu per input, 0 for -S
  const gdouble* h0 = ws + L.h0;
  for (int it = ex.lane; it < P.T * Nc; it += ex.nlanes) {
    const int k = it / Nc, c = it % Nc;
    hv[P.rFx + it] = !qp_rows_on(P, t, k) ? 0.0 : c < P.Ncol ? h0[k * P.Ncol + c] : P.desc.bx[c - P.Ncol];
    hv[P.rPos + it] = 0.0;
  }
  for (int it = ex.lane; it < P.U * P.nFu; it += ex.nlanes) hv[P.rFu + it] = P.desc.bu[it % P.nFu];
  // equality rhs: x0 = x, x_k - A x_src - B u_src = C_src
  const gdouble* Cd = ws + L.Cd;
  for (int k = ex.lane; k < P.T; k += ex.nlanes) {
    const int su = t.x_srcu[k];
    // x_0 = x: robustMPC linearises about the shifted prediction, so x is kept apart
    const gdouble* x0 = robust ? ws + L.misc + MISC_X0 : xbar;
    for (int r = 0; r < NX; ++r) bv[k * NX + r] = su >= 0 ? Cd[su * NX + r] : x0[r];
  }
  ex.sync();
}

// ---- structured operators ------------------------------------------------------------------
// out = P z  (Hx blocks, Hu diagonal blocks + rate couplings, slack quadratic)
template <class X, int NX, int NU>
BMPC_FN void qp_apply_P(const X ex, const QpCtx Cin, const gdouble* zv, gdouble* out) {
  const QpCtx C = Cin.uniform();
  CPlan& P = *C.P;
  CLayout& L = *C.L;
  const auto t = topo_view(P, ex);
  const gdouble* ws = C.ws;
  for (int k = ex.lane; k < P.T; k += ex.nlanes) {
    const gdouble* H = ws + L.hx + k * NX * NX;
    for (int r = 0; r < NX; ++r) {
      double v = 0.0;
      for (int c = 0; c < NX; ++c) v += H[r * NX + c] * zv[P.oX + k * NX + c];
      out[P.oX + k * NX + r] = v;
    }
  }
  for (int u = ex.lane; u < P.U; u += ex.nlanes) {
    const gdouble* Hu = ws + L.hu + u * NU * NU;
    const gdouble* O = ws + L.qo + u * NU * NU;
    const int pu = qp_pred_u(t, u);
    double v[NU];
    for (int r = 0; r < NU; ++r) {
      double a = 0.0;
      for (int c = 0; c < NU; ++c) a += Hu[r * NU + c] * zv[P.oU + u * NU + c];
      if (pu >= 0)
        for (int c = 0; c < NU; ++c) a += O[r * NU + c] * zv[P.oU + pu * NU + c];
      v[r] = a;
    }
    // couplings where u is the predecessor: successors' x nodes carry the inputs that follow
    const int k = t.u_x[u];
    for (int e = t.succ_off[k]; e < t.succ_off[k + 1]; ++e) {
      const int su = t.x_u[t.succ[e]];
      if (su < 0) continue;
      const gdouble* Os = ws + L.qo + su * NU * NU;
      for (int r = 0; r < NU; ++r)
        for (int c = 0; c < NU; ++c) v[r] += Os[c * NU + r] * zv[P.oU + su * NU + c];
    }
    for (int r = 0; r < NU; ++r) out[P.oU + u * NU + r] = v[r];
  }
  const double qs = 2.0 * P.desc.Qslack[0];
  lane_batch(ex, P.oS, P.oJ, [&](int i) { return qs * zv[i]; }, [&](int i, double v) { out[i] = v; });
  ex.sync();
}

// out(rows) = G z
template <class X, int NX, int NU>
BMPC_FN void qp_apply_G(const X ex, const QpCtx Cin, const gdouble* zv, gdouble* out) {
  const QpCtx C = Cin.uniform();
  CPlan& P = *C.P;
  CLayout& L = *C.L;
  const auto t = topo_view(P, ex);
  const int Nc = P.Nc;
  const gdouble* dh = C.ws + L.dh;
  lane_batch(ex, 0, P.T * Nc, [&](int it) {
    const int k = it / Nc, c = it % Nc;
    double v = -zv[P.oS + it];
    const double on = qp_rows_on(P, t, k) ? 1.0 : 0.0;   // multiplier, not a branch around the loads
#pragma unroll
    for (int j = 0; j < NX; ++j) v += on * qp_row<NX>(P, ex, dh, k, c, j) * zv[P.oX + k * NX + j];
    return v;
  }, [&](int it, double v) { out[P.rFx + it] = v; });
  lane_batch(ex, 0, P.U * P.nFu, [&](int it) {
    const int u = it / P.nFu, r = it % P.nFu;
    double v = 0.0;
    for (int j = 0; j < NU; ++j) v += fuv(P, ex, r, j) * zv[P.oU + u * NU + j];
    return v;
  }, [&](int it, double v) { out[P.rFu + it] = v; });
  lane_batch(ex, 0, P.T * Nc, [&](int it) { return -zv[P.oS + it]; }, [&](int it, double v) { out[P.rPos + it] = v; });
  ex.sync();
}

// out(nv) = G' r
template <class X, int NX, int NU>
BMPC_FN void qp_apply_GT(const X ex, const QpCtx Cin, const gdouble* r, gdouble* out) {
  const QpCtx C = Cin.uniform();
  CPlan& P = *C.P;
  CLayout& L = *C.L;
  const auto t = topo_view(P, ex);
  const int Nc = P.Nc;
  const gdouble* dh = C.ws + L.dh;
  for (int k = ex.lane; k < P.T; k += ex.nlanes) {
    double ax[NX];
    for (int j = 0; j < NX; ++j) ax[j] = 0.0;
    const bool term = t.x_u[k] < 0;
    for (int c = 0; c < Nc; ++c) {
      const double rv = r[P.rFx + k * Nc + c];
      if (qp_rows_on(P, t, k))
        for (int j = 0; j < NX; ++j) ax[j] += qp_row<NX>(P, ex, dh, k, c, j) * rv;
      out[P.oS + k * Nc + c] = -rv - r[P.rPos + k * Nc + c];
    }
    for (int j = 0; j < NX; ++j) out[P.oX + k * NX + j] = ax[j];
  }
  for (int u = ex.lane; u < P.U; u += ex.nlanes) {
    double au[NU];
    for (int j = 0; j < NU; ++j) au[j] = 0.0;
    for (int rr = 0; rr < P.nFu; ++rr) {
      const double rv = r[P.rFu + u * P.nFu + rr];
      for (int j = 0; j < NU; ++j) au[j] += P.desc.Fu[rr * NU + j] * rv;
    }
    for (int j = 0; j < NU; ++j) out[P.oU + u * NU + j] = au[j];
  }
  ex.sync();
}

// E z (dynamics rows) and E' y: the first T*NX rows / x,u parts of the CVaR operators
template <class X, int NX, int NU>
BMPC_FN void qp_apply_E(const X ex, const QpCtx Cin, const gdouble* zv, gdouble* out) {
  const QpCtx C = Cin.uniform();
  CPlan& P = *C.P;
  const auto t = topo_view(P, ex);
  const gdouble* Ad = C.ws + C.L->Ad;
  const gdouble* Bd = C.ws + C.L->Bd;
  for (int k = ex.lane; k < P.T; k += ex.nlanes) {
    const int su = t.x_srcu[k], sx = t.x_srcx[k];
    for (int r = 0; r < NX; ++r) {
      double v = zv[P.oX + k * NX + r];
      if (su >= 0) {
        for (int s = 0; s < NX; ++s) v -= Ad[su * NX * NX + r * NX + s] * zv[P.oX + sx * NX + s];
        for (int s = 0; s < NU; ++s) v -= Bd[su * NX * NU + r * NU + s] * zv[P.oU + su * NU + s];
      }
      out[k * NX + r] = v;
    }
  }
  ex.sync();
}

template <class X, int NX, int NU>
BMPC_FN void qp_apply_ET(const X ex, const QpCtx Cin, const gdouble* y, gdouble* out) {
  const QpCtx C = Cin.uniform();
  CPlan& P = *C.P;
  const auto t = topo_view(P, ex);
  const gdouble* Ad = C.ws + C.L->Ad;
  const gdouble* Bd = C.ws + C.L->Bd;
  for (int k = ex.lane; k < P.T; k += ex.nlanes) {
    double ax[NX], au[NU];
    for (int r = 0; r < NX; ++r) ax[r] = y[k * NX + r];
    for (int r = 0; r < NU; ++r) au[r] = 0.0;
    const int u = t.x_u[k];
    if (u >= 0) {
      double ys[NX];
      for (int r = 0; r < NX; ++r) ys[r] = 0.0;
      for (int e = t.succ_off[k]; e < t.succ_off[k + 1]; ++e)
        for (int r = 0; r < NX; ++r) ys[r] += y[t.succ[e] * NX + r];
      for (int s = 0; s < NX; ++s) {
        double v = 0.0;
        for (int r = 0; r < NX; ++r) v += Ad[u * NX * NX + r * NX + s] * ys[r];
        ax[s] -= v;
      }
      for (int s = 0; s < NU; ++s) {
        double v = 0.0;
        for (int r = 0; r < NX; ++r) v += Bd[u * NX * NU + r * NU + s] * ys[r];
        au[s] -= v;
      }
      for (int s = 0; s < NU; ++s) out[P.oU + u * NU + s] = au[s];
    }
    for (int r = 0; r < NX; ++r) out[P.oX + k * NX + r] = ax[r];
  }
  lane_batch(ex, P.oS, P.oJ, [&](int) { return 0.0; }, [&](int i, double v) { out[i] = v; });
  ex.sync();
}

// ---- factorisation: node Hessians of P + G'D^-1G, slack elimination, augmented Riccati -----
// dinv[i] = z_i / s_i (the inverse of the KKT's D = s/z block)
template <class X, int NX, int NU>
BMPC_FN bool qp_factor(const X ex, const QpCtx Cin, const gdouble* dinv) {
  const QpCtx C = Cin.uniform();
  constexpr int NS = NX + NU;
  CPlan& P = *C.P;
  CLayout& L = *C.L;
  const auto t = topo_view(P, ex);
  const int Nc = P.Nc;
  gdouble* ws = C.ws;
  const double qs2 = 2.0 * P.desc.Qslack[0];
  const gdouble* dh = ws + L.dh;
  // slack pivots sd = qs2 + d_f + d_p (stored with d_f for the solves)
  lane_batch(ex, 0, P.T * Nc, [&](int it) { return dinv[P.rFx + it]; }, [&](int it, double df) {
    ws[L.sd + it * 2] = qs2 + df + dinv[P.rPos + it];
    ws[L.sd + it * 2 + 1] = df;
  });
  ex.sync();
  double bad = 0.0;
  for (int dep = P.NB; dep >= 0; --dep) {
    const int b0 = branch_start(P, dep), nbd = branch_count(P, dep);
    for (int bi = ex.lane; bi < nbd; bi += ex.nlanes) {
      const int b = b0 + bi;
      const int ndx = t.br_ndx[b], ndu = t.br_ndu[b], len = t.br_len[b];
      const bool leaf = dep == P.NB;
      const int nnodes = leaf ? len + 1 : len;
      for (int jn = nnodes - 1; jn >= 0; --jn) {
        const int k = ndx + jn;
        const bool term = t.x_u[k] < 0;
        // reduced x Hessian: Hx + sum_c omega_c f_c f_c'
        double Hx[NX][NX];
        mat_load(Hx, ws + L.hx + k * NX * NX);
        if (qp_rows_on(P, t, k))
          for (int c = 0; c < Nc; ++c) {
            const double sd = ws[L.sd + (k * Nc + c) * 2], df = ws[L.sd + (k * Nc + c) * 2 + 1];
            const double om = df - df * df / sd;
            double f[NX];
            for (int j = 0; j < NX; ++j) f[j] = qp_row<NX>(P, ex, dh, k, c, j);
            for (int i = 0; i < NX; ++i)
              for (int j = 0; j < NX; ++j) Hx[i][j] += om * f[i] * f[j];
          }
        double Pt[NS][NS];
        mat_zero(Pt);
        if (term) {
          for (int i = 0; i < NX; ++i)
            for (int j = 0; j < NX; ++j) Pt[i][j] = Hx[i][j];
          mat_store(Pt, ws + L.Pa + k * NS * NS);
          continue;
        }
        const int u = t.x_u[k];
        // P-bar = sum over successors of P~_c
        double Pb[NS][NS];
        mat_zero(Pb);
        for (int e = t.succ_off[k]; e < t.succ_off[k + 1]; ++e) {
          const gdouble* Pc = ws + L.Pa + t.succ[e] * NS * NS;
          for (int i = 0; i < NS; ++i)
            for (int j = 0; j < NS; ++j) Pb[i][j] += Pc[i * NS + j];
        }
        double A[NX][NX], B[NX][NU], D[NU][NU], O[NU][NU];
        mat_load(A, ws + L.Ad + u * NX * NX);
        mat_load(B, ws + L.Bd + u * NX * NU);
        mat_load(D, ws + L.hu + u * NU * NU);
        mat_load(O, ws + L.qo + u * NU * NU);
        for (int r = 0; r < P.nFu; ++r) {
          const double dr = dinv[P.rFu + u * P.nFu + r];
          for (int i = 0; i < NU; ++i)
            for (int j = 0; j < NU; ++j) D[i][j] += dr * P.desc.Fu[r * NU + i] * P.desc.Fu[r * NU + j];
        }
        // PxxA, PxxB
        double PA[NX][NX], PB[NX][NU];
        for (int i = 0; i < NX; ++i) {
          for (int j = 0; j < NX; ++j) {
            double v = 0.0;
            for (int r = 0; r < NX; ++r) v += Pb[i][r] * A[r][j];
            PA[i][j] = v;
          }
          for (int j = 0; j < NU; ++j) {
            double v = 0.0;
            for (int r = 0; r < NX; ++r) v += Pb[i][r] * B[r][j];
            PB[i][j] = v;
          }
        }
        double Qxx[NX][NX], Qux[NU][NX], Quu[NU][NU];
        for (int i = 0; i < NX; ++i)
          for (int j = 0; j < NX; ++j) {
            double v = Hx[i][j];
            for (int r = 0; r < NX; ++r) v += A[r][i] * PA[r][j];
            Qxx[i][j] = v;
          }
        for (int i = 0; i < NU; ++i)
          for (int j = 0; j < NX; ++j) {
            double v = 0.0;
            for (int r = 0; r < NX; ++r) v += B[r][i] * PA[r][j] + Pb[NX + i][r] * A[r][j];
            Qux[i][j] = v;
          }
        for (int i = 0; i < NU; ++i)
          for (int j = 0; j < NU; ++j) {
            double v = D[i][j] + Pb[NX + i][NX + j];
            for (int r = 0; r < NX; ++r) v += B[r][i] * PB[r][j] + B[r][i] * Pb[r][NX + j] + Pb[NX + i][r] * B[r][j];
            Quu[i][j] = v;
          }
        for (int i = 0; i < NU; ++i)   // symmetrise (rounding)
          for (int j = i + 1; j < NU; ++j) {
            const double a = 0.5 * (Quu[i][j] + Quu[j][i]);
            Quu[i][j] = a;
            Quu[j][i] = a;
          }
        if (!chol<NU>(Quu)) bad = 1.0;
        mat_store(Quu, ws + L.Luu + u * NU * NU);
        // K = -Quu^-1 [Qux  Quv],  Quv = O'
        double K[NU][NS];
        for (int j = 0; j < NS; ++j) {
          double col[NU];
          for (int i = 0; i < NU; ++i) col[i] = -(j < NX ? Qux[i][j] : O[j - NX][i]);
          chol_solve<NU>(Quu, col);
          for (int i = 0; i < NU; ++i) K[i][j] = col[i];
        }
        mat_store(K, ws + L.Ka + u * NU * NS);
        // P~ = [[Qxx,0],[0,0]] + S K,  S = [Qux Quv]'  (NS x NU)
        for (int i = 0; i < NS; ++i)
          for (int j = 0; j < NS; ++j) {
            double v = (i < NX && j < NX) ? Qxx[i][j] : 0.0;
            for (int r = 0; r < NU; ++r) v += (i < NX ? Qux[r][i] : O[i - NX][r]) * K[r][j];
            Pt[i][j] = v;
          }
        for (int i = 0; i < NS; ++i)
          for (int j = i + 1; j < NS; ++j) {
            const double a = 0.5 * (Pt[i][j] + Pt[j][i]);
            Pt[i][j] = a;
            Pt[j][i] = a;
          }
        mat_store(Pt, ws + L.Pa + k * NS * NS);
      }
    }
    ex.sync();
  }
  return ex.max(bad) == 0.0;
}

// Solve [H E'; E 0] [v; nu] = [r; e] with H = P + G'D^-1G (slacks eliminated per node)
template <class X, int NX, int NU>
BMPC_FN void qp_tree_solve(const X ex, const QpCtx Cin, const gdouble* r, const gdouble* e, gdouble* out, gdouble* nu) {
  const QpCtx C = Cin.uniform();
  constexpr int NS = NX + NU;
  CPlan& P = *C.P;
  CLayout& L = *C.L;
  const auto t = topo_view(P, ex);
  const int Nc = P.Nc;
  gdouble* ws = C.ws;
  const gdouble* dh = ws + L.dh;
  gdouble* la = ws + L.la;
  gdouble* kf = ws + L.kff;
  // backward
  for (int dep = P.NB; dep >= 0; --dep) {
    const int b0 = branch_start(P, dep), nbd = branch_count(P, dep);
    for (int bi = ex.lane; bi < nbd; bi += ex.nlanes) {
      const int b = b0 + bi;
      const int ndx = t.br_ndx[b], ndu = t.br_ndu[b], len = t.br_len[b];
      const bool leaf = dep == P.NB;
      const int nnodes = leaf ? len + 1 : len;
      for (int jn = nnodes - 1; jn >= 0; --jn) {
        const int k = ndx + jn;
        const bool term = t.x_u[k] < 0;
        double qx[NX];
        for (int j = 0; j < NX; ++j) qx[j] = -r[P.oX + k * NX + j];
        if (qp_rows_on(P, t, k))
          for (int c = 0; c < Nc; ++c) {   // slack elimination
            const double sd = ws[L.sd + (k * Nc + c) * 2], df = ws[L.sd + (k * Nc + c) * 2 + 1];
            const double a = df * r[P.oS + k * Nc + c] / sd;
            for (int j = 0; j < NX; ++j) qx[j] -= qp_row<NX>(P, ex, dh, k, c, j) * a;
          }
        double lt[NS];
        if (term) {
          for (int j = 0; j < NX; ++j) lt[j] = qx[j];
          for (int j = NX; j < NS; ++j) lt[j] = 0.0;
          for (int j = 0; j < NS; ++j) la[k * NS + j] = lt[j];
          continue;
        }
        const int u = t.x_u[k];
        // g = sum_c (P~_c [e_c; 0] + l~_c)
        double g[NS];
        for (int j = 0; j < NS; ++j) g[j] = 0.0;
        for (int s = t.succ_off[k]; s < t.succ_off[k + 1]; ++s) {
          const int c = t.succ[s];
          const gdouble* Pc = ws + L.Pa + c * NS * NS;
          for (int i = 0; i < NS; ++i) {
            double v = la[c * NS + i];
            for (int j = 0; j < NX; ++j) v += Pc[i * NS + j] * e[c * NX + j];
            g[i] += v;
          }
        }
        const gdouble* A = ws + L.Ad + u * NX * NX;
        const gdouble* B = ws + L.Bd + u * NX * NU;
        double qu[NU];
        for (int i = 0; i < NU; ++i) {
          double v = -r[P.oU + u * NU + i] + g[NX + i];
          for (int j = 0; j < NX; ++j) v += B[j * NU + i] * g[j];
          qu[i] = v;
        }
        double Lu[NU][NU], kv[NU];
        mat_load(Lu, ws + L.Luu + u * NU * NU);
        for (int i = 0; i < NU; ++i) kv[i] = -qu[i];
        chol_solve<NU>(Lu, kv);
        for (int i = 0; i < NU; ++i) kf[u * NU + i] = kv[i];
        // l~ = [qx + A'g_x + Qux' k ; Quv' k], with S = -Quu K  =>  S k = -K' Quu k = K' qu
        const gdouble* K = ws + L.Ka + u * NU * NS;
        for (int i = 0; i < NX; ++i) {
          double v = qx[i];
          for (int j = 0; j < NX; ++j) v += A[j * NX + i] * g[j];
          lt[i] = v;
        }
        for (int i = NX; i < NS; ++i) lt[i] = 0.0;
        for (int i = 0; i < NS; ++i) {
          double v = 0.0;
          for (int m2 = 0; m2 < NU; ++m2) v += K[m2 * NS + i] * qu[m2];
          lt[i] += v;
        }
        for (int j = 0; j < NS; ++j) la[k * NS + j] = lt[j];
      }
    }
    ex.sync();
  }
  // forward
  for (int dep = 0; dep <= P.NB; ++dep) {
    const int b0 = branch_start(P, dep), nbd = branch_count(P, dep);
    for (int bi = ex.lane; bi < nbd; bi += ex.nlanes) {
      const int b = b0 + bi;
      const int ndx = t.br_ndx[b], ndu = t.br_ndu[b], len = t.br_len[b];
      const bool leaf = dep == P.NB;
      const int nnodes = leaf ? len + 1 : len;
      double s[NS];
      if (b == 0) {
        for (int j = 0; j < NX; ++j) s[j] = e[j];
        for (int j = NX; j < NS; ++j) s[j] = 0.0;
      } else {
        const int pu = t.x_srcu[ndx];
        for (int j = 0; j < NX; ++j) s[j] = out[P.oX + ndx * NX + j];   // written by the parent lane
        for (int j = 0; j < NU; ++j) s[NX + j] = out[P.oU + pu * NU + j];
      }
      for (int jn = 0; jn < nnodes; ++jn) {
        const int k = ndx + jn;
        const bool term = t.x_u[k] < 0;
        for (int j = 0; j < NX; ++j) out[P.oX + k * NX + j] = s[j];
        const gdouble* Pk = ws + L.Pa + k * NS * NS;
        for (int i = 0; i < NX; ++i) {
          double v = la[k * NS + i];
          for (int j = 0; j < NS; ++j) v += Pk[i * NS + j] * s[j];
          nu[k * NX + i] = -v;
        }
        for (int c = 0; c < Nc; ++c) {   // slack recovery
          const double sd = ws[L.sd + (k * Nc + c) * 2], df = ws[L.sd + (k * Nc + c) * 2 + 1];
          double fx = 0.0;
          if (qp_rows_on(P, t, k))
            for (int j = 0; j < NX; ++j) fx += qp_row<NX>(P, ex, dh, k, c, j) * s[j];
          out[P.oS + k * Nc + c] = (r[P.oS + k * Nc + c] + df * fx) / sd;
        }
        if (term) break;
        const int u = t.x_u[k];
        const gdouble* K = ws + L.Ka + u * NU * NS;
        double uk[NU];
        for (int i = 0; i < NU; ++i) {
          double v = kf[u * NU + i];
          for (int j = 0; j < NS; ++j) v += K[i * NS + j] * s[j];
          uk[i] = v;
          out[P.oU + u * NU + i] = v;
        }
        const gdouble* A = ws + L.Ad + u * NX * NX;
        const gdouble* B = ws + L.Bd + u * NX * NU;
        double xn[NX];
        for (int i = 0; i < NX; ++i) {
          double v = 0.0;
          for (int j = 0; j < NX; ++j) v += A[i * NX + j] * s[j];
          for (int j = 0; j < NU; ++j) v += B[i * NU + j] * uk[j];
          xn[i] = v;
        }
        if (jn < nnodes - 1) {
          for (int i = 0; i < NX; ++i) s[i] = xn[i] + e[(k + 1) * NX + i];
          for (int i = 0; i < NU; ++i) s[NX + i] = uk[i];
        } else {   // branch end: children's first nodes
          const int c0 = t.br_child0[b];
          for (int ci = 0; ci < P.m; ++ci) {
            const int c = t.br_ndx[c0 + ci];
            for (int i = 0; i < NX; ++i) out[P.oX + c * NX + i] = xn[i] + e[c * NX + i];
          }
        }
      }
    }
    ex.sync();
  }
}

// KKT solve [P E' G'; E 0 0; G 0 -D] [dx; dy; dz] = [r1; r2; r3], D = s/z, with iterative
// refinement on the D^-1/2-scaled residual (BMPC_NITREF rounds; oracle: 3 rounds, 1e-15 unscaled)
template <class X, int NX, int NU>
BMPC_FN void qp_kkt_solve(const X ex, const QpCtx Cin, const gdouble* dinv, const gdouble* r1, const gdouble* r2,
                          const gdouble* r3, gdouble* dx, gdouble* dy, gdouble* dz) {
  const QpCtx C = Cin.uniform();
  CPlan& P = *C.P;
  CLayout& L = *C.L;
  gdouble* ws = C.ws;
  gdouble* tr = ws + L.k_r0;
  gdouble* tz = ws + L.k_nv0;
  gdouble* e1 = ws + L.k_e1;
  gdouble* e2 = ws + L.k_e2;
  gdouble* e3 = ws + L.k_e3;
  gdouble* cx = ws + L.k_cx;
  gdouble* cy = ws + L.k_cy;
  gdouble* cz = ws + L.k_cz;
  gdouble* tv = ws + L.k_nv1;
  auto once = [&](const gdouble* a1, const gdouble* a2, const gdouble* a3, gdouble* ox, gdouble* oy, gdouble* oz) {
    // (P + G'D^-1G) ox + E'oy = a1 + G'D^-1 a3 ; E ox = a2 ; oz = D^-1 (G ox - a3)
    lane_batch<16>(ex, 0, P.nrows, [&](int i) { return dinv[i] * a3[i]; }, [&](int i, double v) { tr[i] = v; });
    ex.sync();
    qp_apply_GT<X, NX, NU>(ex, C, tr, tz);
    lane_batch<16>(ex, 0, P.nv, [&](int i) { return tz[i] + a1[i]; }, [&](int i, double v) { tz[i] = v; });
    ex.sync();
    qp_tree_solve<X, NX, NU>(ex, C, tz, a2, ox, oy);
    qp_apply_G<X, NX, NU>(ex, C, ox, tr);
    lane_batch<16>(ex, 0, P.nrows, [&](int i) { return dinv[i] * (tr[i] - a3[i]); }, [&](int i, double v) { oz[i] = v; });
    ex.sync();
  };
  once(r1, r2, r3, dx, dy, dz);
  const double sc = ex.max(fmax(fmax(strided_partial<8, 1>(ex.lane, ex.nlanes, P.nv, [&](int i) { return fabs(r1[i]); }),
                                     strided_partial<8, 1>(ex.lane, ex.nlanes, P.neq, [&](int i) { return fabs(r2[i]); })),
                                strided_partial<8, 1>(ex.lane, ex.nlanes, P.nrows, [&](int i) {
                                  return fabs(r3[i]) * sqrt(dinv[i]);
                                })));
  for (int itr = 0; itr < BMPC_NITREF; ++itr) {
    qp_apply_P<X, NX, NU>(ex, C, dx, e1);
    qp_apply_ET<X, NX, NU>(ex, C, dy, tv);
    lane_batch<16>(ex, 0, P.nv, [&](int i) { return r1[i] - e1[i] - tv[i]; }, [&](int i, double v) { e1[i] = v; });
    qp_apply_GT<X, NX, NU>(ex, C, dz, tv);
    lane_batch<16>(ex, 0, P.nv, [&](int i) { return e1[i] - tv[i]; }, [&](int i, double v) { e1[i] = v; });
    qp_apply_E<X, NX, NU>(ex, C, dx, e2);
    lane_batch<16>(ex, 0, P.neq, [&](int i) { return r2[i] - e2[i]; }, [&](int i, double v) { e2[i] = v; });
    qp_apply_G<X, NX, NU>(ex, C, dx, e3);
    lane_batch<16>(ex, 0, P.nrows, [&](int i) { return r3[i] - e3[i] + dz[i] / dinv[i]; },
                   [&](int i, double v) { e3[i] = v; });
    ex.sync();
    const double err = ex.max(fmax(fmax(strided_partial<8, 1>(ex.lane, ex.nlanes, P.nv, [&](int i) { return fabs(e1[i]); }),
                                        strided_partial<8, 1>(ex.lane, ex.nlanes, P.neq, [&](int i) { return fabs(e2[i]); })),
                                   strided_partial<8, 1>(ex.lane, ex.nlanes, P.nrows, [&](int i) {
                                     return fabs(e3[i]) * sqrt(dinv[i]);
                                   })));
    if (!(err > BMPC_REFTOL * fmax(sc, 1.0))) break;
    once(e1, e2, e3, cx, cy, cz);
    lane_batch<16>(ex, 0, P.nv, [&](int i) { return dx[i] + cx[i]; }, [&](int i, double v) { dx[i] = v; });
    lane_batch<16>(ex, 0, P.neq, [&](int i) { return dy[i] + cy[i]; }, [&](int i, double v) { dy[i] = v; });
    lane_batch<16>(ex, 0, P.nrows, [&](int i) { return dz[i] + cz[i]; }, [&](int i, double v) { dz[i] = v; });
    ex.sync();
  }
}

// ---- Mehrotra loop (oracle/qp_ipm.osqp_like_solve) -------------------------------------------
template <class X, int NX, int NU>
BMPC_FN IpmResult qp_ipm(const X ex, const QpCtx Cin) {
  const QpCtx C = Cin.uniform();
  CPlan& P = *C.P;
  CLayout& L = *C.L;
  gdouble* ws = C.ws;
  const int nv = P.nv, neq = P.neq, m = P.nrows;
  gdouble* x = ws + L.x;
  gdouble* y = ws + L.y;
  gdouble* z = ws + L.z;
  gdouble* s = ws + L.s;
  gdouble* dinv = ws + L.dl;
  gdouble* dx = ws + L.x2;
  gdouble* dy = ws + L.y2;
  gdouble* dz = ws + L.z2;
  gdouble* ds = ws + L.ds;
  gdouble* rd = ws + L.rx;
  gdouble* re = ws + L.ry;
  gdouble* rg = ws + L.rz;
  gdouble* g = ws + L.hvec;
  gdouble* e = ws + L.bvec;
  gdouble* q = ws + L.qq;
  gdouble* t1 = ws + L.ta;
  gdouble* t2 = ws + L.ya;
  gdouble* t3 = ws + L.ra;
  const double tol = 1e-10;
  IpmResult res{-2, 0, 0.0};
  // initial point with D = I
  lane_batch<16>(ex, 0, m, [&](int) { return 1.0; }, [&](int i, double v) { dinv[i] = v; });
  ex.sync();
  if (!qp_factor<X, NX, NU>(ex, C, dinv)) return res;
  lane_batch<16>(ex, 0, nv, [&](int i) { return -q[i]; }, [&](int i, double v) { t1[i] = v; });
  ex.sync();
  qp_kkt_solve<X, NX, NU>(ex, C, dinv, t1, e, g, x, y, z);
  qp_apply_G<X, NX, NU>(ex, C, x, s);
  lane_batch<16>(ex, 0, m, [&](int i) { return g[i] - s[i]; }, [&](int i, double v) { s[i] = v; });
  ex.sync();
  const double a0 = fmax(0.0, -ex.min(strided_partial<8, 2>(ex.lane, ex.nlanes, m, [&](int i) { return s[i]; })));
  struct SZ { double s, z; };
  lane_batch<16>(ex, 0, m, [&](int i) { return SZ{s[i] + a0 + 1.0, fmax(fabs(z[i]), 1.0)}; },
                 [&](int i, SZ v) { s[i] = v.s; z[i] = v.z; });
  ex.sync();
  auto amax_inf = [&](int n, const gdouble* a) {
    return ex.max(strided_partial<8, 1>(ex.lane, ex.nlanes, n, [&](int i) { return fabs(a[i]); }));
  };
  const double nq = fmax(1.0, amax_inf(nv, q));
  const double ne = fmax(1.0, amax_inf(neq, e));
  const double ng = fmax(1.0, amax_inf(m, g));
  auto step_to_boundary = [&](const gdouble* v, const gdouble* dv) {
    return ex.min(strided_partial<8, 2>(ex.lane, ex.nlanes, m, [&](int i) {
      return dv[i] < 0.0 ? -v[i] / dv[i] : 1e300;
    }));
  };
  for (int it = 0; it < P.desc.maxit; ++it) {
    res.iters = it;
    // residuals
    qp_apply_P<X, NX, NU>(ex, C, x, rd);
    qp_apply_ET<X, NX, NU>(ex, C, y, t1);
    lane_batch<16>(ex, 0, nv, [&](int i) { return rd[i] + q[i] + t1[i]; }, [&](int i, double v) { rd[i] = v; });
    qp_apply_GT<X, NX, NU>(ex, C, z, t1);
    lane_batch<16>(ex, 0, nv, [&](int i) { return rd[i] + t1[i]; }, [&](int i, double v) { rd[i] = v; });
    qp_apply_E<X, NX, NU>(ex, C, x, re);
    lane_batch<16>(ex, 0, neq, [&](int i) { return re[i] - e[i]; }, [&](int i, double v) { re[i] = v; });
    qp_apply_G<X, NX, NU>(ex, C, x, rg);
    lane_batch<16>(ex, 0, m, [&](int i) { return rg[i] + s[i] - g[i]; }, [&](int i, double v) { rg[i] = v; });
    ex.sync();
    const double mu = vdot(ex, s, z, m) / m;
#ifdef BMPC_HOST_DEBUG
    printf("qp it %d rd %.3e re %.3e rg %.3e mu %.3e\n", it, amax_inf(nv, rd), amax_inf(neq, re), amax_inf(m, rg), mu);
#endif
    // the inequality residual is judged against max(|g|, |s|) (OSQP's rule scales by the
    // larger of |Ax| and |z|): G x + s - g cancels to the rounding floor of s, which is not
    // bounded by |g| (quadruped config 4 stalled at rg = 9.3e-10 with |g| < 9)
    const double ngs = fmax(ng, amax_inf(m, s));
    if (amax_inf(nv, rd) < tol * nq && amax_inf(neq, re) < tol * ne && amax_inf(m, rg) < tol * ngs && mu < tol) {
      res.exit_flag = 1;
      break;
    }
    lane_batch<16>(ex, 0, m, [&](int i) { return z[i] / s[i]; }, [&](int i, double v) { dinv[i] = v; });
    ex.sync();
    if (!qp_factor<X, NX, NU>(ex, C, dinv)) break;
    // predictor
    lane_batch<16>(ex, 0, nv, [&](int i) { return -rd[i]; }, [&](int i, double v) { t1[i] = v; });
    lane_batch<16>(ex, 0, neq, [&](int i) { return -re[i]; }, [&](int i, double v) { t2[i] = v; });
    lane_batch<16>(ex, 0, m, [&](int i) { return -rg[i] + s[i]; }, [&](int i, double v) { t3[i] = v; });
    ex.sync();
    qp_kkt_solve<X, NX, NU>(ex, C, dinv, t1, t2, t3, dx, dy, dz);
    lane_batch<16>(ex, 0, m, [&](int i) { return -s[i] - s[i] / z[i] * dz[i]; }, [&](int i, double v) { ds[i] = v; });
    ex.sync();
    const double aa = fmin(1.0, fmin(step_to_boundary(s, ds), step_to_boundary(z, dz)));
    const double mua = lane_sum(ex, 0, m, [&](int i) { return (s[i] + aa * ds[i]) * (z[i] + aa * dz[i]); }) / m;
    const double sg = (mua / mu) * (mua / mu) * (mua / mu);
    // corrector: rhs3 = -rg + s + corr, corr = (ds o dz - sigma mu) / z
    lane_batch<16>(ex, 0, m, [&](int i) { return (ds[i] * dz[i] - sg * mu) / z[i]; }, [&](int i, double v) { ds[i] = v; });
    ex.sync();
    lane_batch<16>(ex, 0, m, [&](int i) { return -rg[i] + s[i] + ds[i]; }, [&](int i, double v) { t3[i] = v; });
    ex.sync();
    qp_kkt_solve<X, NX, NU>(ex, C, dinv, t1, t2, t3, dx, dy, dz);
    lane_batch<16>(ex, 0, m, [&](int i) { return -s[i] - s[i] / z[i] * dz[i] - ds[i]; }, [&](int i, double v) { ds[i] = v; });
    ex.sync();
    const double a = 0.99 * fmin(1.0, fmin(step_to_boundary(s, ds), step_to_boundary(z, dz)));
    lane_batch<16>(ex, 0, nv, [&](int i) { return x[i] + a * dx[i]; }, [&](int i, double v) { x[i] = v; });
    lane_batch<16>(ex, 0, neq, [&](int i) { return y[i] + a * dy[i]; }, [&](int i, double v) { y[i] = v; });
    lane_batch<16>(ex, 0, m, [&](int i) { return SZ{s[i] + a * ds[i], z[i] + a * dz[i]}; },
                   [&](int i, SZ v) { s[i] = v.s; z[i] = v.z; });
    ex.sync();
    res.iters = it + 1;
  }
  lane_batch<16>(ex, 0, nv, [&](int i) { return x[i]; }, [&](int i, double v) { ws[L.sol + i] = v; });
  ex.sync();
  qp_apply_P<X, NX, NU>(ex, C, x, t1);     // objective 1/2 x'Px + q'x (reported as J)
  res.pcost = lane_sum(ex, 0, nv, [&](int i) { return x[i] * (0.5 * t1[i] + q[i]); });
  return res;
}

// one BranchMPCProx solve after tree_update: build, IPM, unpack (osqp_solve_qp :461-487,
// unpackSolution :435-442 -- feasible only for status_val == 1, else the old plan stays)
template <class X, class M>
BMPC_HD IpmResult solve_ego_qp(const X& ex, const Plan& P, const Layout& L, EgoView E) {
  constexpr int NX = M::NX, NU = M::NU;
  gdouble* ws = (gdouble*)E.ws;
  QpCtx C{(CPlan*)&P, (CLayout*)&L, ws};
  qp_build<X, M>(ex, C, ws + L.hvec, ws + L.bvec);
  IpmResult r = qp_ipm<X, NX, NU>(ex, C);
  if (P.desc.controller == BMPC_CTRL_ROBUST) {
    // unpackSolution takes the solution whatever the status (:1459-1465); the next solve
    // linearises about the prediction shifted by one step (:1429-1431)
    const gdouble* sol = ws + L.sol;
    for (int i = ex.lane; i < P.U * NU; i += ex.nlanes) {
      ws[L.upred + i] = sol[P.oU + i];
      ws[L.uLin + i] = sol[P.oU + (i / NU + 1 < P.U ? i + NU : i)];
    }
    for (int i = ex.lane; i < P.T * NX; i += ex.nlanes) {
      ws[L.xpred + i] = sol[P.oX + i];
      ws[L.xlin + i] = sol[P.oX + (i / NX + 1 < P.T ? i + NX : i)];
    }
  } else if (r.exit_flag == 1) {
    const gdouble* sol = ws + L.sol;
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
    for (int i = 0; i < NU; ++i) ws[L.misc + MISC_OLDU + i] = ws[L.upred + i];   // OldInput = uPred[0]
  }
  ex.sync();
  return r;
}

}  // namespace bmpc
