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

#include "bmpc_tree.h"

namespace bmpc {

enum {
  EXIT_OPTIMAL = 0, EXIT_PINF = 1, EXIT_DINF = 2, EXIT_INACC = 10,
  EXIT_MAXIT = -1, EXIT_NUMERICS = -2
};

// ------------------------------------------------------------------------------------
// context bundling the per-ego pointers
// ------------------------------------------------------------------------------------
struct Ctx {
  const Plan* P;
  const Layout* L;
  double* ws;
  double qx[BMPC_MAX_N];   // xRef' Q
  double jcons;            // frozen xRef'Q xRef of the first solve (:1939)
  double ralpha;
  BMPC_HD double* at(size_t off) const { return ws + off; }
};

// ------------------------------------------------------------------------------------
// reductions over one cone's rows
// ------------------------------------------------------------------------------------
template <class X>
BMPC_HD double cone_dot(const X& ex, const double* a, const double* b, int off, int q) {
  double s = 0.0;
  for (int i = ex.lane; i < q; i += ex.nlanes) s += a[off + i] * b[off + i];
  return ex.sum(s);
}

// v0^2 - ||v1||^2 without squaring the dominant entry (see oracle.ecos_ipm.cone_res)
template <class X>
BMPC_HD double cone_res(const X& ex, const double* v, int off, int q) {
  double amax = 0.0;
  for (int i = 1 + ex.lane; i < q; i += ex.nlanes) amax = fmax(amax, fabs(v[off + i]));
  amax = ex.max(amax);
  double kidx = 1e300;
  for (int i = 1 + ex.lane; i < q; i += ex.nlanes)
    if (fabs(v[off + i]) == amax) kidx = fmin(kidx, (double)i);
  kidx = ex.min(kidx);
  double ss = 0.0;
  for (int i = 1 + ex.lane; i < q; i += ex.nlanes)
    if ((double)i != kidx) ss += v[off + i] * v[off + i];
  ss = ex.sum(ss);
  return cone_res_parts(v[off], amax, ss);
}

// ------------------------------------------------------------------------------------
// structured operators
// ------------------------------------------------------------------------------------
// x-coefficients of LP row c of state node k: c = 0 -> -dh_k, c >= 1 -> Fx[c-1]
BMPC_HD double fx_coef(const Ctx& C, int k, int c, int j) {
  const Plan& P = *C.P;
  if (c == 0) return -C.ws[C.L->dh + k * P.n + j];
  return P.desc.Fx[(c - 1) * P.n + j];
}

// value of the cone's F1 row dotted with a primal vector zv (unboosted)
template <int NX>
BMPC_HD double cone_f1_dot(const Ctx& C, int k, const double* zv) {
  const Plan& P = *C.P;
  const Topo& t = P.t;
  const int c = t.cone_c[k];
  double acc = 0.0;
  if (c >= 0) {
    const int b = t.cone_b[k], i = t.cone_i[k];
    const int ndx = t.br_ndx[c];
    for (int j = 0; j < P.N; ++j) {
      const int xk = ndx + j;
      for (int r = 0; r < NX; ++r) acc += -2.0 * C.qx[r] * zv[P.oX + xk * NX + r];
      for (int cc = 0; cc < P.Nc; ++cc) acc += P.desc.Qslack[1] * zv[P.oS + xk * P.Nc + cc];
    }
    acc += zv[P.oSig + b] + zv[P.oMup + b + i] - zv[P.oMum + b + i];
    if (t.br_child0[c] >= 0) acc += zv[P.oRho + c];
  } else {
    acc = -zv[P.oJ] + zv[P.oRho + 0];
    for (int cc = 0; cc < P.Nc; ++cc) acc += P.desc.Qslack[1] * zv[P.oS + cc];
  }
  return acc;
}

// out(rows) = G zv, cone rows boosted
template <class X, int NX, int NU>
BMPC_HD void apply_G(const X& ex, const Ctx& C, const double* zv, double* out) {
  const Plan& P = *C.P;
  const Topo& t = P.t;
  const int Nc = P.Nc;
  // Fx rows + positivity rows
  for (int it = ex.lane; it < P.T * Nc; it += ex.nlanes) {
    const int k = it / Nc, c = it % Nc;
    const double S = zv[P.oS + it];
    double v = -S;
    if (t.x_u[k] >= 0) {
      for (int j = 0; j < NX; ++j) v += fx_coef(C, k, c, j) * zv[P.oX + k * NX + j];
    }
    out[P.rFx + it] = v;
    out[P.rPos + it] = -S;
  }
  // Fu rows
  for (int it = ex.lane; it < P.U * P.nFu; it += ex.nlanes) {
    const int u = it / P.nFu, r = it % P.nFu;
    double v = 0.0;
    for (int j = 0; j < NU; ++j) v += P.desc.Fu[r * NU + j] * zv[P.oU + u * NU + j];
    out[P.rFu + it] = v;
  }
  // risk rows: -rho, -mu+, -mu-
  for (int it = ex.lane; it < P.bdim * (2 * P.m + 1); it += ex.nlanes) {
    out[P.rRisk + it] = it < P.bdim ? -zv[P.oRho + it] : -zv[P.oMup + (it - P.bdim)];
  }
  // cones
  const double* boost = C.at(C.L->boost);
  for (int k = ex.lane; k < P.ncones; k += ex.nlanes) {
    const int off = t.cone_off[k], q = t.cone_q[k];
    const double f = cone_f1_dot<NX>(C, k, zv) * exp(-boost[k]);
    out[off] = f;
    out[off + q - 1] = -f;
  }
  for (int k = 0; k < P.ncones; ++k) {
    const int off = t.cone_off[k], c = t.cone_c[k];
    const int nxn = c >= 0 ? P.N * NX : 0;
    const int nmid = c >= 0 ? P.N * (NX + NU) : NU;
    for (int it = ex.lane; it < nmid; it += ex.nlanes) {
      double v = 0.0;
      if (it < nxn) {
        const int j = it / NX, r = it % NX;
        const int xk = t.br_ndx[c] + j;
        for (int s = 0; s < NX; ++s) v += -2.0 * P.W1[r * NX + s] * zv[P.oX + xk * NX + s];
      } else {
        const int jj = it - nxn;
        const int j = jj / NU, r = jj % NU;
        const int uk = c >= 0 ? t.br_ndu[c] + j : 0;
        for (int s = 0; s < NU; ++s) v += -2.0 * P.Wu[r * NU + s] * zv[P.oU + uk * NU + s];
      }
      out[off + 1 + it] = v;
    }
  }
  ex.sync();
}

// out(nv) = G' r
template <class X, int NX, int NU>
BMPC_HD void apply_GT(const X& ex, const Ctx& C, const double* r, double* out) {
  const Plan& P = *C.P;
  const Topo& t = P.t;
  const int Nc = P.Nc;
  const double* boost = C.at(C.L->boost);
  const double Qs = P.desc.Qslack[1];
  // state nodes: x and S parts
  for (int k = ex.lane; k < P.T; k += ex.nlanes) {
    double ax[NX];
    for (int j = 0; j < NX; ++j) ax[j] = 0.0;
    const bool term = t.x_u[k] < 0;
    for (int c = 0; c < Nc; ++c) {
      const double rv = r[P.rFx + k * Nc + c];
      if (!term)
        for (int j = 0; j < NX; ++j) ax[j] += fx_coef(C, k, c, j) * rv;
      out[P.oS + k * Nc + c] = -rv - r[P.rPos + k * Nc + c];
    }
    const int kc = t.x_cone[k];
    if (kc >= 0) {
      const int off = t.cone_off[kc], q = t.cone_q[kc], j = t.x_conepos[k];
      const double f = (r[off] - r[off + q - 1]) * exp(-boost[kc]);
      for (int s = 0; s < NX; ++s) {
        double v = 0.0;
        for (int rr = 0; rr < NX; ++rr) v += -2.0 * P.W1[rr * NX + s] * r[off + 1 + j * NX + rr];
        ax[s] += v - 2.0 * C.qx[s] * f;
      }
      for (int c = 0; c < Nc; ++c) out[P.oS + k * Nc + c] += Qs * f;
    } else if (k == 0) {  // root slack in the root cone
      const int kr = P.ncones - 1;
      const int off = t.cone_off[kr], q = t.cone_q[kr];
      const double f = (r[off] - r[off + q - 1]) * exp(-boost[kr]);
      for (int c = 0; c < Nc; ++c) out[P.oS + c] += Qs * f;
    }
    for (int j = 0; j < NX; ++j) out[P.oX + k * NX + j] = ax[j];
  }
  // input nodes
  for (int u = ex.lane; u < P.U; u += ex.nlanes) {
    double au[NU];
    for (int j = 0; j < NU; ++j) au[j] = 0.0;
    for (int rr = 0; rr < P.nFu; ++rr) {
      const double rv = r[P.rFu + u * P.nFu + rr];
      for (int j = 0; j < NU; ++j) au[j] += P.desc.Fu[rr * NU + j] * rv;
    }
    const int kc = t.u_cone[u];
    if (kc >= 0) {
      const int off = t.cone_off[kc];
      const int c = t.cone_c[kc];
      const int base = c >= 0 ? 1 + P.N * NX + (u - t.br_ndu[c]) * NU : 1;
      for (int s = 0; s < NU; ++s) {
        double v = 0.0;
        for (int rr = 0; rr < NU; ++rr) v += -2.0 * P.Wu[rr * NU + s] * r[off + base + rr];
        au[s] += v;
      }
    }
    for (int j = 0; j < NU; ++j) out[P.oU + u * NU + j] = au[j];
  }
  // globals (one lane; few entries)
  if (ex.lane == 0) {
    for (int i = 0; i < P.ng; ++i) out[i == P.ng - 1 ? P.oJ : P.oRho + i] = 0.0;
    for (int b = 0; b < P.bdim; ++b) out[P.oRho + b] = -r[P.rRisk + b];
    for (int j = 0; j < 2 * P.bdim * P.m; ++j) out[P.oMup + j] = -r[P.rRisk + P.bdim + j];
    for (int k = 0; k < P.ncones; ++k) {
      const int off = t.cone_off[k], q = t.cone_q[k], c = t.cone_c[k];
      const double f = (r[off] - r[off + q - 1]) * exp(-boost[k]);
      if (c >= 0) {
        const int b = t.cone_b[k], i = t.cone_i[k];
        out[P.oSig + b] += f;
        out[P.oMup + b + i] += f;
        out[P.oMum + b + i] -= f;
        if (t.br_child0[c] >= 0) out[P.oRho + c] += f;
      } else {
        out[P.oJ] += -f;
        out[P.oRho + 0] += f;
      }
    }
  }
  ex.sync();
}

// out(neq) = A zv
template <class X, int NX, int NU>
BMPC_HD void apply_A(const X& ex, const Ctx& C, const double* zv, double* out) {
  const Plan& P = *C.P;
  const Topo& t = P.t;
  const double* Ad = C.at(C.L->Ad);
  const double* Bd = C.at(C.L->Bd);
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
  const double* p = C.at(C.L->p);
  for (int b = ex.lane; b < P.bdim; b += ex.nlanes) {
    double v = zv[P.oRho + b] + zv[P.oSig + b];
    for (int i = 0; i < P.m; ++i) v -= p[b * P.m + i] / C.ralpha * zv[P.oMum + b * P.m + i];
    out[P.T * NX + b] = v;
  }
  ex.sync();
}

// out(nv) = A' y
template <class X, int NX, int NU>
BMPC_HD void apply_AT(const X& ex, const Ctx& C, const double* y, double* out) {
  const Plan& P = *C.P;
  const Topo& t = P.t;
  const double* Ad = C.at(C.L->Ad);
  const double* Bd = C.at(C.L->Bd);
  for (int k = ex.lane; k < P.T; k += ex.nlanes) {
    double ax[NX], au[NU];
    for (int r = 0; r < NX; ++r) ax[r] = y[k * NX + r];
    for (int r = 0; r < NU; ++r) au[r] = 0.0;
    const int u = t.x_u[k];
    if (u >= 0) {
      double ys[NX];
      for (int r = 0; r < NX; ++r) ys[r] = 0.0;
      for (int e = t.succ_off[k]; e < t.succ_off[k + 1]; ++e) {
        const int c = t.succ[e];
        for (int r = 0; r < NX; ++r) ys[r] += y[c * NX + r];
      }
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
  for (int it = ex.lane; it < P.T * P.Nc; it += ex.nlanes) out[P.oS + it] = 0.0;
  const double* p = C.at(C.L->p);
  if (ex.lane == 0) {
    for (int i = 0; i < P.ng; ++i) out[i == P.ng - 1 ? P.oJ : P.oRho + i] = 0.0;
    for (int b = 0; b < P.bdim; ++b) {
      const double yb = y[P.T * NX + b];
      out[P.oRho + b] += yb;
      out[P.oSig + b] += yb;
      for (int i = 0; i < P.m; ++i) out[P.oMum + b * P.m + i] += -p[b * P.m + i] / C.ralpha * yb;
    }
  }
  ex.sync();
}

// h (rows) and b (eq) of this solve
template <class X, int NX, int NU>
BMPC_HD void build_hb(const X& ex, const Ctx& C, double* h, double* bv) {
  const Plan& P = *C.P;
  const Topo& t = P.t;
  const int Nc = P.Nc;
  const double* h0 = C.at(C.L->h0);
  for (int it = ex.lane; it < P.T * Nc; it += ex.nlanes) {
    const int k = it / Nc, c = it % Nc;
    double v = 0.0;
    if (t.x_u[k] >= 0) v = c == 0 ? h0[k] : P.desc.bx[c - 1];
    h[P.rFx + it] = v;
    h[P.rPos + it] = 0.0;
  }
  for (int it = ex.lane; it < P.U * P.nFu; it += ex.nlanes) h[P.rFu + it] = P.desc.bu[it % P.nFu];
  for (int it = ex.lane; it < P.bdim * (2 * P.m + 1); it += ex.nlanes) h[P.rRisk + it] = 0.0;
  const double* boost = C.at(C.L->boost);
  for (int k = 0; k < P.ncones; ++k) {
    const int off = t.cone_off[k], q = t.cone_q[k];
    for (int i = ex.lane; i < q; i += ex.nlanes) h[off + i] = 0.0;
  }
  ex.sync();
  for (int k = ex.lane; k < P.ncones; k += ex.nlanes) {
    const int off = t.cone_off[k], q = t.cone_q[k];
    const double a = t.cone_c[k] >= 0 ? C.jcons * P.N : 0.0;
    const double h0v = 1.0 - a, hlv = 1.0 + a;
    const double ch = cosh(boost[k]), sh = sinh(boost[k]);
    h[off] = ch * h0v + sh * hlv;
    h[off + q - 1] = sh * h0v + ch * hlv;
  }
  const double* Cd = C.at(C.L->Cd);
  const double* xbar = C.at(C.L->xbar);
  for (int k = ex.lane; k < P.T; k += ex.nlanes) {
    const int su = t.x_srcu[k];
    for (int r = 0; r < NX; ++r) bv[k * NX + r] = su >= 0 ? Cd[su * NX + r] : xbar[r];
  }
  for (int b = ex.lane; b < P.bdim; b += ex.nlanes) bv[P.T * NX + b] = 0.0;
  ex.sync();
}

// ------------------------------------------------------------------------------------
// Nesterov-Todd scaling
// ------------------------------------------------------------------------------------
// returns false when an iterate left its cone
template <class X>
BMPC_HD bool compute_scaling(const X& ex, const Ctx& C, const double* s, const double* z) {
  const Plan& P = *C.P;
  const Topo& t = P.t;
  double* dl = C.at(C.L->dl);
  double* lam = C.at(C.L->lam);
  double* eta = C.at(C.L->eta);
  double* wb = C.at(C.L->wbar);
  double* vn = C.at(C.L->vnt);
  int bad = 0;
  for (int i = ex.lane; i < P.nlp; i += ex.nlanes) {
    if (!(s[i] > 0.0 && z[i] > 0.0)) bad = 1;
    dl[i] = sqrt(s[i] / z[i]);
    lam[i] = sqrt(s[i] * z[i]);
  }
  if (ex.max((double)bad) > 0.0) return false;
  for (int k = 0; k < P.ncones; ++k) {
    const int off = t.cone_off[k], q = t.cone_q[k];
    const double sres = cone_res(ex, s, off, q);
    const double zres = cone_res(ex, z, off, q);
    if (!(sres > 0.0 && zres > 0.0)) return false;
    const double sn = sqrt(sres), zn = sqrt(zres);
    const double sz = cone_dot(ex, s, z, off, q) / (sn * zn);
    const double gam = sqrt((1.0 + sz) / 2.0);
    for (int i = ex.lane; i < q; i += ex.nlanes) {
      const double jz = i == 0 ? z[off] : -z[off + i];
      wb[off + i] = (s[off + i] / sn + jz / zn) / (2.0 * gam);
    }
    ex.sync();
    const double w0 = wb[off];
    const double nrm = sqrt(2.0 * (w0 + 1.0));
    for (int i = ex.lane; i < q; i += ex.nlanes) vn[off + i] = (wb[off + i] + (i == 0 ? 1.0 : 0.0)) / nrm;
    if (ex.lane == 0) eta[k] = sqrt(sn / zn);
    ex.sync();
    const double e = sqrt(sn / zn);
    const double vz = cone_dot(ex, vn, z, off, q);
    for (int i = ex.lane; i < q; i += ex.nlanes) {
      const double jz = i == 0 ? z[off] : -z[off + i];
      lam[off + i] = e * (2.0 * vn[off + i] * vz - jz);
    }
  }
  ex.sync();
  return true;
}

// identity scaling for the initial point
template <class X>
BMPC_HD void identity_scaling(const X& ex, const Ctx& C) {
  const Plan& P = *C.P;
  const Topo& t = P.t;
  double* dl = C.at(C.L->dl);
  for (int i = ex.lane; i < P.nlp; i += ex.nlanes) dl[i] = 1.0;
  for (int k = 0; k < P.ncones; ++k) {
    const int off = t.cone_off[k], q = t.cone_q[k];
    for (int i = ex.lane; i < q; i += ex.nlanes) {
      C.ws[C.L->wbar + off + i] = i == 0 ? 1.0 : 0.0;
      C.ws[C.L->vnt + off + i] = i == 0 ? 1.0 : 0.0;
    }
  }
  for (int k = ex.lane; k < P.ncones; k += ex.nlanes) C.ws[C.L->eta + k] = 1.0;
  ex.sync();
}

// mode 0: W v, 1: W^-1 v, 2: W^2 v, 3: W^-2 v   (W symmetric NT scaling)
template <class X>
BMPC_HD void apply_W(const X& ex, const Ctx& C, int mode, const double* in, double* out) {
  const Plan& P = *C.P;
  const Topo& t = P.t;
  const double* dl = C.at(C.L->dl);
  for (int i = ex.lane; i < P.nlp; i += ex.nlanes) {
    const double w = dl[i];
    out[i] = mode == 0 ? w * in[i] : mode == 1 ? in[i] / w : mode == 2 ? w * w * in[i] : in[i] / (w * w);
  }
  const double* eta = C.at(C.L->eta);
  const double* wb = C.at(C.L->wbar);
  const double* vn = C.at(C.L->vnt);
  for (int k = 0; k < P.ncones; ++k) {
    const int off = t.cone_off[k], q = t.cone_q[k];
    const double e = eta[k];
    // W = e (2 v v' - J); W^-1 = (2 Jv Jv' - J)/e; W^2 = e^2 (2 wb wb' - J); W^-2 = (2 Jwb Jwb' - J)/e^2
    const double* a = (mode == 0 || mode == 1) ? vn : wb;
    const bool jconj = (mode == 1 || mode == 3);
    double part = 0.0;
    for (int i = ex.lane; i < q; i += ex.nlanes) {
      const double ai = (jconj && i > 0) ? -a[off + i] : a[off + i];
      part += ai * in[off + i];
    }
    const double dot = ex.sum(part);
    const double sc = mode == 0 ? e : mode == 1 ? 1.0 / e : mode == 2 ? e * e : 1.0 / (e * e);
    for (int i = ex.lane; i < q; i += ex.nlanes) {
      const double ai = (jconj && i > 0) ? -a[off + i] : a[off + i];
      const double jv = i == 0 ? in[off] : -in[off + i];
      out[off + i] = sc * (2.0 * ai * dot - jv);
    }
    ex.sync();
  }
  ex.sync();
}

// Jordan product out = u o v
template <class X>
BMPC_HD void jprod(const X& ex, const Ctx& C, const double* u, const double* v, double* out) {
  const Plan& P = *C.P;
  const Topo& t = P.t;
  for (int i = ex.lane; i < P.nlp; i += ex.nlanes) out[i] = u[i] * v[i];
  for (int k = 0; k < P.ncones; ++k) {
    const int off = t.cone_off[k], q = t.cone_q[k];
    const double dot = cone_dot(ex, u, v, off, q);
    const double u0 = u[off], v0 = v[off];
    ex.sync();
    for (int i = 1 + ex.lane; i < q; i += ex.nlanes) out[off + i] = u0 * v[off + i] + v0 * u[off + i];
    if (ex.lane == 0) out[off] = dot;
    ex.sync();
  }
  ex.sync();
}

// out = lam \ v  (lam o out = v)
template <class X>
BMPC_HD void jdiv(const X& ex, const Ctx& C, const double* lam, const double* v, double* out) {
  const Plan& P = *C.P;
  const Topo& t = P.t;
  for (int i = ex.lane; i < P.nlp; i += ex.nlanes) out[i] = v[i] / lam[i];
  for (int k = 0; k < P.ncones; ++k) {
    const int off = t.cone_off[k], q = t.cone_q[k];
    const double rho = cone_res(ex, lam, off, q);
    double part = 0.0;
    for (int i = 1 + ex.lane; i < q; i += ex.nlanes) part += lam[off + i] * v[off + i];
    const double lv = ex.sum(part);
    const double l0 = lam[off];
    const double x0 = (l0 * v[off] - lv) / rho;
    ex.sync();
    for (int i = 1 + ex.lane; i < q; i += ex.nlanes) out[off + i] = (v[off + i] - x0 * lam[off + i]) / l0;
    if (ex.lane == 0) out[off] = x0;
    ex.sync();
  }
  ex.sync();
}

// largest alpha with lam + alpha d in the cone (ECOS lineSearch for one direction)
template <class X>
BMPC_HD double max_step(const X& ex, const Ctx& C, const double* lam, const double* d) {
  const Plan& P = *C.P;
  const Topo& t = P.t;
  double a = 1e300;
  for (int i = ex.lane; i < P.nlp; i += ex.nlanes)
    if (d[i] < 0.0) a = fmin(a, -lam[i] / d[i]);
  a = ex.min(a);
  for (int k = 0; k < P.ncones; ++k) {
    const int off = t.cone_off[k], q = t.cone_q[k];
    const double ln2 = cone_res(ex, lam, off, q);
    if (!(ln2 > 0.0)) return 0.0;
    const double ln = sqrt(ln2);
    double part = 0.0;
    for (int i = 1 + ex.lane; i < q; i += ex.nlanes) part += lam[off + i] * d[off + i];
    const double ld = ex.sum(part);
    const double lb0 = lam[off] / ln;
    const double rho0 = (lam[off] * d[off] - ld) / ln;
    const double fac = (rho0 + d[off]) / (lb0 + 1.0);
    double ss = 0.0;
    for (int i = 1 + ex.lane; i < q; i += ex.nlanes) {
      const double r1 = d[off + i] - fac * lam[off + i] / ln;
      ss += r1 * r1;
    }
    ss = ex.sum(ss);
    const double tt = sqrt(ss) - rho0;
    if (tt > 0.0) a = fmin(a, ln / tt);
  }
  return a;
}

// ------------------------------------------------------------------------------------
// KKT factorisation
// ------------------------------------------------------------------------------------
template <class X, int NX, int NU>
BMPC_HD bool kkt_factor(const X& ex, const Ctx& C) {
  const Plan& P = *C.P;
  const Layout& L = *C.L;
  const Topo& t = P.t;
  const int Nc = P.Nc;
  double* ws = C.ws;
  const double* dl = ws + L.dl;
  const double* eta = ws + L.eta;
  const double* wb = ws + L.wbar;
  const double* boost = ws + L.boost;
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
        for (int j = 0; j < NX; ++j) f[j] = fx_coef(C, k, c, j);
        for (int i = 0; i < NX; ++i)
          for (int j = 0; j < NX; ++j) H[i][j] += om * f[i] * f[j];
      }
    }
    const int kc = t.x_cone[k];
    if (kc >= 0) {
      const double sc = 4.0 / (eta[kc] * eta[kc]);
      for (int i = 0; i < NX; ++i)
        for (int j = 0; j < NX; ++j) H[i][j] += sc * P.QQ[i * NX + j];
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
  for (int k = 0; k < P.ncones; ++k) {
    double* g = ws + L.gk + (size_t)k * P.nv;
    for (int i = ex.lane; i < P.nv; i += ex.nlanes) g[i] = 0.0;
  }
  ex.sync();
  for (int k = 0; k < P.ncones; ++k) {
    double* g = ws + L.gk + (size_t)k * P.nv;
    const int off = t.cone_off[k], q = t.cone_q[k], c = t.cone_c[k];
    const double kap = (wb[off] + wb[off + q - 1]) * exp(-boost[k]);
    if (c >= 0) {
      for (int it = ex.lane; it < P.N; it += ex.nlanes) {
        const int xk = t.br_ndx[c] + it, uk = t.br_ndu[c] + it;
        const double* wx = wb + off + 1 + it * NX;
        const double* wu = wb + off + 1 + P.N * NX + it * NU;
        for (int s = 0; s < NX; ++s) {
          double v = 0.0;
          for (int r = 0; r < NX; ++r) v += P.W1[r * NX + s] * wx[r];
          g[P.oX + xk * NX + s] = kap * (-2.0 * C.qx[s]) + 2.0 * v;
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
        g[P.oSig + b] += kap;
        g[P.oMup + b + i] += kap;
        g[P.oMum + b + i] -= kap;
        if (t.br_child0[c] >= 0) g[P.oRho + c] += kap;
      }
    } else if (ex.lane == 0) {
      g[P.oJ] = -kap;
      g[P.oRho + 0] += kap;
      for (int cc = 0; cc < Nc; ++cc) g[P.oS + cc] = kap * Qs;
      for (int s = 0; s < NU; ++s) {
        double v = 0.0;
        for (int r = 0; r < NU; ++r) v += P.Wu[r * NU + s] * wb[off + 1 + r];
        g[P.oU + s] = 2.0 * v;
      }
    }
  }
  ex.sync();
  // ---- tree Riccati factorisation (leaves -> root) ---------------------------------------
  const double* Ad = ws + L.Ad;
  const double* Bd = ws + L.Bd;
  int bad = 0;
  for (int lv = P.nlevels - 1; lv >= 0; --lv) {
    for (int e = t.lvl_off[lv] + ex.lane; e < t.lvl_off[lv + 1]; e += ex.nlanes) {
      const int k = t.lvl_nodes[e];
      double Pk[NX][NX];
      mat_load(Pk, ws + L.hx + k * NX * NX);
      const int u = t.x_u[k];
      if (u >= 0) {
        double Pb[NX][NX], A[NX][NX], B[NX][NU], M[NX][NX];
        for (int i = 0; i < NX; ++i)
          for (int j = 0; j < NX; ++j) Pb[i][j] = 0.0;
        for (int sidx = t.succ_off[k]; sidx < t.succ_off[k + 1]; ++sidx) {
          const double* Pc = ws + L.P + t.succ[sidx] * NX * NX;
          for (int i = 0; i < NX; ++i)
            for (int j = 0; j < NX; ++j) Pb[i][j] += Pc[i * NX + j];
        }
        mat_load(A, Ad + u * NX * NX);
        mat_load(B, Bd + u * NX * NU);
        for (int i = 0; i < NX; ++i)
          for (int j = 0; j < NX; ++j) {
            double v = 0.0;
            for (int r = 0; r < NX; ++r) v += Pb[i][r] * A[r][j];
            M[i][j] = v;
          }
        double Qux[NU][NX], Quu[NU][NU], PB[NX][NU];
        for (int i = 0; i < NX; ++i)
          for (int j = 0; j < NX; ++j) {
            double v = 0.0;
            for (int r = 0; r < NX; ++r) v += A[r][i] * M[r][j];
            Pk[i][j] += v;
          }
        for (int i = 0; i < NU; ++i)
          for (int j = 0; j < NX; ++j) {
            double v = 0.0;
            for (int r = 0; r < NX; ++r) v += B[r][i] * M[r][j];
            Qux[i][j] = v;
          }
        for (int i = 0; i < NX; ++i)
          for (int j = 0; j < NU; ++j) {
            double v = 0.0;
            for (int r = 0; r < NX; ++r) v += Pb[i][r] * B[r][j];
            PB[i][j] = v;
          }
        mat_load(Quu, ws + L.hu + u * NU * NU);
        for (int i = 0; i < NU; ++i)
          for (int j = 0; j < NU; ++j) {
            double v = 0.0;
            for (int r = 0; r < NX; ++r) v += B[r][i] * PB[r][j];
            Quu[i][j] += v;
          }
        if (!chol<NU>(Quu)) bad = 1;
        mat_store(Quu, ws + L.Luu + u * NU * NU);
        double K[NU][NX];
        for (int j = 0; j < NX; ++j) {
          double col[NU];
          for (int i = 0; i < NU; ++i) col[i] = -Qux[i][j];
          chol_solve<NU>(Quu, col);
          for (int i = 0; i < NU; ++i) K[i][j] = col[i];
        }
        mat_store(K, ws + L.Kg + u * NU * NX);
        for (int i = 0; i < NX; ++i)
          for (int j = 0; j < NX; ++j) {
            double v = 0.0;
            for (int r = 0; r < NU; ++r) v += Qux[r][i] * K[r][j];
            Pk[i][j] += v;
          }
        for (int i = 0; i < NX; ++i)
          for (int j = i + 1; j < NX; ++j) {
            const double a = 0.5 * (Pk[i][j] + Pk[j][i]);
            Pk[i][j] = a;
            Pk[j][i] = a;
          }
      }
      mat_store(Pk, ws + L.P + k * NX * NX);
    }
    ex.sync();
  }
  return ex.max((double)bad) == 0.0;
}

// Tree solve of  [H_t A_dyn'; A_dyn 0] [v; nu] = [r; e]  for nr right-hand sides.
// rhs r_i lives in z-space (x, u, S parts at P.oX/oU/oS), e_i in eq-space (first T*n rows,
// NULL = 0).  Solutions go to out_i (z-space tree parts) and nu_i (eq-space, NULL skips).
template <class X, int NX, int NU>
BMPC_HD void tree_solve(const X& ex, const Ctx& C, int nr, const double* const* r,
                        const double* const* e, double* const* out, double* const* nu) {
  const Plan& P = *C.P;
  const Layout& L = *C.L;
  const Topo& t = P.t;
  const int Nc = P.Nc;
  double* ws = C.ws;
  const double* Ad = ws + L.Ad;
  const double* Bd = ws + L.Bd;
  double* lv_ = ws + L.lvec;   // [nr][T][NX]
  double* kf_ = ws + L.kff;    // [nr][U][NU]
  const size_t lstr = (size_t)P.T * NX, kstr = (size_t)P.U * NU;
  // backward sweep
  for (int lv = P.nlevels - 1; lv >= 0; --lv) {
    const int nlv = t.lvl_off[lv + 1] - t.lvl_off[lv];
    for (int it = ex.lane; it < nlv * nr; it += ex.nlanes) {
      const int k = t.lvl_nodes[t.lvl_off[lv] + it / nr], ri = it % nr;
      const double* rr = r[ri];
      double* lvec = lv_ + ri * lstr;
      double qx[NX];
      for (int j = 0; j < NX; ++j) qx[j] = -rr[P.oX + k * NX + j];
      const bool term = t.x_u[k] < 0;
      if (!term) {  // slack elimination: rx_eff = rx + sum_c df f_c rS_c / sd_c
        for (int c = 0; c < Nc; ++c) {
          const double sd = ws[L.sd + (k * Nc + c) * 2], df = ws[L.sd + (k * Nc + c) * 2 + 1];
          const double a = df * rr[P.oS + k * Nc + c] / sd;
          for (int j = 0; j < NX; ++j) qx[j] -= fx_coef(C, k, c, j) * a;
        }
      }
      if (!term) {
        const int u = t.x_u[k];
        double g[NX];
        for (int j = 0; j < NX; ++j) g[j] = 0.0;
        for (int sidx = t.succ_off[k]; sidx < t.succ_off[k + 1]; ++sidx) {
          const int c = t.succ[sidx];
          const double* Pc = ws + L.P + c * NX * NX;
          const double* lc = lvec + c * NX;
          for (int i = 0; i < NX; ++i) {
            double v = lc[i];
            if (e[ri])
              for (int j = 0; j < NX; ++j) v += Pc[i * NX + j] * e[ri][c * NX + j];
            g[i] += v;
          }
        }
        double qu[NU];
        for (int i = 0; i < NU; ++i) {
          double v = -rr[P.oU + u * NU + i];
          for (int j = 0; j < NX; ++j) v += Bd[u * NX * NU + j * NU + i] * g[j];
          qu[i] = v;
        }
        for (int i = 0; i < NX; ++i) {
          double v = 0.0;
          for (int j = 0; j < NX; ++j) v += Ad[u * NX * NX + j * NX + i] * g[j];
          qx[i] += v;
        }
        double Lu[NU][NU], kf[NU];
        mat_load(Lu, ws + L.Luu + u * NU * NU);
        for (int i = 0; i < NU; ++i) kf[i] = -qu[i];
        chol_solve<NU>(Lu, kf);
        const double* K = ws + L.Kg + u * NU * NX;
        for (int i = 0; i < NX; ++i) {
          double v = 0.0;
          for (int j = 0; j < NU; ++j) v += K[j * NX + i] * qu[j];
          qx[i] += v;
        }
        for (int i = 0; i < NU; ++i) kf_[ri * kstr + u * NU + i] = kf[i];
      }
      for (int j = 0; j < NX; ++j) lvec[k * NX + j] = qx[j];
    }
    ex.sync();
  }
  // forward sweep
  for (int it = ex.lane; it < nr; it += ex.nlanes) {
    for (int j = 0; j < NX; ++j) out[it][P.oX + j] = e[it] ? e[it][j] : 0.0;
  }
  ex.sync();
  for (int lv = 0; lv < P.nlevels; ++lv) {
    const int nlv = t.lvl_off[lv + 1] - t.lvl_off[lv];
    for (int it = ex.lane; it < nlv * nr; it += ex.nlanes) {
      const int k = t.lvl_nodes[t.lvl_off[lv] + it / nr], ri = it % nr;
      double* o = out[ri];
      const double* rr = r[ri];
      double xk[NX];
      for (int j = 0; j < NX; ++j) xk[j] = o[P.oX + k * NX + j];
      const double* Pk = ws + L.P + k * NX * NX;
      const double* lk = lv_ + ri * lstr + k * NX;
      if (nu[ri])
        for (int i = 0; i < NX; ++i) {
          double v = lk[i];
          for (int j = 0; j < NX; ++j) v += Pk[i * NX + j] * xk[j];
          nu[ri][k * NX + i] = -v;
        }
      const bool term = t.x_u[k] < 0;
      for (int c = 0; c < Nc; ++c) {  // slack recovery
        const double sd = ws[L.sd + (k * Nc + c) * 2], df = ws[L.sd + (k * Nc + c) * 2 + 1];
        double fx = 0.0;
        if (!term)
          for (int j = 0; j < NX; ++j) fx += fx_coef(C, k, c, j) * xk[j];
        o[P.oS + k * Nc + c] = (rr[P.oS + k * Nc + c] + df * fx) / sd;
      }
      if (!term) {
        const int u = t.x_u[k];
        const double* K = ws + L.Kg + u * NU * NX;
        double uk[NU];
        for (int i = 0; i < NU; ++i) {
          double v = kf_[ri * kstr + u * NU + i];
          for (int j = 0; j < NX; ++j) v += K[i * NX + j] * xk[j];
          uk[i] = v;
          o[P.oU + u * NU + i] = v;
        }
        double xp[NX];
        for (int i = 0; i < NX; ++i) {
          double v = 0.0;
          for (int j = 0; j < NX; ++j) v += Ad[u * NX * NX + i * NX + j] * xk[j];
          for (int j = 0; j < NU; ++j) v += Bd[u * NX * NU + i * NU + j] * uk[j];
          xp[i] = v;
        }
        for (int sidx = t.succ_off[k]; sidx < t.succ_off[k + 1]; ++sidx) {
          const int c = t.succ[sidx];
          for (int i = 0; i < NX; ++i) o[P.oX + c * NX + i] = xp[i] + (e[ri] ? e[ri][c * NX + i] : 0.0);
        }
      }
    }
    ex.sync();
  }
}

// dense LU with partial pivoting of the coupling system (row-major nsm x nsm)
template <class X>
BMPC_HD bool small_lu(const X& ex, double* M, double* piv, int n) {
  for (int k = 0; k < n; ++k) {
    double best = -1.0, bi = 1e300;
    for (int i = k + ex.lane; i < n; i += ex.nlanes) {
      const double a = fabs(M[i * n + k]);
      if (a > best || (a == best && i < bi)) best = a, bi = (double)i;
    }
    const double amax = ex.max(best);
    double cand = 1e300;
    for (int i = k + ex.lane; i < n; i += ex.nlanes)
      if (fabs(M[i * n + k]) == amax) cand = fmin(cand, (double)i);
    const int p = (int)ex.min(cand);
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
    for (int i = k + 1 + ex.lane; i < n; i += ex.nlanes) {
      const double l = M[i * n + k] / d;
      M[i * n + k] = l;
      for (int j = k + 1; j < n; ++j) M[i * n + j] -= l * M[k * n + j];
    }
    ex.sync();
  }
  return true;
}

template <class X>
BMPC_HD void small_lu_solve(const X& ex, const double* M, const double* piv, double* b, int n) {
  if (ex.lane == 0) {
    for (int k = 0; k < n; ++k) {
      const int p = (int)piv[k];
      if (p != k) {
        const double tmp = b[k];
        b[k] = b[p];
        b[p] = tmp;
      }
    }
    for (int i = 0; i < n; ++i) {
      double v = b[i];
      for (int j = 0; j < i; ++j) v -= M[i * n + j] * b[j];
      b[i] = v;
    }
    for (int i = n - 1; i >= 0; --i) {
      double v = b[i];
      for (int j = i + 1; j < n; ++j) v -= M[i * n + j] * b[j];
      b[i] = v / M[i * n + i];
    }
  }
  ex.sync();
}

// global variable index -> position in the primal vector
BMPC_HD int gvar(const Plan& P, int i) { return i == P.ng - 1 ? P.oJ : P.oRho + i; }

// Woodbury columns, coupling matrix and its LU; returns false on breakdown
template <class X, int NX, int NU>
BMPC_HD bool kkt_coupling(const X& ex, const Ctx& C) {
  const Plan& P = *C.P;
  const Layout& L = *C.L;
  double* ws = C.ws;
  const int nc = P.ncones;
  const double* rr[32];
  const double* ee[32];
  double* oo[32];
  double* nn[32];
  for (int k = 0; k < nc; ++k) {
    rr[k] = ws + L.gk + (size_t)k * P.nv;
    ee[k] = nullptr;
    oo[k] = ws + L.colk + (size_t)k * P.nv;
    nn[k] = ws + L.colnu + (size_t)k * P.neq;
  }
  tree_solve<X, NX, NU>(ex, C, nc, rr, ee, oo, nn);
  const int ng = P.ng, nb = P.bdim, ns = P.nsm;
  double* M = ws + L.Msm;
  const double* eta = ws + L.eta;
  const double* dl = ws + L.dl;
  const double* p = ws + L.p;
  const int ntree = P.oRho;    // x and u parts are [0, oRho); S part [oS, oJ)
  // cone-cone block: c_k (I/c_k + M) with M[k][j] = g_k' col_j over tree variables
  for (int it = 0; it < nc * nc; ++it) {
    const int k = it / nc, j = it % nc;
    const double* g = ws + L.gk + (size_t)k * P.nv;
    const double* col = ws + L.colk + (size_t)j * P.nv;
    double s = 0.0;
    for (int i = ex.lane; i < ntree; i += ex.nlanes) s += g[i] * col[i];
    for (int i = P.oS + ex.lane; i < P.oJ; i += ex.nlanes) s += g[i] * col[i];
    s = ex.sum(s);
    if (ex.lane == 0) {
      const double ck = 2.0 / (eta[k] * eta[k]);
      M[(ng + nb + k) * ns + ng + nb + j] = ck * s + (k == j ? 1.0 : 0.0);
    }
  }
  if (ex.lane == 0) {
    for (int i = 0; i < ng + nb; ++i)
      for (int j = 0; j < ns; ++j) M[i * ns + j] = 0.0;
    for (int k = 0; k < nc; ++k)
      for (int j = 0; j < ng + nb; ++j) M[(ng + nb + k) * ns + j] = 0.0;
    // H_gg diagonal: LP rows -rho, -mu+, -mu-
    for (int b = 0; b < nb; ++b) {
      const double w = dl[P.rRisk + b];
      M[b * ns + b] = 1.0 / (w * w);
    }
    for (int j = 0; j < 2 * nb * P.m; ++j) {
      const double w = dl[P.rRisk + nb + j];
      const int gi = 2 * nb + j;
      M[gi * ns + gi] = 1.0 / (w * w);
    }
    // CVaR equality rows and their transpose
    for (int b = 0; b < nb; ++b) {
      const int row = ng + b;
      M[row * ns + b] = 1.0;
      M[b * ns + row] = 1.0;
      M[row * ns + nb + b] = 1.0;
      M[(nb + b) * ns + row] = 1.0;
      for (int i = 0; i < P.m; ++i) {
        const int gi = 2 * nb + nb * P.m + b * P.m + i;
        const double a = -p[b * P.m + i] / C.ralpha;
        M[row * ns + gi] = a;
        M[gi * ns + row] = a;
      }
    }
    // cone coupling with the globals
    for (int k = 0; k < nc; ++k) {
      const double* g = ws + L.gk + (size_t)k * P.nv;
      const double ck = 2.0 / (eta[k] * eta[k]);
      for (int i = 0; i < ng; ++i) {
        const double gv = g[gvar(P, i)];
        M[i * ns + ng + nb + k] = gv;
        M[(ng + nb + k) * ns + i] = -ck * gv;
      }
    }
  }
  ex.sync();
  return small_lu(ex, M, ws + L.piv, ns);
}

// One pass of the W-scaled KKT system (oracle/ecos_ipm.py KKT)
//   [0 A' G'W^-1; A 0 0; W^-1 G 0 -I] [dx; dy; dzh] = [r1; r2; r3h],   dzh = W dz,
// by the reduced Hessian G'W^-2G (tree Riccati + Woodbury coupling).
template <class X, int NX, int NU>
BMPC_HD void kkt_solve_once(const X& ex, const Ctx& C, const double* r1, const double* r2,
                            const double* r3h, double* dx, double* dy, double* dzh) {
  const Plan& P = *C.P;
  const Layout& L = *C.L;
  double* ws = C.ws;
  double* tr = ws + L.k_r0;
  double* tz = ws + L.k_nv0;
  apply_W(ex, C, 1, r3h, tr);                     // W^-1 r3h
  apply_GT<X, NX, NU>(ex, C, tr, tz);             // G' W^-1 r3h
  for (int i = ex.lane; i < P.nv; i += ex.nlanes) tz[i] += r1[i];
  ex.sync();
  {
    const double* rr[1] = {tz};
    const double* ee[1] = {r2};
    double* oo[1] = {dx};
    double* nn[1] = {dy};
    tree_solve<X, NX, NU>(ex, C, 1, rr, ee, oo, nn);
  }
  const int ng = P.ng, nb = P.bdim, nc = P.ncones, ns = P.nsm;
  double* b = ws + L.smrhs;
  const double* eta = ws + L.eta;
  for (int k = 0; k < nc; ++k) {
    const double* g = ws + L.gk + (size_t)k * P.nv;
    double s = 0.0;
    for (int i = ex.lane; i < P.oRho; i += ex.nlanes) s += g[i] * dx[i];
    for (int i = P.oS + ex.lane; i < P.oJ; i += ex.nlanes) s += g[i] * dx[i];
    s = ex.sum(s);
    if (ex.lane == 0) b[ng + nb + k] = 2.0 / (eta[k] * eta[k]) * s;
  }
  if (ex.lane == 0) {
    for (int i = 0; i < ng; ++i) b[i] = tz[gvar(P, i)];
    for (int j = 0; j < nb; ++j) b[ng + j] = r2[P.T * NX + j];
  }
  ex.sync();
  small_lu_solve(ex, ws + L.Msm, ws + L.piv, b, ns);
  for (int i = ex.lane; i < P.oRho; i += ex.nlanes) {
    double v = dx[i];
    for (int k = 0; k < nc; ++k) v -= b[ng + nb + k] * ws[L.colk + (size_t)k * P.nv + i];
    dx[i] = v;
  }
  for (int i = P.oS + ex.lane; i < P.oJ; i += ex.nlanes) {
    double v = dx[i];
    for (int k = 0; k < nc; ++k) v -= b[ng + nb + k] * ws[L.colk + (size_t)k * P.nv + i];
    dx[i] = v;
  }
  for (int i = ex.lane; i < P.T * NX; i += ex.nlanes) {
    double v = dy[i];
    for (int k = 0; k < nc; ++k) v -= b[ng + nb + k] * ws[L.colnu + (size_t)k * P.neq + i];
    dy[i] = v;
  }
  for (int i = ex.lane; i < ng; i += ex.nlanes) dx[gvar(P, i)] = b[i];
  for (int j = ex.lane; j < nb; j += ex.nlanes) dy[P.T * NX + j] = b[ng + j];
  ex.sync();
  // dzh = W^-1 G dx - r3h
  apply_G<X, NX, NU>(ex, C, dx, tr);
  apply_W(ex, C, 1, tr, dzh);
  for (int i = ex.lane; i < P.nrows; i += ex.nlanes) dzh[i] -= r3h[i];
  ex.sync();
}

// Solve [0 A' G'; A 0 0; G 0 -W^2] [dx; dy; dz] = [r1; r2; r3]: W-scaled solve with
// iterative refinement on the scaled residual (well conditioned, unlike the W^2 form whose
// residual is dominated by the rounding of W^2 dz near the boundary).
template <class X, int NX, int NU>
BMPC_HD void kkt_solve(const X& ex, const Ctx& C, const double* r1, const double* r2,
                       const double* r3, double* dx, double* dy, double* dz) {
  const Plan& P = *C.P;
  const Layout& L = *C.L;
  double* ws = C.ws;
  double* e1 = ws + L.k_e1;
  double* e2 = ws + L.k_e2;
  double* e3 = ws + L.k_e3;
  double* r3h = ws + L.k_t3;
  double* cx = ws + L.k_cx;
  double* cy = ws + L.k_cy;
  double* cz = ws + L.k_cz;
  double* tv = ws + L.k_nv1;
  apply_W(ex, C, 1, r3, r3h);
  kkt_solve_once<X, NX, NU>(ex, C, r1, r2, r3h, dx, dy, dz);   // dz holds dzh until the end
  double sc = 0.0;
  for (int i = ex.lane; i < P.nv; i += ex.nlanes) sc = fmax(sc, fabs(r1[i]));
  for (int i = ex.lane; i < P.neq; i += ex.nlanes) sc = fmax(sc, fabs(r2[i]));
  for (int i = ex.lane; i < P.nrows; i += ex.nlanes) sc = fmax(sc, fabs(r3h[i]));
  sc = ex.max(sc);
  for (int itr = 0; itr < 3; ++itr) {
    // e1 = r1 - A'dy - G'W^-1 dzh
    apply_W(ex, C, 1, dz, e3);
    apply_GT<X, NX, NU>(ex, C, e3, tv);
    apply_AT<X, NX, NU>(ex, C, dy, e1);
    for (int i = ex.lane; i < P.nv; i += ex.nlanes) e1[i] = r1[i] - e1[i] - tv[i];
    // e2 = r2 - A dx
    apply_A<X, NX, NU>(ex, C, dx, e2);
    for (int i = ex.lane; i < P.neq; i += ex.nlanes) e2[i] = r2[i] - e2[i];
    // e3 = r3h - W^-1 G dx + dzh
    apply_G<X, NX, NU>(ex, C, dx, cz);
    apply_W(ex, C, 1, cz, e3);
    for (int i = ex.lane; i < P.nrows; i += ex.nlanes) e3[i] = r3h[i] - e3[i] + dz[i];
    ex.sync();
    double err = 0.0;
    for (int i = ex.lane; i < P.nv; i += ex.nlanes) err = fmax(err, fabs(e1[i]));
    for (int i = ex.lane; i < P.neq; i += ex.nlanes) err = fmax(err, fabs(e2[i]));
    for (int i = ex.lane; i < P.nrows; i += ex.nlanes) err = fmax(err, fabs(e3[i]));
    err = ex.max(err);
#ifdef BMPC_HOST_DEBUG
    printf("   refine %d err %.3e sc %.3e\n", itr, err, sc);
#endif
    if (!(err > 1e-14 * fmax(sc, 1.0))) break;
    kkt_solve_once<X, NX, NU>(ex, C, e1, e2, e3, cx, cy, cz);
    for (int i = ex.lane; i < P.nv; i += ex.nlanes) dx[i] += cx[i];
    for (int i = ex.lane; i < P.neq; i += ex.nlanes) dy[i] += cy[i];
    for (int i = ex.lane; i < P.nrows; i += ex.nlanes) dz[i] += cz[i];
    ex.sync();
  }
  // dz = W^-1 dzh
  apply_W(ex, C, 1, dz, e3);
  for (int i = ex.lane; i < P.nrows; i += ex.nlanes) dz[i] = e3[i];
  ex.sync();
}

// ECOS bring2cone: s = r + (1 + alpha) e
template <class X>
BMPC_HD void bring2cone(const X& ex, const Ctx& C, const double* r, double* s) {
  const Plan& P = *C.P;
  const Topo& t = P.t;
  double alpha = -0.99;
  double mn = 1e300;
  for (int i = ex.lane; i < P.nlp; i += ex.nlanes) mn = fmin(mn, r[i]);
  mn = -ex.min(mn);
  if (P.nlp > 0 && mn >= 0.0 && mn > alpha) alpha = mn;
  for (int k = 0; k < P.ncones; ++k) {
    const int off = t.cone_off[k], q = t.cone_q[k];
    double ss = 0.0;
    for (int i = 1 + ex.lane; i < q; i += ex.nlanes) ss += r[off + i] * r[off + i];
    ss = ex.sum(ss);
    const double cres = r[off] - sqrt(ss);
    if (cres <= 0.0 && -cres > alpha) alpha = -cres;
  }
  ex.sync();
  for (int i = ex.lane; i < P.nlp; i += ex.nlanes) s[i] = r[i] + 1.0 + alpha;
  for (int k = 0; k < P.ncones; ++k) {
    const int off = t.cone_off[k], q = t.cone_q[k];
    for (int i = ex.lane; i < q; i += ex.nlanes) s[off + i] = r[off + i] + (i == 0 ? 1.0 + alpha : 0.0);
  }
  ex.sync();
}

template <class X>
BMPC_HD double vdot(const X& ex, const double* a, const double* b, int n) {
  double s = 0.0;
  for (int i = ex.lane; i < n; i += ex.nlanes) s += a[i] * b[i];
  return ex.sum(s);
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
BMPC_HD IpmResult ipm_solve(const X& ex, const Ctx& C) {
  const Plan& P = *C.P;
  const Layout& L = *C.L;
  double* ws = C.ws;
  const int nv = P.nv, neq = P.neq, nr = P.nrows;
  double* x = ws + L.x;
  double* y = ws + L.y;
  double* z = ws + L.z;
  double* s = ws + L.s;
  double* lam = ws + L.lam;
  double* x1 = ws + L.x1;
  double* y1 = ws + L.y1;
  double* z1 = ws + L.z1;
  double* x2 = ws + L.x2;
  double* y2 = ws + L.y2;
  double* z2 = ws + L.z2;
  double* dz = ws + L.dz;
  double* ds = ws + L.ds;
  double* rx = ws + L.rx;
  double* ry = ws + L.ry;
  double* rz = ws + L.rz;
  double* hv = ws + L.hvec;
  double* bv = ws + L.bvec;
  double* tA = ws + L.ta;
  double* ya = ws + L.ya;
  double* ra = ws + L.ra;
  double* rb = ws + L.rb;
  double* rc = ws + L.rc;
  const double feastol = P.desc.feastol, abstol = P.desc.abstol, reltol = P.desc.reltol;
  const double deg = (double)(P.nlp + P.ncones);
  IpmResult res{EXIT_MAXIT, 0, 0.0};

  build_hb<X, NX, NU>(ex, C, hv, bv);
  // ---- initial point with W = I ----------------------------------------------------------
  identity_scaling(ex, C);
  if (!kkt_factor<X, NX, NU>(ex, C) || !kkt_coupling<X, NX, NU>(ex, C)) {
    res.exit_flag = EXIT_NUMERICS;
    return res;
  }
  for (int i = ex.lane; i < nv; i += ex.nlanes) tA[i] = 0.0;
  ex.sync();
  kkt_solve<X, NX, NU>(ex, C, tA, bv, hv, x, y2, z2);
  for (int i = ex.lane; i < nr; i += ex.nlanes) ra[i] = -z2[i];
  ex.sync();
  bring2cone(ex, C, ra, s);
  for (int i = ex.lane; i < nv; i += ex.nlanes) tA[i] = i == P.oJ ? -1.0 : 0.0;
  for (int i = ex.lane; i < neq; i += ex.nlanes) ya[i] = 0.0;
  for (int i = ex.lane; i < nr; i += ex.nlanes) ra[i] = 0.0;
  ex.sync();
  kkt_solve<X, NX, NU>(ex, C, tA, ya, ra, x2, y, z2);
  bring2cone(ex, C, z2, z);
  double tau = 1.0, kap = 1.0;
  const double resx0 = 1.0;   // max(1, ||c||), c = e_J
  const double resy0 = fmax(1.0, sqrt(vdot(ex, bv, bv, neq)));
  const double resz0 = fmax(1.0, sqrt(vdot(ex, hv, hv, nr)));
  double best_score = 1e300, best_tau = 1.0;
  int stall = 0;
  int best_it = 0;
  double bs_pres = 0, bs_dres = 0, bs_relgap = 0, bs_gap = 0, bs_pcost = 0;
  bool bs_ok_cx = false;

  for (int it = 0; it <= P.desc.maxit; ++it) {
    // residuals
    apply_AT<X, NX, NU>(ex, C, y, rx);
    apply_GT<X, NX, NU>(ex, C, z, tA);
    for (int i = ex.lane; i < nv; i += ex.nlanes) rx[i] += tA[i] + (i == P.oJ ? tau : 0.0);
    apply_A<X, NX, NU>(ex, C, x, ry);
    for (int i = ex.lane; i < neq; i += ex.nlanes) ry[i] = bv[i] * tau - ry[i];
    apply_G<X, NX, NU>(ex, C, x, rz);
    for (int i = ex.lane; i < nr; i += ex.nlanes) rz[i] = hv[i] * tau - rz[i] - s[i];
    ex.sync();
    const double cx = x[P.oJ];
    const double by = vdot(ex, bv, y, neq), hz = vdot(ex, hv, z, nr);
    const double rt = kap + cx + by + hz;
    const double nx = sqrt(vdot(ex, x, x, nv)), ny = sqrt(vdot(ex, y, y, neq));
    const double nz = sqrt(vdot(ex, z, z, nr)), ns = sqrt(vdot(ex, s, s, nr));
    const double sz = vdot(ex, s, z, nr);
    const double mu = (sz + kap * tau) / (deg + 1.0);
    const double gap = sz / (tau * tau);
    const double pcost = cx / tau, dcost = -(hz + by) / tau;
    double relgap = -1.0;   // -1 = NaN
    if (pcost < 0.0) relgap = gap / (-pcost);
    else if (dcost > 0.0) relgap = gap / dcost;
    const double nry = neq ? sqrt(vdot(ex, ry, ry, neq)) / fmax(resy0 + nx, 1.0) : 0.0;
    const double nrz = sqrt(vdot(ex, rz, rz, nr)) / fmax(resz0 + nx + ns, 1.0);
    const double pres = fmax(nry, nrz) / tau;
    const double dres = sqrt(vdot(ex, rx, rx, nv)) / fmax(resx0 + ny + nz, 1.0) / tau;
    // infeasibility certificates (only evaluated when their preconditions hold)
    double pinfres = -1.0, dinfres = -1.0;
    if ((hz + by) / fmax(ny + nz, 1.0) < -reltol) {
      for (int i = ex.lane; i < nv; i += ex.nlanes) ra[i] = rx[i] - (i == P.oJ ? tau : 0.0);
      ex.sync();
      pinfres = sqrt(vdot(ex, ra, ra, nv)) / fmax(ny + nz, 1.0);
    }
    if (cx / fmax(nx, 1.0) < -reltol) {
      apply_A<X, NX, NU>(ex, C, x, rb);
      const double a1 = sqrt(vdot(ex, rb, rb, neq)) / fmax(nx, 1.0);
      apply_G<X, NX, NU>(ex, C, x, ra);
      for (int i = ex.lane; i < nr; i += ex.nlanes) ra[i] += s[i];
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
    // stall counter: only in the end game (best iterate within the inaccurate tolerances)
    if (score < 0.5 * best_score || best_score > 1e-4) stall = 0;
    else ++stall;
    if (score < best_score) {
      best_score = score;
      best_it = it;
      best_tau = tau;
      bs_pres = pres, bs_dres = dres, bs_relgap = relgap, bs_gap = gap, bs_pcost = pcost;
      bs_ok_cx = (-cx > 0.0 || -by - hz >= -5e-5);
      for (int i = ex.lane; i < nv; i += ex.nlanes) ws[L.bestx + i] = x[i];
      ex.sync();
    }
#ifdef BMPC_HOST_DEBUG
    printf("it %3d pcost %+.9e dcost %+.9e gap %.2e pres %.2e dres %.2e k/t %.2e tau %.2e nx %.2e\n", it, pcost,
           dcost, gap, pres, dres, kap / tau, tau, nx);
#endif
    int code = check(feastol, abstol, reltol);
    if (code == 99 && stall >= 5) {    // no progress for 5 end-game iterations: precision floor
      const int c2 = check(1e-4, 5e-5, 5e-5);
      if (c2 != 99) code = c2 + EXIT_INACC;
      else if (best_score < 1e300) {
        const bool inacc = bs_ok_cx && bs_pres < 1e-4 && bs_dres < 1e-4 &&
                           (bs_gap < 5e-5 || (bs_relgap >= 0.0 && bs_relgap < 5e-5));
        for (int i = ex.lane; i < nv; i += ex.nlanes) ws[L.sol + i] = ws[L.bestx + i] / best_tau;
        ex.sync();
        res.exit_flag = inacc ? EXIT_OPTIMAL + EXIT_INACC : EXIT_MAXIT;
        res.iters = it;
        res.pcost = bs_pcost;
        return res;
      }
    }
    if (code == 99 && it == P.desc.maxit) {
      const int c2 = check(1e-4, 5e-5, 5e-5);
      code = c2 == 99 ? EXIT_MAXIT : c2 + EXIT_INACC;
    }
    if (code != 99) {
      for (int i = ex.lane; i < nv; i += ex.nlanes) ws[L.sol + i] = x[i] / tau;
      ex.sync();
      res.exit_flag = code;
      res.iters = it;
      res.pcost = pcost;
      return res;
    }
    // ---- Newton step ---------------------------------------------------------------------
    bool ok = compute_scaling(ex, C, s, z);
    if (ok) ok = kkt_factor<X, NX, NU>(ex, C) && kkt_coupling<X, NX, NU>(ex, C);
    double alpha = 0.0, dtau = 0.0, dkap = 0.0;
    if (ok) {
      // c vector
      for (int i = ex.lane; i < nv; i += ex.nlanes) tA[i] = i == P.oJ ? -1.0 : 0.0;
      ex.sync();
      kkt_solve<X, NX, NU>(ex, C, tA, bv, hv, x1, y1, z1);
      const double den = kap / tau - (x1[P.oJ] + vdot(ex, bv, y1, neq) + vdot(ex, hv, z1, nr));
      // affine: xi = -lam
      for (int i = ex.lane; i < nr; i += ex.nlanes) ra[i] = -lam[i];
      ex.sync();
      apply_W(ex, C, 0, ra, rb);                               // W xi
      for (int i = ex.lane; i < nr; i += ex.nlanes) rb[i] = rz[i] - rb[i];
      for (int i = ex.lane; i < nv; i += ex.nlanes) tA[i] = -rx[i];
      ex.sync();
      kkt_solve<X, NX, NU>(ex, C, tA, ry, rb, x2, y2, z2);
      const double dk_aff = -kap * tau;
      const double dtau_a = (rt + dk_aff / tau + x2[P.oJ] + vdot(ex, bv, y2, neq) + vdot(ex, hv, z2, nr)) / den;
      for (int i = ex.lane; i < nr; i += ex.nlanes) dz[i] = z2[i] + dtau_a * z1[i];
      ex.sync();
      apply_W(ex, C, 0, dz, rb);                               // W dz_aff
      for (int i = ex.lane; i < nr; i += ex.nlanes) ds[i] = ra[i] - rb[i];   // dsW_aff
      ex.sync();
      const double dkap_a = (dk_aff - kap * dtau_a) / tau;
      double a_aff = fmin(max_step(ex, C, lam, ds), max_step(ex, C, lam, rb));
      if (dtau_a < 0.0) a_aff = fmin(a_aff, -tau / dtau_a);
      if (dkap_a < 0.0) a_aff = fmin(a_aff, -kap / dkap_a);
      a_aff = fmax(0.0, fmin(a_aff, 0.999));
      double sigma = (1.0 - a_aff) * (1.0 - a_aff) * (1.0 - a_aff);
      sigma = fmin(1.0, fmax(1e-4, sigma));
      const double eta1 = 1.0 - sigma;
      // combined: ds_comb = -lam o lam - dsW_a o Wdz_a + sigma mu e
      jprod(ex, C, lam, lam, ra);
      jprod(ex, C, ds, rb, rc);
      for (int i = ex.lane; i < nr; i += ex.nlanes) ra[i] = -ra[i] - rc[i];
      ex.sync();
      for (int i = ex.lane; i < P.nlp; i += ex.nlanes) ra[i] += sigma * mu;
      for (int k = ex.lane; k < P.ncones; k += ex.nlanes) ra[P.t.cone_off[k]] += sigma * mu;
      ex.sync();
      jdiv(ex, C, lam, ra, ds);                                // xi (kept in ds)
      apply_W(ex, C, 0, ds, rb);                               // W xi
      for (int i = ex.lane; i < nr; i += ex.nlanes) rb[i] = eta1 * rz[i] - rb[i];
      for (int i = ex.lane; i < nv; i += ex.nlanes) tA[i] = -eta1 * rx[i];
      for (int i = ex.lane; i < neq; i += ex.nlanes) ya[i] = eta1 * ry[i];
      ex.sync();
      kkt_solve<X, NX, NU>(ex, C, tA, ya, rb, x2, y2, z2);
      const double dk_c = -kap * tau - dtau_a * dkap_a + sigma * mu;
      dtau = (eta1 * rt + dk_c / tau + x2[P.oJ] + vdot(ex, bv, y2, neq) + vdot(ex, hv, z2, nr)) / den;
      for (int i = ex.lane; i < nv; i += ex.nlanes) x2[i] += dtau * x1[i];
      for (int i = ex.lane; i < neq; i += ex.nlanes) y2[i] += dtau * y1[i];
      for (int i = ex.lane; i < nr; i += ex.nlanes) z2[i] += dtau * z1[i];
      ex.sync();
      apply_W(ex, C, 0, z2, rb);                               // W dz
      for (int i = ex.lane; i < nr; i += ex.nlanes) ds[i] = ds[i] - rb[i];   // dsW
      ex.sync();
      dkap = (dk_c - kap * dtau) / tau;
      double a = fmin(max_step(ex, C, lam, ds), max_step(ex, C, lam, rb));
      if (dtau < 0.0) a = fmin(a, -tau / dtau);
      if (dkap < 0.0) a = fmin(a, -kap / dkap);
      a = fmin(a, 0.999);
      alpha = a * 0.99;           // never step onto or past the cone / tau / kappa boundary
      apply_W(ex, C, 0, ds, rb);                               // ds = W dsW
      double fin = 0.0;
      for (int i = ex.lane; i < nv; i += ex.nlanes) fin += isfinite(x2[i]) ? 0.0 : 1.0;
      fin = ex.max(fin);
      ok = fin == 0.0 && isfinite(dtau) && alpha > 1e-10;
      if (ok) {
        for (int i = ex.lane; i < nv; i += ex.nlanes) x[i] += alpha * x2[i];
        for (int i = ex.lane; i < neq; i += ex.nlanes) y[i] += alpha * y2[i];
        for (int i = ex.lane; i < nr; i += ex.nlanes) {
          z[i] += alpha * z2[i];
          s[i] += alpha * rb[i];
        }
        tau += alpha * dtau;
        kap += alpha * dkap;
        ex.sync();
      }
    }
    if (!ok) {   // numerical failure: ECOS backtracks to the best iterate
      const bool inacc = bs_ok_cx && bs_pres < 1e-4 && bs_dres < 1e-4 &&
                         (bs_gap < 5e-5 || (bs_relgap >= 0.0 && bs_relgap < 5e-5));
      for (int i = ex.lane; i < nv; i += ex.nlanes) ws[L.sol + i] = ws[L.bestx + i] / best_tau;
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
