// bmpc_hmm.h -- HMM belief-augmented linearisation (HMM_backup_dyn.PredictiveModel).
//
// regressionAndLinearization (HMM_backup_dyn.py:216-237) of the graph built by
// calc_xp_expr (:238-276), evaluated with forward-mode dual numbers over (xb, u):
//   xb = [x; vec_colmajor(b)], b in R^{M x m};  xbp = [x + dubin(x,u) dt; vec_colmajor(b H_i rows)]
//   h_i[j] = softmin_{col_alpha}(veh_col(x, xbackup[m i + j], [L+1, W+0.2]), lane_bdry(xbackup row))
//   H_i = (1 - tau) 1 (s_i / sum s_i)' + tau I,  s_i = softsat(h_i, s1)     (backup_trans :96-101)
// The SX veh_col of this module normalises by the size and does not clip (:140-149).
#pragma once

#include "bmpc_model.h"

namespace bmpc {

constexpr int HMM_MAX_AGENTS = 4;
constexpr int HMM_MAX_BACKUPS = 4;
constexpr int HMM_MAX_NB = 4 + HMM_MAX_AGENTS * HMM_MAX_BACKUPS;
constexpr int HMM_K = HMM_MAX_NB + 2;   // derivative directions: xb then u

// hc = {dt, L, W, ylb, yub, col_alpha, s1, tran_diag}
template <int K>
BMPC_HD Dual<K> hmm_softmin2(const Dual<K>& x, const Dual<K>& y, double g) {
  const Dual<K> ex = dexp(-g * x), ey = dexp(-g * y);
  return (ex * x + ey * y) / (ex + ey);
}

BMPC_HD void hmm_linearize(int M, int m, const double* hc, const double* xb, const double* u,
                           const double* xbackup, double* xbp, double* A, double* Bm, double* C,
                           double* h0, double* Jh) {
  using DD = Dual<HMM_K>;
  const int nb = 4 + M * m;
  const double dt = hc[0], sx = hc[1] + 1.0, sy = hc[2] + 0.2, ylb = hc[3], yub = hc[4];
  const double calpha = hc[5], s1 = hc[6], tau = hc[7];
  DD v[HMM_MAX_NB], uu[2];
  for (int k = 0; k < nb; ++k) v[k] = dvar<HMM_K>(xb[k], k);
  for (int k = 0; k < 2; ++k) uu[k] = dvar<HMM_K>(u[k], nb + k);
  DD out[HMM_MAX_NB];
  out[0] = v[0] + v[2] * dcos(v[3]) * dt;
  out[1] = v[1] + v[2] * dsin(v[3]) * dt;
  out[2] = v[2] + uu[0] * dt;
  out[3] = v[3] + uu[1] * dt;
  for (int i = 0; i < M; ++i) {
    DD h[HMM_MAX_BACKUPS], s[HMM_MAX_BACKUPS];
    for (int j = 0; j < m; ++j) {
      const double* xr = xbackup + (size_t)(m * i + j) * 4;
      const DD dx = (dfabs(v[0] - xr[0]) - sx) / sx;
      const DD dy = (dfabs(v[1] - xr[1]) - sy) / sy;
      const DD ex = dexp(dx), ey = dexp(dy);
      const DD vc = (dx * ex + dy * ey) / (ex + ey);
      const DD lb = hmm_softmin2(dconst<HMM_K>(xr[1] - ylb), dconst<HMM_K>(yub - xr[1]), 5.0);
      h[j] = hmm_softmin2(vc, lb, calpha);
      const DD e = dexp(s1 * h[j]);
      s[j] = (e - 1.0) / (e + 1.0) * 0.5 + 0.5;
    }
    DD tot = s[0];
    for (int j = 1; j < m; ++j) tot = tot + s[j];
    for (int c = 0; c < m; ++c) {
      DD acc = dconst<HMM_K>(0.0);
      for (int r = 0; r < m; ++r) {
        DD Hrc = (1.0 - tau) * (s[c] / tot);
        if (r == c) Hrc = Hrc + tau;
        acc = acc + v[4 + r * M + i] * Hrc;
      }
      out[4 + c * M + i] = acc;
    }
    for (int j = 0; j < m; ++j) {
      double jx = 0.0;
      for (int k = 0; k < nb; ++k) {
        if (Jh) Jh[((size_t)i * m + j) * nb + k] = h[j].g[k];
        jx += h[j].g[k] * xb[k];
      }
      if (h0) h0[i * m + j] = h[j].v - jx;
    }
  }
  for (int r = 0; r < nb; ++r) {
    double c = out[r].v;
    for (int k = 0; k < nb; ++k) {
      if (A) A[r * nb + k] = out[r].g[k];
      c -= out[r].g[k] * xb[k];
    }
    for (int k = 0; k < 2; ++k) {
      if (Bm) Bm[r * 2 + k] = out[r].g[nb + k];
      c -= out[r].g[nb + k] * u[k];
    }
    if (C) C[r] = c;
    if (xbp) xbp[r] = out[r].v;
  }
}

}  // namespace bmpc
