"""NumPy restatement of ``HMM_backup_dyn.PredictiveModel`` (oracle; test-only).

The reference module cannot be imported (``HMM_constants`` is missing from utils and
casadi is absent), so this follows the text of ``calc_xp_expr``
(``HMM_backup_dyn.py:238-276``) and ``regressionAndLinearization`` (:216-237):

* belief state ``xb = [x; reshape(b, -1, 1)]`` -- CasADi ``reshape`` is column-major, so
  ``xb[4 + j*M + i] = b[i, j]`` (:244);
* per uncontrolled agent i and backup policy j:
  ``h[j] = softmin(veh_col(x, xbackup[m*i+j], [L+1, W+0.2]), lane_bdry_h(xbackup[m*i+j],
  ylb, yub), col_alpha)`` (:255) with the SX ``veh_col`` that normalises by the size
  (:142-149, alpha = 1) and ``lane_bdry_h = softmin(y-lb, ub-y, 5)`` (:133-134);
* ``H = kron((1-tau) 1, m'/sum(m)) + tau I`` with ``m = softsat(h, s1)`` (``backup_trans``
  :96-101), ``bp[i,:] = b[i,:] @ H`` (:257);
* ``xbp = [x + dubin(x,u) dt; reshape(bp,-1,1)]``; A, B are its Jacobians; C = xbp - A xb - B u;
* ``h0_i = h_i - Jh_i xb`` with ``Jh_i = dh_i/dxb`` (:226-229).

Parity with the reference's output is unpinned (the module never ran); the restatement is
pinned by sympy-exact derivatives and central differences (tests/test_oracle_hmm.py).
"""
from __future__ import annotations

import numpy as np

from .model import D, _cos, _exp, _fabs, _sin, softsat


def _softmin2(x, y, gamma):
    """HMM_backup_dyn.softmin(x, y, gamma) (:114-115)."""
    ex, ey = _exp(-gamma * x), _exp(-gamma * y)
    return (ex * x + ey * y) / (ex + ey)


def veh_col_sx(x1, x2, size, alpha=1.0):
    """SX branch of HMM_backup_dyn.veh_col (:140-149): size-normalised, no clipping."""
    dx = (_fabs(x1[0] - x2[0]) - size[0]) / size[0]
    dy = (_fabs(x1[1] - x2[1]) - size[1]) / size[1]
    ex, ey = _exp(alpha * dx), _exp(alpha * dy)
    return (dx * ex + dy * ey) / (ex + ey)


def lane_bdry_h(x, lb, ub):
    return _softmin2(x[1] - lb, ub - x[1], 5.0)


class HMMModel:
    """Belief-augmented linearisation of one ego against M agents with m backups each."""

    def __init__(self, M, m, dt, L=4.0, W=2.5, ylb=0.0, yub=7.2, col_alpha=5.0, s1=2.0, tran_diag=0.3):
        self.M, self.m, self.dt = M, m, dt
        self.L, self.W, self.ylb, self.yub = L, W, ylb, yub
        self.col_alpha, self.s1, self.tran_diag = col_alpha, s1, tran_diag
        self.nb = 4 + M * m

    def _graph(self, xb, u, xbackup):
        """Dual-number evaluation of (xbp, h[M][m]) w.r.t. (xb, u)."""
        M, m, nb = self.M, self.m, self.nb
        K = nb + 2
        eye = np.eye(K)
        v = [D(float(xb[k]), eye[k].copy()) for k in range(nb)]
        uu = [D(float(u[k]), eye[nb + k].copy()) for k in range(2)]
        x = v[0:4]
        b = [[v[4 + j * M + i] for j in range(m)] for i in range(M)]      # column-major reshape
        f = [x[2] * _cos(x[3]), x[2] * _sin(x[3]), uu[0], uu[1]]
        xp = [x[k] + f[k] * self.dt for k in range(4)]
        size = [self.L + 1.0, self.W + 0.2]
        bp = [[None] * m for _ in range(M)]
        hs = []
        tau = self.tran_diag
        for i in range(M):
            h = []
            for j in range(m):
                xr = xbackup[m * i + j]
                h.append(_softmin2(veh_col_sx(x, xr, size), lane_bdry_h(xr, self.ylb, self.yub), self.col_alpha))
            hs.append(h)
            ms = [softsat(hj, self.s1) for hj in h]
            tot = ms[0]
            for mj in ms[1:]:
                tot = tot + mj
            for c in range(m):
                acc = 0.0
                for r in range(m):
                    Hrc = (1.0 - tau) * (ms[c] / tot) + (tau if r == c else 0.0)
                    acc = acc + b[i][r] * Hrc
                bp[i][c] = acc
        xbp = xp + [bp[i][j] for j in range(m) for i in range(M)]        # column-major reshape
        return xbp, hs

    def linearize(self, xb, u, xbackup):
        """(A, B, C, h0 [M][m], Jh [M][m x nb]) of regressionAndLinearization (:216-237)."""
        xb = np.asarray(xb, float)
        u = np.asarray(u, float)
        nb = self.nb
        xbp, hs = self._graph(xb, u, np.asarray(xbackup, float))
        A = np.array([e.g[:nb] for e in xbp])
        B = np.array([e.g[nb:nb + 2] for e in xbp])
        xv = np.array([e.v for e in xbp])
        C = xv - A @ xb - B @ u
        h0, Jh = [], []
        for i in range(self.M):
            J = np.array([h.g[:nb] for h in hs[i]])
            hv = np.array([h.v for h in hs[i]])
            Jh.append(J)
            h0.append(hv - J @ xb)
        return A, B, C, np.array(h0), np.array(Jh), xv
