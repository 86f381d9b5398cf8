"""HMM belief-augmented predictive model -- drop-in for the reference's ``HMM_backup_dyn``.

The reference module (HMM_backup_dyn.py) builds CasADi graphs in ``calc_xp_expr``
(:238-276) and evaluates them in ``regressionAndLinearization`` (:216-237).  Here the same
linearisation runs on the GPU (``bmpc_hmm_eval``, csrc/bmpc_hmm.h), batched over points.
NumPy helpers keep the reference's NumPy-branch semantics (``veh_col`` clips to +-5 there).
``HMM_constants`` is the reference's missing import; ``Branch_constants`` carries every
field the model reads (utils.HMM_constants).
"""
from __future__ import annotations

import numpy as np

from highway_branch_dyn import backup_brake, backup_maintain, dubin, lane_bdry_h, propagate_backup  # noqa: F401
from highway_branch_dyn import softmax, softmin, softsat  # noqa: F401

__all__ = ["np", "PredictiveModel", "backup_trans", "veh_col", "dubin", "propagate_backup", "softsat",
           "backup_maintain", "backup_brake", "softmin", "softmax", "X_bdry", "veh_con", "dubin_fg", "dubin_f_x",
           "generate_backup_traj", "backup_input_prob"]


def softmin(x, y, gamma=1):
    """Two-argument soft minimum of this module (:117-118; highway_branch_dyn's takes a vector)."""
    return (np.exp(-gamma * x) * x + np.exp(-gamma * y) * y) / (np.exp(-gamma * x) + np.exp(-gamma * y))


def softmax(x, y, gamma=1):
    """Two-argument soft maximum (:120-121)."""
    return (np.exp(gamma * x) * x + np.exp(gamma * y) * y) / (np.exp(gamma * x) + np.exp(gamma * y))


def X_bdry(x, bdry, width):
    """Distance to the nearer road edge and its gradient (:10-16)."""
    dy1 = x[1] - bdry[0] - width / 2
    dy2 = bdry[1] - x[1] - width / 2
    return (dy1, np.array([0, 1, 0, 0])) if dy1 < dy2 else (dy2, np.array([0, -1, 0, 0]))


def veh_con(x, x0, umax, ignore_x=True):
    """LQR-like lane keeping toward x0, clipped to +-umax (:18-28)."""
    if ignore_x:
        u = np.array([-0.8558 * (x[2] - x0[2]), -0.3162 * (x[1] - x0[1]) - 3.9889 * (x[3] - x0[3])])
    else:
        u = np.array([-0.3162 * (x[0] - x0[0]) - 0.8558 * (x[2] - x0[2]),
                      -0.3162 * (x[1] - x0[1]) - 3.9889 * (x[3] - x0[3])])
    return np.minimum(umax, np.maximum(-umax, u))


def dubin_fg(x):
    """Control-affine split of the unicycle (:39-42): xdot = f(x) + g u."""
    f = np.array([x[2] * np.cos(x[3]), x[2] * np.sin(x[3]), 0.0, 0.0])
    g = np.array([[0, 0], [0, 0], [1, 0], [0, 1]], float)
    return f, g


def dubin_f_x(x, con, h=1e-6):
    """Closed-loop Jacobian d(f(x, con(x)))/dx with central differences of con (:43-54)."""
    dudx = np.zeros([4, 2])
    for k in range(4):
        e = np.zeros(4)
        e[k] = h
        dudx[k] = (con(x + e) - con(x - e)) / 2 / h
    return np.concatenate((np.array([[0, 0, np.cos(x[3]), -x[2] * np.sin(x[3])],
                                     [0, 0, np.sin(x[3]), x[2] * np.cos(x[3])]]), dudx.transpose()))


def generate_backup_traj(x, con, stop_crit, f0, ts=0.05, sensitivity=True):
    """Euler rollout of x under con until stop_crit(x, t) (:56-94), with the sensitivity
    Q = dx_t/dx_0 and Qt = xdot - f0 per step when asked: (tt, xx, uu, QQ, Qt)."""
    t, tt, xx, uu, QQ, Qt = 0, [], [], [], [], []
    Q = np.identity(4)
    while not stop_crit(x, t):
        u = con(x)
        xdot = np.array([x[2] * np.cos(x[3]), x[2] * np.sin(x[3]), u[0], u[1]])
        if sensitivity:
            QQ.append(Q)
            ja = dubin_f_x(x, con)
            Qt.append(xdot - f0)
        tt.append(t)
        xx.append(x)
        uu.append(u)
        x = x + xdot * ts
        if sensitivity:
            Q = Q + np.matmul(ja, Q) * ts
        t = t + ts
    return tt, xx, uu, QQ, Qt


def backup_input_prob(cbfcond, cons):
    """Likelihood of a backup given its CBF condition (:103-104)."""
    return softsat(cbfcond - cons.c2, cons.s2)


def backup_trans(h, cons):
    """NumPy branch of backup_trans (:96-101): kron((1-tau) 1, m'/sum m) + tau I."""
    h = np.asarray(h, float).reshape(-1)
    m = softsat(h, cons.s1)
    return np.kron((1 - cons.tran_diag) * np.ones([h.shape[0], 1]), m / m.sum()) + cons.tran_diag * np.eye(h.shape[0])


def veh_col(x1, x2, size, alpha=1):
    """NumPy branch (:150-160): size-normalised and clipped to +-5."""
    a, b = np.atleast_2d(np.asarray(x1, float)), np.atleast_2d(np.asarray(x2, float))
    dx = np.clip((np.abs(a[:, 0] - b[:, 0]) - size[0]) / size[0], -5, 5)
    dy = np.clip((np.abs(a[:, 1] - b[:, 1]) - size[1]) / size[1], -5, 5)
    h = (dx * np.exp(alpha * dx) + dy * np.exp(alpha * dy)) / (np.exp(alpha * dx) + np.exp(alpha * dy))
    return h[0] if np.ndim(x1) == 1 else h


class PredictiveModel:
    """HMM_backup_dyn.PredictiveModel (:180-276) with the linearisation on the GPU."""

    def __init__(self, n, d, M, backupcons, dt, cons):
        self.n, self.d, self.M = n, d, M
        self.m = len(backupcons)
        self.dt, self.cons = dt, cons
        self.backupcons = backupcons
        self.alpha = cons.alpha
        self.lamb = 0.0

    def constants(self):
        c = self.cons
        return (self.dt, c.L, c.W, c.ylb, c.yub, c.col_alpha, c.s1, c.tran_diag)

    def generate_backup_traj(self, x0, N):
        """Backup rollouts of every agent under every policy (:199-214), NumPy."""
        xbackup = np.empty([self.M * self.m, N * self.n])
        for i in range(self.M):
            for j in range(self.m):
                con = self.backupcons[j]
                xs = propagate_backup(np.asarray(x0[i], float), lambda x: dubin(x, con(x)), N, self.dt)
                xbackup[self.m * i + j, :] = np.reshape(xs, (1, -1))
        return xbackup

    def regressionAndLinearization(self, xb, xbackup, u):
        """(A, B, C, h0[M], Jh[M]) at one point (:216-237), or batched over a leading axis."""
        from bmpc.plan import hmm_eval
        single = np.ndim(xb) == 1
        r = hmm_eval(self.M, self.m, self.constants(), xb, u,
                     np.asarray(xbackup, float).reshape(-1, self.M * self.m, self.n))
        if single:
            return (r["A"][0], r["B"][0], r["C"][0], [r["h0"][0, i] for i in range(self.M)],
                    [r["Jh"][0, i] for i in range(self.M)])
        return r["A"], r["B"], r["C"], r["h0"], r["Jh"]
