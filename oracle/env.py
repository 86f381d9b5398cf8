"""Closed-loop scene restatements (oracle; test-only).

``HighwayOvertake`` restates ``Highway_env_branch.Highway_env`` + ``Highway_sim`` for
``sim_overtake`` (``Highway_env_branch.py:48-184,393-445,719-725``):

* obstacle policy choice with the NumPy (clipped) ``veh_col`` and ``lane_bdry_h``
  (``:137-149``) against the env boundary ``LB = [W/2, N_lane*3.6 - W/2]`` (``:63``);
* obstacle inputs from the env's *construction-time* policy list (``:60``; the model's
  later ``update_backup`` replaces the model's list, not the env's), NumPy branches
  (``backup_brake`` NumPy = softmax([-5,-v], 3), ``highway_branch_dyn.py:121``);
* lane bookkeeping with Python's round-half-even ``round`` (``:103``) and the
  ``update_backup`` re-targeting of the lane-change policy (``:99-118``);
* the x_ref rule (``:153-167``) and Euler ``vehicle.step`` (``:39-41``);
* the collision flag of ``Highway_sim`` (``:421-429``; only the last pair's distance is
  tested, which for two vehicles is the only pair).

The RNG draws of ``:121-133`` only write ``desired_x``, which nothing reads, so the scene
is deterministic.
"""
from __future__ import annotations

import numpy as np

from .model import highway_policies

V0 = 20.0


def softmin_np(x, gamma):
    return np.sum(np.exp(-gamma * x) * x) / np.sum(np.exp(-gamma * x))


def softmax_np(x, gamma):
    return np.sum(np.exp(gamma * x) * x) / np.sum(np.exp(gamma * x))


def veh_col_np(x1, x2, size, alpha=1.0):
    """NumPy branch of ``veh_col`` (highway_branch_dyn.py:243-254), rows clipped to +-5."""
    dx = np.clip(np.abs(x1[:, 0] - x2[:, 0]) - size[0], -5, 5)
    dy = np.clip(np.abs(x1[:, 1] - x2[:, 1]) - size[1], -5, 5)
    return (dx * np.exp(alpha * dx) + dy * np.exp(dy * alpha)) / (np.exp(alpha * dx) + np.exp(dy * alpha))


def lane_bdry_np(x, lb, ub):
    return np.array([softmin_np(np.array([r[1] - lb, ub - r[1]]), 5) for r in x])


def policy_u_np(kind, x, Kpsi, target):
    """NumPy branches of the backup policies (highway_branch_dyn.py:67,121,148)."""
    if kind == 0:
        return np.array([0.0, -Kpsi * x[3]])
    if kind == 1:
        return np.array([softmax_np(np.array([-5.0, -x[2]]), 3), -Kpsi * x[3]])
    return np.array([-0.8558 * (x[2] - target[2]), -0.3162 * (x[1] - target[1]) - 3.9889 * (x[3] - target[3])])


class HighwayOvertake:
    """Two-vehicle overtake scene; ``mpc`` exposes ``solve(x, z, xRef)``, ``uPred`` and
    ``model`` (with ``zpred_eval`` / ``update_backup``)."""

    def __init__(self, mpc, model, N_lane=4, L=4.0, W=2.5, Kpsi=0.1,
                 lc_target0=(0.5, 1.8, 15.0, 0.0), dt=0.1,
                 x0=((0.0, 1.8, V0, 0.0), (5.0, 5.4, V0, 0.0))):
        self.mpc, self.model = mpc, model
        self.N_lane, self.L, self.W, self.Kpsi, self.dt = N_lane, L, W, Kpsi, dt
        self.LB = [W / 2.0, N_lane * 3.6 - W / 2.0]
        self.env_target = np.array(lc_target0, float)      # env.backupcons keeps main's list
        self.state = [np.array(v, float) for v in x0]
        self.laneidx = [0, 0]
        self.backupidx = [0, 0]
        self.vlen, self.vwid = 4.0, 2.4                     # vehicle() defaults (:29)
        self.collision = False
        self.lc_target = None

    def step(self, t):
        xx = [None, None]
        for i in range(2):
            z = self.state[i]
            xx[i] = self.model.zpred_eval(z)
            new = round((z[1] - 1.8) / 3.6)
            if t == 0 or (new != self.laneidx[i] and abs(z[1] - 1.8 - 3.6 * new) < 1.4):
                self.laneidx[i] = new
                if i == 1:
                    l0, l1 = self.laneidx
                    if l0 < l1:
                        tgt = [0, 1.8 + 3.6 * (l1 - 1), V0, 0]
                    elif l0 > l1:
                        tgt = [0, 1.8 + 3.6 * (l1 + 1), V0, 0]
                    elif l1 > 0:
                        tgt = [0, 1.8 + 3.6 * (l1 - 1), V0, 0]
                    else:
                        tgt = [0, 1.8 + 3.6 * (l1 + 1), V0, 0]
                    self.lc_target = np.array(tgt, float)
                    self.model.update_backup(highway_policies(self.Kpsi, self.lc_target))
        n = 4
        x1 = xx[0][:, 0:n]
        hi = np.zeros(3)
        for j in range(3):
            hi[j] = min(np.append(veh_col_np(x1, xx[1][:, j * n:(j + 1) * n], [self.L + 1, self.W + 0.2]),
                                  lane_bdry_np(x1, self.LB[0], self.LB[1])))
        self.backupidx[1] = int(np.argmax(hi))
        u_obs = policy_u_np(self.backupidx[1], self.state[1], self.Kpsi, self.env_target)
        e, o = self.state
        Ydes = 1.8 + self.laneidx[0] * 3.6 if e[0] < o[0] else o[1]
        if abs(e[1] - Ydes) < 1 and e[0] > o[0] + 3:
            vdes = V0
        else:
            vdes = o[2] + 1 * (o[0] + 1.5 - e[0])
        xRef = np.array([0.0, Ydes, vdes, 0.0])
        x_in, z_in = e.copy(), o.copy()
        self.mpc.solve(x_in, z_in, xRef)
        u = np.array(self.mpc.uPred[0], float)
        self.state[0] = e + np.array([e[2] * np.cos(e[3]), e[2] * np.sin(e[3]), u[0], u[1]]) * self.dt
        self.state[1] = o + np.array([o[2] * np.cos(o[3]), o[2] * np.sin(o[3]), u_obs[0], u_obs[1]]) * self.dt
        return dict(x=x_in, z=z_in, xRef=xRef, u=u, u_obs=u_obs, obs_policy=self.backupidx[1],
                    lc_target=self.lc_target.copy())

    def check_collision(self):
        a, b = self.state
        dis = max(abs(a[0] - b[0]) - self.vlen, abs(a[1] - b[1]) - self.vwid)
        if dis < 0:
            self.collision = True
        return self.collision

    def run(self, steps):
        rec = []
        for t in range(steps):
            if not self.collision:
                self.check_collision()
            rec.append(self.step(t))
        return rec
