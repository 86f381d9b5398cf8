"""Quadruped closed-loop scene -- drop-in for the reference's ``quadruped_env`` module.

``main_quadruped.py`` (reference ``:7,43``) imports this module and calls ``sim(mpc)``.  The
rules are the reference's (``quadruped_env.py:24-164,326-331``): body-frame Euler steps of
both robots, obstacle rollouts under every backup policy (``zpred_eval``, on the GPU), the
obstacle's backup choice from the NumPy ``robot_col`` clearance along the ego's predicted
path (policy 0 while that clearance exceeds 0.5, else the argmax), the x_ref rule towards
``x_des`` (5 m look-ahead, heading wrapped towards ``x_des[2]``), and one ``mpc.solve`` per
step.

One deliberate difference: the reference's ``Quad_env.step`` unpacks three values from
``BT2array()`` (``:120``), which returns four (``MPC_branch.py:459``), so the reference loop
raises ``ValueError`` after its first solve (SURVEY §8(a) quirk register).  This loop keeps
the 4-tuple and records it.  The ``pdb.set_trace()`` at ``:330`` and the matplotlib
animation are not part of the build (plotting is out of scope).
"""
from __future__ import annotations

import numpy as np
from numpy.linalg import norm

from quadruped_branch_dyn import robot_col


def with_probability(P=1):
    return np.random.uniform() <= P


class robot:
    """Planar robot with body-frame velocity inputs (``quadruped_env.py:24-37``)."""

    def __init__(self, state=(0, 0, 0), L=1, W=0.5, dt=0.05, backupidx=0):
        self.state = np.array(state, float)
        self.dt, self.L, self.W = dt, L, W
        self.x_pred, self.y_pred, self.xbackup = [], [], None
        self.backupidx = backupidx

    def step(self, u):
        s = self.state
        c, sn = np.cos(s[2]), np.sin(s[2])
        self.state = s + np.array([u[0] * c - u[1] * sn, u[1] * c + u[0] * sn, u[2]]) * self.dt


class Quad_env:
    """Two-robot scene (``quadruped_env.py:40-130``); robot 0 is the controlled ego."""

    def __init__(self, NR, mpc, x_des):
        self.dt = mpc.predictiveModel.dt
        self.NR, self.mpc = NR, mpc
        self.desired_x = [None] * NR
        self.predictiveModel = mpc.predictiveModel
        self.backupcons = mpc.predictiveModel.backupcons
        self.m = len(self.backupcons)
        self.cons = mpc.predictiveModel.cons
        x0 = np.array([[0, 1.8, 0], [2.5, 2.5, -np.pi / 2]])
        self.robot_set = [robot(x0[0], L=self.cons.L1, W=self.cons.W1, dt=self.dt, backupidx=0)]
        self.desired_x[0] = np.asarray(x_des, float)
        for i in range(1, NR):
            self.robot_set.append(robot(x0[i], L=self.cons.L2, W=self.cons.W2, dt=self.dt, backupidx=0))
            self.desired_x[i] = x0[i]

    def x_ref(self):
        """Reference point 5 m towards x_des, heading wrapped towards x_des[2] (:97-115)."""
        ego, des = self.robot_set[0].state, self.desired_x[0]
        dx = des[0:2] - ego[0:2]
        dx = dx / norm(dx) * min(norm(dx), 5.0)
        if norm(dx) > 0.1:
            psi = np.arctan2(dx[1], dx[0])
            while psi - des[2] > np.pi:
                psi -= 2 * np.pi
            while psi - des[2] < -np.pi:
                psi += 2 * np.pi
        else:
            psi = ego[2]
        xRef = ego.copy()
        xRef[0:2] += dx
        xRef[2] = psi
        return xRef

    def step(self, t_):
        n = self.predictiveModel.n
        u_set, x_set, u0_set = [None] * self.NR, [None] * self.NR, [None] * self.NR
        zz = self.predictiveModel.zpred_eval(np.stack([np.asarray(r.state, float) for r in self.robot_set]))
        xx_set = [zz[i] for i in range(self.NR)]   # every robot's rollouts in one batched call
        idx0 = self.robot_set[0].backupidx
        x1 = xx_set[0][:, idx0 * n:(idx0 + 1) * n]
        ego = self.robot_set[0]
        for i in range(1, self.NR):
            ob = self.robot_set[i]
            hi = np.array([np.min(robot_col(x1, xx_set[i][:, j * n:(j + 1) * n], ego.L, ego.W, ob.L, ob.W,
                                            self.cons.col_tol)) for j in range(self.m)])
            ob.backupidx = 0 if hi[0] > 0.5 else int(np.argmax(hi))
            u0_set[i] = self.backupcons[ob.backupidx](ob.state)
        xRef = self.x_ref()
        self.mpc.solve(ego.state, self.robot_set[1].state, xRef)
        u_set[0] = self.mpc.uPred[0]
        xPred, zPred, uPred, branch_w = self.mpc.BT2array()
        ego.step(u_set[0])
        x_set[0] = ego.state
        for i in range(1, self.NR):
            u_set[i] = u0_set[i]
            self.robot_set[i].step(u_set[i])
            x_set[i] = self.robot_set[i].state
        return u_set, x_set, xx_set, xPred, zPred


def Robot_sim(env, T):
    """Closed loop of T seconds (``quadruped_env.py:133-164``); the reference's records."""
    N = int(round(T / env.dt))
    state_rec = np.zeros([env.NR, N, 3])
    input_rec = np.zeros([env.NR, N, 3])
    backup_rec = [[None] * N for _ in range(env.NR)]
    backup_choice_rec = [[None] * N for _ in range(env.NR)]
    xPred_rec, zPred_rec = [None] * N, [None] * N
    for i, r in enumerate(env.robot_set):
        state_rec[i][0] = r.state
    for t in range(N):
        u_set, x_set, xx_set, xPred, zPred = env.step(t)
        xPred_rec[t], zPred_rec[t] = xPred, zPred
        for i in range(env.NR):
            input_rec[i][t] = u_set[i]
            state_rec[i][t] = x_set[i]
            backup_rec[i][t] = xx_set[i]
            backup_choice_rec[i][t] = env.robot_set[i].backupidx
    return state_rec, input_rec, backup_rec, backup_choice_rec, xPred_rec, zPred_rec


def plot_snapshot(*args, **kwargs):
    """Plotting is out of scope for the MI355X build (``quadruped_env.py:166``)."""
    return None


def animate_scenario(*args, **kwargs):
    """Animation is out of scope for the MI355X build (``quadruped_env.py:245-323``)."""
    print("[quadruped_env] animate_scenario: plotting is not part of the MI355X build; skipped")
    return None


def sim(mpc, T=40):
    """The ``main_quadruped.py`` scene (``quadruped_env.py:326-331``): 2 robots, 40 s."""
    x_des = np.array([5., -3., 0.])
    env = Quad_env(NR=2, mpc=mpc, x_des=x_des)
    rec = Robot_sim(env, T)
    animate_scenario(env, *rec[:1], *rec[2:], x_des)
    return rec
