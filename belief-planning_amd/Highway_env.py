"""Belief-MPC highway scene -- drop-in for the reference's ``Highway_env`` (:1-475).

The ego runs ``PredictiveControllers.MPC`` (the belief LTV-MPC: HMM linearisation and the QP
on the GPU).  Every other vehicle tracks a lane with ``veh_con`` filtered by a backup-CBF
quadratic program -- the reference hands each one to a fresh ``osqp.OSQP`` (:193-216); here
each goes to ``bmpc_qp_solve`` on the GPU.  The vehicles are handled in turn, as in the
reference: vehicle i's QP reads the backup choices vehicles 1..i-1 re-drew this step.  The
HMM belief over each vehicle's backup policy is then updated from the CBF conditions along
the ego's plan (:224-259).

Same class and function names, arguments, random-number consumption (``random`` and
``np.random`` in the reference's order, so a seeded run replays the reference's scene) and
records.  Reference behaviour kept as is: the belief update's second finite difference
overwrites ``dh[0]`` (:241-244, so the y-gradient lands in the x slot); ``Highway_sim``
checks the collision distance of the last (i, j) pair of each i only (:334-341);
animation is replaced by a no-op (plotting is out of scope).  The reference module is
unreachable as shipped (its MPC raises at ``PredictiveControllers.py:121``); the compat MPC
fixes that line (see ``PredictiveControllers``).
"""
from __future__ import annotations

import math
import random

import numpy as np
from numpy.linalg import norm

from HMM_backup_dyn import (X_bdry, backup_input_prob, backup_trans, dubin, dubin_fg,  # noqa: F401
                            generate_backup_traj, veh_col, veh_con)

v0 = 15
lane_width = 3.6
lm = [0, 3.6, 7.2, 10.8, 14.4, 18, 21.6]
f0 = np.array([v0, 0, 0, 0])


def with_probability(P=1):
    return np.random.uniform() <= P


class vehicle:
    """Highway_env.vehicle (:27-42): Euler-stepped unicycle."""

    def __init__(self, state=(0, 0, v0, 0), v_length=4, v_width=2.4, dt=0.05, backupidx=0, laneidx=0):
        self.state = np.array(state)
        self.dt = dt
        self.v_length, self.v_width = v_length, v_width
        self.x_pred, self.y_pred, self.obs_rec_x, self.obs_rec_y = [], [], [], []
        self.xbackup = None
        self.backupidx, self.laneidx = backupidx, laneidx

    def step(self, u):
        s = self.state
        self.state = s + np.array([s[2] * np.cos(s[3]), s[2] * np.sin(s[3]), u[0], u[1]]) * self.dt


def _cbf_qp_solve(A, b, u0, umax):
    """One vehicle's backup-CBF QP on the GPU (:193-207): min 1/2 u'u - u0'u + 1e6 s subject to
    the CBF rows (A | -1)(u, s) <= b, -umax <= u <= umax, s >= 0.  Returns (x, status)."""
    from bmpc import plan
    AA = np.concatenate((np.append(A, -np.ones([A.shape[0], 1]), 1), np.identity(3)))
    ub = np.append(np.append(b, umax), np.inf)
    lb = np.append(np.append(-np.inf * np.ones(len(b)), -umax), 0.0)
    r = plan.qp_solve(np.diag([1.0, 1.0, 0.0]), np.append(-u0, 1e6), AA, lb, ub)
    return r["x"][0], int(r["status"][0])


class Highway_env:
    """Highway_env.Highway_env (:48-302)."""

    def __init__(self, NV, mpc, N_lane=6):
        self.dt = mpc.predictiveModel.dt
        self.veh_set = []
        self.NV = NV
        self.N_lane = N_lane
        self.desired_x = [None] * NV
        self.mpc = mpc
        self.backupcons = mpc.predictiveModel.backupcons
        self.b = np.ones([NV - 1, len(self.backupcons)]) / len(self.backupcons)
        self.m = len(self.backupcons)
        self.cons = mpc.predictiveModel.cons
        UB, LB = 30, 0
        for i in range(NV):
            lane_number = math.floor(random.random() * N_lane)
            while True:
                Y = (lane_number + 0.5) * lane_width + np.random.normal(0, 0.1)
                X = random.random() * (UB - LB) + LB
                if not any(abs(Y - v.state[1]) <= 3 and abs(X - v.state[0]) <= 8 for v in self.veh_set):
                    break
            self.veh_set.append(vehicle([X, Y, v0, 0], dt=self.dt, backupidx=0, laneidx=lane_number))
            lane_des = np.random.choice(N_lane)
            v_des = v0 + np.random.normal(0, 5)
            if i == 0:
                v_des = v0
            self.desired_x[i] = np.array([0, lm[lane_des] + lane_width / 2, v_des, 0])

    def step(self):
        """One scene step (:89-260): backup rollouts, the ego's belief-MPC solve, every other
        vehicle's CBF-filtered input, belief update / replacement."""
        NV, m, N, veh = self.NV, self.m, self.mpc.N, self.veh_set
        u_set, xx_set, QQ_set, u0_set, Qt_set, x_set = ([None] * NV for _ in range(6))
        umax = np.array([self.cons.am, self.cons.rm])
        self.xbackup = np.empty([0, (N + 1) * 4])
        for i in range(NV):
            xx_set[i], QQ_set[i], Qt_set[i] = [None] * m, [None] * m, [None] * m
            if abs(veh[i].state[1] - (1.8 + veh[i].laneidx * 3.6)) < 0.4:
                if i == 0:
                    mindis, idx = 1000, 0
                    for ii in range(1, NV):
                        d = abs(veh[ii].state[0] - veh[0].state[0])
                        if veh[ii].laneidx != veh[0].laneidx and d < mindis:
                            mindis, idx = d, ii
                    if mindis < 4:
                        veh[0].laneidx = veh[idx].laneidx
                elif with_probability(0.05):
                    if veh[i].laneidx == 0:
                        veh[i].laneidx = 1
                    elif veh[i].laneidx == self.N_lane - 1:
                        veh[i].laneidx = self.N_lane - 2
                    elif with_probability(0.5):
                        veh[i].laneidx += 1
                    else:
                        veh[i].laneidx -= 1
            x0 = veh[i].state.copy()
            x0[1] = 1.8 + veh[i].laneidx * 3.6
            x0[2] = veh[0].state[2] + 0.5 * (veh[0].state[0] - veh[i].state[0])
            x0[3] = 0
            con = (lambda x0_: (lambda x: veh_con(x, x0_, umax)))(x0)
            u0_set[i] = con(veh[i].state)
            stop_crit = lambda x, t: t > self.dt * N + 2
            for j in range(m):
                tt, xx, uu, QQ, Qt = generate_backup_traj(veh[i].state, self.backupcons[j], stop_crit, f0, self.dt, True)
                xx_set[i][j], Qt_set[i][j], QQ_set[i][j] = xx, Qt, QQ
                if i > 0:
                    self.xbackup = np.vstack((self.xbackup, np.reshape(np.array(xx[0:N + 1]), [1, -1])))
        xRef = np.array([0, 1.8 + veh[0].laneidx * 3.6, v0, 0])
        self.mpc.solve(veh[0].state, self.b, self.xbackup, xRef)
        u_set[0] = self.mpc.uPred[0]
        veh[0].step(u_set[0])
        x_set[0] = veh[0].state

        # each other vehicle in turn (:160-259): its backup-CBF QP -- built on the host from the
        # backup choices of the vehicles before it, already re-drawn this step, as in the
        # reference's sequential loop -- solved on the GPU, then its step and belief update
        eps = 1e-6
        for i in range(1, NV):
            A, b = [], []
            x = veh[i].state
            fi, g = dubin_fg(x)
            bi_ = veh[i].backupidx
            for t in range(len(xx_set[i][bi_])):
                if t % 3 != 0:
                    continue
                xi = xx_set[i][bi_][t]
                h, dh = X_bdry(xi, [0, lm[self.N_lane]], veh[i].v_width)
                if h < 0.5:
                    dhdx = np.matmul(dh, QQ_set[i][bi_][t])
                    if norm(dhdx.dot(g)) > 1e-6:
                        A.append(-dhdx.dot(g))
                        b.append(dhdx.dot(fi - f0) - np.matmul(dh, Qt_set[i][bi_][t]) + self.cons.alpha * h)
                for j in range(NV):
                    if j == i:
                        continue
                    bj = veh[j].backupidx
                    if t >= len(xx_set[j][bj]):
                        continue   # (:178-179: the reference extrapolates xj and never uses it)
                    xj = xx_set[j][bj][t]
                    size = [(veh[i].v_length + veh[j].v_length) / 2 + 1, (veh[i].v_width + veh[j].v_width) / 2 + 0.2]
                    h = veh_col(xi, xj, size)
                    if h < 2:
                        dh = np.zeros(4)
                        dh[0] = (veh_col(xi + [eps, 0, 0, 0], xj, size) - h) / eps
                        dh[1] = (veh_col(xi + [0, eps, 0, 0], xj, size) - h) / eps
                        dhdx = np.matmul(dh, QQ_set[i][bi_][t])
                        if norm(dhdx.dot(g)) > 1e-6:
                            A.append(-dhdx.dot(g))
                            b.append(dhdx.dot(fi - f0) + self.cons.alpha * h - np.matmul(dh, Qt_set[i][bi_][t]))
            if A:
                x_qp, _ = _cbf_qp_solve(np.array(A), np.array(b, float).reshape(-1), u0_set[i], umax)
                u_set[i] = x_qp[0:2]   # status 1/2 or any returned x (:210-216): the solution's inputs
            else:
                u_set[i] = np.minimum(np.maximum(u0_set[i], -umax), umax)
            veh[i].step(u_set[i])
            x_set[i] = veh[i].state
            if veh[i].state[0] - veh[0].state[0] > 15 or veh[i].state[0] - veh[0].state[0] < -15:
                if not self.replace_veh(i, 0):
                    self.replace_veh(i, 2)
                continue
            cbfcond, hi = np.zeros(m), np.zeros(m)
            xdot = dubin(x_set[i], u_set[i])
            size = [(veh[i].v_length + veh[0].v_length) / 2, (veh[i].v_width + veh[0].v_width) / 2]
            for j in range(m):
                hij, dhij = np.zeros(N), np.zeros(N)
                for tt in range(N):
                    xp = self.mpc.xPred[tt][0:4]
                    hij[tt] = veh_col(xx_set[i][j][tt], xp, size, self.cons.col_alpha)
                    dh = np.zeros(4)
                    dh[0] = (veh_col(xx_set[i][j][tt] + [eps, 0, 0, 0], xp, size, self.cons.col_alpha) - hij[tt]) / eps
                    dh[0] = (veh_col(xx_set[i][j][tt] + [0, eps, 0, 0], xp, size, self.cons.col_alpha) - hij[tt]) / eps
                    dhij[tt] = dh @ (QQ_set[i][j][tt] @ (xdot - f0) - Qt_set[i][j][tt])
                hi[j] = np.min(hij)
                cbfcond[j] = np.mean(hij + dhij)
            bi = self.b[i - 1].copy()
            H = backup_trans(hi, self.cons)
            bi = bi @ H
            for j in range(m):
                bi[j] = bi[j] * backup_input_prob(cbfcond[j], self.cons)
            self.b[i - 1] = bi / np.sum(bi)
            veh[i].backupidx = np.random.choice(range(0, m), 1, p=H[veh[i].backupidx])[0]
            if np.isnan(self.b).any():
                raise FloatingPointError("belief became NaN")   # (the reference drops into pdb)
        return u_set, x_set, xx_set, self.mpc.xPred[1:, 0:4]

    def replace_veh(self, idx, dir=2):
        """Respawn vehicle idx around the ego (:262-302)."""
        if idx == 0:
            return
        ego = self.veh_set[0]
        if dir == 0:
            UB, LB = ego.state[0] + 13, ego.state[0] + 8
        elif dir == 1:
            UB, LB = ego.state[0] - 5, ego.state[0] - 13
        else:
            UB, LB = ego.state[0] + 15, ego.state[0] - 15
        if ego.laneidx == 0:
            laneidx = 1
        elif ego.laneidx == self.N_lane - 1:
            laneidx = self.N_lane - 2
        else:
            laneidx = ego.laneidx - 1 if with_probability(0.5) else ego.laneidx + 1
        count = 0
        while True:
            count += 1
            Y = (laneidx + 0.5) * lane_width + np.random.normal(0, 0.1)
            X = random.random() * (UB - LB) + LB
            if not any(i != idx and abs(Y - self.veh_set[i].state[1]) <= 2.2 and abs(X - self.veh_set[i].state[0]) <= 5
                       for i in range(self.NV)):
                break
            if count > 20:
                return False
        self.veh_set[idx] = vehicle([X, Y, ego.state[2], 0], dt=self.dt, backupidx=0, laneidx=laneidx)
        self.b[idx - 1] = np.ones(self.m) / self.m
        return True


def Highway_sim(env, T):
    """Closed loop for T seconds (:308-382): desired lane / speed re-drawn every 4 s,
    collision flag, records (state, input, backup, backup choice, belief, ego plan)."""
    collision = False
    dt = env.dt
    t = 0
    N_update = int(round(4 / dt))
    N = int(round(T / dt))
    state_rec = np.zeros([env.NV, N, 4])
    b_rec, xPred_rec = [None] * N, [None] * N
    backup_rec = [[None] * N for _ in range(env.NV)]
    backup_choice_rec = [[None] * N for _ in range(env.NV)]
    input_rec = np.zeros([env.NV, N, 2])
    for i in range(len(env.veh_set)):
        state_rec[i][t] = env.veh_set[i].state
    dis = 100
    while t < N:
        if not collision:
            for i in range(env.NV):
                for j in range(env.NV):
                    if i != j:
                        vi, vj = env.veh_set[i], env.veh_set[j]
                        dis = max(abs(vi.state[0] - vj.state[0]) - 0.5 * (vi.v_length + vj.v_length),
                                  abs(vi.state[1] - vj.state[1]) - 0.5 * (vi.v_width + vj.v_width))
                if dis < 0:
                    collision = True
        if t % N_update == 0:
            for i in range(env.NV):
                if np.random.random() > 0.5:
                    lane_des = np.random.choice(env.N_lane)
                else:
                    lane_des = min(max(int(env.veh_set[i].state[1] / 3.6), 0), env.N_lane - 1)
                if i == 0:
                    v_des = v0 + np.random.randn() * 8
                    env.desired_x[i] = np.array([0, lm[lane_des] + lane_width / 2, v_des, 0])
                else:
                    if env.veh_set[i].state[0] > env.veh_set[0].state[0] + 6:
                        v_des = env.desired_x[0][2] - np.random.random() * 4
                    elif env.veh_set[i].state[0] < env.veh_set[0].state[0] - 6:
                        v_des = env.desired_x[0][2] + np.random.random() * 4
                    else:
                        v_des = env.desired_x[i][2] + np.random.randn() * 4
                    env.desired_x[i][1] = lm[lane_des] + lane_width / 2
                    env.desired_x[i][2] = v_des
        u_set, x_set, xx_set, xPred = env.step()
        xPred_rec[t] = xPred
        for i in range(env.NV):
            input_rec[i][t] = u_set[i]
            state_rec[i][t] = x_set[i]
            backup_rec[i][t] = xx_set[i]
            backup_choice_rec[i][t] = env.veh_set[i].backupidx
        b_rec[t] = env.b.copy()
        t += 1
    return state_rec, input_rec, backup_rec, backup_choice_rec, b_rec, xPred_rec, collision


def animate_scenario(env, state_rec, backup_rec, backup_choice_rec, b_rec, xPred_rec, lm, output=None):
    """Plotting is out of scope: a no-op with the reference's signature (:383-469)."""
    return None


def sim(mpc, N_lane, T=15):
    """Highway_env.sim (:472-475): NV = M + 1 vehicles for T seconds (the reference: 15)."""
    env = Highway_env(NV=mpc.M + 1, mpc=mpc, N_lane=N_lane)
    recs = Highway_sim(env, T)
    animate_scenario(env, recs[0], recs[2], recs[3], recs[4], recs[5], lm)
    return recs
