"""Highway closed-loop scene -- drop-in for the reference's ``Highway_env_branch`` module.

Host-side driver of one ego (scalar ``mpc.solve`` per step) with the reference's rules
(``Highway_env_branch.py:48-184,393-445,719-725``): obstacle policy selection with the
NumPy ``veh_col`` / ``lane_bdry_h`` against the env boundary, obstacle inputs from the
env's construction-time policy list, lane bookkeeping with round-half-even, lane-change
re-targeting through ``update_backup``, the x_ref rule and Euler vehicle steps.
Plotting/animation are out of scope (``animate_scenario`` and ``plot_snapshot`` only
report that).  The batched, on-device version of this loop is ``bench.py``'s env step.
"""
from __future__ import annotations

import random

import numpy as np

from highway_branch_dyn import backup_brake, backup_lc, backup_maintain, interpolant, lane_bdry_h, veh_col

v0 = 20
f0 = np.array([v0, 0, 0, 0])
lane_width = 3.6
lm = np.arange(0, 7) * lane_width


def with_probability(P=1):
    return np.random.uniform() <= P


class vehicle:
    """Euler-integrated unicycle (:28-41)."""

    def __init__(self, state=(0, 0, v0, 0), v_length=4, v_width=2.4, dt=0.05, backupidx=0, laneidx=0):
        self.state = np.array(state, float)
        self.dt, self.v_length, self.v_width = dt, v_length, v_width
        self.x_pred, self.y_pred, self.xbackup = [], [], None
        self.backupidx, self.laneidx = backupidx, laneidx

    def step(self, u):
        s = self.state
        self.state = s + np.array([s[2] * np.cos(s[3]), s[2] * np.sin(s[3]), u[0], u[1]]) * self.dt


class Highway_env:
    """Overtake scene (:48-184)."""

    def __init__(self, NV, mpc, N_lane=6):
        self.dt = mpc.predictiveModel.dt
        self.NV, self.N_lane, self.mpc = NV, N_lane, mpc
        self.predictiveModel = mpc.predictiveModel
        self.backupcons = mpc.predictiveModel.backupcons       # kept: later update_backup
        self.m = len(self.backupcons)                            # replaces the model's list only
        self.cons = mpc.predictiveModel.cons
        self.LB = [self.cons.W / 2, N_lane * 3.6 - self.cons.W / 2]
        x0 = np.array([[0, 1.8, v0, 0], [5, 5.4, v0, 0]], float)
        self.veh_set = [vehicle(x0[i], dt=self.dt, backupidx=0) for i in range(NV)]
        self.desired_x = [np.array([0, x0[i, 1], v0, 0], float) for i in range(NV)]

    def _retarget(self):
        """Lane-change target of the ego relative to the obstacle lane (:103-116)."""
        l0, l1 = self.veh_set[0].laneidx, self.veh_set[1].laneidx
        if l0 < l1 or (l0 == l1 and l1 > 0):
            y = 1.8 + 3.6 * (l1 - 1)
        else:
            y = 1.8 + 3.6 * (l1 + 1)
        return np.array([0, y, v0, 0], float)

    def step(self, t_):
        n = self.predictiveModel.n
        xx_set = [None] * self.NV
        # the vehicles' backup rollouts in batched calls (one bmpc_model_eval launch each): vehicles
        # 0 and 1 together -- update_backup below runs at i == 1 only, after that vehicle's
        # rollout -- and the rest after it, as the reference's per-vehicle loop sees the policies
        states = [np.asarray(v.state, float) for v in self.veh_set]
        head = self.predictiveModel.zpred_eval(np.stack(states[:2]))
        tail = None
        for i, veh in enumerate(self.veh_set):
            z = veh.state
            if i < 2:
                xx_set[i] = head[i]
            else:
                if tail is None:
                    tail = self.predictiveModel.zpred_eval(np.stack(states[2:]))
                xx_set[i] = tail[i - 2]
            new = round((z[1] - 1.8) / 3.6)
            if t_ == 0 or (new != veh.laneidx and abs(z[1] - 1.8 - 3.6 * new) < 1.4):
                veh.laneidx = new
                self.desired_x[i][1] = 1.8 + new * 3.6
                if i == 1:
                    tgt = self._retarget()
                    cons = self.cons
                    self.predictiveModel.update_backup([lambda x: backup_maintain(x, cons),
                                                        lambda x: backup_brake(x, cons),
                                                        lambda x: backup_lc(x, tgt)])
            if t_ % 10 == 0 and i != 0 and with_probability(0.5):
                pass   # the reference only rewrites desired_x here, which nothing reads (:121-133)
        ego = self.veh_set[0]
        x1 = xx_set[0][:, ego.backupidx * n:(ego.backupidx + 1) * n]
        u0_set = [None] * self.NV
        for i in range(1, self.NV):
            hi = np.array([min(np.append(veh_col(x1, xx_set[i][:, j * n:(j + 1) * n],
                                                 [self.cons.L + 1, self.cons.W + 0.2]),
                                         lane_bdry_h(x1, self.LB[0], self.LB[1]))) for j in range(self.m)])
            self.veh_set[i].backupidx = int(np.argmax(hi))
            u0_set[i] = self.backupcons[self.veh_set[i].backupidx](self.veh_set[i].state)
        e, o = self.veh_set[0].state, self.veh_set[1].state
        Ydes = 1.8 + ego.laneidx * 3.6 if e[0] < o[0] else o[1]
        vdes = v0 if (abs(e[1] - Ydes) < 1 and e[0] > o[0] + 3) else o[2] + 1 * (o[0] + 1.5 - e[0])
        xRef = np.array([0, Ydes, vdes, 0], float)
        self.mpc.solve(e, o, xRef)
        u_set = [self.mpc.uPred[0]] + u0_set[1:]
        xPred, zPred, uPred, branch_w = self.mpc.BT2array()
        ego.step(u_set[0])
        for i in range(1, self.NV):
            self.veh_set[i].step(u_set[i])
        x_set = [v.state for v in self.veh_set]
        return u_set, x_set, xx_set, xPred, zPred, branch_w


def Highway_sim(env, T):
    """Closed loop of T seconds (:393-445); returns the reference's record tuple."""
    collision = False
    N = int(round(T / env.dt))
    state_rec = np.zeros([env.NV, N, 4])
    input_rec = np.zeros([env.NV, N, 2])
    backup_rec = [[None] * N for _ in range(env.NV)]
    backup_choice_rec = [[None] * N for _ in range(env.NV)]
    xPred_rec, zPred_rec, branch_w_rec = [None] * N, [None] * N, [None] * N
    for i, veh in enumerate(env.veh_set):
        state_rec[i][0] = veh.state
    dis = 100
    for t in range(N):
        if not collision:
            for i in range(env.NV):
                for j in range(env.NV):
                    if i != j:
                        a, b = env.veh_set[i], env.veh_set[j]
                        dis = max(abs(a.state[0] - b.state[0]) - 0.5 * (a.v_length + b.v_length),
                                  abs(a.state[1] - b.state[1]) - 0.5 * (a.v_width + b.v_width))
                if dis < 0:   # after each i: the distance to vehicle i's last partner (:427-428)
                    collision = True
        u_set, x_set, xx_set, xPred, zPred, branch_w = env.step(t)
        xPred_rec[t], zPred_rec[t], branch_w_rec[t] = xPred, zPred, branch_w
        for i in range(env.NV):
            input_rec[i][t] = u_set[i]
            state_rec[i][t] = x_set[i]
            backup_rec[i][t] = xx_set[i]
            backup_choice_rec[i][t] = env.veh_set[i].backupidx
    return state_rec, input_rec, backup_rec, backup_choice_rec, xPred_rec, zPred_rec, branch_w_rec, collision


def merge_geometry(N_lane, merge_lane, merge_s, merge_R, merge_side=0):
    """Ramp geometry of the merge scene (:447-...): straight lead-in + circular arc."""
    th = np.arccos(1 - lane_width * merge_lane / merge_R)
    if merge_side == 0:
        center = np.array([merge_s + merge_R * np.sin(th), (N_lane - merge_lane) * lane_width + merge_R])
        start = np.array([merge_s - merge_s * np.cos(th), N_lane * lane_width + np.sin(th) * merge_s])
    else:
        center = np.array([merge_s + merge_R * np.sin(th), merge_lane * lane_width - merge_R])
        start = np.array([merge_s - merge_s * np.cos(th), -np.sin(th) * merge_s - lane_width * merge_lane])
    s1 = np.linspace(0, merge_s, num=int(merge_s / 0.5), endpoint=False)
    s2 = merge_s + np.linspace(0, merge_R * th, num=int(merge_R * th / 0.5))
    sgn = 1.0 if merge_side == 0 else -1.0
    X1 = start[0] + s1 * np.cos(th)
    Y1 = start[1] - sgn * s1 * np.sin(th)
    psi1 = -sgn * np.ones(s1.shape) * th
    psi2 = sgn * (s2 - s2[-1]) / merge_R
    X2 = center[0] + sgn * np.sin(psi2) * merge_R
    if merge_side == 0:
        Y2 = center[1] - np.cos(psi2) * merge_R
    else:
        Y2 = center[1] + np.cos(psi2) * merge_R - merge_lane * lane_width
    return X1, X2, Y1, Y2, psi1, psi2


class Highway_env_merge:
    """Merge scene (Highway_env_branch.py:271-390): the ego starts on the ramp (laneID 1),
    the obstacle on the main road.

    Per step: a vehicle past merge_s + 8 switches to laneID 0; every vehicle's backup
    rollouts come from pred_model[laneID] (:326-331); the obstacle keeps backup policy 0 --
    the reference computes an argmax over its policies and then overwrites every backupidx
    with 0 (:334-345), so only the overwrite is kept here; the ego solves with the S, x_ref and
    bx of its lane: identity / the last lane centre / the plan's bound on the main road, the
    ramp's tangent transformation and bounds from the lane-reference interpolants on the
    ramp (:350-364)."""

    def __init__(self, NV, N_lane, mpc, pred_model, merge_lane=2, merge_s=50, merge_R=300, merge_side=0, dt=0.05):
        self.dt, self.NV, self.N_lane = dt, NV, N_lane
        self.laneID = [1] + [0] * (NV - 1)
        self.merge_lane, self.merge_s, self.merge_R, self.merge_side = merge_lane, merge_s, merge_R, merge_side
        self.pred_model, self.mpc = pred_model, mpc
        self.backupcons = [pm.backupcons for pm in pred_model]
        self.m = [len(b) for b in self.backupcons]
        self.cons = mpc.predictiveModel.cons
        self.LB = [self.cons.W / 2, N_lane * 3.6 - self.cons.W / 2]
        X1, X2, Y1, Y2, psi1, psi2 = merge_geometry(N_lane, merge_lane, merge_s, merge_R, merge_side)
        self.merge_theta = np.arccos(1 - lane_width * merge_lane / merge_R)
        self.merge_end = merge_s + merge_R * np.sin(self.merge_theta)
        self.merge_lane_ref_X = np.append(X1, X2)
        self.merge_lane_ref_Y = np.append(Y1, Y2)
        self.merge_lane_ref_psi = np.append(psi1, psi2)
        self.refY = interpolant("refY", "linear", [self.merge_lane_ref_X], self.merge_lane_ref_Y)
        self.refpsi = interpolant("refY", "linear", [self.merge_lane_ref_X], self.merge_lane_ref_psi)
        x0 = np.array([[24, 13, v0, -0.2], [15, 5.4, v0, 0]], float)
        self.veh_set = [vehicle(x0[i], dt=self.dt, backupidx=0) for i in range(NV)]
        self.desired_x = [np.array([0, x0[i, 1], v0, 0], float) for i in range(NV)]

    def transform(self, x):
        """(S, x_ref, bx) of the ego's lane (:350-364)."""
        if self.laneID[0] == 0:
            return np.eye(4), np.array([0, (self.N_lane - 0.5) * 3.6, v0, 0], float), self.mpc.param.bx
        y0, psi0 = float(self.refY(x[0])), float(self.refpsi(x[0]))
        t = np.tan(psi0)
        S = np.array([[1., 0, 0, 0], [-t, 1., 0, 0], [0, 0, 1, 0], [0, 0, 0, 1]])
        xRef = np.array([0, -t * x[0] + y0 + 1.8, v0, psi0])
        bx = np.array([-t * x[0] + y0 + 3.6 * self.merge_lane - self.cons.W / 2, t * x[0] - y0 - self.cons.W / 2,
                       psi0 + self.mpc.psimax, -psi0 + self.mpc.psimax])
        return S, xRef, bx

    def step(self, t_):
        xx_set, u0_set = [None] * self.NV, [None] * self.NV
        for i, veh in enumerate(self.veh_set):
            if veh.state[0] > self.merge_s + 8:
                self.laneID[i] = 0
        # one batched rollout call per lane model (the ramp's psiref model runs on the GPU too)
        for lid in sorted(set(self.laneID)):
            idx = [i for i in range(self.NV) if self.laneID[i] == lid]
            zz = self.pred_model[lid].zpred_eval(np.stack([np.asarray(self.veh_set[i].state, float) for i in idx]))
            for j, i in enumerate(idx):
                xx_set[i] = zz[j]
        for i, veh in enumerate(self.veh_set):
            veh.backupidx = 0
            u0_set[i] = self.backupcons[self.laneID[i]][0](veh.state)
        x = self.veh_set[0].state
        S, xRef, bx = self.transform(x)
        self.mpc.solve(self.veh_set[0].state, self.veh_set[1].state, xRef, S, Fx=None, bx=bx)
        u_set = [self.mpc.uPred[0]] + u0_set[1:]
        xPred, zPred, uPred, branch_w = self.mpc.BT2array()
        for i, veh in enumerate(self.veh_set):
            veh.step(u_set[i])
        x_set = [v.state for v in self.veh_set]
        return u_set, x_set, xx_set, xPred, zPred, branch_w


def plot_snapshot(*args, **kwargs):
    """Plotting is out of scope for the MI355X build (matplotlib snapshot, :447)."""
    return None


def animate_scenario(*args, **kwargs):
    """Animation is out of scope for the MI355X build (:566-709)."""
    print("[Highway_env_branch] animate_scenario: plotting is not part of the MI355X build; skipped")
    return None


def sim_overtake(mpc, N_lane):
    """The main_branch.py scene (:719-725): 2 vehicles, 10 s; returns the records."""
    env = Highway_env(NV=2, mpc=mpc, N_lane=N_lane)
    rec = Highway_sim(env, 10)
    state_rec, input_rec, backup_rec, backup_choice_rec, xPred_rec, zPred_rec, branch_w_rec, collision = rec
    animate_scenario(env, state_rec, backup_rec, backup_choice_rec, xPred_rec, zPred_rec, lm)
    return rec


def sim_merge(mpc, pred_model, N_lane, merge_lane, merge_s, merge_R, merge_side, T=6):
    """The main_branch.py merge scene (:727-733): 2 vehicles, 6 s; returns the records."""
    env = Highway_env_merge(2, N_lane, mpc, pred_model, merge_lane, merge_s, merge_R, merge_side, pred_model[0].dt)
    rec = Highway_sim(env, T)
    state_rec, input_rec, backup_rec, backup_choice_rec, xPred_rec, zPred_rec, branch_w_rec, collision = rec
    animate_scenario(env, state_rec, backup_rec, backup_choice_rec, xPred_rec, zPred_rec, lm)
    return rec
