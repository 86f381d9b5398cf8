"""Synthetic workloads of the headline benchmark and the plan descriptions
of the reference's scenes (Init_MPC.initBranchMPC + Branch_constants, main_branch.py:37)."""
from __future__ import annotations

import numpy as np

from . import abi


def highway_desc(N=20, NB=1, N_lane=4, am=6.0, rm=0.3, L=4.0, W=2.5, s1=2.0, model_lanes=3):
    """initBranchMPC(n=4,d=2,N,NB,...) + Branch_constants of main_branch.py:37."""
    Fx = np.array([[0., 1, 0, 0], [0, -1, 0, 0], [0, 0, 0, 1], [0, 0, 0, -1]])
    bx = np.array([N_lane * 3.6 - W / 2, -W / 2, 0.25, 0.25])
    Fu = np.kron(np.eye(2), np.array([1, -1])).T
    bu = np.array([am, am, rm, rm])
    return abi.make_desc(abi.CTRL_CVAR, abi.MODEL_HIGHWAY, 4, 2, N, NB, 3, 0.1,
                         np.diag([0., 3, 3, 10]), np.diag([1., 100]), Fx, bx, Fu, bu, [0., 300.],
                         [L, W, s1, float(model_lanes)], ralpha=0.9)


def highway_desc_from_golden(g):
    return highway_desc(N=int(g["N"]), NB=int(g["NB"]), N_lane=int(g["N_lane"]), am=float(g["am"]),
                        rm=float(g["rm"]), L=float(g["L"]), W=float(g["W"]), s1=float(g["s1"]))


def highway_policy_rows(targets, Kpsi=0.1):
    return [[(abi.POL_MAINTAIN, (Kpsi,)), (abi.POL_BRAKE, (Kpsi,)), (abi.POL_LC, tuple(map(float, t)))]
            for t in np.atleast_2d(targets)]


LANES = np.array([1.8, 5.4, 9.0, 12.6])


def seeded_batch(B, seed=0):
    """SURVEY §8(d) synthetic inputs; row 0 is the sim_overtake initial state."""
    rng = np.random.default_rng(seed)
    x = np.zeros((B, 4))
    z = np.zeros((B, 4))
    li = rng.integers(0, 4, B)
    x[:, 0] = rng.uniform(-5, 5, B)
    x[:, 1] = LANES[li] + rng.normal(0, 0.1, B)
    x[:, 2] = rng.uniform(15, 25, B)
    x[:, 3] = np.clip(rng.normal(0, 0.02, B), -0.2, 0.2)
    lo = (li + rng.integers(1, 4, B)) % 4
    z[:, 0] = x[:, 0] + rng.uniform(-10, 30, B)
    z[:, 1] = LANES[lo]
    z[:, 2] = rng.uniform(15, 25, B)
    x[0] = [0, 1.8, 20, 0]
    z[0] = [5, 5.4, 20, 0]
    xref, tgt = xref_rule(x, z)
    return x, z, xref, tgt


def xref_rule(x, z, v0=20.0):
    """x_ref of Highway_env.step (Highway_env_branch.py:153-167) and the lane-change target
    of update_backup (:103-116), vectorised over egos (first step, t == 0)."""
    B = x.shape[0]
    l0 = np.array([round((v - 1.8) / 3.6) for v in x[:, 1]])
    l1 = np.array([round((v - 1.8) / 3.6) for v in z[:, 1]])
    tgt = np.zeros((B, 4))
    tgt[:, 2] = v0
    for i in range(B):
        if l0[i] < l1[i]:
            tgt[i, 1] = 1.8 + 3.6 * (l1[i] - 1)
        elif l0[i] > l1[i]:
            tgt[i, 1] = 1.8 + 3.6 * (l1[i] + 1)
        elif l1[i] > 0:
            tgt[i, 1] = 1.8 + 3.6 * (l1[i] - 1)
        else:
            tgt[i, 1] = 1.8 + 3.6 * (l1[i] + 1)
    Ydes = np.where(x[:, 0] < z[:, 0], 1.8 + l0 * 3.6, z[:, 1])
    vdes = np.where((np.abs(x[:, 1] - Ydes) < 1) & (x[:, 0] > z[:, 0] + 3), v0,
                    z[:, 2] + 1 * (z[:, 0] + 1.5 - x[:, 0]))
    xref = np.stack([np.zeros(B), Ydes, vdes, np.zeros(B)], axis=1)
    return xref, tgt


def quadruped_desc(N=25, NB=2, vxm=0.2, vym=0.1, rm=0.5, dt=0.2, L1=0.5, W1=0.3, L2=1.0, W2=0.6,
                   col_tol=0.2, s1=2.0):
    """initquadBranchMPC(3,3,N,NB,...) + the main_quadruped.py:15-30 constants
    (BranchMPCProx controller, 2 policies)."""
    Fu = np.kron(np.eye(3), np.array([1, -1])).T
    bu = np.array([vxm, 0.0, vym, vym, rm, rm])
    return abi.make_desc(abi.CTRL_PROX, abi.MODEL_QUADRUPED, 3, 3, N, NB, 2, dt, np.eye(3),
                         np.diag([1., 100., 1.]), np.zeros((0, 3)), [], Fu, bu, [0., 300.],
                         [L1, W1, L2, W2, col_tol, s1], dR=[0.9, 5.0, 1.0])


def quadruped_policy_rows(B, v0=0.2):
    return [[(abi.POL_FORWARD, (v0,)), (abi.POL_STOP, ())] for _ in range(B)]


def seeded_quadruped_batch(B, seed=1):
    """Synthetic quadruped egos (BASELINE config 4): ego in a 6 m x 6 m yard heading anywhere,
    obstacle 1-4 m away walking at any heading; goal x_des = (5, -3, 0) as in the recorded
    loop.  Row 0 is main_quadruped's state (ego (0, 1.8, 0), obstacle (2.5, 2.5, -pi/2))."""
    rng = np.random.default_rng(seed)
    x = np.stack([rng.uniform(-1, 1, B), rng.uniform(0, 3, B), rng.uniform(-np.pi, np.pi, B)], 1)
    r, a = rng.uniform(1, 4, B), rng.uniform(-np.pi, np.pi, B)
    z = np.stack([x[:, 0] + r * np.cos(a), x[:, 1] + r * np.sin(a), rng.uniform(-np.pi, np.pi, B)], 1)
    x[0] = [0, 1.8, 0]
    z[0] = [2.5, 2.5, -np.pi / 2]
    return x, z, quadruped_xref(x)


def quadruped_xref(x, x_des=(5.0, -3.0, 0.0)):
    """Reference of the recorded quadruped loop (tools/gen_golden.py, after quadruped_env.py):
    a point at most 5 m towards x_des, heading along the way."""
    x = np.atleast_2d(x)
    xd = np.asarray(x_des, float)
    dx = xd[None, 0:2] - x[:, 0:2]
    nrm = np.linalg.norm(dx, axis=1)
    dx = dx / np.maximum(nrm, 1e-300)[:, None] * np.minimum(nrm, 5.0)[:, None]
    psi = np.arctan2(dx[:, 1], dx[:, 0])
    psi = np.where(np.linalg.norm(dx, axis=1) > 0.1, psi, x[:, 2])
    psi = psi - 2 * np.pi * np.round((psi - xd[2]) / (2 * np.pi))
    xr = x.copy()
    xr[:, 0:2] += dx
    xr[:, 2] = psi
    return xr
