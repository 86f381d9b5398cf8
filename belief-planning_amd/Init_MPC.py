"""Parameter factories of the reference (``Init_MPC.py:7-94``), same signatures and numbers.

Quirk kept: ``bx`` is returned as a 1-tuple holding the (4,1) column (the trailing comma
of ``Init_MPC.py:48-51``); ``BranchMPC_CVaR`` reads ``psimax = bx[0][2][0]`` from it.
"""
from __future__ import annotations

import numpy as np

from MPC_branch import BranchMPCParams
from PredictiveControllers import MPC  # noqa: F401  (Init_MPC.py:4 re-exports the belief MPC)
from utils import MPCParams

LANE_WIDTH = 3.6


def _lane_box(N_lane, W):
    """Rows y <= N_lane*3.6 - W/2, -y <= -W/2, psi <= 0.25, -psi <= 0.25."""
    Fx = np.zeros((4, 4))
    Fx[0, 1], Fx[1, 1], Fx[2, 3], Fx[3, 3] = 1.0, -1.0, 1.0, -1.0
    bx = np.array([[N_lane * LANE_WIDTH - W / 2], [-W / 2], [0.25], [0.25]])
    return Fx, bx


def _box_rows(k):
    """Fu = kron(I_k, [1, -1])': +-1 rows per input."""
    return np.kron(np.eye(k), np.array([1, -1])).T


def initMPCParams(nx, d, N, M, m, ydes, vdes, am, rm, N_lane, W):
    """Belief-MPC parameters (Init_MPC.py:7-34); state augmented by M*m belief entries."""
    Fx, bx = _lane_box(N_lane, W)
    Fx = np.hstack((Fx, np.zeros((4, m * M))))
    Fu = _box_rows(2)
    bu = np.array([[am], [0.5 * am], [rm], [rm]])
    Q = np.zeros((nx + M * m, nx + M * m))
    Q[:4, :4] = np.diag([0.0, 0.5, 0.2, 5.0])
    R = np.diag([30.0, 100.0])
    xRef = np.concatenate([[0.0, ydes, vdes, 0.0], np.zeros(M * m)])
    return MPCParams(n=nx + M * m, d=d, N=N, Q=Q, R=R, Fx=Fx, bx=(bx,), Fu=Fu, bu=bu, xRef=xRef,
                     slacks=True, Qslack=np.array([0, 1000]), timeVarying=True)


def initBranchMPC(n, d, N, NB, xRef, am, rm, N_lane, W):
    """Highway branch-MPC parameters (Init_MPC.py:40-72)."""
    Fx, bx = _lane_box(N_lane, W)
    bu = np.array([[am], [am], [rm], [rm]])
    return BranchMPCParams(n=n, d=d, N=N, NB=NB, Q=np.diag([0.0, 3.0, 3.0, 10.0]),
                           R=np.diag([1.0, 100.0]), Fx=Fx, bx=(bx,), Fu=_box_rows(2), bu=bu,
                           xRef=xRef, slacks=True, Qslack=np.array([0, 300]), timeVarying=True)


def initquadBranchMPC(n, d, N, NB, xRef, vxm, vym, rm):
    """Quadruped branch-MPC parameters (Init_MPC.py:74-94): no state rows (Nc = 1)."""
    bu = np.array([[vxm], [0], [vym], [vym], [rm], [rm]])
    return BranchMPCParams(n=n, d=d, N=N, NB=NB, Q=np.diag([1.0, 1.0, 1.0]),
                           R=np.diag([1.0, 100.0, 1.0]), dR=np.array([0.9, 5, 1]),
                           Fx=np.empty([0, n]), bx=(np.empty([0, 1]),), Fu=_box_rows(3), bu=bu,
                           xRef=xRef, slacks=True, Qslack=np.array([0, 300]), timeVarying=True)
