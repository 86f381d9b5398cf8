"""Quadruped predictive model -- drop-in for the reference's ``quadruped_branch_dyn``.

Planar body-velocity kinematics (x, y, theta) with inputs (vx, vy, omega) and the two
backup policies forward(v0) / stop (``quadruped_branch_dyn.py:14-248``).  The NumPy
helpers keep the reference's NumPy-branch semantics (``robot_col`` is an L2 norm there,
``:145-150``); the traced graph form -- evaluated on the GPU -- uses the SX branch's L1
norm (``:135-144``) and no ``softsat`` in the branch probability (``:212-216``).
"""
from __future__ import annotations

import numpy as np

from bmpc import abi
from bmpc.tracing import PolicySpec, Tracer
from highway_branch_dyn import PredictiveModel as _HighwayModel
from highway_branch_dyn import propagate_backup, softmax, softmin, softsat  # noqa: F401
from utils import Quad_constants  # noqa: F401  (re-exported: the reference star-imports it, :7)

__all__ = ["np", "Quad_constants", "quad_kinetics", "softsat", "backup_forward", "backup_stop", "softmin", "softmax",
           "propagate_backup", "robot_col", "PredictiveModel"]


def quad_kinetics(x, u):
    c, s = np.cos(x[2]), np.sin(x[2])
    return np.array([u[0] * c - u[1] * s, u[0] * s + u[1] * c, u[2]])


def backup_forward(x, v0):
    if isinstance(x, Tracer):
        return PolicySpec(abi.POL_FORWARD, (float(v0),))
    return np.array([v0, 0, 0])


def backup_stop(x):
    if isinstance(x, Tracer):
        return PolicySpec(abi.POL_STOP, ())
    return np.array([0, 0, 0])


def robot_col(x1, x2, L1, W1, L2, W2, tol, alpha=1):
    """NumPy form (:145-150): Euclidean clearance per row."""
    a, b = np.atleast_2d(np.asarray(x1, float)), np.atleast_2d(np.asarray(x2, float))
    return np.linalg.norm(a[:, 0:2] - b[:, 0:2], axis=1) - (L1 + L2) / 2 - tol


class PredictiveModel(_HighwayModel):
    """``quadruped_branch_dyn.PredictiveModel`` (:154-248) on the GPU."""

    model_kind = abi.MODEL_QUADRUPED

    def __init__(self, n, d, N, backupcons, dt, cons):
        if (n, d) != (3, 3):
            raise ValueError("the quadruped model is 3-state / 3-input")
        self.n, self.d, self.N, self.dt, self.cons = n, d, N, dt, cons
        self.update_backup(backupcons)

    def model_constants(self):
        c = self.cons
        return [float(c.L1), float(c.W1), float(c.L2), float(c.W2), float(c.col_tol), float(c.s1)]
