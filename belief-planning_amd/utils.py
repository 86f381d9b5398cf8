"""Constants containers of the reference surface (``utils.py:14-90``).

Same class names, field names and defaults as the reference so driver scripts that build
``Branch_constants(...)`` / ``Quad_constants(...)`` / ``MPCParams(...)`` run unchanged.
``HMM_constants`` is provided as well: the reference's ``HMM_backup_dyn.py:5`` imports it
but ``utils.py`` never defines it (its fields are the subset of ``Branch_constants`` the
HMM model reads).
"""
from __future__ import annotations

from dataclasses import dataclass, field, fields

import numpy as np


@dataclass
class PythonMsg:
    """Frozen-field guard: assigning an attribute that is not a declared field raises."""

    def __setattr__(self, key, value):
        if key not in {f.name for f in fields(self)} and not hasattr(self, key):
            raise TypeError(f'Cannot add new field "{key}" to frozen class {self}')
        object.__setattr__(self, key, value)


def _none():
    return field(default=None)


@dataclass
class Branch_constants:
    """Highway model constants (branch probability, collision, lane keeping)."""

    s1: float = _none()
    s2: float = _none()
    c2: float = _none()
    tran_diag: float = _none()
    alpha: float = _none()
    R: float = _none()
    am: float = _none()
    rm: float = _none()
    J_c: float = _none()
    s_c: float = _none()
    ylb: float = _none()
    yub: float = _none()
    W: float = _none()
    L: float = _none()
    col_alpha: float = _none()
    Kpsi: float = _none()


HMM_constants = Branch_constants


@dataclass
class Quad_constants:
    """Quadruped model constants."""

    s1: float = _none()
    s2: float = _none()
    c2: float = _none()
    alpha: float = _none()
    R: float = _none()
    vxm: float = _none()
    vym: float = _none()
    rm: float = _none()
    W1: float = _none()
    L1: float = _none()
    W2: float = _none()
    L2: float = _none()
    col_tol: float = _none()
    col_alpha: float = _none()


@dataclass
class MPCParams(PythonMsg):
    """Parameters of the belief MPC (PredictiveControllers.MPC)."""

    n: int = _none()
    d: int = _none()
    N: int = _none()
    M: int = _none()
    m: int = _none()
    A: np.ndarray = _none()
    B: np.ndarray = _none()
    Q: np.ndarray = _none()
    R: np.ndarray = _none()
    Qf: np.ndarray = _none()
    dR: np.ndarray = _none()
    Qslack: np.ndarray = _none()
    Fx: np.ndarray = _none()
    bx: np.ndarray = _none()
    Fu: np.ndarray = _none()
    bu: np.ndarray = _none()
    xRef: np.ndarray = _none()
    slacks: bool = field(default=True)
    timeVarying: bool = field(default=False)

    def __post_init__(self):
        if self.Qf is None:
            self.Qf = np.zeros((self.n, self.n))
        if self.dR is None:
            self.dR = np.zeros(self.d)
        if self.xRef is None:
            self.xRef = np.zeros(self.n)
