"""NumPy restatement of the reference's CasADi predictive models (oracle; test-only).

The reference builds CasADi ``SX`` graphs once per policy set and evaluates them through
``Function`` objects (``highway_branch_dyn.py:363-398``, ``quadruped_branch_dyn.py:218-248``).
CasADi is not installed here, so this module re-evaluates the *same* expressions
numerically, following the ``casadi.SX`` branch of every helper (that is the branch the
graphs are built from), and differentiates them with a small forward-mode dual number
class instead of CasADi's ``jacobian``.

Quirks kept on purpose:
* ``backup_brake`` on SX uses ``softmax(vertcat(-7,-v), 5)`` (``highway_branch_dyn.py:117``),
  not the NumPy branch's ``(-5, 3)`` (``:121``);
* ``veh_col`` on SX does **not** clip dx/dy (``:228-235``); the NumPy branch clips to +-5;
* ``PredictiveModel.LB`` uses the constructor default ``N_lane=3`` (``:264,:279``);
* ``BF_traj`` checks the *obstacle* rollout against the lane boundary (``:346-348``);
* quadruped ``robot_col`` on SX is an L1 norm (``quadruped_branch_dyn.py:144``) and the
  branch probability has no ``softsat`` (``:212-216``);
* CasADi's derivative of ``fabs`` is ``sign`` with ``sign(0)=0``.
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import Sequence

import numpy as np


# ---------------------------------------------------------------------------------------
# forward-mode dual numbers (value + gradient w.r.t. the ego state)
# ---------------------------------------------------------------------------------------
class D:
    __slots__ = ("v", "g")

    def __init__(self, v, g):
        self.v = float(v)
        self.g = g

    @staticmethod
    def _lift(o, n):
        return o if isinstance(o, D) else D(o, np.zeros(n))

    def __add__(self, o):
        if isinstance(o, D):
            return D(self.v + o.v, self.g + o.g)
        return D(self.v + o, self.g)

    __radd__ = __add__

    def __sub__(self, o):
        if isinstance(o, D):
            return D(self.v - o.v, self.g - o.g)
        return D(self.v - o, self.g)

    def __rsub__(self, o):
        return D(o - self.v, -self.g)

    def __mul__(self, o):
        if isinstance(o, D):
            return D(self.v * o.v, self.g * o.v + o.g * self.v)
        return D(self.v * o, self.g * o)

    __rmul__ = __mul__

    def __truediv__(self, o):
        if isinstance(o, D):
            return D(self.v / o.v, (self.g * o.v - o.g * self.v) / (o.v * o.v))
        return D(self.v / o, self.g / o)

    def __rtruediv__(self, o):
        return D(o / self.v, -o * self.g / (self.v * self.v))

    def __neg__(self):
        return D(-self.v, -self.g)


def _exp(a):
    if isinstance(a, D):
        e = math.exp(a.v)
        return D(e, a.g * e)
    return math.exp(a)


def _cos(a):
    if isinstance(a, D):
        return D(math.cos(a.v), -math.sin(a.v) * a.g)
    return math.cos(a)


def _sin(a):
    if isinstance(a, D):
        return D(math.sin(a.v), math.cos(a.v) * a.g)
    return math.sin(a)


def _sign(v):
    return 1.0 if v > 0 else (-1.0 if v < 0 else 0.0)


def _fabs(a):
    if isinstance(a, D):
        return D(abs(a.v), _sign(a.v) * a.g)
    return abs(a)


def _val(a):
    return a.v if isinstance(a, D) else float(a)


def _grad(a, n):
    return a.g if isinstance(a, D) else np.zeros(n)


def _seed(x):
    n = len(x)
    return [D(float(x[i]), np.eye(n)[i].copy()) for i in range(n)]


# ---------------------------------------------------------------------------------------
# scalar helpers (SX branches)
# ---------------------------------------------------------------------------------------
def softmin(vals, gamma):
    """``softmin`` SX branch: sum(exp(-g*x)*x)/sum(exp(-g*x)) (highway_branch_dyn.py:151-155)."""
    num = 0.0
    den = 0.0
    for v in vals:
        e = _exp(-gamma * v)
        num = num + e * v
        den = den + e
    return num / den


def softmax(vals, gamma):
    """``softmax`` SX branch (highway_branch_dyn.py:158-162)."""
    num = 0.0
    den = 0.0
    for v in vals:
        e = _exp(gamma * v)
        num = num + e * v
        den = den + e
    return num / den


def softsat(x, s):
    """``softsat`` (highway_branch_dyn.py:38-39)."""
    e = _exp(s * x)
    return (e - 1) / (e + 1) * 0.5 + 0.5


# ---------------------------------------------------------------------------------------
# policies: descriptor = (kind, params)
# ---------------------------------------------------------------------------------------
MAINTAIN, BRAKE, LC, MAINTAIN_TRACKV, FORWARD, STOP = 0, 1, 2, 3, 4, 5
MAINTAIN_PSIREF, MAINTAIN_TRACKV_PSIREF, BRAKE_PSIREF = 6, 7, 8


@dataclass(frozen=True)
class Policy:
    kind: int
    params: tuple = ()
    lane_ref: object = None     # psiref kinds: LaneRef


class LaneRef:
    """``casadi.interpolant(name, 'linear', [grid], values)`` (main_branch.py:78-79): linear on
    the cell [g_i, g_i+1) holding t (the last grid point <= t, clamped to the first / last
    cell, so the end cells extend beyond the grid); d/dt = the cell's slope."""

    def __init__(self, grid, values):
        self.g = np.asarray(grid, float).reshape(-1)
        self.v = np.asarray(values, float).reshape(-1)

    def __call__(self, t):
        tv = _val(t)
        i = int(np.clip(np.searchsorted(self.g, tv, side="right") - 1, 0, self.g.size - 2))
        g0, g1, v0, v1 = self.g[i], self.g[i + 1], self.v[i], self.v[i + 1]
        return (t - g0) / (g1 - g0) * (v1 - v0) + v0


def policy_u(pol: Policy, x):
    """Input of a backup policy at state ``x`` (SX semantics).

    * MAINTAIN  -- ``backup_maintain`` :54-67   u=[0, -Kpsi*psi]
    * BRAKE     -- ``backup_brake`` :108-119    u=[softmax([-7,-v],5), -Kpsi*psi]
    * LC        -- ``backup_lc`` :136-146       u=[-0.8558(v-v*), -0.3162(y-y*)-3.9889(psi-psi*)]
    * MAINTAIN_TRACKV -- ``backup_maintain_trackV`` :80-88 u=[0.5(v0-v), -Kpsi*psi]
    * FORWARD/STOP -- ``quadruped_branch_dyn.backup_forward/stop`` :34-54
    * *_PSIREF -- the MX branches with psiref (:66-77, :89-96, :122-130): the second input is
      psiref(X) - Kpsi*psi, brake's first softmax([-5,-v],3)
    """
    k, p = pol.kind, pol.params
    if k == MAINTAIN_PSIREF:
        return [0.0, pol.lane_ref(x[0]) - x[3] * p[0]]
    if k == MAINTAIN_TRACKV_PSIREF:
        return [0.5 * (p[1] - x[2]), pol.lane_ref(x[0]) - x[3] * p[0]]
    if k == BRAKE_PSIREF:
        return [softmax([-5.0, -x[2]], 3.0), pol.lane_ref(x[0]) - x[3] * p[0]]
    if k == MAINTAIN:
        return [0.0, -p[0] * x[3]]
    if k == BRAKE:
        return [softmax([-7.0, -x[2]], 5.0), -p[0] * x[3]]
    if k == LC:
        t = p
        return [-0.8558 * (x[2] - t[2]), -0.3162 * (x[1] - t[1]) - 3.9889 * (x[3] - t[3])]
    if k == MAINTAIN_TRACKV:
        return [0.5 * (p[1] - x[2]), -p[0] * x[3]]
    if k == FORWARD:
        return [p[0], 0.0, 0.0]
    if k == STOP:
        return [0.0, 0.0, 0.0]
    raise ValueError(f"unknown policy kind {k}")


# ---------------------------------------------------------------------------------------
# dynamics
# ---------------------------------------------------------------------------------------
def dubin(x, u):
    """``dubin`` (highway_branch_dyn.py:17-34)."""
    return [x[2] * _cos(x[3]), x[2] * _sin(x[3]), u[0], u[1]]


def quad_kinetics(x, u):
    """``quad_kinetics`` (quadruped_branch_dyn.py:14-27)."""
    return [u[0] * _cos(x[2]) - u[1] * _sin(x[2]), u[0] * _sin(x[2]) + u[1] * _cos(x[2]), u[2]]


class _ModelBase:
    """Common part of the two predictive models (duck-typed interface of the reference)."""

    n: int
    d: int

    def f(self, x, u):
        raise NotImplementedError

    def step(self, x, u):
        fx = self.f(x, u)
        return [x[i] + fx[i] * self.dt for i in range(self.n)]

    # --- PredictiveModel.dyn_linearization (highway_branch_dyn.py:284-291) --------------
    def dyn_linearization(self, x, u):
        x = np.asarray(x, float)
        u = np.asarray(u, float)
        n, d = self.n, self.d
        xs = _seed(np.concatenate([x, u]))
        xpD = self.step(xs[:n], xs[n:])
        J = np.array([_grad(v, n + d) for v in xpD])
        A = J[:, :n].copy()
        B = J[:, n:].copy()
        xp = np.array([_val(v) for v in xpD])
        C = xp - A @ x - B @ u
        return A, B, C, xp

    def rollout(self, x, pol, N=None):
        """``propagate_backup`` (highway_branch_dyn.py:174-187): rows are x_1..x_N."""
        N = self.N if N is None else N
        out = []
        for _ in range(N):
            x = self.step(x, policy_u(pol, x))
            out.append(x)
        return out

    # --- zpred_eval (:310-311) ----------------------------------------------------------
    def zpred_eval(self, z):
        z = [float(v) for v in z]
        cols = []
        for pol in self.policies:
            cols.append(np.array([[_val(v) for v in row] for row in self.rollout(z, pol)]))
        return np.hstack(cols)

    def xpred_eval(self, x):
        x = [float(v) for v in x]
        traj = np.array([[_val(v) for v in row] for row in self.rollout(x, self.policies[0])])
        return traj, np.array([_val(v) for v in policy_u(self.policies[0], x)])

    # --- branch_eval (:298-301) ---------------------------------------------------------
    def branch_eval(self, x, z):
        n = self.n
        xD = _seed(np.asarray(x, float))
        x1 = self.rollout(xD, self.policies[0])            # ego rollout, policy 0 (:371-372)
        zf = [float(v) for v in z]
        hi = []
        for pol in self.policies:
            x2 = self.rollout(zf, pol)                        # obstacle rollout (:374-377)
            hi.append(self.bf_traj(x2, x1))
        p = self.branch_prob(hi)
        pv = np.array([_val(v) for v in p])
        dp = np.array([_grad(v, n) for v in p])
        return pv, dp

    # --- col_eval (:322-325) ------------------------------------------------------------
    def col_eval(self, x, z):
        x = np.asarray(x, float)
        hD = self.col_h(_seed(x), [float(v) for v in z])
        dh = _grad(hD, self.n).copy()
        h = _val(hD)
        return h - np.dot(dh, x), dh

    def update_backup(self, policies):
        self.policies = list(policies)
        self.m = len(self.policies)


class HighwayModel(_ModelBase):
    """``highway_branch_dyn.PredictiveModel`` (highway_branch_dyn.py:262-398)."""

    def __init__(self, N, dt, policies, L=4.0, W=2.5, s1=2.0, N_lane=3, n=4, d=2):
        self.n, self.d, self.N, self.dt = n, d, N, dt
        self.L, self.W, self.s1 = L, W, s1
        self.LB = [W / 2.0, N_lane * 3.6 - W / 2.0]          # :279
        self.policies = list(policies)
        self.m = len(self.policies)

    def f(self, x, u):
        return dubin(x, u)

    @staticmethod
    def veh_col(a, b, size, alpha=1.0):
        """``veh_col`` SX branch (:228-235), one row, no clipping."""
        dx = _fabs(a[0] - b[0]) - size[0]
        dy = _fabs(a[1] - b[1]) - size[1]
        ex = _exp(alpha * dx)
        ey = _exp(dy * alpha)
        return (dx * ex + dy * ey) / (ex + ey)

    @staticmethod
    def lane_bdry_h(x, lb, ub):
        """``lane_bdry_h`` SX branch (:195-201), one row."""
        return softmin([x[1] - lb, ub - x[1]], 5.0)

    def bf_traj(self, x2, x1):
        """``BF_traj(x1=obstacle, x2=ego)`` (:337-349)."""
        size = [self.L + 2.0, self.W + 0.2]
        h = [self.veh_col(x2[k], x1[k], size) for k in range(len(x2))]
        h += [self.lane_bdry_h(x2[k], self.LB[0], self.LB[1]) for k in range(len(x2))]
        return softmin(h, 5.0)

    def branch_prob(self, hi):
        """``branch_prob`` (:355-359)."""
        mm = [_exp(self.s1 * softsat(h, 1.0)) for h in hi]
        s = 0.0
        for v in mm:
            s = s + v
        return [v / s for v in mm]

    def col_h(self, x, z):
        """``h = veh_col(x.T, z.T, [L+1, W+0.2], 1)`` (:386)."""
        return self.veh_col(x, z, [self.L + 1.0, self.W + 0.2], 1.0)


class HighwayMergeModel(HighwayModel):
    """``highway_branch_dyn.PredictiveModel_merge`` (highway_branch_dyn.py:400-502): same
    dynamics, collision row and branch probabilities as the highway model; ``BF_traj``
    (:463-467) is softmin_5 over veh_col(obs, ego, [L+1, W+0.2]) only -- no lane-boundary term.
    Its policies are the merge scene's (main_branch.py:82-85): maintain_trackV(v0) / brake
    (pred_model[0]) or their lane-reference tracking forms (*_PSIREF, pred_model[1])."""

    def bf_traj(self, x2, x1):
        size = [self.L + 1.0, self.W + 0.2]
        return softmin([self.veh_col(x2[k], x1[k], size) for k in range(len(x2))], 5.0)


class QuadrupedModel(_ModelBase):
    """``quadruped_branch_dyn.PredictiveModel`` (quadruped_branch_dyn.py:154-248)."""

    def __init__(self, N, dt, policies, L1=0.5, W1=0.3, L2=1.0, W2=0.6, col_tol=0.2, s1=2.0,
                 n=3, d=3):
        self.n, self.d, self.N, self.dt = n, d, N, dt
        self.L1, self.W1, self.L2, self.W2, self.col_tol, self.s1 = L1, W1, L2, W2, col_tol, s1
        self.policies = list(policies)
        self.m = len(self.policies)

    def f(self, x, u):
        return quad_kinetics(x, u)

    def robot_col(self, a, b):
        """``robot_col`` SX branch (:135-144): L1 norm."""
        return _fabs(a[0] - b[0]) + _fabs(a[1] - b[1]) - (self.L1 + self.L2) / 2.0 - self.col_tol

    def bf_traj(self, x2, x1):
        """``BF_traj`` (:204-211) -- obstacle vs ego, softmin over N."""
        return softmin([self.robot_col(x2[k], x1[k]) for k in range(len(x2))], 5.0)

    def branch_prob(self, hi):
        """``branch_prob`` (:212-216) -- no softsat."""
        mm = [_exp(self.s1 * h) for h in hi]
        s = 0.0
        for v in mm:
            s = s + v
        return [v / s for v in mm]

    def col_h(self, x, z):
        return self.robot_col(x, z)


def highway_policies(Kpsi: float, lc_target: Sequence[float]):
    """The ``main_branch.py:39`` policy set [maintain, brake, lc(xRef)]."""
    return [Policy(MAINTAIN, (Kpsi,)), Policy(BRAKE, (Kpsi,)),
            Policy(LC, tuple(float(v) for v in lc_target))]


def quadruped_policies(v0: float):
    """The ``main_quadruped.py:21`` policy set [forward(v0), stop]."""
    return [Policy(FORWARD, (v0,)), Policy(STOP, ())]
