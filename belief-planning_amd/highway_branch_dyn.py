"""Highway predictive model -- drop-in for the reference's ``highway_branch_dyn``.

NumPy helpers keep the reference's NumPy-branch semantics (the environment uses them on
plain arrays: ``Highway_env_branch.py:137-149,181``).  Called with a policy tracer they
lower to GPU policy descriptors (the role the ``casadi.SX`` branch plays in the
reference).  ``PredictiveModel`` evaluates dynamics, Jacobians, obstacle rollouts, branch
probabilities and the linearised collision constraint with the gfx950 kernels of
libbmpc.so (``bmpc_model_eval``); there is no CPU fallback.
"""
from __future__ import annotations

import numpy as np

from bmpc import abi
from bmpc.tracing import PolicySpec, Tracer, lane_ref_of, trace

__all__ = ["np", "dubin", "softsat", "backup_maintain", "backup_maintain_trackV", "backup_brake",
           "backup_lc", "softmin", "softmax", "propagate_backup", "lane_bdry_h", "veh_col",
           "PredictiveModel", "PredictiveModel_merge", "interpolant"]


def dubin(x, u):
    """Unicycle kinematics [v cos psi, v sin psi, a, r] (highway_branch_dyn.py:17-34)."""
    return np.array([x[2] * np.cos(x[3]), x[2] * np.sin(x[3]), u[0], u[1]])


def softsat(x, s):
    return (np.exp(s * x) - 1) / (np.exp(s * x) + 1) * 0.5 + 0.5


def softmin(x, gamma=1):
    x = np.asarray(x, float)
    e = np.exp(-gamma * x)
    return np.sum(e * x) / np.sum(e)


def softmax(x, gamma=1):
    x = np.asarray(x, float)
    e = np.exp(gamma * x)
    return np.sum(e * x) / np.sum(e)


class PsirefPolicy(NotImplementedError):
    """A backup policy whose lane reference is not a 1-D linear interpolant (the only form the
    kernels evaluate)."""


def _lane_ref(psiref):
    if not isinstance(psiref, LinearInterpolant):
        raise PsirefPolicy("psiref must be a 1-D linear interpolant (interpolant(name, 'linear', [grid], values))")
    if psiref.g.size < 2 or psiref.g.size > abi.MAX_LANE_REF or not np.all(np.diff(psiref.g) > 0):
        raise PsirefPolicy("the lane reference's grid must be strictly increasing, 2 .. MAX_LANE_REF points")
    return psiref


class LinearInterpolant:
    """``casadi.interpolant(name, 'linear', [grid], values)`` for the merge scene's lane
    reference (main_branch.py:76-77, Highway_env_branch.py:312-313): piecewise linear on the
    grid cells, the end cells extended beyond the grid (CasADi's 'linear' plugin).  Policies
    that track it lower to *_PSIREF descriptors; the kernels evaluate the same interpolant."""

    def __init__(self, name, grid, values):
        self.name = name
        self.g = np.asarray(grid, float).reshape(-1)
        self.v = np.asarray(values, float).reshape(-1)

    def __call__(self, t):
        t = np.asarray(t, float)
        i = np.clip(np.searchsorted(self.g, t, side="right") - 1, 0, self.g.size - 2)
        g0, g1, v0, v1 = self.g[i], self.g[i + 1], self.v[i], self.v[i + 1]
        r = v0 + (t - g0) / (g1 - g0) * (v1 - v0)
        return float(r) if r.ndim == 0 else r


def interpolant(name, solver, grid, values, *opts):
    """CasADi ``interpolant`` subset used by the reference (1-D, 'linear')."""
    if solver != "linear" or len(grid) != 1:
        raise NotImplementedError("only 1-D linear interpolants (the merge lane reference)")
    return LinearInterpolant(name, grid[0], values)


def backup_maintain(x, cons, psiref=None):
    """Keep speed, steer psi to 0 (:54-78); with psiref, steer to the lane reference."""
    if isinstance(x, Tracer):
        if psiref is not None:
            return PolicySpec(abi.POL_MAINTAIN_PSIREF, (float(cons.Kpsi),), _lane_ref(psiref))
        return PolicySpec(abi.POL_MAINTAIN, (float(cons.Kpsi),))
    r = -cons.Kpsi * x[3] if psiref is None else psiref(x[0]) - cons.Kpsi * x[3]
    return np.array([0.0, r])


def backup_maintain_trackV(x, cons, v0, psiref=None):
    """Track speed v0 (:80-96)."""
    if isinstance(x, Tracer):
        if psiref is not None:
            return PolicySpec(abi.POL_MAINTAIN_TRACKV_PSIREF, (float(cons.Kpsi), float(v0)), _lane_ref(psiref))
        return PolicySpec(abi.POL_MAINTAIN_TRACKV, (float(cons.Kpsi), float(v0)))
    r = -cons.Kpsi * x[3] if psiref is None else psiref(x[0]) - cons.Kpsi * x[3]
    return np.array([0.5 * (v0 - x[2]), r])


def backup_brake(x, cons, psiref=None):
    """Brake.  Traced (graph) form: softmax([-7, -v], 5); NumPy form: softmax([-5, -v], 3)
    -- the two branches of the reference differ (:117 vs :121) and both are kept; the psiref
    graph form uses softmax([-5, -v], 3) (:122-126)."""
    if isinstance(x, Tracer):
        if psiref is not None:
            return PolicySpec(abi.POL_BRAKE_PSIREF, (float(cons.Kpsi),), _lane_ref(psiref))
        return PolicySpec(abi.POL_BRAKE, (float(cons.Kpsi),))
    r = -cons.Kpsi * x[3] if psiref is None else psiref(x[0]) - cons.Kpsi * x[3]
    return np.array([softmax(np.array([-5.0, -x[2]]), 3), r])


def backup_lc(x, x0):
    """Lane change towards x0 (:136-148)."""
    if isinstance(x, Tracer):
        return PolicySpec(abi.POL_LC, tuple(float(v) for v in np.asarray(x0, float)[:4]))
    return np.array([-0.8558 * (x[2] - x0[2]), -0.3162 * (x[1] - x0[1]) - 3.9889 * (x[3] - x0[3])])


def propagate_backup(x, dyn, N, ts):
    """Euler rollout, rows x_1..x_N (:174-187)."""
    x = np.asarray(x, float)
    out = np.empty((N, x.shape[0]))
    for i in range(N):
        x = x + dyn(x) * ts
        out[i] = x
    return out


def lane_bdry_h(x, lb=0, ub=7.2):
    """Soft distance to the road boundary (NumPy form, :207-214)."""
    x = np.asarray(x, float)
    if x.ndim == 1:
        return softmin(np.array([x[1] - lb, ub - x[1]]), 5)
    return np.array([softmin(np.array([r[1] - lb, ub - r[1]]), 5) for r in x])


def veh_col(x1, x2, size, alpha=1):
    """Soft vehicle clearance, NumPy form with dx, dy clipped to +-5 (:243-254)."""
    a, b = np.asarray(x1, float), np.asarray(x2, float)
    one = a.ndim == 1
    a, b = np.atleast_2d(a), np.atleast_2d(b)
    dx = np.clip(np.abs(a[:, 0] - b[:, 0]) - size[0], -5, 5)
    dy = np.clip(np.abs(a[:, 1] - b[:, 1]) - size[1], -5, 5)
    h = (dx * np.exp(alpha * dx) + dy * np.exp(dy * alpha)) / (np.exp(alpha * dx) + np.exp(dy * alpha))
    return h[0] if one else h


class PredictiveModel:
    """``highway_branch_dyn.PredictiveModel`` (:262-398) on the GPU.

    Same constructor and duck-typed interface; ``backupcons`` are traced into policy
    descriptors instead of being compiled into CasADi graphs.  All evaluation methods
    accept a single point or a batch (leading axis)."""

    model_kind = abi.MODEL_HIGHWAY

    def __init__(self, n, d, N, backupcons, dt, cons, N_lane=3):
        if (n, d) != (4, 2):
            raise ValueError("the highway model is 4-state / 2-input")
        self.n, self.d, self.N, self.dt, self.cons = n, d, N, dt, cons
        self.N_lane = N_lane
        self.LB = [cons.W / 2, N_lane * 3.6 - cons.W / 2]
        self.update_backup(backupcons)

    # ---- policies ------------------------------------------------------------------------
    def update_backup(self, backupcons):
        """Re-trace the policy lambdas (the reference rebuilds its graphs, :331-334)."""
        self.backupcons = backupcons
        self.m = len(backupcons)
        self.policies = trace(backupcons)

    def policy_rows(self):
        return [p.as_row() for p in self.policies]

    def model_constants(self):
        return [float(self.cons.L), float(self.cons.W), float(self.cons.s1), float(self.N_lane)]

    def desc(self):
        return abi.make_desc(abi.CTRL_CVAR, self.model_kind, self.n, self.d, self.N, 1, self.m, self.dt,
                             np.eye(self.n), np.eye(self.d), np.zeros((0, self.n)), [],
                             np.zeros((0, self.d)), [], [0, 0], self.model_constants())

    # ---- evaluation (GPU) -------------------------------------------------------------------
    def _eval(self, x, u, z):
        from bmpc import plan
        x = np.atleast_2d(np.asarray(x, float))
        B = x.shape[0]
        u = np.zeros((B, self.d)) if u is None else np.broadcast_to(np.atleast_2d(u), (B, self.d))
        z = x if z is None else np.broadcast_to(np.atleast_2d(np.asarray(z, float)), (B, self.n))
        rows = [self.policy_rows()] * B
        return plan.model_eval(self.desc(), rows, x, u, z)

    def dyn_linearization(self, x, u):
        """(A, B, C, x+) of x+ = x + f(x,u) dt with C = x+ - A x - B u (:284-291)."""
        r = self._eval(x, u, None)
        sq = np.ndim(x) == 1
        out = (r["A"], r["B"], r["C"], r["xp"])
        return tuple(v[0] for v in out) if sq else out

    def branch_eval(self, x, z):
        """Branch probabilities p[m] and dp/dx [m, n] (:298-301)."""
        r = self._eval(x, None, z)
        return (r["p"][0], r["dp"][0]) if np.ndim(x) == 1 else (r["p"], r["dp"])

    def zpred_eval(self, z):
        """Obstacle rollouts under the m policies, (N, m*n) (:310-311)."""
        r = self._eval(z, None, z)
        return r["zpred"][0] if np.ndim(z) == 1 else r["zpred"]

    def xpred_eval(self, x):
        """Ego rollout under policy 0 and that policy's input at x (:314-315)."""
        traj = self.zpred_eval(x)[..., :self.n]
        return traj, self.backupcons[0](np.asarray(x, float))

    def col_eval(self, x, z):
        """Linearised collision constraint: (h - dh.x, dh) (:322-325)."""
        r = self._eval(x, None, z)
        return (r["h0"][0], r["dh"][0]) if np.ndim(x) == 1 else (r["h0"], r["dh"])


class PredictiveModel_merge(PredictiveModel):
    """``highway_branch_dyn.PredictiveModel_merge`` (:400-502): the highway model whose
    ``BF_traj`` is softmin_5 of veh_col(obstacle, ego, [L+1, W+0.2]) only (:463-467), model
    kind HIGHWAY_MERGE (its plans take the per-solve S / bx of ``BranchMPC_CVaR.solve``).

    Both of the merge scene's models run on the GPU: ``pred_model[0]`` (maintain_trackV(v0),
    brake -- the controller's model, main_branch.py:84-88) and ``pred_model[1]`` whose backups
    track the ramp's lane reference (psiref, :82-85; the scene asks it for the ramp vehicles'
    rollouts, Highway_env_branch.py:331): its policies lower to *_PSIREF descriptors and the
    kernels evaluate psiref(X) from the interpolant's grid (bmpc_model_eval_ref; a controller
    plan over it gets the reference through bmpc_set_lane_ref)."""

    model_kind = abi.MODEL_HIGHWAY_MERGE

    def __init__(self, n, d, N, backupcons, dt, cons, merge_ref, laneID=0, N_lane1=3, N_lane2=2):
        if (n, d) != (4, 2):
            raise ValueError("the highway model is 4-state / 2-input")
        self.n, self.d, self.N, self.dt, self.cons = n, d, N, dt, cons
        self.N_lane2, self.laneID = N_lane2, laneID
        self.refY, self.refpsi = merge_ref[0], merge_ref[1]
        self.LB1 = [cons.W / 2, N_lane1 * 3.6 - cons.W / 2]
        self.N_lane, self.LB = N_lane1, self.LB1
        self.update_backup(backupcons)

    def update_backup(self, backupcons):
        super().update_backup(backupcons)
        self.lane_ref = lane_ref_of(self.policies)

    def _eval(self, x, u, z):
        from bmpc import plan
        x = np.atleast_2d(np.asarray(x, float))
        B = x.shape[0]
        u = np.zeros((B, self.d)) if u is None else np.broadcast_to(np.atleast_2d(u), (B, self.d))
        z = x if z is None else np.broadcast_to(np.atleast_2d(np.asarray(z, float)), (B, self.n))
        return plan.model_eval(self.desc(), [self.policy_rows()] * B, x, u, z, lane_ref=self.lane_ref)
