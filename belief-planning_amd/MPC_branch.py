"""Branch-MPC controllers -- drop-in for the reference's ``MPC_branch`` module.

``BranchMPC_CVaR`` keeps the reference's constructor, ``solve`` signature and the
attributes drivers read (``uPred``, ``xPred``, ``xLin``, ``uLin``, ``feasible``,
``solverTime``, ``OldInput``, ``BT``, ``BT2array()``, ``psimax``, ...), but one solve is
one call into libbmpc.so: the tree update, linearisation, SOCP assembly and the
interior-point solve all run in the gfx950 kernels (one wavefront per ego).  Passing
``batch=B`` to the constructor turns the object into a B-ego controller
(``solve_batch``).  There is no CPU fallback: without a HIP device the first solve raises
``bmpc._lib.BmpcUnavailable``.
"""
from __future__ import annotations

import datetime
from dataclasses import dataclass, field, fields

import numpy as np
from scipy import linalg

from bmpc import abi
from bmpc.topology import TreeIndex


@dataclass
class PythonMsg:
    def __setattr__(self, key, value):
        if key not in {f.name for f in fields(self)} and not hasattr(self, key):
            raise TypeError(f'Cannot add new field "{key}" to frozen class {self}')
        object.__setattr__(self, key, value)


@dataclass
class BranchMPCParams(PythonMsg):
    """Branch-MPC parameters (MPC_branch.py:27-54); Qf defaults to Q."""

    n: int = field(default=None)
    d: int = field(default=None)
    NB: int = field(default=None)
    N: int = field(default=None)
    A: np.ndarray = field(default=None)
    B: np.ndarray = field(default=None)
    Q: np.ndarray = field(default=None)
    R: np.ndarray = field(default=None)
    Qf: np.ndarray = field(default=None)
    dR: np.ndarray = field(default=None)
    Qslack: np.ndarray = field(default=None)
    Fx: np.ndarray = field(default=None)
    bx: np.ndarray = field(default=None)
    Fu: np.ndarray = field(default=None)
    bu: np.ndarray = field(default=None)
    xRef: np.ndarray = field(default=None)
    slacks: bool = field(default=True)
    timeVarying: bool = field(default=False)

    def __post_init__(self):
        if self.Qf is None:
            self.Qf = self.Q
        if self.dR is None:
            self.dR = np.zeros(self.d)
        if self.xRef is None:
            self.xRef = np.zeros(self.n)


class BranchTree:
    """One branch of the scenario tree (MPC_branch.py:65-78), filled from the GPU tree."""

    def __init__(self, xtraj, ztraj, utraj, w, depth=0):
        self.xtraj, self.ztraj, self.utraj = xtraj, ztraj, utraj
        self.dynmatr = [None] * xtraj.shape[0]
        self.w = w
        self.children = []
        self.depth = depth
        self.p = None
        self.dp = None
        self.J = 0

    def addchild(self, BT):
        self.children.append(BT)


def _weight_root(M):
    """cholesky(M).T with the sqrtm fallback (MPC_branch.py:1628-1643)."""
    try:
        return np.linalg.cholesky(M).T
    except np.linalg.LinAlgError:
        return np.real(linalg.sqrtm(M))


def _flat_bx(bx):
    return np.asarray(bx[0] if isinstance(bx, tuple) else bx, float).reshape(-1)


class BranchMPC_CVaR:
    """Branch MPC with a CVaR objective (MPC_branch.py:1598-2152) on MI355X."""

    controller_kind = abi.CTRL_CVAR

    def __init__(self, mpcParameters, predictiveModel, ralpha, S=None, batch=1, device=0):
        p = mpcParameters
        self.N, self.NB, self.n, self.d = p.N, p.NB, p.n, p.d
        self.Qslack, self.Q, self.Qf, self.R, self.dR = p.Qslack, p.Q, p.Qf, p.R, p.dR
        self.Fx, self.Fu, self.bx, self.bu = p.Fx, p.Fu, p.bx, p.bu
        self.xRef = p.xRef
        self.m = predictiveModel.m
        self.psimax = p.bx[0][2][0] if np.size(_flat_bx(p.bx)) > 2 else None
        self.S = S
        self.ralpha = ralpha
        self.param = p
        self.Wx = _weight_root(np.asarray(self.Q, float))
        self.Wu = _weight_root(np.asarray(self.R, float))
        if self.dR is not None:
            self.Wdu = _weight_root(np.diag(np.asarray(self.dR, float)))
        self.slacks, self.timeVarying = p.slacks, p.timeVarying
        self.predictiveModel = predictiveModel
        self.batch, self.device = int(batch), device
        self.tree_index = TreeIndex(self.N, self.NB, self.m)
        self.totalx, self.totalu = self.tree_index.T, self.tree_index.U
        self.branchdim = self.tree_index.bdim
        self._bt = None
        self.xPred = self.uPred = self.xLin = self.uLin = None
        self.OldInput = np.zeros(self.d)
        self.feasible = 0
        self.J = None
        self.status = None
        self.iters = None
        zero = datetime.timedelta(0)
        self.solverTime = zero
        self.linearizationTime = zero
        self.timeStep = 0
        self._plan = None
        self._pol_rows = None
        self._last = None

    # ---- plan ------------------------------------------------------------------------------
    def _takes_transform(self):
        """Plans of this controller accept solve's S / Fx / bx (MPC_branch.py:2043-2057): the
        CVaR controller over the highway models (HIGHWAY plans get BMPC_PLAN_TRANSFORM, the
        merge model always has it)."""
        kind = getattr(self.predictiveModel, "model_kind", None)
        return self.controller_kind == abi.CTRL_CVAR and kind in (abi.MODEL_HIGHWAY, abi.MODEL_HIGHWAY_MERGE)

    def plan_desc(self):
        mdl = self.predictiveModel
        Fx = np.asarray(self.Fx, float).reshape(-1, self.n)
        flags = abi.PLAN_TRANSFORM if (self._takes_transform() and mdl.model_kind == abi.MODEL_HIGHWAY) else 0
        return abi.make_desc(self.controller_kind, mdl.model_kind, self.n, self.d, self.N, self.NB, self.m,
                             mdl.dt, self.Q, self.R, Fx, _flat_bx(self.bx), self.Fu,
                             np.asarray(self.bu, float).reshape(-1), self.Qslack, mdl.model_constants(),
                             ralpha=self.ralpha, Qf=self.Qf, dR=self.dR, flags=flags)

    def _ensure_plan(self):
        if self._plan is None:
            from bmpc.plan import BatchPlan
            self._plan = BatchPlan(self.plan_desc(), self.batch, self.device)
        rows = self.predictiveModel.policy_rows()
        lref = getattr(self.predictiveModel, "lane_ref", None)   # psiref policies (merge ramp)
        if lref is not None and lref is not getattr(self, "_lref", None):
            self._plan.set_lane_ref(*lref)
            self._lref = lref
        if rows != self._pol_rows:               # update_backup happened
            self._plan.set_policies([rows] * self.batch)
            self._pol_rows = rows
        return self._plan

    # ---- solve -----------------------------------------------------------------------------
    def _transform(self, pl, S, Fx, bx, B):
        """The S / Fx / bx arguments of solve (MPC_branch.py:2052-2057): S is reset on every
        call, Fx and bx are kept when None.  The state rows they form follow the reference's
        build / update split (bmpc_set_transform, include/bmpc.h)."""
        if not self._takes_transform():
            if S is not None or Fx is not None or bx is not None:
                raise NotImplementedError("solve's S / Fx / bx need the CVaR controller over a highway model")
            return
        if Fx is not None:
            F = np.asarray(Fx, float).reshape(-1, self.n)
            if F.shape[0] != np.asarray(self.param.Fx, float).reshape(-1, self.n).shape[0]:
                raise ValueError("a per-step Fx must keep the row count of mpcParameters.Fx")
            pl.set_fx(np.broadcast_to(F, (B,) + F.shape))
        S_arr = None if S is None else np.broadcast_to(np.asarray(S, float), (B, self.n, self.n))
        bx_arr = None if bx is None else np.broadcast_to(_flat_bx(bx), (B, _flat_bx(bx).size))
        pl.set_transform(S_arr, bx_arr)

    def solve(self, x, z, xRef=None, S=None, Fx=None, bx=None):
        """One controller step (MPC_branch.py:2043-2092), including solve's S (state
        transformation), Fx and bx (state constraints)."""
        if self.batch != 1:
            raise ValueError("this controller holds a batch; use solve_batch")
        if not self._takes_transform() and (S is not None or Fx is not None or bx is not None):
            # checked before any attribute changes: a refused call leaves the controller as it was
            raise NotImplementedError("solve's S / Fx / bx need the CVaR controller over a highway model")
        if xRef is not None:
            self.xRef = xRef
        self.S = S
        if Fx is not None:
            self.Fx = Fx
        if bx is not None:
            self.bx = bx
        pl = self._ensure_plan()
        self._transform(pl, S, Fx, bx, 1)
        t0 = datetime.datetime.now()
        r = pl.solve(np.asarray(x, float)[None], np.asarray(z, float)[None],
                     np.asarray(self.xRef, float)[None])
        self.solverTime = datetime.datetime.now() - t0
        self._unpack(r, 0)
        self.timeStep += 1

    def _unpack(self, r, e):
        self._last = r
        st = int(r["status"][e])
        self.status, self.iters, self.J = st, int(r["iters"][e]), float(r["J"][e])
        self.feasible = 1 if st >= 0 else 0       # ECOS exitFlag >= 0 (MPC_branch.py:2141)
        # the library keeps the previous prediction when a solve is infeasible (:2098)
        self.xPred = r["xpred"][e]
        self.uPred = r["upred"][e]
        self.xLin = self.xPred
        self.uLin = np.vstack((self.uPred, self.uPred[-1]))
        self.OldInput = self.uPred[0, :]
        self._bt = None            # rebuilt from the device tree on first access of .BT
        self._tree = None

    def solve_batch(self, X, Z, XREF, S=None, bx=None, Fx=None):
        """Batched step for all egos of the plan: returns the raw result dict
        (upred [B,U,d], xpred [B,T,n], branch_w, J, status, iters); S [B,n,n], bx [B,nFx],
        Fx [B,nFx,n] (or one for all) as in solve."""
        pl = self._ensure_plan()
        self._transform(pl, S, Fx, bx, self.batch)
        t0 = datetime.datetime.now()
        r = pl.solve(X, Z, XREF)
        self.solverTime = datetime.datetime.now() - t0
        self._last = r
        self.timeStep += 1
        return r

    # ---- scenario tree views ------------------------------------------------------------------
    def _tree_arrays(self, e=0):
        if getattr(self, "_tree", None) is None:
            self._tree = self._plan.tree()
            if self.tree_index.bdim > 0 and self.controller_kind != abi.CTRL_ROBUST:
                self._tree["dp"] = self._plan.branch_dp()
        return {k: v[e] for k, v in self._tree.items()}

    def BT2array(self, e=0):
        """(xtraj, ztraj, utraj, branch_w) over non-root branches, BFS order (:2108-2122)."""
        t = self.tree_index
        a = self._tree_arrays(e)
        xs, zs, us, ws = [], [], [], []
        for b in range(t.nbranch):
            lx, lu = t.ndx[b] + t.length[b] - 1, t.ndu[b] + t.length[b] - 1
            for c in t.children[b]:
                sl = slice(t.ndx[c], t.ndx[c] + t.N)
                su = slice(t.ndu[c], t.ndu[c] + t.N)
                ws.append(a["w"][c])
                xs.append(np.vstack((a["xbar"][lx], a["xbar"][sl])))
                zs.append(np.vstack((a["zbar"][lx], a["zbar"][sl])))
                us.append(np.vstack((a["ubar"][lu], a["ubar"][su])))
        return xs, zs, us, ws

    @property
    def BT(self):
        """The live scenario tree of the last solve (``MPC_branch.py:65-78,2062-2064``):
        built from the device tree on first access after a solve (``None`` before any)."""
        if self._bt is None and self._last is not None and self._plan is not None:
            try:
                self.build_tree()
            except NotImplementedError:
                return None
        return self._bt

    @BT.setter
    def BT(self, tree):
        self._bt = tree

    def build_tree(self, e=0):
        """BranchTree objects of the last solve (the reference's ``self.BT``)."""
        t = self.tree_index
        a = self._tree_arrays(e)
        nodes = []
        for b in range(t.nbranch):
            sl = slice(t.ndx[b], t.ndx[b] + t.length[b])
            su = slice(t.ndu[b], t.ndu[b] + t.length[b])
            br = BranchTree(a["xbar"][sl].copy(), a["zbar"][sl].copy(), a["ubar"][su].copy(), a["w"][b],
                            t.depth[b])
            if not t.is_leaf(b):
                br.p = a["p"][b].copy()
                br.dp = a["dp"][b].copy()      # (m, n), MPC_branch.py:1711,1842
            nodes.append(br)
        for b in range(t.nbranch):
            for c in t.children[b]:
                nodes[b].addchild(nodes[c])
        self._bt = nodes[0]
        return self._bt

    @property
    def Solution(self):
        return self._tree_arrays()["sol"]


class BranchMPCProx(BranchMPC_CVaR):
    """Proximal branch QP (MPC_branch.py:82-488) on MI355X: the OSQP problem of
    buildCost/buildEqConstr/buildIneqConstr solved by the device QP interior point.
    ``feasible`` follows osqp_solve_qp: only status_val == 1 (:482); otherwise the previous
    prediction is kept, and OldInput = uPred[0] either way (:421)."""

    controller_kind = abi.CTRL_PROX

    def __init__(self, mpcParameters, predictiveModel, batch=1, device=0):
        super().__init__(mpcParameters, predictiveModel, ralpha=0.0, batch=batch, device=device)

    def solve(self, x, z, xRef=None):
        """One controller step (MPC_branch.py:384-423)."""
        super().solve(x, z, xRef)

    def _unpack(self, r, e):
        super()._unpack(r, e)
        self.feasible = 1 if self.status == 1 else 0


class BranchMPC(BranchMPCProx):
    """Branch QP -- the active (second) definition, MPC_branch.py:881-1274 -- on MI355X.
    Same tree, constraints, OSQP feasibility rule and OldInput update as BranchMPCProx; the
    cost is buildCost :1063-1110 (dQ = 0.5 Q, no rate couplings)."""

    controller_kind = abi.CTRL_QP


class robustMPC(BranchMPCProx):
    """Robust MPC (MPC_branch.py:1275-1595) on MI355X: one input sequence over a chain of
    Nx = N*NB+2 states / Nu = N*NB+1 inputs that must clear every obstacle prediction of the
    scenario tree, solved by the device QP interior point (controller kind ROBUST).  The
    solution is taken whatever the OSQP status (unpackSolution :1459); the next solve
    linearises about the prediction shifted by one step (:1429-1431); OldInput = uPred[0]."""

    controller_kind = abi.CTRL_ROBUST

    def __init__(self, mpcParameters, predictiveModel, batch=1, device=0):
        super().__init__(mpcParameters, predictiveModel, batch=batch, device=device)
        self.Nx, self.Nu = self.N * self.NB + 2, self.N * self.NB + 1
        self.totalx, self.totalu, self.branchdim = self.Nx, self.Nu, 0
        self.slackdim = None
        self._z = None

    def solve(self, x, z, xRef=None):
        """One controller step (MPC_branch.py:1397-1435)."""
        self._z = np.asarray(z, float).copy()
        super().solve(x, z, xRef)

    def _unpack(self, r, e):
        super()._unpack(r, e)
        self.xLin = np.vstack((self.xPred[1:], self.xPred[-1]))
        self.uLin = np.vstack((self.uPred[1:], self.uPred[-1]))
        self.zt, self.zt_u = self.xPred[-1, :], self.uPred[-1, :]

    def BT2array(self, e=0):
        """([xPred], ztraj, [uPred], []) with ztraj the obstacle branches in BFS order, each
        prefixed by its parent's last prediction (:1385-1396)."""
        n, m = self.n, self.m
        ztraj, q = [], [(0, np.reshape(self._z, (1, n)))]
        while q:
            depth, zt = q.pop(0)
            if depth < self.NB:
                zp = self.predictiveModel.zpred_eval(zt[-1])
                for i in range(m):
                    child = zp[:, n * i:n * (i + 1)]
                    ztraj.append(np.vstack((zt[-1], child)))
                    q.append((depth + 1, child))
        return [self.xPred], ztraj, [self.uPred], []

    def build_tree(self, e=0):
        raise NotImplementedError("robustMPC keeps no branch tree of states (MPC_branch.py:1336)")
