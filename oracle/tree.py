"""Scenario-tree bookkeeping and problem assembly of the reference controllers (oracle).

Restates, with sparse COO assembly instead of dense ``np.eye``/``block_diag`` + CSC
conversion, what these reference methods hand to their solvers:

* ``BranchTree`` + ``inittree`` / ``updatetree``      -- ``MPC_branch.py:65-78,1678-1747,1811-1858``
* ``BranchMPC_CVaR.buildEqConstr``                     -- ``MPC_branch.py:1752-1804``
* ``BranchMPC_CVaR.buildIneqConstr/updateIneqConstr``  -- ``MPC_branch.py:1869-2036``
* ``BranchMPC_CVaR.solve/unpackSolution/BT2array``     -- ``MPC_branch.py:2043-2122``
* ``BranchMPCProx.buildCost/buildIneqConstr/solve``    -- ``MPC_branch.py:185-487``

The topology (BFS branch order, ``ndx``/``ndu`` offsets, leaf terminal nodes) is
identical to the reference, so the solution vector layout ``sol['x']`` is the same.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field

import numpy as np
import scipy.linalg as sla
import scipy.sparse as sp


# ---------------------------------------------------------------------------------------
# topology
# ---------------------------------------------------------------------------------------
@dataclass
class Topology:
    """BFS scenario tree of ``inittree`` (MPC_branch.py:1678-1747)."""

    N: int
    NB: int
    m: int
    depth: list = field(default_factory=list)      # per branch
    length: list = field(default_factory=list)     # xtraj rows (1 for root, N otherwise)
    parent: list = field(default_factory=list)     # parent branch (-1 root)
    children: list = field(default_factory=list)   # list of child branch ids
    ndx: list = field(default_factory=list)
    ndu: list = field(default_factory=list)
    T: int = 0                                      # totalx
    U: int = 0                                      # totalu
    bdim: int = 0                                   # non-leaf branches

    @classmethod
    def build(cls, N, NB, m):
        t = cls(N, NB, m)
        t.depth, t.length, t.parent, t.children = [0], [1], [-1], [[]]
        t.ndx, t.ndu = [0], [0]
        cx, cu = 1, 1
        q = [0]
        while q:
            b = q.pop(0)
            if t.depth[b] < NB:
                for _ in range(m):
                    c = len(t.depth)
                    t.depth.append(t.depth[b] + 1)
                    t.length.append(N)
                    t.parent.append(b)
                    t.children.append([])
                    t.children[b].append(c)
                    t.ndx.append(cx)
                    t.ndu.append(cu)
                    cx += N + 1 if t.depth[c] == NB else N
                    cu += N
                    q.append(c)
        t.T, t.U = cx, cu
        t.bdim = sum(1 for d in t.depth if d < NB)
        return t

    @property
    def nbranch(self):
        return len(self.depth)

    def is_leaf(self, b):
        return self.depth[b] == self.NB

    def xnode(self, b, j):
        return self.ndx[b] + j

    def unode(self, b, j):
        return self.ndu[b] + j

    def src_of_first(self, b):
        """(branch, position) whose dynmatr links into branch ``b``'s first node."""
        p = self.parent[b]
        return p, self.length[p] - 1


# ---------------------------------------------------------------------------------------
# persistent per-controller tree state
# ---------------------------------------------------------------------------------------
class TreeState:
    """Per-branch trajectories (``BranchTree`` fields) for one ego."""

    def __init__(self, topo: Topology, n, d):
        self.topo = topo
        self.n, self.d = n, d
        nb = topo.nbranch
        self.xtraj = [np.zeros((topo.length[b], n)) for b in range(nb)]
        self.ztraj = [np.zeros((topo.length[b], n)) for b in range(nb)]
        self.utraj = [np.zeros((topo.length[b], d)) for b in range(nb)]
        self.dyn = [[None] * topo.length[b] for b in range(nb)]   # (A, B, C)
        self.w = np.zeros(nb)
        self.p = [None] * nb
        self.dp = [None] * nb

    def warm_shift(self, uLin):
        """Input shift of ``updatetree`` (MPC_branch.py:1813-1823) -- uses the *old* p."""
        t = self.topo
        for b in range(t.nbranch):
            l = t.length[b]
            ndu = t.ndu[b]
            self.utraj[b][0:l - 1] = uLin[ndu + 1:ndu + l]
            if not t.is_leaf(b):
                k = int(np.argmax(self.p[b]))
                self.utraj[b][-1] = uLin[t.ndu[t.children[b][k]]]
            else:
                self.utraj[b][-1] = self.utraj[b][-2]

    def rollout(self, model, x, z):
        """BFS rebuild of trajectories, probabilities and linearisations
        (inittree :1694-1724 and updatetree :1826-1858; identical arithmetic)."""
        t = self.topo
        self.xtraj[0][0] = x
        self.ztraj[0][0] = z
        self.w[0] = 1.0
        A, B, C, _ = model.dyn_linearization(x, self.utraj[0][0])
        self.dyn[0][0] = (A, B, C)
        q = [0]
        while q:
            b = q.pop(0)
            if t.is_leaf(b):
                continue
            zPred = model.zpred_eval(self.ztraj[b][-1])
            p, dp = model.branch_eval(self.xtraj[b][-1], self.ztraj[b][-1])
            self.p[b], self.dp[b] = p, dp
            for i, c in enumerate(t.children[b]):
                self.w[c] = self.w[b] * p[i]
                self.ztraj[c] = zPred[:, self.n * i:self.n * (i + 1)].copy()
                _, _, _, xp = model.dyn_linearization(self.xtraj[b][-1], self.utraj[b][-1])
                self.xtraj[c][0] = xp
                for j in range(t.N):
                    A, B, C, xp = model.dyn_linearization(self.xtraj[c][j], self.utraj[c][j])
                    self.dyn[c][j] = (A, B, C)
                    if j < t.N - 1:
                        self.xtraj[c][j + 1] = xp
                q.append(c)

    def bt2array(self):
        """``BT2array`` (MPC_branch.py:2108-2122)."""
        t = self.topo
        xs, zs, us, ws = [], [], [], []
        q = [0]
        while q:
            b = q.pop(0)
            for c in t.children[b]:
                ws.append(self.w[c])
                zs.append(np.vstack((self.ztraj[b][-1], self.ztraj[c])))
                xs.append(np.vstack((self.xtraj[b][-1], self.xtraj[c])))
                us.append(np.vstack((self.utraj[b][-1], self.utraj[c])))
                q.append(c)
        return xs, zs, us, ws


def _sqrt_psd(M):
    """``cholesky(M).T`` with the ``sqrtm`` fallback (MPC_branch.py:1628-1643)."""
    try:
        return np.linalg.cholesky(M).T
    except np.linalg.LinAlgError:
        return np.real(sla.sqrtm(M))


def _coo(rows, cols, vals, shape):
    return sp.csc_matrix((vals, (rows, cols)), shape=shape)


# ---------------------------------------------------------------------------------------
# problem containers
# ---------------------------------------------------------------------------------------
@dataclass
class ConeProblem:
    """ECOS problem: min c'z s.t. A z = b, G z + s = h, s in K(dims)."""

    c: np.ndarray
    G: sp.csc_matrix
    h: np.ndarray
    dims: dict
    A: sp.csc_matrix
    b: np.ndarray
    cone_boost: list = None


@dataclass
class QPProblem:
    """OSQP problem: min 1/2 z'Pz + q'z s.t. l <= Az <= u."""

    P: sp.csc_matrix
    q: np.ndarray
    A: sp.csc_matrix
    l: np.ndarray
    u: np.ndarray
    n_ineq: int


# ---------------------------------------------------------------------------------------
# BranchMPC_CVaR
# ---------------------------------------------------------------------------------------
class CVaRController:
    """Oracle restatement of ``BranchMPC_CVaR`` (MPC_branch.py:1598-2152)."""

    def __init__(self, model, N, NB, Q, R, Fx, bx, Fu, bu, Qslack, xRef, ralpha, solver=None):
        self.model = model
        self.n, self.d, self.m = model.n, model.d, model.m
        self.N, self.NB = N, NB
        self.Q, self.R = np.asarray(Q, float), np.asarray(R, float)
        self.Fx = np.asarray(Fx, float)
        self.bx = np.asarray(bx, float).reshape(-1)        # the 1-tuple of Init_MPC.py:48-51
        self.Fu = np.asarray(Fu, float)
        self.bu = np.asarray(bu, float).reshape(-1)
        self.Qslack = np.asarray(Qslack, float)
        self.xRef = np.asarray(xRef, float)
        self.ralpha = float(ralpha)
        self.Wx = _sqrt_psd(self.Q)
        self.Wu = _sqrt_psd(self.R)
        self.topo = Topology.build(N, NB, self.m)
        self.tree = None
        self.Jcons = None
        self.uLin = None
        self.xPred = self.uPred = None
        self.OldInput = np.zeros(self.d)
        self.feasible = 0
        self.solver = solver
        self.last_problem = None
        self.last_info = None
        self.Solution = None
        self.S = None            # state transformation of the current solve (merge scene)
        self._first = True
        self._rows = self._brows = None   # state rows / bound in force (None: not built yet)

    # ---- sizes ---------------------------------------------------------------------
    @property
    def Nc(self):
        return self.Fx.shape[0] + 1

    def layout(self):
        t, n, d, m = self.topo, self.n, self.d, self.m
        bd = t.bdim
        oX = 0
        oU = t.T * n
        oR = oU + t.U * d                       # rho | sigma | mu+ | mu-
        oS = oR + bd * (2 * m + 2)
        oJ = oS + t.T * self.Nc
        return dict(X=oX, U=oU, rho=oR, sig=oR + bd, mup=oR + 2 * bd, mum=oR + bd * (2 + m),
                    S=oS, J=oJ, nv=oJ + 1)

    # ---- equality rows (buildEqConstr :1752-1804) --------------------------------------
    def build_eq(self, x):
        t, n, d, m = self.topo, self.n, self.d, self.m
        L = self.layout()
        tr = self.tree
        rows, cols, vals = [], [], []
        rhs = np.zeros(t.T * n + t.bdim)
        for k in range(t.T * n):
            rows.append(k); cols.append(k); vals.append(1.0)
        rhs[0:n] = x

        def link(row_node, b, j):
            A, B, C = tr.dyn[b][j]
            xs, us = t.xnode(b, j), t.unode(b, j)
            for r in range(n):
                for c in range(n):
                    if A[r, c] != 0.0:
                        rows.append(row_node * n + r); cols.append(L['X'] + xs * n + c); vals.append(-A[r, c])
                for c in range(d):
                    if B[r, c] != 0.0:
                        rows.append(row_node * n + r); cols.append(L['U'] + us * d + c); vals.append(-B[r, c])
            rhs[row_node * n:(row_node + 1) * n] = C

        for b in range(t.nbranch):
            for j in range(1, t.length[b]):
                link(t.xnode(b, j), b, j - 1)
            last = t.length[b] - 1
            if not t.is_leaf(b):
                for c in t.children[b]:
                    link(t.ndx[c], b, last)
            else:
                link(t.ndx[b] + t.length[b], b, last)
        bd = t.bdim
        for b in range(bd):
            r = t.T * n + b
            rows += [r, r]; cols += [L['rho'] + b, L['sig'] + b]; vals += [1.0, 1.0]
            for i in range(m):
                rows.append(r); cols.append(L['mum'] + b * m + i); vals.append(-tr.p[b][i] / self.ralpha)
        A = _coo(rows, cols, vals, (t.T * n + bd, L['nv']))
        return A, rhs

    # ---- inequality rows (buildIneqConstr :1869-1990 / updateIneqConstr :1993-2036) -----
    def build_ineq(self):
        t, n, d, m = self.topo, self.n, self.d, self.m
        L = self.layout()
        tr = self.tree
        Nc, nFu = self.Nc, self.Fu.shape[0]
        bd = t.bdim
        rows, cols, vals = [], [], []
        h = []
        r0 = 0
        # Fxtot with slack (-I) ; only nodes i < len(utraj) get rows (terminal rows empty)
        hx = np.zeros(t.T * Nc)
        # with a state transformation S (MPC_branch.py:1894-1901, :2025-2036): Fx S rows, and on
        # updates dh[0] <- sign(dh0) max(0.1, |dh0|) in the row while h keeps the unclipped dh
        FxS, bxr = self._rows, self._brows       # the state rows as built / last updated
        for b in range(t.nbranch):
            for j in range(t.length[b]):
                h0, dh = self.model.col_eval(tr.xtraj[b][j], tr.ztraj[b][j])
                if self.S is not None and not self._first:
                    dh = dh.copy()
                    dh[0] = np.sign(dh[0]) * max(0.1, abs(dh[0]))
                k = t.xnode(b, j)
                blk = np.vstack((-dh, FxS))
                for r in range(Nc):
                    for c in range(n):
                        if blk[r, c] != 0.0:
                            rows.append(k * Nc + r); cols.append(L['X'] + k * n + c); vals.append(blk[r, c])
                hx[k * Nc:(k + 1) * Nc] = np.append(h0, bxr)
        for k in range(t.T * Nc):
            rows.append(k); cols.append(L['S'] + k); vals.append(-1.0)
        h.append(hx)
        r0 = t.T * Nc
        # Futot
        for u in range(t.U):
            for r in range(nFu):
                for c in range(d):
                    if self.Fu[r, c] != 0.0:
                        rows.append(r0 + u * nFu + r); cols.append(L['U'] + u * d + c); vals.append(self.Fu[r, c])
        h.append(np.tile(self.bu, t.U))
        r0 += t.U * nFu
        # Frisk: -rho, -mu+, -mu-
        for b in range(bd):
            rows.append(r0 + b); cols.append(L['rho'] + b); vals.append(-1.0)
        for k in range(2 * bd * m):
            rows.append(r0 + bd + k); cols.append(L['mup'] + k); vals.append(-1.0)
        h.append(np.zeros(bd * (2 * m + 1)))
        r0 += bd * (2 * m + 1)
        # positivity of slacks
        for k in range(t.T * Nc):
            rows.append(r0 + k); cols.append(L['S'] + k); vals.append(-1.0)
        h.append(np.zeros(t.T * Nc))
        r0 += t.T * Nc
        n_lp = r0
        # SOC cones (:1940-1984)
        qdims = []
        xq = self.xRef @ self.Q
        W1 = self.Wx if self.S is None else self.Wx @ self.S      # :1935-1937
        for b in range(bd):
            for i, c in enumerate(t.children[b]):
                nx = nu = t.length[c]
                f1r = r0
                # F1 row (and F3 = -F1)
                f1 = {}
                f1[L['sig'] + b] = 1.0
                f1[L['mup'] + b + i] = f1.get(L['mup'] + b + i, 0.0) + 1.0      # quirk: b+i
                f1[L['mum'] + b + i] = f1.get(L['mum'] + b + i, 0.0) - 1.0
                if not t.is_leaf(c):
                    f1[L['rho'] + c] = 1.0
                for j in range(nx):
                    k = t.xnode(c, j)
                    for cc in range(n):
                        f1[L['X'] + k * n + cc] = -2.0 * xq[cc]
                    for cc in range(Nc):
                        f1[L['S'] + k * Nc + cc] = self.Qslack[1]
                q = 2 + nx * n + nu * d
                for col, v in f1.items():
                    if v != 0.0:
                        rows += [f1r, f1r + q - 1]; cols += [col, col]; vals += [v, -v]
                for j in range(nx):
                    k = t.xnode(c, j)
                    for r in range(n):
                        for cc in range(n):
                            if W1[r, cc] != 0.0:
                                rows.append(f1r + 1 + j * n + r); cols.append(L['X'] + k * n + cc)
                                vals.append(-2.0 * W1[r, cc])
                for j in range(nu):
                    u = t.unode(c, j)
                    for r in range(d):
                        for cc in range(d):
                            if self.Wu[r, cc] != 0.0:
                                rows.append(f1r + 1 + nx * n + j * d + r); cols.append(L['U'] + u * d + cc)
                                vals.append(-2.0 * self.Wu[r, cc])
                hq = np.zeros(q)
                hq[0] = 1.0 - self.Jcons * nx
                hq[-1] = 1.0 + self.Jcons * nx
                h.append(hq)
                qdims.append(q)
                r0 += q
        # root cone: J >= rho_0 + u0'Ru0 + Qs*sum(S_0)
        q = 2 + d
        f1 = {L['J']: -1.0, L['rho'] + 0: 1.0}
        for cc in range(Nc):
            f1[L['S'] + cc] = self.Qslack[1]
        for col, v in f1.items():
            rows += [r0, r0 + q - 1]; cols += [col, col]; vals += [v, -v]
        for r in range(d):
            for cc in range(d):
                if self.Wu[r, cc] != 0.0:
                    rows.append(r0 + 1 + r); cols.append(L['U'] + cc); vals.append(-2.0 * self.Wu[r, cc])
        hq = np.zeros(q)
        hq[0] = 1.0
        hq[-1] = 1.0
        h.append(hq)
        qdims.append(q)
        r0 += q
        G = _coo(rows, cols, vals, (r0, L['nv']))
        return G, np.concatenate(h), {'l': n_lp, 'q': qdims}

    # ---- solve (:2043-2092) ------------------------------------------------------------
    def setup_problem(self, x, z, xRef=None, S=None, bx=None, Fx=None):
        """``solve`` (:2043-2057): xRef, Fx and bx kept when None, S reset every solve.  The
        state rows (Fx S | bx) are written by buildIneqConstr on the first solve (:1894-1901)
        and by updateIneqConstr only when S is not None (:2025-2036); with S None a later solve
        keeps the rows it finds (:2016-2024 patch the collision row alone)."""
        x = np.asarray(x, float)
        z = np.asarray(z, float)
        if xRef is not None:
            self.xRef = np.asarray(xRef, float)
        self.S = None if S is None else np.asarray(S, float)
        if Fx is not None:
            self.Fx = np.asarray(Fx, float).reshape(-1, self.n)
        if bx is not None:
            self.bx = np.asarray(bx, float).reshape(-1)
        first = self.tree is None
        self._first = first
        if first or self.S is not None or self._rows is None:   # (a resumed controller builds them)
            self._rows = self.Fx if self.S is None else self.Fx @ self.S
            self._brows = self.bx.copy()
        if first:
            self.tree = TreeState(self.topo, self.n, self.d)
            self.Jcons = float(self.xRef @ self.Q @ self.xRef)
        else:
            self.tree.warm_shift(self.uLin)
        self.tree.rollout(self.model, x, z)
        G, h, dims = self.build_ineq()
        A, b = self.build_eq(x)
        c = np.zeros(self.layout()['nv'])
        c[-1] = 1.0
        self.last_problem = ConeProblem(c, G, h, dims, A, b, self.cone_boost())
        return self.last_problem

    def cone_boost(self):
        """Per-cone Lorentz boost used inside the IPM (see ``ecos_ipm.boost_rows``):
        beta = 1/2 log(max(1, c)) with c = sum_j xbar'Q xbar + ubar'R ubar over the cone's
        branch on the linearisation trajectory, i.e. ~|a| of the rotated cone rows."""
        t, tr = self.topo, self.tree
        out = []
        for b in range(t.bdim):
            for c in t.children[b]:
                est = 0.0
                for j in range(t.length[c]):
                    xb, ub = tr.xtraj[c][j], tr.utraj[c][j]
                    est += xb @ self.Q @ xb + ub @ self.R @ ub
                out.append(0.5 * math.log(max(1.0, est)))
        ub = tr.utraj[0][0]
        out.append(0.5 * math.log(max(1.0, ub @ self.R @ ub)))
        return out

    def solve(self, x, z, xRef=None, S=None, bx=None, Fx=None):
        prob = self.setup_problem(x, z, xRef, S, bx, Fx)
        sol, info = self.solver(prob)
        self.last_info = info
        self.accept(sol, info['exitFlag'])

    def accept(self, sol, exit_flag):
        """``ecos_solve_socp`` feasibility rule + ``unpackSolution`` (:2096-2106,:2141)."""
        t, n, d = self.topo, self.n, self.d
        self.feasible = 1 if exit_flag >= 0 else 0
        self.Solution = sol
        if self.feasible:
            self.xPred = sol[:t.T * n].reshape(t.T, n).copy()
            self.uPred = sol[t.T * n:t.T * n + t.U * d].reshape(t.U, d).copy()
            self.uLin = np.vstack((self.uPred, self.uPred[-1]))
        self.OldInput = self.uPred[0, :].copy()

    def BT2array(self):
        return self.tree.bt2array()


# ---------------------------------------------------------------------------------------
# BranchMPCProx (quadruped)
# ---------------------------------------------------------------------------------------
class ProxController:
    """Oracle restatement of ``BranchMPCProx`` (MPC_branch.py:82-487)."""

    def __init__(self, model, N, NB, Q, R, dR, Fx, bx, Fu, bu, Qslack, xRef, Qf=None, solver=None):
        self.model = model
        self.n, self.d, self.m = model.n, model.d, model.m
        self.N, self.NB = N, NB
        self.Q, self.R = np.asarray(Q, float), np.asarray(R, float)
        self.Qf = self.Q if Qf is None else np.asarray(Qf, float)
        self.dR = np.asarray(dR, float)
        self.Fx = np.asarray(Fx, float).reshape(-1, self.n)
        self.bx = np.asarray(bx, float).reshape(-1)
        self.Fu = np.asarray(Fu, float)
        self.bu = np.asarray(bu, float).reshape(-1)
        self.Qslack = np.asarray(Qslack, float)
        self.xRef = np.asarray(xRef, float)
        self.topo = Topology.build(N, NB, self.m)
        self.tree = None
        self.uLin = None
        self.xPred = self.uPred = None
        self.OldInput = np.zeros(self.d)
        self.feasible = 0
        self.solver = solver
        self.last_problem = None
        self.Solution = None

    @property
    def Nc(self):
        return self.Fx.shape[0] + 1

    def build_cost(self):
        """``buildCost`` (:265-325), quirks kept: dR broadcast rows (:312), scalar qu (:311)."""
        t, n, d = self.topo, self.n, self.d
        tr = self.tree
        dQ = 3.0 * self.Q
        dRm = np.diag(self.dR)
        Hx = [np.zeros((n, n)) for _ in range(t.T)]
        Hu = np.zeros((t.U * d, t.U * d))
        qx = np.zeros(t.T * n)
        xq = self.xRef @ self.Q

        def ublk(a, b):
            return (slice(a * d, (a + 1) * d), slice(b * d, (b + 1) * d))

        for b in range(t.nbranch):
            w = tr.w[b]
            ndx, ndu, l = t.ndx[b], t.ndu[b], t.length[b]
            for i in range(l - 1):
                Hx[ndx + i] = (dQ + self.Q) * w
                qx[(ndx + i) * n:(ndx + i + 1) * n] = -2 * w * (xq + tr.xtraj[b][i] @ dQ)
                Hu[ublk(ndu + i, ndu + i)] += w * self.R
                Hu[ublk(ndu + i, ndu + i)] += w * dRm
                Hu[ublk(ndu + i, ndu + i + 1)] -= w * dRm
                Hu[ublk(ndu + i + 1, ndu + i)] -= w * dRm
                Hu[ublk(ndu + i + 1, ndu + i + 1)] += w * dRm
            if not t.is_leaf(b):
                Hu[ublk(ndu + l - 1, ndu + l - 1)] += w * (self.R + dRm)
                Hx[ndx + l - 1] = (dQ + self.Q) * w
                childJ = np.zeros(self.m)                    # BranchTree.J is always 0 (:76)
                for j, c in enumerate(t.children[b]):
                    wc = tr.w[c]
                    nc = t.ndu[c]
                    Hu[ublk(ndu + l - 1, nc)] -= wc * dRm
                    Hu[ublk(nc, ndu + l - 1)] -= wc * dRm
                    Hu[ublk(nc, nc)] += wc * dRm
                qx[(ndx + l - 1) * n:(ndx + l) * n] = w * (-2 * xq - 2 * tr.xtraj[b][-1] @ dQ
                                                          + childJ @ tr.dp[b])
            else:
                Hu[ublk(ndu + l - 1, ndu + l - 1)] = w * self.R
                Hx[ndx + l - 1] = (dQ + self.Q) * w
                Hx[ndx + l] = self.Qf * w
                qx[(ndx + l - 1) * n:(ndx + l) * n] = -2 * w * (xq + tr.xtraj[b][l - 1] @ dQ)
                qx[(ndx + l) * n:(ndx + l + 1) * n] = -2 * w * (self.xRef @ self.Qf)
        qu = np.zeros(t.U * d)
        qu[0:d] = -2 * (self.OldInput @ self.dR)           # scalar broadcast (:311)
        Hu[0:d, 0:d] += self.dR                             # row broadcast (:312)
        nS = t.T * self.Nc
        H = sp.block_diag([sp.block_diag(Hx), sp.csc_matrix(Hu),
                           self.Qslack[0] * sp.eye(nS)], format='csc')
        qv = np.concatenate([qx, qu, self.Qslack[1] * self.slackweight])
        return 2.0 * H, qv

    def build_ineq(self):
        t, n, d = self.topo, self.n, self.d
        tr = self.tree
        Nc, nFu = self.Nc, self.Fu.shape[0]
        nX, nU, nS = t.T * n, t.U * d, t.T * Nc
        rows, cols, vals = [], [], []
        bx = np.zeros(nS)
        self.slackweight = np.zeros(nS)
        for b in range(t.nbranch):
            for j in range(t.length[b]):
                h0, dh = self.model.col_eval(tr.xtraj[b][j], tr.ztraj[b][j])
                k = t.xnode(b, j)
                blk = np.vstack((-dh, self.Fx))
                for r in range(Nc):
                    for c in range(n):
                        if blk[r, c] != 0.0:
                            rows.append(k * Nc + r); cols.append(k * n + c); vals.append(blk[r, c])
                bx[k * Nc:(k + 1) * Nc] = np.append(h0, self.bx)
                self.slackweight[k * Nc:(k + 1) * Nc] = tr.w[b]
        for k in range(nS):
            rows.append(k); cols.append(nX + nU + k); vals.append(-1.0)
        r0 = nS
        for u in range(t.U):
            for r in range(nFu):
                for c in range(d):
                    if self.Fu[r, c] != 0.0:
                        rows.append(r0 + u * nFu + r); cols.append(nX + u * d + c); vals.append(self.Fu[r, c])
        r0 += t.U * nFu
        for k in range(nS):
            rows.append(r0 + k); cols.append(nX + nU + k); vals.append(-1.0)
        r0 += nS
        F = _coo(rows, cols, vals, (r0, nX + nU + nS))
        b = np.concatenate([bx, np.tile(self.bu, t.U), np.zeros(nS)])
        return F, b

    def build_eq(self, x):
        t, n, d = self.topo, self.n, self.d
        tr = self.tree
        nX, nU, nS = t.T * n, t.U * d, t.T * self.Nc
        rows, cols, vals = list(range(nX)), list(range(nX)), [1.0] * nX
        rhs = np.zeros(nX)
        rhs[0:n] = x

        def link(row_node, b, j):
            A, B, C = tr.dyn[b][j]
            xs, us = t.xnode(b, j), t.unode(b, j)
            for r in range(n):
                for c in range(n):
                    if A[r, c] != 0.0:
                        rows.append(row_node * n + r); cols.append(xs * n + c); vals.append(-A[r, c])
                for c in range(d):
                    if B[r, c] != 0.0:
                        rows.append(row_node * n + r); cols.append(nX + us * d + c); vals.append(-B[r, c])
            rhs[row_node * n:(row_node + 1) * n] = C

        for b in range(t.nbranch):
            for j in range(1, t.length[b]):
                link(t.xnode(b, j), b, j - 1)
            last = t.length[b] - 1
            if not t.is_leaf(b):
                for c in t.children[b]:
                    link(t.ndx[c], b, last)
            else:
                link(t.ndx[b] + t.length[b], b, last)
        return _coo(rows, cols, vals, (nX, nX + nU + nS)), rhs

    def setup_problem(self, x, z, xRef=None):
        x = np.asarray(x, float)
        z = np.asarray(z, float)
        if xRef is not None:
            self.xRef = np.asarray(xRef, float)
        if self.tree is None:
            self.tree = TreeState(self.topo, self.n, self.d)
        else:
            self.tree.warm_shift(self.uLin)
        self.tree.rollout(self.model, x, z)
        F, bineq = self.build_ineq()
        P, q = self.build_cost()
        G, beq = self.build_eq(x)
        A = sp.vstack([F, G]).tocsc()
        lo = np.concatenate([-np.inf * np.ones(len(bineq)), beq])
        hi = np.concatenate([bineq, beq])
        self.last_problem = QPProblem(P, q, A, lo, hi, len(bineq))
        return self.last_problem

    def solve(self, x, z, xRef=None):
        prob = self.setup_problem(x, z, xRef)
        sol, info = self.solver(prob)
        self.last_info = info
        self.accept(sol, info['status_val'])

    def accept(self, sol, status_val):
        """``osqp_solve_qp`` feasibility rule + ``unpackSolution`` (:435-442,:482)."""
        t, n, d = self.topo, self.n, self.d
        self.feasible = 1 if status_val == 1 else 0
        self.Solution = sol
        if self.feasible:
            self.xPred = sol[:t.T * n].reshape(t.T, n).copy()
            self.uPred = sol[t.T * n:t.T * n + t.U * d].reshape(t.U, d).copy()
            self.uLin = np.vstack((self.uPred, self.uPred[-1]))
        self.OldInput = self.uPred[0, :].copy()

    def BT2array(self):
        return self.tree.bt2array()


class BranchQPController(ProxController):
    """Oracle restatement of ``BranchMPC`` -- the active (second) definition,
    MPC_branch.py:881-1274.  Same tree, constraints and OSQP call as ``BranchMPCProx``; the
    cost differs (``buildCost`` :1063-1110): dQ = 0.5 Q, Hu blocks are *assigned* w R (no
    rate couplings, no dR broadcast), the leaf's last node tracks xRef with Qf and the leaf
    terminal node has no linear term; qu[0:d] = -2 OldInput.dR stays (:1102)."""

    def build_cost(self):
        t, n, d = self.topo, self.n, self.d
        tr = self.tree
        dQ = 0.5 * self.Q
        Hx = [np.zeros((n, n)) for _ in range(t.T)]
        Hu = np.zeros((t.U * d, t.U * d))
        qx = np.zeros(t.T * n)
        xq = self.xRef @ self.Q

        def ublk(a):
            return (slice(a * d, (a + 1) * d), slice(a * d, (a + 1) * d))

        for b in range(t.nbranch):
            w = tr.w[b]
            ndx, ndu, l = t.ndx[b], t.ndu[b], t.length[b]
            for i in range(l - 1):
                Hx[ndx + i] = (dQ + self.Q) * w
                qx[(ndx + i) * n:(ndx + i + 1) * n] = -2 * w * (xq + tr.xtraj[b][i] @ dQ)
                Hu[ublk(ndu + i)] = w * self.R
            Hu[ublk(ndu + l - 1)] = w * self.R
            Hx[ndx + l - 1] = (dQ + self.Q) * w
            if not t.is_leaf(b):
                childJ = np.zeros(self.m)                    # BranchTree.J is always 0 (:76)
                qx[(ndx + l - 1) * n:(ndx + l) * n] = w * (-2 * xq - 2 * tr.xtraj[b][l - 1] @ dQ
                                                          + childJ @ tr.dp[b])
            else:
                Hx[ndx + l] = self.Qf * w
                qx[(ndx + l - 1) * n:(ndx + l) * n] = -2 * w * (self.xRef @ self.Qf + tr.xtraj[b][l - 1] @ dQ)
        qu = np.zeros(t.U * d)
        qu[0:d] = -2 * (self.OldInput @ self.dR)           # scalar broadcast (:1102)
        nS = t.T * self.Nc
        H = sp.block_diag([sp.block_diag(Hx), sp.csc_matrix(Hu),
                           self.Qslack[0] * sp.eye(nS)], format='csc')
        qv = np.concatenate([qx, qu, self.Qslack[1] * self.slackweight])
        return 2.0 * H, qv


# ---------------------------------------------------------------------------------------
# robustMPC
# ---------------------------------------------------------------------------------------
class RobustController:
    """Oracle restatement of ``robustMPC`` (MPC_branch.py:1275-1595).

    One input sequence over a chain of Nx = N*NB + 2 states / Nu = N*NB + 1 inputs must clear
    every obstacle prediction of the scenario tree: at time slot t (0 <= t <= N*NB) there is
    one collision row per prediction of the obstacle at t -- the measured z at t = 0, then
    m**depth rows (BFS order of the branches, ``inittree`` :1336-1360).  Every state row gets
    a slack (``buildIneqConstr`` :1467-1510); the cost is unweighted (``buildCost``
    :1540-1569).  The linearisation trajectory is the previous prediction shifted by one
    step (``solve`` :1429-1431); the first solve rolls out u = 0 from x (``get_xLin`` :1326).
    The branch probabilities the reference computes on an uninitialised root trajectory
    (:1337, :1353) only feed branch weights that nothing reads, so they are not restated."""

    def __init__(self, model, N, NB, Q, R, dR, Fx, bx, Fu, bu, Qslack, xRef, Qf=None, solver=None):
        self.model = model
        self.n, self.d, self.m = model.n, model.d, model.m
        self.N, self.NB = N, NB
        self.Nx, self.Nu = N * NB + 2, N * NB + 1
        self.Q, self.R = np.asarray(Q, float), np.asarray(R, float)
        self.Qf = self.Q if Qf is None else np.asarray(Qf, float)
        self.dR = np.asarray(dR, float)
        self.Fx = np.asarray(Fx, float).reshape(-1, self.n)
        self.bx = np.asarray(bx, float).reshape(-1)
        self.Fu = np.asarray(Fu, float)
        self.bu = np.asarray(bu, float).reshape(-1)
        self.Qslack = np.asarray(Qslack, float)
        self.xRef = np.asarray(xRef, float)
        self.xLin = self.uLin = None
        self.xPred = self.uPred = None
        self.OldInput = np.zeros(self.d)
        self.feasible = 0
        self.solver = solver
        self.last_problem = None
        self.zPred = None
        self.ztraj = None

    def predictions(self, z):
        """Obstacle predictions per time slot (``inittree`` / ``updatetree``) and the BFS
        branch trajectories that ``BT2array`` returns (parent's last z prepended)."""
        n, m, N = self.n, self.m, self.N
        zPred = [np.zeros((0, n)) for _ in range(self.N * self.NB + 1)]
        zPred[0] = np.array([z])
        ztraj = []
        q = [(0, np.reshape(z, (1, n)))]
        while q:
            depth, zt = q.pop(0)
            if depth > 0:
                for i in range(zt.shape[0]):
                    t = (depth - 1) * N + i + 1
                    zPred[t] = np.vstack((zPred[t], zt[i]))
            if depth < self.NB:
                zp = self.model.zpred_eval(zt[-1])
                for i in range(m):
                    child = zp[:, n * i:n * (i + 1)]
                    ztraj.append(np.vstack((zt[-1], child)))
                    q.append((depth + 1, child))
        return zPred, ztraj

    def linearisation(self, x):
        """``get_xLin`` on the first solve, then the carried shifted prediction; the dynamics
        of every input node (``computeLTVdynamics`` :1438-1443)."""
        if self.xLin is None:
            self.uLin = np.vstack((np.zeros((self.Nu, self.d)), np.zeros((1, self.d))))
            self.xLin = np.zeros((self.Nx, self.n))
            self.xLin[0] = x
            for i in range(self.Nx - 1):
                self.xLin[i + 1] = self.model.dyn_linearization(self.xLin[i], self.uLin[i])[3]
        return [self.model.dyn_linearization(self.xLin[i], self.uLin[i])[:3] for i in range(self.Nu)]

    def setup_problem(self, x, z, xRef=None):
        x = np.asarray(x, float)
        z = np.asarray(z, float)
        if xRef is not None:
            self.xRef = np.asarray(xRef, float)
        n, d, Nx, Nu = self.n, self.d, self.Nx, self.Nu
        self.zPred, self.ztraj = self.predictions(z)
        dyn = self.linearisation(x)
        nFx, nFu = self.Fx.shape[0], self.Fu.shape[0]
        # inequalities: [Fx rows of every node | collision rows | Fu rows | -S <= 0]
        colrows = []
        for i, zs in enumerate(self.zPred):
            for j in range(zs.shape[0]):
                h, dh = self.model.col_eval(self.xLin[i], zs[j])
                colrows.append((i, -np.asarray(dh, float), float(h)))
        nS = Nx * nFx + len(colrows)
        nX, nU = Nx * n, Nu * d
        rows, cols, vals = [], [], []
        for k in range(Nx):
            for r in range(nFx):
                for c in range(n):
                    if self.Fx[r, c] != 0.0:
                        rows.append(k * nFx + r); cols.append(k * n + c); vals.append(self.Fx[r, c])
        r0 = Nx * nFx
        for e, (i, a, _) in enumerate(colrows):
            for c in range(n):
                if a[c] != 0.0:
                    rows.append(r0 + e); cols.append(i * n + c); vals.append(a[c])
        for k in range(nS):
            rows.append(k); cols.append(nX + nU + k); vals.append(-1.0)
        r0 = nS
        for u in range(Nu):
            for r in range(nFu):
                for c in range(d):
                    if self.Fu[r, c] != 0.0:
                        rows.append(r0 + u * nFu + r); cols.append(nX + u * d + c); vals.append(self.Fu[r, c])
        r0 += Nu * nFu
        for k in range(nS):
            rows.append(r0 + k); cols.append(nX + nU + k); vals.append(-1.0)
        r0 += nS
        F = _coo(rows, cols, vals, (r0, nX + nU + nS))
        bineq = np.concatenate([np.tile(self.bx, Nx), [h for _, _, h in colrows], np.tile(self.bu, Nu), np.zeros(nS)])
        # equalities: x_0 = x, x_{i+1} - A_i x_i - B_i u_i = C_i
        rows, cols, vals = list(range(nX)), list(range(nX)), [1.0] * nX
        beq = np.zeros(nX)
        beq[:n] = x
        for i, (A, B, C) in enumerate(dyn):
            for r in range(n):
                for c in range(n):
                    if A[r, c] != 0.0:
                        rows.append((i + 1) * n + r); cols.append(i * n + c); vals.append(-A[r, c])
                for c in range(d):
                    if B[r, c] != 0.0:
                        rows.append((i + 1) * n + r); cols.append(nX + i * d + c); vals.append(-B[r, c])
            beq[(i + 1) * n:(i + 2) * n] = C
        G = _coo(rows, cols, vals, (nX, nX + nU + nS))
        # cost: 2 blockdiag(Q .. Q, Qf, Hu, Qs0 I); Hu = R + 2 dR (last block R + dR), -dR couplings
        dRm = np.diag(self.dR)
        Hu = np.zeros((nU, nU))
        for u in range(Nu):
            Hu[u * d:(u + 1) * d, u * d:(u + 1) * d] = self.R + (2 * dRm if u < Nu - 1 else dRm)
            if u + 1 < Nu:
                Hu[(u + 1) * d:(u + 2) * d, u * d:(u + 1) * d] = -dRm
                Hu[u * d:(u + 1) * d, (u + 1) * d:(u + 2) * d] = -dRm
        H = sp.block_diag([sp.block_diag([self.Q] * (Nx - 1) + [self.Qf]), sp.csc_matrix(Hu),
                           self.Qslack[0] * sp.eye(nS)], format='csc')
        qx = np.concatenate([-2 * (self.xRef @ self.Q)] * (Nx - 1) + [-2 * (self.xRef @ self.Qf)])
        qu = np.zeros(nU)
        qu[:d] = -2 * (np.reshape(self.OldInput, -1) * self.dR)
        qv = np.concatenate([qx, qu, self.Qslack[1] * np.ones(nS)])
        A = sp.vstack([F, G]).tocsc()
        lo = np.concatenate([-np.inf * np.ones(len(bineq)), beq])
        hi = np.concatenate([bineq, beq])
        self.last_problem = QPProblem((2.0 * H).tocsc(), qv, A, lo, hi, len(bineq))
        return self.last_problem

    def solve(self, x, z, xRef=None):
        prob = self.setup_problem(x, z, xRef)
        sol, info = self.solver(prob)
        self.last_info = info
        self.accept(sol, info['status_val'])

    def accept(self, sol, status_val):
        """``osqp_solve_qp`` (:1591-1595), ``unpackSolution`` (:1459-1465) -- the solution is
        taken whatever the status -- then the time-varying shift (:1429-1434)."""
        n, d = self.n, self.d
        self.feasible = 1 if status_val == 1 else 0
        self.Solution = sol
        self.xPred = sol[:self.Nx * n].reshape(self.Nx, n).copy()
        self.uPred = sol[self.Nx * n:self.Nx * n + self.Nu * d].reshape(self.Nu, d).copy()
        self.xLin = np.vstack((self.xPred[1:], self.xPred[-1]))
        self.uLin = np.vstack((self.uPred[1:], self.uPred[-1]))
        self.OldInput = self.uPred[0, :].copy()

    def BT2array(self):
        return [self.xPred], self.ztraj, [self.uPred], []
