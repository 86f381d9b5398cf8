"""Belief LTV-MPC -- drop-in for the reference's ``PredictiveControllers`` (:1-340).

``MPC`` plans over the belief-augmented state xb = [x; b] (n = nx + M*m) of the HMM model
(``HMM_backup_dyn.PredictiveModel``).  Each ``solve`` (reference :130-163):

1. rolls the belief model out along the last input plan (``get_xLin``, :116-128) and
   linearises it at every stage (``computeLTVdynamics``, :166-171) -- both on the GPU
   (``bmpc_hmm_eval``, csrc/bmpc_hmm.h), the N stage linearisations in one batched launch;
2. assembles the condensed-free QP on the host exactly as the reference does
   (``buildIneqConstr`` :195-249, ``buildCost`` :279-308, ``buildEqConstr`` :251-277):
   state box rows, collision rows -Jh xb <= h0 only where the belief exceeds 0.1, input
   box rows, slacks on every state row, the dR rate coupling;
3. solves it on the GPU with ``bmpc_qp_solve`` (csrc/bmpc_bandqp.h: interior point on the
   band-ordered KKT matrix) in place of a fresh ``OSQP().setup(..., polish=True)`` (:320-340).

Reference behaviour kept, and documented where it is a defect:

* ``get_xLin`` :121 calls ``np.reshape(b0, -1, 1)``, which raises TypeError on every call --
  the belief path is unreachable as shipped.  The evident intent, flattening
  b0, is implemented: ``np.reshape(b0, -1)``.
* b is flattened ROW-major here (:121, :146) and reshaped row-major at :208, while the HMM
  model packs it COLUMN-major (``HMM_backup_dyn.py:244``).  For M = 1 the two agree; for
  M > 1 the model reads agent/backup transposed.  Kept as the reference has it.
* ``computeLTVdynamics`` linearises stage i at (xLin[i+1], uLin[i+1]) with the backups of
  stage i (:170) -- one stage ahead of the stage it constrains.  Kept.
* With ``timeVarying`` False, ``uLin`` grows by one row per solve (:119, :193).  Kept.

Parity: the assembly is pinned to the reference's own class run over the reference's own
HMM model (tests/golden/belief_*.npz, tools/gen_golden.py); OSQP itself is absent, so the
solution is pinned to the exact QP optimum (oracle/qp_ipm.py), not to OSQP's ADMM iterate.
"""
from __future__ import annotations

import datetime

import numpy as np
from scipy import linalg, sparse

from utils import MPCParams, PythonMsg  # noqa: F401  (the reference defines both here)

__all__ = ["MPC", "MPCParams", "PythonMsg"]


class MPC:
    """Belief LTV-MPC (PredictiveControllers.py:56-340); same constructor and attributes."""

    def __init__(self, mpcParameters, predictiveModel):
        p = mpcParameters
        self.N, self.Qslack, self.Q, self.Qf, self.R, self.dR = p.N, p.Qslack, p.Q, p.Qf, p.R, p.dR
        self.n, self.d, self.A, self.B = p.n, p.d, p.A, p.B
        self.Fx, self.Fu, self.bx, self.bu, self.xRef = p.Fx, p.Fu, p.bx, p.bu, p.xRef
        self.M, self.m = predictiveModel.M, predictiveModel.m
        self.nx = self.n - self.M * self.m
        self.h0, self.Jh = [], []
        self.thres = 0.1
        self.alphad = np.exp(-predictiveModel.alpha * predictiveModel.dt)
        self.slacks = p.slacks
        self.slackdim = self.Fx.shape[0] * self.N + (self.N - 1) * self.M * self.m
        self.timeVarying = p.timeVarying
        self.predictiveModel = predictiveModel
        self.osqp = None
        self.OldInput = np.zeros((1, 2))
        self.xPred = None
        self.uLin = None
        self.feasible = 0
        zero = datetime.timedelta(0)
        self.solverTime = zero
        self.linearizationTime = zero
        self.timeStep = 0

    # ---- linearisation (GPU) -------------------------------------------------------------
    def _stage_backups(self, xbackup):
        """xbackup [M*m][N*nx] -> [N][M*m][nx] (the column block of stage i, :125 / :170)."""
        xbk = np.asarray(xbackup, float)
        return xbk[:, :self.N * self.nx].reshape(self.M * self.m, self.N, self.nx).transpose(1, 0, 2)

    def get_xLin(self, x0, xbackup, b0):
        """Roll the belief model along uLin (:116-128; :121's reshape fixed, see module doc)."""
        if self.uLin is None:
            self.uLin = np.zeros([self.N, self.d])
        self.uLin = np.vstack((self.uLin, self.uLin[-1]))
        self.xLin = np.zeros([self.N + 1, self.n])
        xb = np.append(x0, np.reshape(b0, -1))
        self.xLin[0] = xb
        stages = self._stage_backups(xbackup)
        for i in range(self.N):
            A, B, C, _, _ = self.predictiveModel.regressionAndLinearization(xb, stages[i], self.uLin[i])
            xb = C + A.dot(xb) + B.dot(self.uLin[i])
            self.xLin[i + 1] = xb

    def computeLTVdynamics(self, xbackup):
        """(A, B, C, h0, Jh) of every stage at (xLin[i+1], uLin[i+1]) (:166-171), one launch."""
        A, B, C, h0, Jh = self.predictiveModel.regressionAndLinearization(
            self.xLin[1:self.N + 1], self._stage_backups(xbackup), self.uLin[1:self.N + 1])
        self.A, self.B, self.C = list(A), list(B), list(C)
        self.h0, self.Jh = list(h0), list(Jh)

    # ---- QP assembly (host, the reference's matrices) ------------------------------------
    def buildIneqConstr(self):
        """F z <= b (:195-249): state boxes (last state free), belief-gated collision rows,
        input boxes, then the slacks of every state row and their positivity."""
        N, n, M, m = self.N, self.n, self.M, self.m
        Fxtot = np.hstack((linalg.block_diag(*([self.Fx] * N)), np.zeros((self.Fx.shape[0] * N, n))))
        bxtot = np.tile(np.squeeze(self.bx), N)
        rows, rhs = [], []
        for i in range(N - 1):
            b = np.reshape(self.xLin[i + 1][self.nx:], [M, m])     # row-major (:208)
            for j in range(M):
                for k in range(m):
                    if b[j, k] > self.thres:
                        r = np.zeros(n * (N + 1))
                        r[(i + 1) * n:(i + 2) * n] = -np.asarray(self.Jh[i + 1][j][k], float).reshape(-1)
                        rows.append(r)
                        rhs.append(float(np.asarray(self.h0[i + 1][j][k]).reshape(-1)[0]))
        if rows:
            Fxtot = np.vstack((Fxtot, np.array(rows)))
            bxtot = np.append(bxtot, rhs)
        self.slackdim = Fxtot.shape[0]
        Futot = linalg.block_diag(*([self.Fu] * N))
        butot = np.tile(np.squeeze(self.bu), N)
        F_hard = linalg.block_diag(Fxtot, Futot)
        if self.slacks:
            nc = Fxtot.shape[0]
            soft = np.zeros((F_hard.shape[0], nc))
            soft[:nc, :nc] = -np.eye(nc)
            self.F = np.vstack((np.hstack((F_hard, soft)), np.hstack((np.zeros((nc, F_hard.shape[1])), -np.eye(nc)))))
            self.b = np.hstack((bxtot, butot, np.zeros(nc)))
        else:
            self.F = F_hard
            self.b = np.hstack((bxtot, butot))

    def buildEqConstr(self):
        """G z = E x(t) + L (:251-277): x0 pinned, x_{i+1} = A_i x_i + B_i u_i + C_i."""
        N, n, d = self.N, self.n, self.d
        Gx = np.eye(n * (N + 1))
        Gu = np.zeros((n * (N + 1), d * N))
        E = np.zeros((n * (N + 1), n))
        E[:n] = np.eye(n)
        L = np.zeros(n * (N + 1))
        for i in range(N):
            r = slice(n + i * n, 2 * n + i * n)
            Gx[r, i * n:(i + 1) * n] = -(self.A[i] if self.timeVarying else self.A)
            Gu[r, i * d:(i + 1) * d] = -(self.B[i] if self.timeVarying else self.B)
            if self.timeVarying:
                L[r] = self.C[i]
        self.G = np.hstack((Gx, Gu, np.zeros((Gx.shape[0], self.slackdim)))) if self.slacks else np.hstack((Gx, Gu))
        self.E, self.L = E, L

    def buildCost(self):
        """1/2 z'Hz + q'z (:279-308): stage Q, terminal Qf, R + the dR rate coupling (the
        first input against OldInput), quadratic / linear slack weights; H doubled."""
        N, d = self.N, self.d
        Hx = linalg.block_diag(*([self.Q] * N))
        dR = np.asarray(self.dR, float)
        Hu = linalg.block_diag(*([self.R + 2 * np.diag(dR)] * N))
        for i in range(d):
            Hu[i - d, i - d] -= dR[i]               # the last input enters one difference only
        off = -np.tile(dR, N - 1)
        np.fill_diagonal(Hu[d:], off)
        np.fill_diagonal(Hu[:, d:], off)
        q = -2 * np.dot(np.append(np.tile(self.xRef, N + 1), np.zeros(self.R.shape[0] * N)),
                        linalg.block_diag(Hx, self.Qf, Hu))
        q[self.n * (N + 1):self.n * (N + 1) + d] = -2 * np.dot(self.OldInput, np.diag(dR))
        if self.slacks:
            self.H = linalg.block_diag(Hx, self.Qf, Hu, self.Qslack[0] * np.eye(self.slackdim))
            self.q = np.append(q, self.Qslack[1] * np.ones(self.slackdim))
        else:
            self.H = linalg.block_diag(Hx, self.Qf, Hu)
            self.q = q
        self.H = 2 * self.H

    def addTerminalComponents(self, x0):
        """(:173-181) no terminal components: the FTOCP matrices are the built ones."""
        self.H_FTOCP = sparse.csc_matrix(self.H)
        self.q_FTOCP = self.q
        self.F_FTOCP = sparse.csc_matrix(self.F)
        self.b_FTOCP = self.b
        self.G_FTOCP = sparse.csc_matrix(self.G)
        self.E_FTOCP = self.E
        self.L_FTOCP = self.L

    # ---- solve ---------------------------------------------------------------------------
    def osqp_solve_qp(self, P, q, G=None, h=None, A=None, b=None, initvals=None):
        """min 1/2 x'Px + q'x s.t. G x <= h, A x == b (:310-340) on the GPU; feasible iff the
        solver reports solved (OSQP status_val 1).  ``initvals`` is accepted and, as the
        interior point starts from its own point, unused."""
        from bmpc import plan
        Aq = sparse.vstack([G, A]).tocsc()
        lo = np.hstack([-np.inf * np.ones(len(h)), b])
        hi = np.hstack([h, b])
        r = plan.qp_solve(P, q, Aq, lo, hi)
        self.osqp = r
        self.feasible = 1 if int(r["status"][0]) == 1 else 0
        self.Solution = r["x"][0]

    def unpackSolution(self):
        """xPred [N+1][n], uPred [N][d] from the solution (:187-193)."""
        nxs = self.n * (self.N + 1)
        self.xPred = self.Solution[:nxs].reshape(self.N + 1, self.n)
        self.uPred = self.Solution[nxs:nxs + self.d * self.N].reshape(self.N, self.d)
        self.xLin = self.xPred
        self.uLin = np.vstack((self.uPred, self.uPred[-1]))

    def feasibleStateInput(self):
        self.zt = self.xPred[-1, :]
        self.zt_u = self.uPred[-1, :]

    def solve(self, x0, b0, xbackup, xRef=None):
        """One receding-horizon step (:130-163) from ego state x0, beliefs b0 [M][m] and the
        backup rollouts xbackup [M*m][N*nx] (``PredictiveModel.generate_backup_traj``)."""
        if xRef is not None:
            self.xRef = np.append(xRef, np.zeros(self.M * self.m))
        t0 = datetime.datetime.now()
        self.get_xLin(x0, xbackup, b0)
        self.computeLTVdynamics(xbackup)
        self.linearizationTime = datetime.datetime.now() - t0
        self.buildIneqConstr()
        self.buildCost()
        self.buildEqConstr()
        xb0 = np.append(x0, np.reshape(b0, [-1, 1]))
        self.addTerminalComponents(xb0)
        t1 = datetime.datetime.now()
        self.osqp_solve_qp(self.H_FTOCP, self.q_FTOCP, self.F_FTOCP, self.b_FTOCP, self.G_FTOCP,
                           np.add(np.dot(self.E_FTOCP, xb0), self.L_FTOCP))
        self.unpackSolution()
        self.solverTime = datetime.datetime.now() - t1
        self.feasibleStateInput()
        if self.timeVarying:
            self.xLin = np.vstack((self.xPred[1:, :], self.zt))
            self.uLin = np.vstack((self.uPred[1:, :], self.zt_u))
        self.OldInput = self.uPred[0, :]
        self.timeStep += 1
