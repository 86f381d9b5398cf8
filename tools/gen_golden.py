"""Generate golden fixtures from the reference's own controller code (run HERE only).

The reference's ``MPC_branch`` / ``Init_MPC`` / ``utils`` import fine once the three
solver packages they name are replaced by import stubs (SURVEY §8c route 1):

* ``cvxopt`` -- only ``solvers.options`` is touched (``MPC_branch.py:3,15``);
* ``ecos``   -- ``ecos.solve`` is replaced by a recorder that captures the exact
  ``(c, G, h, dims, A, b)`` the reference assembles and answers with the oracle's
  ECOS-algorithm restatement (``oracle/ecos_ipm.py``);
* ``osqp``   -- likewise for ``OSQP.setup/solve`` (quadruped ``BranchMPCProx``).

The predictive model handed to the reference controller is the reference's OWN
``highway_branch_dyn`` / ``quadruped_branch_dyn`` ``PredictiveModel``, built over the CasADi
API stand-in ``tools/casadi_shim`` (CasADi is absent; ``tools/gen_golden_model.py``).  So
the *model values, tree bookkeeping, warm start, linearisation schedule and problem
assembly* in the fixtures are produced by the reference code itself; the solutions come
from the oracle's ECOS-algorithm / QP interior points behind the solver stubs.

Outputs ``tests/golden/*.npz`` (data only, no reference source).  Usage:
    python tools/gen_golden.py [--quick]
"""
from __future__ import annotations

import argparse
import os
import sys
import time
import types

import numpy as np
import scipy.sparse as sp

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
REF = "/root/reference"
sys.path.insert(0, REPO)
sys.path.insert(0, HERE)

from oracle import ecos_ipm, qp_ipm  # noqa: E402
from oracle.env import HighwayOvertake  # noqa: E402
from oracle.model import HighwayModel, QuadrupedModel, highway_policies, quadruped_policies  # noqa: E402
from oracle.tree import ConeProblem, QPProblem  # noqa: E402

CURRENT = {}
REFMOD = {}


def ref_models():
    """The reference's highway / quadruped model modules over the CasADi shim."""
    if not REFMOD:
        from gen_golden_model import import_reference_models
        H, Q, _, _ = import_reference_models()
        REFMOD.update(H=H, Q=Q)
    return REFMOD["H"], REFMOD["Q"]


class RefHighwayModel:
    """The reference's ``highway_branch_dyn.PredictiveModel`` (its own lambdas and graphs)
    behind the oracle env's ``update_backup(policy list)`` call: the lane-change target of
    the oracle's third policy is re-issued as the reference's ``backup_lc`` lambda
    (``Highway_env_branch.py:117-118``)."""

    def __init__(self, N, dt, cons, lc_target):
        self.H, _ = ref_models()
        self.cons = cons
        self.inner = self.H.PredictiveModel(4, 2, N, self._lambdas(lc_target), dt, cons)

    def _lambdas(self, tgt):
        H, cons, t = self.H, self.cons, np.array(tgt, float)
        return [lambda x: H.backup_maintain(x, cons), lambda x: H.backup_brake(x, cons), lambda x: H.backup_lc(x, t)]

    def update_backup(self, policies):
        self.inner.update_backup(self._lambdas(policies[2].params))

    def __getattr__(self, k):
        return getattr(self.inner, k)


def ref_quadruped_model(N, dt, v0, L1, W1, L2, W2, col_tol):
    _, Q = ref_models()
    import utils
    cons = utils.Quad_constants(s1=2, s2=3, c2=0.5, alpha=1, R=1.2, vxm=0.2, vym=0.1, rm=0.5, L1=L1, W1=W1, L2=L2,
                                W2=W2, col_tol=col_tol, col_alpha=5)
    return Q.PredictiveModel(3, 3, N, [lambda x: Q.backup_forward(x, v0), lambda x: Q.backup_stop(x)], dt, cons)


def install_stubs():
    cv = types.ModuleType("cvxopt")
    cvs = types.ModuleType("cvxopt.solvers")
    cvs.options = {}
    cvs.qp = None
    cv.solvers, cv.spmatrix, cv.matrix = cvs, None, None
    sys.modules["cvxopt"], sys.modules["cvxopt.solvers"] = cv, cvs

    ec = types.ModuleType("ecos")

    def ecos_solve(c, G, h, dims, A=None, b=None, **kw):
        mpc = CURRENT["mpc"]
        prob = ConeProblem(np.array(c, float), sp.csc_matrix(G, copy=True), np.array(h, float),
                           {"l": int(dims["l"]), "q": [int(v) for v in dims["q"]]},
                           sp.csc_matrix(A, copy=True), np.array(b, float), ref_cone_boost(mpc))
        x, info = ecos_ipm.ecos_solve(prob)
        CURRENT["captured"] = (prob, x, info, kw)
        return {"x": x, "y": info["y"], "z": info["z"], "s": info["s"],
                "info": {"exitFlag": info["exitFlag"], "iter": info["iter"]}}

    ec.solve = ecos_solve
    sys.modules["ecos"] = ec

    oq = types.ModuleType("osqp")

    class OSQP:
        def setup(self, P, q, A, l, u, **kw):
            self.prob = QPProblem(sp.csc_matrix(P, copy=True), np.array(q, float), sp.csc_matrix(A, copy=True),
                                  np.array(l, float), np.array(u, float),
                                  int(np.sum(~np.isfinite(l))))
            self.kw = kw

        def warm_start(self, **kw):
            pass

        def solve(self):
            x, info = qp_ipm.osqp_like_solve(self.prob)
            CURRENT["captured"] = (self.prob, x, info, self.kw)
            return types.SimpleNamespace(x=x, info=types.SimpleNamespace(status_val=info["status_val"]))

    oq.OSQP = OSQP
    sys.modules["osqp"] = oq
    sys.path.insert(0, REF)


def ref_cone_boost(mpc):
    """Same rule as ``oracle.tree.CVaRController.cone_boost`` on the reference's own tree."""
    out = []
    q = [mpc.BT]
    while q:
        br = q.pop(0)
        if br.depth < mpc.NB:
            for ch in br.children:
                est = 0.0
                for j in range(ch.xtraj.shape[0]):
                    est += ch.xtraj[j] @ mpc.Q @ ch.xtraj[j] + ch.utraj[j] @ mpc.R @ ch.utraj[j]
                out.append(0.5 * np.log(max(1.0, est)))
                q.append(ch)
    u0 = mpc.BT.utraj[0]
    out.append(0.5 * np.log(max(1.0, u0 @ mpc.R @ u0)))
    return out


def coo(M, name, d):
    M = sp.coo_matrix(M)
    d[name + "_data"] = M.data
    d[name + "_row"] = M.row.astype(np.int32)
    d[name + "_col"] = M.col.astype(np.int32)
    d[name + "_shape"] = np.array(M.shape, np.int64)


def bt_arrays(mpc):
    xs, zs, us, ws = mpc.BT2array()[:4]
    return np.array(xs), np.array(zs), np.array(us), np.array(ws)


def gen_highway(name, N, NB, steps, keep, out):
    import Init_MPC
    import MPC_branch
    from utils import Branch_constants

    n, d, dt, am, rm, N_lane = 4, 2, 0.1, 6.0, 0.3, 4
    xRef0 = np.array([0.5, 1.8, 15, 0])
    cons = Branch_constants(s1=2, s2=3, c2=0.5, tran_diag=0.3, alpha=1, R=1.2, am=am, rm=rm, J_c=20,
                            s_c=1, ylb=0., yub=7.2, L=4, W=2.5, col_alpha=5, Kpsi=0.1)
    model = RefHighwayModel(N, dt, cons, xRef0)
    param = Init_MPC.initBranchMPC(n, d, N, NB, xRef0, am, rm, N_lane, cons.W)
    mpc = MPC_branch.BranchMPC_CVaR(param, model, ralpha=0.9)
    CURRENT["mpc"] = mpc
    env = HighwayOvertake(mpc, model, N_lane=N_lane, L=cons.L, W=cons.W, Kpsi=cons.Kpsi,
                          lc_target0=xRef0, dt=dt)
    d_out = dict(N=N, NB=NB, m=3, n=n, d=d, dt=dt, am=am, rm=rm, N_lane=N_lane, ralpha=0.9,
                 L=cons.L, W=cons.W, Kpsi=cons.Kpsi, s1=cons.s1, xRef0=xRef0,
                 Q=param.Q, R=param.R, Fx=param.Fx, bx=np.asarray(param.bx, float).reshape(-1),
                 Fu=param.Fu, bu=np.asarray(param.bu, float).reshape(-1), Qslack=param.Qslack)
    traj = {k: [] for k in ("x", "z", "xRef", "u", "lc_target", "exit", "J", "iters", "collision",
                            "ws_uLin", "ws_p")}
    bdim = sum(3 ** k for k in range(NB))
    t0 = time.time()
    for t in range(steps):
        if not env.collision:
            env.check_collision()
        # warm start the controller carries into this solve (updatetree inputs,
        # MPC_branch.py:1813-1823): uLin and the old p of the non-leaf branches (BFS order)
        if mpc.uLin is None:
            traj["ws_uLin"].append(None)
            traj["ws_p"].append(None)
        else:
            traj["ws_uLin"].append(np.array(mpc.uLin, float).copy())
            traj["ws_p"].append(np.array([np.ravel(b.p) for b in mpc.ndx if b.depth < NB], float))
        r = env.step(t)
        prob, sol, info, kw = CURRENT["captured"]
        assert kw == {"verbose": False}, kw
        for k in ("x", "z", "xRef", "u", "lc_target"):
            traj[k].append(r[k])
        traj["exit"].append(info["exitFlag"])
        traj["J"].append(sol[-1])
        traj["iters"].append(info["iter"])
        traj["collision"].append(env.collision)
        if t in keep:
            p = f"s{t}_"
            coo(prob.G, p + "G", d_out)
            coo(prob.A, p + "A", d_out)
            d_out[p + "c"] = prob.c
            d_out[p + "h"] = prob.h
            d_out[p + "b"] = prob.b
            d_out[p + "dims_l"] = np.array(prob.dims["l"])
            d_out[p + "dims_q"] = np.array(prob.dims["q"])
            d_out[p + "cone_boost"] = np.array(prob.cone_boost)
            d_out[p + "sol"] = sol
            d_out[p + "exit"] = np.array(info["exitFlag"])
            d_out[p + "uPred"] = mpc.uPred
            d_out[p + "xPred"] = mpc.xPred
            xs, zs, us, ws = bt_arrays(mpc)
            d_out[p + "bt_x"], d_out[p + "bt_z"], d_out[p + "bt_u"], d_out[p + "bt_w"] = xs, zs, us, ws
        print(f"[{name}] t={t:3d} exit={info['exitFlag']:3d} it={info['iter']:3d} J={sol[-1]:.6f} "
              f"u0={mpc.uPred[0]} ({time.time() - t0:.0f}s)", flush=True)
    for k in ("ws_uLin", "ws_p"):    # first solve has no warm start (inittree): NaN rows
        shape = next(v.shape for v in traj[k] if v is not None)
        traj[k] = [np.full(shape, np.nan) if v is None else v for v in traj[k]]
    for k, v in traj.items():
        d_out["traj_" + k] = np.array(v)
    d_out["keep"] = np.array(sorted(keep))
    np.savez_compressed(os.path.join(out, f"{name}.npz"), **d_out)


# solve's S / Fx / bx schedule of the transform fixture (MPC_branch.py:2043-2057): S on some
# steps and None on others, a new Fx and a new bx on steps with S off (the reference keeps the
# state rows then: updateIneqConstr :2016-2024) and with S on (:2025-2036)
XF_S1 = np.array([[1.0, 0.0, 0.0, 0.0], [0.0, 1.0, 0.01, 0.0], [0.0, 0.0, 1.0, 0.0], [0.0, 0.0, 0.0, 1.0]])
XF_S2 = np.array([[1.0, 0.0, 0.0, 0.0], [0.0, 0.98, 0.0, 0.0], [0.0, 0.0, 1.0, 0.0], [0.0, 0.0, 0.05, 1.0]])
XF_FX2 = np.diag([1.0, 1.0, 2.0, 2.0]) @ np.array([[0., 1, 0, 0], [0, -1, 0, 0], [0, 0, 0, 1], [0, 0, 0, -1]])


def xform_schedule(t):
    """(S, Fx, bx) passed to solve at step t (None = argument omitted)."""
    S = {1: XF_S1, 6: XF_S2, 8: np.eye(4), 9: XF_S1, 12: XF_S2, 13: XF_S2, 16: np.eye(4)}.get(t)
    Fx = XF_FX2 if t in (5, 14) else None
    bx = {7: [4 * 3.6 - 1.0, -1.0, 0.2, 0.2], 13: [4 * 3.6 - 1.25, -1.25, 0.25, 0.25]}.get(t)
    return S, Fx, bx


class XformProxy:
    """The controller as the overtake env sees it, passing the schedule's S / Fx / bx."""

    def __init__(self, mpc):
        self.mpc, self.t = mpc, 0

    def solve(self, x, z, xRef):
        S, Fx, bx = xform_schedule(self.t)
        self.mpc.solve(x, z, xRef, S=S, Fx=Fx, bx=bx)
        self.t += 1

    def __getattr__(self, k):
        return getattr(self.mpc, k)


def gen_highway_xform(name, N, NB, steps, keep, out):
    """The overtake scene with solve's S / Fx / bx arguments (xform_schedule) and the live
    tree's dp recorded every step: the reference's own BranchMPC_CVaR under its build / update
    rules for the state rows."""
    import Init_MPC
    import MPC_branch
    from utils import Branch_constants

    n, d, dt, am, rm, N_lane = 4, 2, 0.1, 6.0, 0.3, 4
    xRef0 = np.array([0.5, 1.8, 15, 0])
    cons = Branch_constants(s1=2, s2=3, c2=0.5, tran_diag=0.3, alpha=1, R=1.2, am=am, rm=rm, J_c=20,
                            s_c=1, ylb=0., yub=7.2, L=4, W=2.5, col_alpha=5, Kpsi=0.1)
    model = RefHighwayModel(N, dt, cons, xRef0)
    param = Init_MPC.initBranchMPC(n, d, N, NB, xRef0, am, rm, N_lane, cons.W)
    mpc = MPC_branch.BranchMPC_CVaR(param, model, ralpha=0.9)
    CURRENT["mpc"] = mpc
    env = HighwayOvertake(XformProxy(mpc), model, N_lane=N_lane, L=cons.L, W=cons.W, Kpsi=cons.Kpsi,
                          lc_target0=xRef0, dt=dt)
    d_out = dict(N=N, NB=NB, m=3, n=n, d=d, dt=dt, am=am, rm=rm, N_lane=N_lane, ralpha=0.9,
                 L=cons.L, W=cons.W, Kpsi=cons.Kpsi, s1=cons.s1, xRef0=xRef0,
                 Q=param.Q, R=param.R, Fx=param.Fx, bx=np.asarray(param.bx, float).reshape(-1),
                 Fu=param.Fu, bu=np.asarray(param.bu, float).reshape(-1), Qslack=param.Qslack)
    traj = {k: [] for k in ("x", "z", "xRef", "u", "lc_target", "exit", "J", "iters", "S", "S_on", "Fx", "Fx_on",
                            "bx", "bx_on", "dp", "ws_uLin", "ws_p")}
    t0 = time.time()
    for t in range(steps):
        if not env.collision:
            env.check_collision()
        S, Fx, bx = xform_schedule(t)
        # the warm start the controller carries into this solve (as gen_highway records it), so a
        # replay can hand every step the reference's own warm start
        if mpc.uLin is None:
            traj["ws_uLin"].append(None)
            traj["ws_p"].append(None)
        else:
            traj["ws_uLin"].append(np.array(mpc.uLin, float).copy())
            traj["ws_p"].append(np.array([np.ravel(b.p) for b in mpc.ndx if b.depth < NB], float))
        r = env.step(t)
        prob, sol, info, kw = CURRENT["captured"]
        for k in ("x", "z", "xRef", "u", "lc_target"):
            traj[k].append(r[k])
        traj["exit"].append(info["exitFlag"])
        traj["J"].append(sol[-1])
        traj["iters"].append(info["iter"])
        traj["S"].append(np.eye(n) if S is None else np.asarray(S, float))
        traj["S_on"].append(S is not None)
        traj["Fx"].append(np.zeros((4, n)) if Fx is None else np.asarray(Fx, float))
        traj["Fx_on"].append(Fx is not None)
        traj["bx"].append(np.zeros(4) if bx is None else np.asarray(bx, float))
        traj["bx_on"].append(bx is not None)
        traj["dp"].append(np.array([np.asarray(b.dp, float) for b in mpc.ndx if b.depth < NB]))
        if t in keep:
            p = f"s{t}_"
            coo(prob.G, p + "G", d_out)
            coo(prob.A, p + "A", d_out)
            d_out[p + "c"] = prob.c
            d_out[p + "h"] = prob.h
            d_out[p + "b"] = prob.b
            d_out[p + "dims_l"] = np.array(prob.dims["l"])
            d_out[p + "dims_q"] = np.array(prob.dims["q"])
            d_out[p + "cone_boost"] = np.array(prob.cone_boost)
            d_out[p + "sol"] = sol
            d_out[p + "exit"] = np.array(info["exitFlag"])
        print(f"[{name}] t={t:3d} exit={info['exitFlag']:3d} it={info['iter']:3d} J={sol[-1]:.6f} "
              f"u0={mpc.uPred[0]} ({time.time() - t0:.0f}s)", flush=True)
    for k in ("ws_uLin", "ws_p"):    # first solve has no warm start (inittree): NaN rows
        shape = next(v.shape for v in traj[k] if v is not None)
        traj[k] = [np.full(shape, np.nan) if v is None else v for v in traj[k]]
    for k, v in traj.items():
        d_out["traj_" + k] = np.array(v)
    d_out["keep"] = np.array(sorted(keep))
    np.savez_compressed(os.path.join(out, f"{name}.npz"), **d_out)


def gen_highway_qp(name, N, NB, steps, keep, out):
    """main_branch.py's overtake scene with the (commented-out) ``BranchMPC`` controller
    (main_branch.py:46; the active class definition is MPC_branch.py:881)."""
    import Init_MPC
    import MPC_branch
    from utils import Branch_constants

    n, d, dt, am, rm, N_lane = 4, 2, 0.1, 6.0, 0.3, 4
    xRef0 = np.array([0.5, 1.8, 15, 0])
    cons = Branch_constants(s1=2, s2=3, c2=0.5, tran_diag=0.3, alpha=1, R=1.2, am=am, rm=rm, J_c=20,
                            s_c=1, ylb=0., yub=7.2, L=4, W=2.5, col_alpha=5, Kpsi=0.1)
    model = RefHighwayModel(N, dt, cons, xRef0)
    param = Init_MPC.initBranchMPC(n, d, N, NB, xRef0, am, rm, N_lane, cons.W)
    mpc = MPC_branch.BranchMPC(param, model)
    CURRENT["mpc"] = mpc
    env = HighwayOvertake(mpc, model, N_lane=N_lane, L=cons.L, W=cons.W, Kpsi=cons.Kpsi,
                          lc_target0=xRef0, dt=dt)
    d_out = dict(N=N, NB=NB, m=3, n=n, d=d, dt=dt, am=am, rm=rm, N_lane=N_lane,
                 L=cons.L, W=cons.W, Kpsi=cons.Kpsi, s1=cons.s1, xRef0=xRef0,
                 Q=param.Q, R=param.R, dR=param.dR, Fx=param.Fx, bx=np.asarray(param.bx, float).reshape(-1),
                 Fu=param.Fu, bu=np.asarray(param.bu, float).reshape(-1), Qslack=param.Qslack)
    traj = {k: [] for k in ("x", "z", "xRef", "u", "lc_target", "status", "collision", "ws_uLin", "ws_p", "ws_old")}
    for t in range(steps):
        if not env.collision:
            env.check_collision()
        traj["ws_uLin"].append(None if mpc.uLin is None else np.array(mpc.uLin, float).copy())
        traj["ws_p"].append(None if mpc.BT is None else
                            np.array([np.ravel(b.p) for b in mpc.ndx if b.depth < NB], float))
        traj["ws_old"].append(np.array(mpc.OldInput, float).reshape(-1).copy())
        r = env.step(t)
        prob, sol, info, kw = CURRENT["captured"]
        assert kw == {"verbose": False, "polish": True}, kw
        for k in ("x", "z", "xRef", "u", "lc_target"):
            traj[k].append(r[k])
        traj["status"].append(info["status_val"])
        traj["collision"].append(env.collision)
        if t in keep:
            p = f"s{t}_"
            coo(prob.P, p + "P", d_out)
            coo(prob.A, p + "A", d_out)
            d_out[p + "q"], d_out[p + "l"], d_out[p + "u"] = prob.q, prob.l, prob.u
            d_out[p + "sol"] = sol
            d_out[p + "uPred"], d_out[p + "xPred"] = mpc.uPred, mpc.xPred
            xs, zs, us, ws = bt_arrays(mpc)
            d_out[p + "bt_x"], d_out[p + "bt_z"], d_out[p + "bt_u"], d_out[p + "bt_w"] = xs, zs, us, ws
        print(f"[{name}] t={t:3d} status={info['status_val']} it={info['iter']} u0={mpc.uPred[0]}", flush=True)
    for k in ("ws_uLin", "ws_p"):
        shape = next(v.shape for v in traj[k] if v is not None)
        traj[k] = [np.full(shape, np.nan) if v is None else v for v in traj[k]]
    for k, v in traj.items():
        d_out["traj_" + k] = np.array(v)
    d_out["keep"] = np.array(sorted(keep))
    np.savez_compressed(os.path.join(out, f"{name}.npz"), **d_out)


def gen_highway_robust(name, N, NB, steps, keep, out):
    """The overtake scene with ``robustMPC`` (MPC_branch.py:1275-1595): one input sequence
    that must clear every obstacle prediction of the scenario tree."""
    import Init_MPC
    import MPC_branch
    from utils import Branch_constants

    n, d, dt, am, rm, N_lane = 4, 2, 0.1, 6.0, 0.3, 4
    xRef0 = np.array([0.5, 1.8, 15, 0])
    cons = Branch_constants(s1=2, s2=3, c2=0.5, tran_diag=0.3, alpha=1, R=1.2, am=am, rm=rm, J_c=20,
                            s_c=1, ylb=0., yub=7.2, L=4, W=2.5, col_alpha=5, Kpsi=0.1)
    model = RefHighwayModel(N, dt, cons, xRef0)
    param = Init_MPC.initBranchMPC(n, d, N, NB, xRef0, am, rm, N_lane, cons.W)
    mpc = MPC_branch.robustMPC(param, model)
    CURRENT["mpc"] = mpc
    env = HighwayOvertake(mpc, model, N_lane=N_lane, L=cons.L, W=cons.W, Kpsi=cons.Kpsi,
                          lc_target0=xRef0, dt=dt)
    d_out = dict(N=N, NB=NB, m=3, n=n, d=d, dt=dt, am=am, rm=rm, N_lane=N_lane,
                 L=cons.L, W=cons.W, Kpsi=cons.Kpsi, s1=cons.s1, xRef0=xRef0,
                 Q=param.Q, Qf=param.Qf, R=param.R, dR=param.dR, Fx=param.Fx,
                 bx=np.asarray(param.bx, float).reshape(-1),
                 Fu=param.Fu, bu=np.asarray(param.bu, float).reshape(-1), Qslack=param.Qslack)
    traj = {k: [] for k in ("x", "z", "xRef", "u", "lc_target", "status", "collision",
                            "ws_xLin", "ws_uLin", "ws_old", "xPred", "uPred")}
    Nx, Nu = N * NB + 2, N * NB + 1
    for t in range(steps):
        if not env.collision:
            env.check_collision()
        # warm start carried into this solve: the shifted previous prediction
        # (MPC_branch.py:1429-1431) and the rate-cost OldInput (:1434)
        first = mpc.BT is None
        traj["ws_xLin"].append(np.full((Nx, n), np.nan) if first else np.array(mpc.xLin, float).copy())
        traj["ws_uLin"].append(np.full((Nu, d), np.nan) if first else np.array(mpc.uLin, float).copy())
        traj["ws_old"].append(np.array(mpc.OldInput, float).reshape(-1).copy())
        r = env.step(t)
        prob, sol, info, kw = CURRENT["captured"]
        assert kw == {"verbose": False, "polish": True}, kw
        for k in ("x", "z", "xRef", "u", "lc_target"):
            traj[k].append(r[k])
        traj["status"].append(info["status_val"])
        traj["collision"].append(env.collision)
        traj["xPred"].append(np.array(mpc.xPred, float))
        traj["uPred"].append(np.array(mpc.uPred, float))
        if t in keep:
            p = f"s{t}_"
            coo(prob.P, p + "P", d_out)
            coo(prob.A, p + "A", d_out)
            d_out[p + "q"], d_out[p + "l"], d_out[p + "u"] = prob.q, prob.l, prob.u
            d_out[p + "sol"] = sol
            d_out[p + "bt_z"] = np.array(mpc.BT2array()[1])
        print(f"[{name}] t={t:3d} status={info['status_val']} it={info['iter']} u0={mpc.uPred[0]}", flush=True)
    for k, v in traj.items():
        d_out["traj_" + k] = np.array(v)
    d_out["keep"] = np.array(sorted(keep))
    np.savez_compressed(os.path.join(out, f"{name}.npz"), **d_out)


def gen_quadruped(name, steps, keep, out):
    import Init_MPC
    import MPC_branch

    n, d, N, NB, dt = 3, 3, 25, 2, 0.2
    vxm, vym, rm, v0 = 0.2, 0.1, 0.5, 0.2
    L1, L2, W1, W2, col_tol = 0.5, 1.0, 0.3, 0.6, 0.2
    xRef = np.array([5., 5., 0.])
    model = ref_quadruped_model(N, dt, v0, L1, W1, L2, W2, col_tol)
    param = Init_MPC.initquadBranchMPC(n, d, N, NB, xRef, vxm, vym, rm)
    mpc = MPC_branch.BranchMPCProx(param, model)
    CURRENT["mpc"] = mpc
    d_out = dict(N=N, NB=NB, m=2, n=n, d=d, dt=dt, vxm=vxm, vym=vym, rm=rm, v0=v0, L1=L1, L2=L2, W1=W1,
                 W2=W2, col_tol=col_tol, Q=param.Q, R=param.R, dR=param.dR,
                 Fu=param.Fu, bu=np.asarray(param.bu, float).reshape(-1), Qslack=param.Qslack, xRef0=xRef)
    # the build's own quadruped loop (quadruped_env.py:67-130 crashes at :120; same rules)
    x_des = np.array([5., -3., 0.])
    ego = np.array([0, 1.8, 0.]); obs = np.array([2.5, 2.5, -np.pi / 2])
    traj = {k: [] for k in ("x", "z", "xRef", "u", "status", "ws_uLin", "ws_p", "ws_old")}
    for t in range(steps):
        dx = x_des[0:2] - ego[0:2]
        dx = dx / np.linalg.norm(dx) * min(np.linalg.norm(dx), 5.0)
        if np.linalg.norm(dx) > 0.1:
            psiRef = np.arctan2(dx[1], dx[0])
            while psiRef - x_des[2] > np.pi:
                psiRef -= 2 * np.pi
            while psiRef - x_des[2] < -np.pi:
                psiRef += 2 * np.pi
        else:
            psiRef = ego[2]
        xr = ego.copy(); xr[0:2] += dx; xr[2] = psiRef
        # warm start carried into this solve (updatetree inputs) and the rate-cost OldInput
        traj["ws_uLin"].append(None if mpc.uLin is None else np.array(mpc.uLin, float).copy())
        traj["ws_p"].append(None if mpc.BT is None else
                            np.array([np.ravel(b.p) for b in mpc.ndx if b.depth < NB], float))
        traj["ws_old"].append(np.array(mpc.OldInput, float).reshape(-1).copy())
        mpc.solve(ego.copy(), obs.copy(), xr)
        prob, sol, info, kw = CURRENT["captured"]
        assert kw == {"verbose": False, "polish": True}, kw
        u = mpc.uPred[0].copy()
        traj["x"].append(ego.copy()); traj["z"].append(obs.copy()); traj["xRef"].append(xr)
        traj["u"].append(u); traj["status"].append(info["status_val"])
        if t in keep:
            p = f"s{t}_"
            coo(prob.P, p + "P", d_out)
            coo(prob.A, p + "A", d_out)
            d_out[p + "q"] = prob.q
            d_out[p + "l"] = prob.l
            d_out[p + "u"] = prob.u
            d_out[p + "sol"] = sol
            d_out[p + "uPred"] = mpc.uPred
            d_out[p + "xPred"] = mpc.xPred
            xs, zs, us, ws = bt_arrays(mpc)
            d_out[p + "bt_x"], d_out[p + "bt_z"], d_out[p + "bt_u"], d_out[p + "bt_w"] = xs, zs, us, ws
        # robot.step (quadruped_env.py:34-37); obstacle: forward policy (v0) as chosen by
        # the env's rule when the L2 clearance of the forward branch exceeds 0.5
        ego = ego + np.array([u[0] * np.cos(ego[2]) - u[1] * np.sin(ego[2]),
                              u[1] * np.cos(ego[2]) + u[0] * np.sin(ego[2]), u[2]]) * dt
        uo = np.array([v0, 0, 0])
        obs = obs + np.array([uo[0] * np.cos(obs[2]) - uo[1] * np.sin(obs[2]),
                              uo[1] * np.cos(obs[2]) + uo[0] * np.sin(obs[2]), uo[2]]) * dt
        print(f"[{name}] t={t} status={info['status_val']} u0={u}", flush=True)
    for k in ("ws_uLin", "ws_p"):
        shape = next(v.shape for v in traj[k] if v is not None)
        traj[k] = [np.full(shape, np.nan) if v is None else v for v in traj[k]]
    for k, v in traj.items():
        d_out["traj_" + k] = np.array(v)
    d_out["keep"] = np.array(sorted(keep))
    np.savez_compressed(os.path.join(out, f"{name}.npz"), **d_out)


def gen_merge(name, steps, keep, out):
    """main_branch.sim_merge (main_branch.py:53-88): the reference's own merge scene --
    PredictiveModel_merge over the CasADi shim (MX graphs with linear interpolants), the
    reference's Highway_env_merge (Highway_env_branch.py:271-390) stepping it, and its
    BranchMPC_CVaR taking the per-step S / bx (the S path of buildIneqConstr /
    updateIneqConstr) with the oracle ECOS-algorithm IPM behind the ecos stub."""
    ref_models()
    import Highway_env_branch as HE
    import highway_branch_dyn as H
    import Init_MPC
    import MPC_branch
    from utils import Branch_constants

    N, n, d, dt, NB, N_lane = 40, 4, 2, 0.1, 1, 2
    xRef = np.array([0.5, 1.8, 15, 0])
    am, rm = 7.0, 0.3
    cons = Branch_constants(s1=2, s2=3, c2=0.5, tran_diag=0.3, alpha=1, R=1.2, am=am, rm=rm, J_c=20, s_c=1,
                            ylb=0., yub=7.2, L=4, W=2.5, col_alpha=5, Kpsi=0.1)
    merge_lane, merge_s, merge_R, merge_side = 1, 50, 300, 0
    X1, X2, Y1, Y2, psi1, psi2 = HE.merge_geometry(N_lane, merge_lane, merge_s, merge_R, merge_side)
    refX, refYv, refpsiv = np.append(X1, X2), np.append(Y1, Y2), np.append(psi1, psi2)
    refY = H.interpolant('refY', 'linear', [refX], refYv)
    refpsi = H.interpolant('refpsi', 'linear', [refX], refpsiv)
    v0 = HE.v0
    bc_merge = [lambda x: H.backup_maintain_trackV(x, cons, v0, refpsi), lambda x: H.backup_brake(x, cons, refpsi)]
    bc_normal = [lambda x: H.backup_maintain_trackV(x, cons, v0), lambda x: H.backup_brake(x, cons)]
    pred_model = [H.PredictiveModel_merge(n, d, N, bc_normal, dt, cons, (refY, refpsi), laneID=0, N_lane1=N_lane,
                                          N_lane2=merge_lane),
                  H.PredictiveModel_merge(n, d, N, bc_merge, dt, cons, (refY, refpsi), laneID=1, N_lane1=N_lane,
                                          N_lane2=merge_lane)]
    param = Init_MPC.initBranchMPC(n, d, N, NB, xRef, am, rm, N_lane, cons.W)
    mpc = MPC_branch.BranchMPC_CVaR(param, pred_model[0], ralpha=0.1)
    CURRENT["mpc"] = mpc
    env = HE.Highway_env_merge(2, N_lane, mpc, pred_model, merge_lane, merge_s, merge_R, merge_side,
                               pred_model[0].dt)
    args = {}
    orig = mpc.solve

    def recording_solve(x, z, xRef=None, S=None, Fx=None, bx=None):
        args.update(x=np.array(x, float), z=np.array(z, float), xRef=np.array(xRef, float),
                    S=np.array(S, float), bx=np.asarray(bx[0] if isinstance(bx, tuple) else bx, float).reshape(-1))
        return orig(x, z, xRef, S, Fx, bx)
    mpc.solve = recording_solve
    d_out = dict(N=N, NB=NB, m=2, n=n, d=d, dt=dt, am=am, rm=rm, N_lane=N_lane, ralpha=0.1, v0=float(v0),
                 L=cons.L, W=cons.W, Kpsi=cons.Kpsi, s1=cons.s1, xRef0=xRef, Q=param.Q, R=param.R, Fx=param.Fx,
                 bx=np.asarray(param.bx, float).reshape(-1), Fu=param.Fu, bu=np.asarray(param.bu, float).reshape(-1),
                 Qslack=param.Qslack, refX=refX, refY=refYv, refpsi=refpsiv)
    traj = {k: [] for k in ("x", "z", "xRef", "S", "bx", "u", "exit", "J", "iters", "laneID", "ws_uLin", "ws_p",
                            "obs_u", "ego_backup")}
    for t in range(steps):
        traj["ws_uLin"].append(None if mpc.uLin is None else np.array(mpc.uLin, float).copy())
        traj["ws_p"].append(None if mpc.BT is None else
                            np.array([np.ravel(b.p) for b in mpc.ndx if b.depth < NB], float))
        u_set, x_set, xx_set, xPred, zPred, branch_w = env.step(t)
        prob, sol, info, kw = CURRENT["captured"]
        for k in ("x", "z", "xRef", "S", "bx"):
            traj[k].append(args[k])
        traj["u"].append(np.array(u_set[0], float))
        traj["obs_u"].append(np.array(u_set[1], float))
        traj["ego_backup"].append(np.array(xx_set[0], float))
        traj["exit"].append(info["exitFlag"])
        traj["J"].append(sol[-1])
        traj["iters"].append(info["iter"])
        traj["laneID"].append(int(env.laneID[0]))
        if t in keep:
            p = f"s{t}_"
            coo(prob.G, p + "G", d_out)
            coo(prob.A, p + "A", d_out)
            d_out[p + "c"], d_out[p + "h"], d_out[p + "b"] = prob.c, prob.h, prob.b
            d_out[p + "dims_l"] = np.array(prob.dims["l"])
            d_out[p + "dims_q"] = np.array(prob.dims["q"])
            d_out[p + "cone_boost"] = np.array(prob.cone_boost)
            d_out[p + "sol"] = sol
            d_out[p + "uPred"], d_out[p + "xPred"] = mpc.uPred, mpc.xPred
        print(f"[{name}] t={t:3d} lane={env.laneID[0]} exit={info['exitFlag']:3d} it={info['iter']:3d} "
              f"J={sol[-1]:.6f} u0={mpc.uPred[0]}", flush=True)
    for k in ("ws_uLin", "ws_p"):
        shape = next(v.shape for v in traj[k] if v is not None)
        traj[k] = [np.full(shape, np.nan) if v is None else v for v in traj[k]]
    for k, v in traj.items():
        d_out["traj_" + k] = np.array(v)
    d_out["keep"] = np.array(sorted(keep))
    np.savez_compressed(os.path.join(out, f"{name}.npz"), **d_out)


def belief_scene_step(x, z, u, true_j, xbackup, m, dt):
    """The recording's scene (not the reference's: Highway_env.py, its only caller, is dead
    code): the ego integrates its input with Highway_env.vehicle.step's Euler rule (:40-42);
    agent i moves to the first state of its backup rollout under its true policy."""
    x = x + dt * np.array([x[2] * np.cos(x[3]), x[2] * np.sin(x[3]), u[0], u[1]])
    z = [xbackup[m * i + true_j[i], 0:4].copy() for i in range(len(z))]
    return x, z


def belief_next(xpred1, nx, M, m):
    """Next beliefs: the MPC's own one-step belief prediction, read row-major as it reads
    them (:208), clipped at 0 and renormalised per agent."""
    b = np.maximum(np.reshape(np.asarray(xpred1[nx:], float), (M, m)), 0.0) + 1e-9
    return b / b.sum(axis=1, keepdims=True)


def gen_belief(name, M, m, N, z0, true_j, steps, keep, out):
    """PredictiveControllers.MPC (:56-340), the reference's own class over the reference's
    own HMM model (HMM_backup_dyn.py over the CasADi shim, its backup_maintain / backup_brake
    and a constant -2 m/s^2 brake as the third policy), parameters from the reference's
    Init_MPC.initMPCParams (:7-34).  get_xLin :121 raises TypeError as shipped; the recording
    subclass replaces only that line's np.reshape(b0, -1, 1) by np.reshape(b0, -1).  OSQP is
    the oracle QP interior point behind the stub (install_stubs)."""
    from gen_golden_model import import_reference_models
    _, _, HM, utils = import_reference_models()
    import Init_MPC
    import PredictiveControllers as RPC
    assert os.path.dirname(os.path.abspath(RPC.__file__)) == REF

    class FixedMPC(RPC.MPC):
        def get_xLin(self, x0, xbackup, b0):
            if self.uLin is None:
                self.uLin = np.zeros([self.N, self.d])
            self.uLin = np.vstack((self.uLin, self.uLin[-1]))
            self.xLin = np.zeros([self.N + 1, self.n])
            xb = np.append(x0, np.reshape(b0, -1))
            self.xLin[0] = xb
            for i in range(0, self.N):
                A, B, C, h0, Jh = self.predictiveModel.regressionAndLinearization(
                    xb, xbackup[:, i * self.nx:(i + 1) * self.nx], self.uLin[i])
                xbp = C + A.dot(xb) + B.dot(self.uLin[i])
                self.xLin[i + 1] = xbp
                xb = xbp

    cons = utils.Branch_constants(s1=2, s2=3, c2=0.5, tran_diag=0.3, alpha=1, R=1.2, am=6.0, rm=0.3, J_c=20, s_c=1,
                                  ylb=0., yub=7.2, L=4, W=2.5, col_alpha=5, Kpsi=0.1)
    pols = [lambda x: HM.backup_maintain(x, cons), lambda x: HM.backup_brake(x, cons),
            lambda x: np.array([-2.0, -cons.Kpsi * x[3]])][:m]
    dt, nx, N_lane, ydes, vdes = 0.1, 4, 2, 1.8, 15.0
    model = HM.PredictiveModel(nx, 2, M, pols, dt, cons)
    param = Init_MPC.initMPCParams(nx, 2, N, M, m, ydes, vdes, cons.am, cons.rm, N_lane, cons.W)
    mpc = FixedMPC(param, model)
    x = np.array([0.0, 1.8, 15.0, 0.0])
    z = [np.array(v, float) for v in z0]
    b = np.ones([M, m]) / m
    xRef = np.array([0.0, ydes, vdes, 0.0])
    d_out = dict(M=M, m=m, N=N, nx=nx, dt=dt, N_lane=N_lane, ydes=ydes, vdes=vdes, am=cons.am, rm=cons.rm,
                 W=cons.W, true_j=np.array(true_j), hc=np.array([dt, cons.L, cons.W, cons.ylb, cons.yub,
                                                                 cons.col_alpha, cons.s1, cons.tran_diag]))
    traj = {k: [] for k in ("x", "z", "b", "xbackup", "uLin_in", "old_in", "u", "status", "sol", "slackdim")}
    for t in range(steps):
        xbackup = np.array(model.generate_backup_traj(np.array(z), N), float)
        traj["uLin_in"].append(np.full((N + 1, 2), np.nan) if mpc.uLin is None else
                               np.vstack((mpc.uLin, np.full((N + 1 - len(mpc.uLin), 2), np.nan))))
        traj["old_in"].append(np.asarray(mpc.OldInput, float).reshape(-1))
        for k, v in (("x", x), ("z", np.array(z)), ("b", b), ("xbackup", xbackup)):
            traj[k].append(np.array(v, float))
        mpc.solve(x, b, xbackup, xRef)
        prob, sol, info, kw = CURRENT["captured"]
        traj["u"].append(np.array(mpc.uPred[0], float))
        traj["status"].append(info["status_val"])
        traj["sol"].append(np.array(sol, float))
        traj["slackdim"].append(mpc.slackdim)
        if t in keep:
            p = f"s{t}_"
            coo(prob.P, p + "P", d_out)
            coo(prob.A, p + "A", d_out)
            d_out[p + "q"], d_out[p + "l"], d_out[p + "u"] = prob.q, prob.l, prob.u
            d_out[p + "xLin"] = np.array(mpc.xPred, float)   # (kept for the record)
            d_out[p + "uPred"] = np.array(mpc.uPred, float)
        print(f"[{name}] t={t:3d} status={info['status_val']} it={info['iter']:3d} rows={mpc.slackdim} "
              f"u0={mpc.uPred[0]}", flush=True)
        x, z = belief_scene_step(x, z, mpc.uPred[0], true_j, xbackup, m, dt)
        b = belief_next(mpc.xPred[1], nx, M, m)
    L = max(len(v) for v in traj["sol"])
    traj["sol"] = [np.append(v, np.full(L - len(v), np.nan)) for v in traj["sol"]]
    for k, v in traj.items():
        d_out["traj_" + k] = np.array(v)
    d_out["keep"] = np.array(sorted(keep))
    np.savez_compressed(os.path.join(out, f"{name}.npz"), **d_out)


def gen_belief_env(name, M, m, N, T, seed, N_lane, out):
    """Highway_env.sim's scene (Highway_env.py:48-382), the reference's own env driving the
    reference's PredictiveControllers.MPC (:121 fixed as in gen_belief) over its HMM model,
    the backup-CBF QPs of the other vehicles through the osqp stub (oracle QP, general
    bounds), random and np.random seeded with ``seed`` before the env is built.  matplotlib
    (plotting only) is stubbed when absent."""
    from gen_golden_model import import_reference_models
    _, _, HM, utils = import_reference_models()
    import importlib
    try:
        importlib.import_module("matplotlib")
    except ImportError:
        for mod in ("matplotlib", "matplotlib.pyplot", "matplotlib.patches", "matplotlib.animation"):
            sys.modules.setdefault(mod, types.ModuleType(mod))
        sys.modules["matplotlib"].pyplot = sys.modules["matplotlib.pyplot"]
        sys.modules["matplotlib"].patches = sys.modules["matplotlib.patches"]
        sys.modules["matplotlib"].animation = sys.modules["matplotlib.animation"]
    import random
    import Highway_env as RHE
    import Init_MPC
    import PredictiveControllers as RPC
    assert os.path.dirname(os.path.abspath(RHE.__file__)) == REF

    class FixedMPC(RPC.MPC):
        def get_xLin(self, x0, xbackup, b0):
            if self.uLin is None:
                self.uLin = np.zeros([self.N, self.d])
            self.uLin = np.vstack((self.uLin, self.uLin[-1]))
            self.xLin = np.zeros([self.N + 1, self.n])
            xb = np.append(x0, np.reshape(b0, -1))
            self.xLin[0] = xb
            for i in range(0, self.N):
                A, B, C, h0, Jh = self.predictiveModel.regressionAndLinearization(
                    xb, xbackup[:, i * self.nx:(i + 1) * self.nx], self.uLin[i])
                xbp = C + A.dot(xb) + B.dot(self.uLin[i])
                self.xLin[i + 1] = xbp
                xb = xbp

    cons = utils.Branch_constants(s1=2, s2=3, c2=0.5, tran_diag=0.3, alpha=1, R=1.2, am=6.0, rm=0.3, J_c=20, s_c=1,
                                  ylb=0., yub=7.2, L=4, W=2.5, col_alpha=5, Kpsi=0.1)
    pols = [lambda x: HM.backup_maintain(x, cons), lambda x: HM.backup_brake(x, cons),
            lambda x: np.array([-2.0, -cons.Kpsi * x[3]])][:m]
    dt = 0.1
    model = HM.PredictiveModel(4, 2, M, pols, dt, cons)
    param = Init_MPC.initMPCParams(4, 2, N, M, m, 1.8, RHE.v0, cons.am, cons.rm, N_lane, cons.W)
    mpc = FixedMPC(param, model)
    random.seed(seed)
    np.random.seed(seed)
    env = RHE.Highway_env(NV=M + 1, mpc=mpc, N_lane=N_lane)
    init = np.array([v.state for v in env.veh_set])
    lanes0 = np.array([v.laneidx for v in env.veh_set])
    state_rec, input_rec, backup_rec, choice_rec, b_rec, xPred_rec, collision = RHE.Highway_sim(env, T)
    d_out = dict(M=M, m=m, N=N, dt=dt, T=T, seed=seed, N_lane=N_lane, am=cons.am, rm=cons.rm, W=cons.W,
                 init=init, lanes0=lanes0, state_rec=state_rec, input_rec=input_rec,
                 choice_rec=np.array(choice_rec, float), b_rec=np.array(b_rec), xPred_rec=np.array(xPred_rec),
                 collision=int(collision))
    print(f"[{name}] {state_rec.shape[1]} steps, collision={collision}, final states {state_rec[:, -1]}")
    np.savez_compressed(os.path.join(out, f"{name}.npz"), **d_out)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--quick", action="store_true")
    ap.add_argument("--only", default="")
    ap.add_argument("--out", default=os.path.join(REPO, "tests", "golden"))
    a = ap.parse_args()
    install_stubs()
    out = a.out
    os.makedirs(out, exist_ok=True)
    jobs = {
        "highway_n20_nb1": lambda: gen_highway("highway_n20_nb1", 20, 1, 8 if a.quick else 100, {0, 1, 2, 5, 50}, out),
        "highway_n8_nb2": lambda: gen_highway("highway_n8_nb2", 8, 2, 5 if a.quick else 40, {0, 1, 2, 30}, out),
        "highway_n10_nb1": lambda: gen_highway("highway_n10_nb1", 10, 1, 5 if a.quick else 20, {0, 1}, out),
        "highway_n30_nb2": lambda: gen_highway("highway_n30_nb2", 30, 2, 3 if a.quick else 24, {0, 1, 12}, out),
        "highway_xform_n8_nb2": lambda: gen_highway_xform("highway_xform_n8_nb2", 8, 2, 5 if a.quick else 18,
                                                          {0, 1, 2, 5, 6, 7, 8}, out),
        "highway_qp_n8_nb2": lambda: gen_highway_qp("highway_qp_n8_nb2", 8, 2, 5 if a.quick else 30, {0, 1, 2, 15}, out),
        "highway_robust_n20_nb1": lambda: gen_highway_robust("highway_robust_n20_nb1", 20, 1, 5 if a.quick else 30, {0, 1, 2, 15}, out),
        "highway_robust_n8_nb2": lambda: gen_highway_robust("highway_robust_n8_nb2", 8, 2, 5 if a.quick else 20, {0, 1, 10}, out),
        "quadruped_n25_nb2": lambda: gen_quadruped("quadruped_n25_nb2", 3 if a.quick else 40, {0, 1, 2, 20}, out),
        "merge_n40_nb1": lambda: gen_merge("merge_n40_nb1", 4 if a.quick else 60, {0, 1, 2, 30, 45}, out),
        "belief_env_m2": lambda: gen_belief_env("belief_env_m2", 2, 3, 10, 3.0, 7, 3, out),
        "belief_m1": lambda: gen_belief("belief_m1", 1, 3, 10, [[10.0, 1.8, 12.0, 0.0]], [1], 12, {0, 1, 6}, out),
        "belief_m2": lambda: gen_belief("belief_m2", 2, 2, 8, [[12.0, 1.8, 12.0, 0.0], [-6.0, 5.4, 17.0, 0.0]], [1, 0],
                                        10, {0, 4}, out),
    }
    for k, f in jobs.items():
        if a.only and k not in a.only.split(","):
            continue
        f()


if __name__ == "__main__":
    main()
