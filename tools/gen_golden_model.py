"""Golden model vectors produced by the REFERENCE's own model code (run HERE only).

The reference's ``highway_branch_dyn.py``, ``quadruped_branch_dyn.py`` and
``HMM_backup_dyn.py`` are imported from /root/reference unchanged, with CasADi replaced
by ``tools/casadi_shim`` (a CasADi-API stand-in that evaluates the graphs those files
build; SURVEY §8(c) route 2) and the solver packages their siblings import by empty
stubs.  ``HMM_backup_dyn.py:5`` imports ``utils.HMM_constants``, which the reference's
``utils.py`` never defines: the reference's own ``Branch_constants`` (it has every field the
HMM model reads) is attached under that name before the import.

Each model's ``PredictiveModel`` is built with the reference's own backup-policy
functions and evaluated through its public methods (``dyn_linearization``,
``branch_eval``, ``zpred_eval``, ``col_eval``; HMM: ``regressionAndLinearization``) on
seeded points and on the inputs of the commented smoke test at
``quadruped_branch_dyn.py:250-272``.  Outputs: ``tests/golden/model_{highway,quadruped,
hmm,merge,merge_psiref}.npz`` (inputs and outputs only).  Usage:  python tools/gen_golden_model.py
"""
from __future__ import annotations

import os
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
REF = "/root/reference"
OUT = os.path.join(REPO, "tests", "golden")


def import_reference_models():
    """The three reference model modules over the CasADi shim (and solver-package stubs)."""
    sys.path.insert(0, os.path.join(HERE, "casadi_shim"))
    import casadi  # noqa: F401  (the shim)
    cv, cvs = types.ModuleType("cvxopt"), types.ModuleType("cvxopt.solvers")
    cvs.options, cvs.qp = {}, None
    cv.solvers, cv.spmatrix, cv.matrix = cvs, None, None
    sys.modules.setdefault("cvxopt", cv)
    sys.modules.setdefault("cvxopt.solvers", cvs)
    oq = types.ModuleType("osqp")
    oq.OSQP = object
    sys.modules.setdefault("osqp", oq)
    if REF not in sys.path:
        sys.path.insert(1, REF)
    import utils
    if not hasattr(utils, "HMM_constants"):
        utils.HMM_constants = utils.Branch_constants
    import HMM_backup_dyn
    import highway_branch_dyn
    import quadruped_branch_dyn
    for mod in (highway_branch_dyn, quadruped_branch_dyn, HMM_backup_dyn):
        assert os.path.dirname(os.path.abspath(mod.__file__)) == REF, mod.__file__
    return highway_branch_dyn, quadruped_branch_dyn, HMM_backup_dyn, utils


def seeded_highway_points(K, rng):
    lanes = np.array([1.8, 5.4, 9.0, 12.6])
    x = np.stack([rng.uniform(-5, 5, K), lanes[rng.integers(0, 4, K)] + rng.normal(0, 0.3, K),
                  rng.uniform(12, 26, K), rng.normal(0, 0.05, K)], 1)
    z = np.stack([x[:, 0] + rng.uniform(-12, 30, K), lanes[rng.integers(0, 4, K)], rng.uniform(12, 26, K),
                  rng.normal(0, 0.03, K)], 1)
    u = np.stack([rng.uniform(-6, 6, K), rng.uniform(-0.3, 0.3, K)], 1)
    # edge cases: the sim_overtake start, coincident positions (|.|' = sign(0) = 0), a
    # near-collision, a stopped obstacle
    x[0], z[0], u[0] = [0, 1.8, 20, 0], [5, 5.4, 20, 0], [0, 0]
    x[1], z[1] = [3.0, 5.4, 18, 0.01], [3.0, 5.4, 22, 0.0]
    x[2], z[2] = [0.5, 1.9, 20, 0.0], [4.4, 4.5, 15, 0.0]
    z[3, 2] = 0.0
    return x, z, u


def gen_highway(H, utils, rng):
    cons = utils.Branch_constants(s1=2, s2=3, c2=0.5, tran_diag=0.3, alpha=1, R=1.2, am=6.0, rm=0.3, J_c=20, s_c=1,
                                  ylb=0., yub=7.2, L=4, W=2.5, col_alpha=5, Kpsi=0.1)
    out = {}
    cases = [(20, np.array([0.5, 1.8, 15, 0.0]), 24), (8, np.array([0.0, 5.4, 20, 0.0]), 12),
             (10, np.array([0.0, 9.0, 20, 0.0]), 12)]
    for ci, (N, tgt, K) in enumerate(cases):
        model = H.PredictiveModel(4, 2, N, [lambda x: H.backup_maintain(x, cons), lambda x: H.backup_brake(x, cons),
                                            lambda x, t=tgt: H.backup_lc(x, t)], 0.1, cons)
        x, z, u = seeded_highway_points(K, rng)
        rec = {k: [] for k in ("A", "B", "C", "xp", "p", "dp", "zpred", "h0", "dh")}
        for k in range(K):
            A, B, C, xp = model.dyn_linearization(x[k], u[k])
            p, dp = model.branch_eval(x[k], z[k])
            zp = model.zpred_eval(z[k])
            h0, dh = model.col_eval(x[k], z[k])
            for key, v in zip(rec, (A, B, C, xp, p, dp, zp, h0, dh)):
                rec[key].append(np.asarray(v, float))
        pre = f"c{ci}_"
        out[pre + "N"], out[pre + "lc_target"] = N, tgt
        out[pre + "x"], out[pre + "z"], out[pre + "u"] = x, z, u
        for key, v in rec.items():
            out[pre + key] = np.array(v)
    out["ncases"] = len(cases)
    out["dt"], out["L"], out["W"], out["s1"], out["Kpsi"], out["N_lane"] = 0.1, 4.0, 2.5, 2.0, 0.1, 3
    return out


def gen_merge_model(H, utils, rng):
    """PredictiveModel_merge (highway_branch_dyn.py:400-502) as sim_merge's controller builds it:
    pred_model[0] with [maintain_trackV(v0), brake] and no psiref (main_branch.py:85-88)."""
    cons = utils.Branch_constants(s1=2, s2=3, c2=0.5, tran_diag=0.3, alpha=1, R=1.2, am=7.0, rm=0.3, J_c=20, s_c=1,
                                  ylb=0., yub=7.2, L=4, W=2.5, col_alpha=5, Kpsi=0.1)
    out = {}
    for ci, (N, v0, K) in enumerate([(40, 20.0, 12), (10, 18.0, 8)]):
        grid = np.linspace(0.0, 100.0, 11)
        ref = (H.interpolant('refY', 'linear', [grid], np.linspace(9.0, 5.4, 11)),
               H.interpolant('refpsi', 'linear', [grid], np.full(11, -0.05)))
        model = H.PredictiveModel_merge(4, 2, N, [lambda x, v=v0: H.backup_maintain_trackV(x, cons, v),
                                                  lambda x: H.backup_brake(x, cons)], 0.1, cons, ref, laneID=0,
                                        N_lane1=2, N_lane2=1)
        x, z, u = seeded_highway_points(K, rng)
        rec = {k: [] for k in ("A", "B", "C", "xp", "p", "dp", "zpred", "h0", "dh")}
        for k in range(K):
            A, B, C, xp = model.dyn_linearization(x[k], u[k])
            p, dp = model.branch_eval(x[k], z[k])
            zp = model.zpred_eval(z[k])
            h0, dh = model.col_eval(x[k], z[k])
            for key, v in zip(rec, (A, B, C, xp, p, dp, zp, h0, dh)):
                rec[key].append(np.asarray(v, float))
        pre = f"c{ci}_"
        out[pre + "N"], out[pre + "v0"] = N, v0
        out[pre + "x"], out[pre + "z"], out[pre + "u"] = x, z, u
        for key, v in rec.items():
            out[pre + key] = np.array(v)
    out["ncases"] = 2
    out["dt"], out["L"], out["W"], out["s1"], out["Kpsi"] = 0.1, 4.0, 2.5, 2.0, 0.1
    return out


def merge_reference_geometry():
    """sim_merge's lane reference (main_branch.py:53-79): the reference's own merge_geometry
    (Highway_env_branch.py:227-270) with N_lane 2, merge_lane 1, merge_s 50, merge_R 300."""
    import importlib
    try:
        importlib.import_module("matplotlib")
    except ImportError:   # plotting only; stubbed when absent
        for mod in ("matplotlib", "matplotlib.pyplot", "matplotlib.patches", "matplotlib.animation"):
            sys.modules.setdefault(mod, types.ModuleType(mod))
        for sub in ("pyplot", "patches", "animation"):
            setattr(sys.modules["matplotlib"], sub, sys.modules["matplotlib." + sub])
    import Highway_env_branch as HE
    assert os.path.dirname(os.path.abspath(HE.__file__)) == REF
    X1, X2, Y1, Y2, psi1, psi2 = HE.merge_geometry(2, 1, 50, 300, 0)
    return np.append(X1, X2), np.append(Y1, Y2), np.append(psi1, psi2), HE.v0


def gen_merge_psiref(H, utils, rng):
    """PredictiveModel_merge with the ramp's psiref-tracking backups -- sim_merge's pred_model[1]
    (main_branch.py:82-85): [maintain_trackV(v0, refpsi), brake(refpsi)], refpsi the linear
    interpolant of the ramp heading over the ramp's X grid (highway_branch_dyn.py:54-130,
    400-502).  Points on, before and after the ramp grid and exactly on grid nodes."""
    cons = utils.Branch_constants(s1=2, s2=3, c2=0.5, tran_diag=0.3, alpha=1, R=1.2, am=7.0, rm=0.3, J_c=20, s_c=1,
                                  ylb=0., yub=7.2, L=4, W=2.5, col_alpha=5, Kpsi=0.1)
    gX, gY, gpsi, v0 = merge_reference_geometry()
    refY = H.interpolant('refY', 'linear', [gX], gY)
    refpsi = H.interpolant('refpsi', 'linear', [gX], gpsi)
    out = {"grid": gX, "refY": gY, "refpsi": gpsi, "v0": v0}
    for ci, (N, K) in enumerate([(40, 14), (10, 8)]):
        model = H.PredictiveModel_merge(4, 2, N, [lambda x: H.backup_maintain_trackV(x, cons, v0, refpsi),
                                                  lambda x: H.backup_brake(x, cons, refpsi)], 0.1, cons,
                                        (refY, refpsi), laneID=1, N_lane1=2, N_lane2=1)
        X = rng.uniform(gX[0] - 10, gX[-1] + 10, K)
        X[0], X[1], X[2] = gX[0] - 3.0, gX[-1] + 2.0, gX[len(gX) // 3]   # before / after the grid, on a node
        y = np.interp(X, gX, gY) + rng.normal(0, 0.3, K)
        psi = np.interp(X, gX, gpsi) + rng.normal(0, 0.02, K)
        x = np.stack([X, y, rng.uniform(12, 24, K), psi], 1)
        z = np.stack([X + rng.uniform(-15, 25, K), rng.choice([1.8, 5.4], K), rng.uniform(12, 24, K),
                      rng.normal(0, 0.02, K)], 1)
        z[3, 0:2] = x[3, 0:2]        # coincident positions: sign(0) = 0
        u = np.stack([rng.uniform(-6, 6, K), rng.uniform(-0.3, 0.3, K)], 1)
        rec = {k: [] for k in ("A", "B", "C", "xp", "p", "dp", "zpred", "h0", "dh")}
        for k in range(K):
            A, B, C, xp = model.dyn_linearization(x[k], u[k])
            p, dp = model.branch_eval(x[k], z[k])
            zp = model.zpred_eval(z[k])
            h0, dh = model.col_eval(x[k], z[k])
            for key, v in zip(rec, (A, B, C, xp, p, dp, zp, h0, dh)):
                rec[key].append(np.asarray(v, float))
        pre = f"c{ci}_"
        out[pre + "N"] = N
        out[pre + "x"], out[pre + "z"], out[pre + "u"] = x, z, u
        for key, v in rec.items():
            out[pre + key] = np.array(v)
    out["ncases"] = 2
    out["dt"], out["L"], out["W"], out["s1"], out["Kpsi"] = 0.1, 4.0, 2.5, 2.0, 0.1
    return out


def gen_quadruped(Q, utils, rng):
    out = {}
    # (N, dt, v0, L1, W1, L2, W2, col_tol, K): main_quadruped.py:15-30, then the smoke test
    # block of quadruped_branch_dyn.py:250-272 (its Quad_constants leaves col_tol at None,
    # which robot_col cannot subtract; the main_quadruped value 0.2 is used)
    cases = [(25, 0.2, 0.2, 0.5, 0.3, 1.0, 0.6, 0.2, 16), (10, 0.05, 1.0, 3.0, 2.0, 2.0, 1.5, 0.2, 6)]
    for ci, (N, dt, v0, L1, W1, L2, W2, tol, K) in enumerate(cases):
        cons = utils.Quad_constants(s1=2, s2=3, c2=0.5, alpha=1, R=1.2, vxm=0.2, vym=0.1, rm=0.5, L1=L1, W1=W1, L2=L2,
                                    W2=W2, col_tol=tol, col_alpha=5)
        model = Q.PredictiveModel(3, 3, N, [lambda x, v=v0: Q.backup_forward(x, v), lambda x: Q.backup_stop(x)],
                                  dt, cons)
        x = np.stack([rng.uniform(-1, 2, K), rng.uniform(0, 3, K), rng.uniform(-np.pi, np.pi, K)], 1)
        r, a = rng.uniform(0.5, 4, K), rng.uniform(-np.pi, np.pi, K)
        z = np.stack([x[:, 0] + r * np.cos(a), x[:, 1] + r * np.sin(a), rng.uniform(-np.pi, np.pi, K)], 1)
        u = np.stack([rng.uniform(-0.2, 0.2, K), rng.uniform(-0.1, 0.1, K), rng.uniform(-0.5, 0.5, K)], 1)
        if ci == 0:
            x[0], z[0] = [0, 1.8, 0], [2.5, 2.5, -np.pi / 2]
        else:   # the smoke-test inputs
            x[0], z[0], u[0] = [1, 1, 0.2], [4, 3, -0.2], [0.5, 0.1, 0.2]
        x[1, 0:2] = z[1, 0:2]          # coincident positions: sign(0) = 0 in the L1 norm
        rec = {k: [] for k in ("A", "B", "C", "xp", "p", "dp", "zpred", "h0", "dh")}
        for k in range(K):
            A, B, C, xp = model.dyn_linearization(x[k], u[k])
            p, dp = model.branch_eval(x[k], z[k])
            zp = model.zpred_eval(z[k])
            h0, dh = model.col_eval(x[k], z[k])
            for key, v in zip(rec, (A, B, C, xp, p, dp, zp, h0, dh)):
                rec[key].append(np.asarray(v, float))
        pre = f"c{ci}_"
        out[pre + "N"], out[pre + "dt"], out[pre + "v0"] = N, dt, v0
        out[pre + "consts"] = np.array([L1, W1, L2, W2, tol, 2.0])
        out[pre + "x"], out[pre + "z"], out[pre + "u"] = x, z, u
        for key, v in rec.items():
            out[pre + key] = np.array(v)
    out["ncases"] = len(cases)
    return out


def gen_hmm(HM, utils, rng):
    out = {}
    cases = [(1, 3, 6), (2, 3, 6), (4, 4, 4), (1, 2, 4)]
    for ci, (M, m, K) in enumerate(cases):
        cons = utils.Branch_constants(s1=2, s2=3, c2=0.5, tran_diag=0.3, alpha=1, R=1.2, am=6.0, rm=0.3, J_c=20,
                                      s_c=1, ylb=0., yub=7.2, L=4, W=2.5, col_alpha=5, Kpsi=0.1)
        # the HMM graph reads only len(backupcons) (calc_xp_expr :238-276)
        model = HM.PredictiveModel(4, 2, M, [lambda x, j=j: HM.backup_maintain(x, cons) for j in range(m)], 0.1, cons)
        nb = 4 + M * m
        recs = {k: [] for k in ("xb", "u", "xbackup", "A", "B", "C", "h0", "Jh")}
        for k in range(K):
            x = np.array([rng.uniform(-3, 3), rng.uniform(0.5, 7), rng.uniform(10, 25), rng.normal(0, 0.05)])
            b = rng.dirichlet(np.ones(m), size=M)                    # M x m beliefs
            xb = np.concatenate([x, b.reshape(-1, order="F")])      # CasADi reshape: column-major
            u = np.array([rng.uniform(-3, 3), rng.uniform(-0.2, 0.2)])
            xbk = np.stack([np.array([x[0] + rng.uniform(-8, 12), rng.uniform(0, 7.2), rng.uniform(10, 25),
                                      rng.normal(0, 0.03)]) for _ in range(M * m)])
            if k == 0:
                xbk[0, 0:2] = x[0:2]                                 # sign(0) = 0 edge
            A, B, C, h0, Jh = model.regressionAndLinearization(xb, xbk, u)
            recs["xb"].append(xb)
            recs["u"].append(u)
            recs["xbackup"].append(xbk)
            recs["A"].append(np.asarray(A, float))
            recs["B"].append(np.asarray(B, float))
            recs["C"].append(np.asarray(C, float).reshape(nb))
            recs["h0"].append(np.stack([np.asarray(h, float).reshape(m) for h in h0]))
            recs["Jh"].append(np.stack([np.asarray(j, float).reshape(m, nb) for j in Jh]))
        pre = f"c{ci}_"
        out[pre + "M"], out[pre + "m"] = M, m
        for key, v in recs.items():
            out[pre + key] = np.array(v)
    out["ncases"] = len(cases)
    out["consts"] = np.array([0.1, 4.0, 2.5, 0.0, 7.2, 5.0, 2.0, 0.3])   # dt L W ylb yub col_alpha s1 tran_diag
    return out


def main():
    H, Q, HM, utils = import_reference_models()
    rng = np.random.default_rng(2024)
    os.makedirs(OUT, exist_ok=True)
    np.savez_compressed(os.path.join(OUT, "model_highway.npz"), **gen_highway(H, utils, rng))
    np.savez_compressed(os.path.join(OUT, "model_quadruped.npz"), **gen_quadruped(Q, utils, rng))
    np.savez_compressed(os.path.join(OUT, "model_hmm.npz"), **gen_hmm(HM, utils, rng))
    np.savez_compressed(os.path.join(OUT, "model_merge.npz"), **gen_merge_model(H, utils, np.random.default_rng(77)))
    np.savez_compressed(os.path.join(OUT, "model_merge_psiref.npz"),
                        **gen_merge_psiref(H, utils, np.random.default_rng(78)))
    print("wrote", [f for f in os.listdir(OUT) if f.startswith("model_")])


if __name__ == "__main__":
    main()
