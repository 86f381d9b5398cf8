"""BASELINE config 4 (quadruped BranchMPCProx closed loop, bench.py --workload quadruped):
find the solves whose status is not 1 (OSQP "solved") and re-solve exactly those problems with
the oracle -- the reference's own BranchMPCProx structure restated (oracle/tree.py
ProxController) driven through the same inputs from step 0, with the exact-optimum QP
interior point (oracle/qp_ipm.py) standing in for OSQP.

The kernel's algorithm runs here as the host build (tests/hostsim, the same csrc templates as
libbmpc); pass --gpu to run libbmpc instead.  Output: one JSON line per failing solve
(ego, step, kernel status / iterations, the oracle's status / iterations, and the distance
between the two solutions) and a summary."""
import argparse
import json
import math
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "belief-planning_amd"), os.path.join(REPO, "tests")]

from bmpc.scenarios import quadruped_desc, quadruped_policy_rows, quadruped_xref, seeded_quadruped_batch  # noqa: E402

QDT, QV0 = 0.2, 0.2


def env_step(x, z, u0):
    """bench.py quad_env_step: robot.step of ego and obstacle (forward policy), new reference."""
    c, s = np.cos(x[:, 2]), np.sin(x[:, 2])
    x = x + QDT * np.stack([u0[:, 0] * c - u0[:, 1] * s, u0[:, 1] * c + u0[:, 0] * s, u0[:, 2]], 1)
    z = z + QDT * np.stack([QV0 * np.cos(z[:, 2]), QV0 * np.sin(z[:, 2]), np.zeros(len(z))], 1)
    xr = quadruped_xref(x)
    psi = xr[:, 2] - 2 * math.pi * np.round((xr[:, 2] - 0.0) / (2 * math.pi))
    xr[:, 2] = psi
    return x, z, xr


def oracle_controller():
    from oracle.model import QuadrupedModel, quadruped_policies
    from oracle.qp_ipm import osqp_like_solve
    from oracle.tree import ProxController
    mdl = QuadrupedModel(25, 0.2, quadruped_policies(QV0), L1=0.5, W1=0.3, L2=1.0, W2=0.6, col_tol=0.2, s1=2.0)
    Fu = np.kron(np.eye(3), np.array([1, -1])).T
    bu = np.array([0.2, 0.0, 0.1, 0.1, 0.5, 0.5])
    return ProxController(mdl, 25, 2, np.eye(3), np.diag([1., 100., 1.]), [0.9, 5.0, 1.0], np.zeros((0, 3)), [],
                          Fu, bu, [0., 300.], np.zeros(3), solver=osqp_like_solve)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--egos", type=int, default=1024)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--gpu", action="store_true")
    a = ap.parse_args()
    x, z, xr = seeded_quadruped_batch(a.egos, seed=1)
    desc = quadruped_desc()
    if a.gpu:
        from bmpc import plan
        pl = plan.BatchPlan(desc, a.egos)
    else:
        import hostsim_lib as H
        pl = H.HostSim(desc, a.egos)
    pl.set_policies(quadruped_policy_rows(a.egos))
    hist, fails = [], []
    for t in range(a.steps):
        hist.append((x.copy(), z.copy(), xr.copy()))
        r = pl.solve(x, z, xr)
        for e in np.where(r["status"] != 1)[0]:
            fails.append((int(e), t, int(r["status"][e]), int(r["iters"][e]), r["upred"][e].copy()))
        x, z, xr = env_step(x, z, r["upred"][:, 0])
    out = []
    for e, t, st, it, up in fails:
        c = oracle_controller()
        for s in range(t + 1):
            hx, hz, hr = hist[s]
            c.solve(hx[e], hz[e], hr[e])
        info = c.last_info
        rec = dict(ego=e, step=t, kernel_status=st, kernel_iters=it, oracle_status=int(info["status_val"]),
                   oracle_iters=int(info["iter"]), u0_kernel=up[0].tolist(),
                   u0_oracle=(c.uPred[0].tolist() if c.feasible else None))
        out.append(rec)
        print(json.dumps(rec), flush=True)
    both = sum(1 for o in out if o["oracle_status"] != 1)
    print(json.dumps(dict(summary=True, solves=a.egos * a.steps, kernel_failures=len(fails),
                          oracle_also_fails=both, backend="libbmpc" if a.gpu else "host build")))


if __name__ == "__main__":
    main()
