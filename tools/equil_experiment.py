"""ECOS equilibration on / off in the oracle (oracle/ecos_ipm.py): exit codes, iterations and J of
the first closed-loop solves of seeded egos (SURVEY §8(d) batch, seed 0).  CPU, test tooling.
    python tools/equil_experiment.py EGOS N NB STEPS > profiles/r05/equil_oracle_*.log"""
import os
import sys
import multiprocessing as mp

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "belief-planning_amd")]


def episode(args):
    i, G, N, NB, steps, eq = args
    os.environ["OMP_NUM_THREADS"] = "1"
    from bmpc.scenarios import seeded_batch
    from oracle import ecos_ipm
    from oracle.model import HighwayModel, highway_policies
    from oracle.tree import CVaRController
    x, z, xref, tgt = seeded_batch(G, seed=0)
    x, z, xr = x[i].copy(), z[i].copy(), xref[i].copy()
    solver = lambda p: ecos_ipm.ecos_solve(p, equilibrate=eq)
    c = CVaRController(HighwayModel(N, 0.1, highway_policies(0.1, tgt[i])), N, NB, np.diag([0., 3, 3, 10]),
                       np.diag([1., 100]), np.array([[0., 1, 0, 0], [0, -1, 0, 0], [0, 0, 0, 1], [0, 0, 0, -1]]),
                       [4 * 3.6 - 1.25, -1.25, .25, .25], np.kron(np.eye(2), [1, -1]).T, [6., 6., .3, .3], [0, 300],
                       xr, 0.9, solver=solver)
    out = []
    for k in range(steps):
        c.solve(x, z, xr)
        inf = c.last_info
        out.append((inf["exitFlag"], inf["iter"], inf["x"][-1]))
        u = c.uPred[0]
        x = x + 0.1 * np.array([x[2] * np.cos(x[3]), x[2] * np.sin(x[3]), u[0], u[1]])
        z = z + 0.1 * np.array([z[2] * np.cos(z[3]), z[2] * np.sin(z[3]), 0.0, 0.0])
    return out


def main():
    E, N, NB, steps = (int(v) for v in sys.argv[1:5])
    res = {}
    with mp.get_context("spawn").Pool(8) as pool:
        for eq in (False, True):
            res[eq] = np.array(pool.map(episode, [(i, E, N, NB, steps, eq) for i in range(E)]))   # [E, steps, 3]
    for eq in (False, True):
        r = res[eq]
        ex = r[:, :, 0].astype(int)
        vals, cnt = np.unique(ex, return_counts=True)
        print(f"equilibrate={eq}: exits {dict(zip(vals.tolist(), cnt.tolist()))}  exit-0 share {np.mean(ex == 0):.4f}  "
              f"iters mean {r[:, :, 1].mean():.2f}")
    a, b = res[False], res[True]
    both0 = (a[:, :, 0] == 0) & (b[:, :, 0] == 0)
    dJ = np.abs(a[:, :, 2] - b[:, :, 2]) / np.maximum(1, np.abs(a[:, :, 2]))
    print(f"exit agreement off/on {np.mean(a[:, :, 0] == b[:, :, 0]):.4f}; max rel |dJ| where both exit 0 "
          f"{dJ[both0].max() if both0.any() else float('nan'):.2e}; egos {E}, steps {steps}, N={N} NB={NB}")


if __name__ == "__main__":
    main()
