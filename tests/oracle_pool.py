"""Test infrastructure: CPU oracle re-solves of sampled egos in parallel worker processes.

The oracle (oracle/, the ECOS-algorithm restatement on the reference's assembly) takes seconds
per highway N=20 ego and ~40 s per N=30 NB=2 ego on one core, so the GPU tests that check
sampled egos of a 4096-ego launch against it spread the solves over spawned workers (fresh
interpreters that import only numpy / scipy / oracle -- never the HIP library or torch).
"""
from __future__ import annotations

import os


def _init():
    for k in ("OMP_NUM_THREADS", "OPENBLAS_NUM_THREADS", "MKL_NUM_THREADS"):
        os.environ[k] = "1"


def solve_cvar(case):
    """case = (N, NB, lane-change target, xref, x, z) -> (exitFlag, J, uPred[0])."""
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    repo = os.path.dirname(here)
    for p in (repo, os.path.join(repo, "belief-planning_amd")):
        if p not in sys.path:
            sys.path.insert(0, p)
    import numpy as np
    from oracle.ecos_ipm import ecos_solve
    from oracle.model import HighwayModel, highway_policies
    from oracle.tree import CVaRController
    N, NB, tgt, xref, x, z = case
    Fx = np.array([[0., 1, 0, 0], [0, -1, 0, 0], [0, 0, 0, 1], [0, 0, 0, -1]])
    mdl = HighwayModel(N, 0.1, highway_policies(0.1, tgt))
    c = CVaRController(mdl, N, NB, np.diag([0., 3, 3, 10]), np.diag([1., 100]), Fx,
                       [4 * 3.6 - 1.25, -1.25, .25, .25], np.kron(np.eye(2), [1, -1]).T,
                       [6., 6., .3, .3], [0, 300], xref, 0.9, solver=ecos_solve)
    c.solve(x, z, xref)
    return int(c.last_info["exitFlag"]), float(c.last_info["x"][-1]), np.asarray(c.uPred[0], float).copy()


def solve_many(cases, workers=None):
    """Oracle solves of every case, in order, on `workers` spawned processes."""
    import multiprocessing as mp
    from concurrent.futures import ProcessPoolExecutor
    workers = workers or min(8, len(cases), max(1, (os.cpu_count() or 2) // 2))
    with ProcessPoolExecutor(max_workers=workers, mp_context=mp.get_context("spawn"), initializer=_init) as ex:
        return list(ex.map(solve_cvar, cases))
