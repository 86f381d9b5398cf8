"""How tightly ECOS's default tolerances pin uPred[0] (CPU, oracle; test tooling): each kept solver
problem of a recording solved at feastol = abstol = reltol = 1e-8 (what the reference runs) and at
1e-10 / 1e-12, with the difference of uPred[0] and J between the 1e-8 point and the tighter ones.
A closed loop whose steps carry their own solutions forward can only be held to that precision.
    python tools/optimum_precision.py [recording ...] > profiles/r06/optimum_precision.log"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "tests"), REPO, os.path.join(REPO, "belief-planning_amd")]
from common import cone_problem, golden  # noqa: E402
from oracle.ecos_ipm import ecos_solve  # noqa: E402
from oracle.tree import Topology  # noqa: E402

for name in sys.argv[1:] or ("merge_n40_nb1", "highway_n20_nb1", "highway_xform_n8_nb2"):
    g = golden(name)
    m = 2 if name.startswith("merge") else 3
    top = Topology.build(int(g["N"]), int(g["NB"]), m)
    oU = top.T * 4
    for t in (int(k) for k in g["keep"]):
        prob = cone_problem(g, t)
        res = [(tol,) + ecos_solve(prob, feastol=tol, abstol=tol, reltol=tol) for tol in (1e-8, 1e-10, 1e-12)]
        x8 = res[0][1]
        line = f"{name} step {t:3d}: exit {res[0][2]['exitFlag']:2d} J {x8[-1]:.10e}"
        for tol, x, info in res[1:]:
            line += (f" | tol {tol:.0e} exit {info['exitFlag']:2d} |du0| {np.abs(x[oU:oU + 2] - x8[oU:oU + 2]).max():.1e}"
                     f" |dJ|/J {abs(x[-1] - x8[-1]) / abs(x8[-1]):.1e}")
        print(line, flush=True)
