"""ECOS's Ruiz equilibration (ECOS_setup -> set_equilibration; oracle/ecos_ipm.py:equilibration,
csrc/bmpc_ipm.h:equilibrate).

* The kernel never assembles A or G: it enumerates their entries from the structured operators.
  Its factors (host build of the kernel templates) must equal the oracle's, computed on the
  problem the reference itself assembled (the fixtures' recorded (A, G) of kept steps), to the
  rounding of the three sqrt(max) rounds.
* The oracle's equilibrated IPM returns a point certified by the unscaled KKT residuals and the
  unscaled problem's optimum (J) of the unequilibrated solve.
ECOS is absent from this image: equilibration is restated from ECOS 2.0.x's published source
(equil.c, RUIZ_EQUIL, EQUIL_ITERS = 3); parity of ECOS's iterates stays unpinned.
"""
import numpy as np
import pytest

import hostsim_lib as H
from common import cone_problem, golden, highway_desc_from_golden, replay_batch


@pytest.mark.parametrize("name", ["highway_n10_nb1", "highway_n8_nb2", "highway_n30_nb2"])
def test_kernel_equilibration_matches_oracle(name):
    from oracle.ecos_ipm import Cones, equilibration
    g = golden(name)
    steps = [int(k) for k in g["keep"]][:2]
    rb = replay_batch(g, max(steps) + 1)
    hs = H.HostSim(highway_desc_from_golden(g), rb["T"])
    hs.set_policies(rb["rows"])
    hs.set_warm_start(rb["uLin"], rb["p"], rb["jcons"])
    hs.reset_mask(~rb["warm"])
    hs.solve(rb["x"], rb["z"], rb["xref"])
    lay = hs.layout()
    for t in steps:
        prob = cone_problem(g, t)
        xe, ae, ge = equilibration(prob.A, prob.G, Cones(prob.dims))
        w = hs.workspace(t)
        kx, ka, kg = (w[lay[f]:lay[f] + len(v)] for f, v in (("xeq", xe), ("aeq", ae), ("geq", ge)))
        for lab, a, b in (("x", kx, xe), ("A rows", ka, ae), ("G rows", kg, ge)):
            err = np.max(np.abs(a - b) / np.abs(b))
            assert err < 1e-12, (name, t, lab, err, int(np.argmax(np.abs(a - b) / np.abs(b))))
        assert not np.allclose(xe, 1.0) and not np.allclose(ge, 1.0)   # the problem is not already balanced


def test_oracle_equilibrated_solve_is_certified():
    from oracle.ecos_ipm import ecos_solve, kkt_residuals
    g = golden("highway_n10_nb1")
    for t in (int(k) for k in g["keep"]):
        prob = cone_problem(g, t)
        x0, i0 = ecos_solve(prob, equilibrate=False)
        x1, i1 = ecos_solve(prob, equilibrate=True)
        assert i1["exitFlag"] in (0, 10), i1["exitFlag"]
        r = kkt_residuals(prob, i1["x"], i1["y"], i1["z"], i1["s"])
        tol = 1e-6 if i1["exitFlag"] == 0 else 1e-3
        assert r["dual"] < tol and r["eq"] < tol and r["ineq"] < tol and r["cone"] > -tol, r
        assert abs(x1[-1] - x0[-1]) <= 1e-6 * max(1.0, abs(x0[-1])), (x1[-1], x0[-1])
