"""BranchMPCProx (quadruped, BASELINE config 4): the device QP algorithm compiled for the
host (TEST-ONLY build) against the reference's recorded closed loop
(tests/golden/quadruped_n25_nb2.npz: the reference's own tree/cost/constraint code, the
oracle quadruped model and the oracle QP solver behind the osqp stub).

OSQP itself is absent and unpinned; the oracle returns the exact QP optimum
(interior point to 1e-10), so the recorded uPred is that optimum.  Tolerances: status_val
must be 1 on every step; uPred[0] to 1e-6 absolute (|u| <= 0.5); the full primal vector of
the kept steps to 1e-6 relative to max(1, |z|)."""
import numpy as np

import hostsim_lib as H
from common import golden, quad_replay_batch, quadruped_desc_from_golden, quadruped_policy_rows


def test_quadruped_prox_replay():
    g = golden("quadruped_n25_nb2")
    rb = quad_replay_batch(g)
    hs = H.HostSim(quadruped_desc_from_golden(g), rb["T"])
    hs.set_policies(quadruped_policy_rows(rb["T"]))
    hs.set_warm_start(rb["uLin"], rb["p"], None, rb["old"])
    hs.reset_mask(~rb["warm"])
    r = hs.solve(rb["x"], rb["z"], rb["xref"])
    np.testing.assert_array_equal(r["status"], np.ones(rb["T"]))
    np.testing.assert_allclose(r["upred"][:, 0], g["traj_u"][:rb["T"]], atol=1e-6)
    sol = hs.tree()["sol"]
    for t in (int(k) for k in g["keep"]):
        ref = g[f"s{t}_sol"]
        np.testing.assert_allclose(sol[t], ref, atol=1e-6 * max(1.0, np.abs(ref).max()), err_msg=f"step {t}")
        np.testing.assert_allclose(r["upred"][t], g[f"s{t}_uPred"], atol=1e-6)
