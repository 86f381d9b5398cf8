"""BranchMPCProx (quadruped, BASELINE config 4): the device QP algorithm compiled for the
host (TEST-ONLY build) against the reference's recorded closed loop
(tests/golden/quadruped_n25_nb2.npz: the reference's own tree/cost/constraint code, the
oracle quadruped model and the oracle QP solver behind the osqp stub).

OSQP itself is absent and unpinned; the oracle returns the exact QP optimum
(interior point to 1e-10), so the recorded uPred is that optimum.  Tolerances: status_val
must be 1 on every step; uPred[0] to 1e-6 absolute (|u| <= 0.5); the full primal vector of
the kept steps to 1e-6 relative to max(1, |z|)."""
import numpy as np
import pytest

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


def test_branch_mpc_qp_replay():
    """BranchMPC (MPC_branch.py:881) on the highway scene: every recorded step replayed."""
    from common import highway_desc_from_golden, highway_policy_rows
    from bmpc import abi
    g = golden("highway_qp_n8_nb2")
    T = len(g["traj_x"])
    desc = highway_desc_from_golden(g)
    desc.controller = abi.CTRL_QP
    hs = H.HostSim(desc, T)
    hs.set_policies(highway_policy_rows(g["traj_lc_target"], float(g["Kpsi"])))
    ws_u = np.asarray(g["traj_ws_uLin"], float)
    warm = ~np.isnan(ws_u).any(axis=(1, 2))
    hs.set_warm_start(np.nan_to_num(ws_u), np.nan_to_num(g["traj_ws_p"]), None, g["traj_ws_old"])
    hs.reset_mask(~warm)
    r = hs.solve(g["traj_x"], g["traj_z"], g["traj_xRef"])
    np.testing.assert_array_equal(r["status"], g["traj_status"])
    np.testing.assert_allclose(r["upred"][:, 0], g["traj_u"], atol=1e-6)
    sol = hs.tree()["sol"]
    for t in (int(k) for k in g["keep"]):
        ref = g[f"s{t}_sol"]
        np.testing.assert_allclose(sol[t], ref, atol=1e-6 * max(1.0, np.abs(ref).max()), err_msg=f"step {t}")


def _robust_desc(g):
    from common import highway_desc_from_golden
    from bmpc import abi
    desc = highway_desc_from_golden(g)
    desc.controller = abi.CTRL_ROBUST
    return desc


@pytest.mark.parametrize("name", ["highway_robust_n20_nb1", "highway_robust_n8_nb2"])
def test_robust_mpc_replay(name):
    """robustMPC (MPC_branch.py:1275): every recorded step replayed as one ego carrying the
    reference's warm start (shifted prediction, OldInput); uPred/xPred of every step to 1e-6
    (the oracle QP optimum stands in for OSQP + polish), the kept steps' full primal
    vector against the reference's OSQP problem solution on its x/u part."""
    from common import highway_policy_rows
    g = golden(name)
    T = len(g["traj_x"])
    hs = H.HostSim(_robust_desc(g), T)
    assert (hs.T, hs.U) == (g["traj_xPred"].shape[1], g["traj_uPred"].shape[1])
    hs.set_policies(highway_policy_rows(g["traj_lc_target"], float(g["Kpsi"])))
    xl = np.asarray(g["traj_ws_xLin"], float)
    warm = ~np.isnan(xl).any(axis=(1, 2))
    hs.set_robust_warm_start(np.nan_to_num(xl), np.nan_to_num(g["traj_ws_uLin"]), g["traj_ws_old"])
    hs.reset_mask(~warm)
    r = hs.solve(g["traj_x"], g["traj_z"], g["traj_xRef"])
    np.testing.assert_array_equal(r["status"], g["traj_status"])
    np.testing.assert_allclose(r["upred"], g["traj_uPred"], atol=1e-6)
    np.testing.assert_allclose(r["xpred"], g["traj_xPred"], atol=1e-6)


def test_quadruped_closed_loop_precision_floor():
    """BASELINE config 4, seeded ego 311 of 1024: at step 7 the inequality residual
    G x + s - g stalls at the rounding floor of s (9.3e-10) while |g| < 9, so a test scaled by
    |g| alone never passed and the factorisation broke down at mu ~ 1e-17 (status -2).  Judged
    against max(|g|, |s|) (OSQP scales by max(|Ax|, |z|)) every step solves
    (tools/quad_failures.py: 0 of 20,480 closed-loop solves fail, host build and GPU)."""
    import sys
    import os
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
    from quad_failures import env_step
    from bmpc.scenarios import quadruped_desc, seeded_quadruped_batch
    x, z, xr = (v[311:312] for v in seeded_quadruped_batch(1024, seed=1))
    hs = H.HostSim(quadruped_desc(), 1)
    hs.set_policies(quadruped_policy_rows(1))
    for t in range(8):
        r = hs.solve(x, z, xr)
        assert r["status"][0] == 1, (t, r["status"], r["iters"])
        x, z, xr = env_step(x, z, r["upred"][:, 0])
