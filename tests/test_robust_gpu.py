"""robustMPC (MPC_branch.py:1275-1595) on the GPU, through the C ABI.

Fixtures: tests/golden/highway_robust_*.npz, made by the reference's own robustMPC (tree,
linearisation schedule, OSQP problem assembly) with the oracle QP solver behind the osqp
stub (tools/gen_golden.py).  OSQP itself is absent and unpinned; the oracle
returns the exact QP optimum (interior point to 1e-10), so the recorded predictions are that
optimum.  Tolerances: status_val 1 on every step; uPred / xPred of every step to 1e-6
absolute; the GPU against the host build of the same kernel source to 1e-9."""
import numpy as np
import pytest

import hostsim_lib as H
from common import golden, highway_desc_from_golden, highway_policy_rows
from conftest import assert_solver_path

pytestmark = pytest.mark.gpu

CASES = ["highway_robust_n20_nb1", "highway_robust_n8_nb2"]


@pytest.fixture(scope="module")
def gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from bmpc import plan
    plan.context(0)
    return plan


def _desc(g):
    from bmpc import abi
    desc = highway_desc_from_golden(g)
    desc.controller = abi.CTRL_ROBUST
    return desc


@pytest.mark.parametrize("name", CASES)
def test_robust_replay_gpu(gpu, name, qp_path):
    """Every recorded step in one launch, each ego carrying the reference's warm start."""
    g = golden(name)
    T = len(g["traj_x"])
    pl = gpu.BatchPlan(_desc(g), T)
    assert (pl.T, pl.U) == (g["traj_xPred"].shape[1], g["traj_uPred"].shape[1])
    pl.set_policies(highway_policy_rows(g["traj_lc_target"], float(g["Kpsi"])))
    xl = np.asarray(g["traj_ws_xLin"], float)
    warm = ~np.isnan(xl).any(axis=(1, 2))
    pl.set_robust_warm_start(np.nan_to_num(xl), np.nan_to_num(g["traj_ws_uLin"]), g["traj_ws_old"], mask=warm)
    r = pl.solve(g["traj_x"], g["traj_z"], g["traj_xRef"])
    assert_solver_path(pl, qp_path)
    np.testing.assert_array_equal(r["status"], g["traj_status"])
    np.testing.assert_allclose(r["upred"], g["traj_uPred"], atol=1e-6)
    np.testing.assert_allclose(r["xpred"], g["traj_xPred"], atol=1e-6)
    # the carried warm start of the next step = this step's prediction shifted by one
    ws = pl.get_robust_warm_start()
    np.testing.assert_allclose(ws["xLin"][:-1], g["traj_ws_xLin"][1:], atol=1e-6)
    np.testing.assert_allclose(ws["uLin"][:-1], g["traj_ws_uLin"][1:], atol=1e-6)
    np.testing.assert_allclose(ws["old_input"][:-1], g["traj_ws_old"][1:], atol=1e-6)
    # and the host build of the same source agrees tightly
    hs = H.HostSim(_desc(g), T)
    hs.set_policies(highway_policy_rows(g["traj_lc_target"], float(g["Kpsi"])))
    hs.set_robust_warm_start(np.nan_to_num(xl), np.nan_to_num(g["traj_ws_uLin"]), g["traj_ws_old"])
    hs.reset_mask(~warm)
    rh = hs.solve(g["traj_x"], g["traj_z"], g["traj_xRef"])
    np.testing.assert_allclose(r["upred"], rh["upred"], atol=1e-9)


def test_robust_dropin_closed_loop(gpu):
    """The drop-in ``MPC_branch.robustMPC`` (built as Init_MPC.initBranchMPC builds its
    parameters) driven through the overtake scene reproduces the recorded loop."""
    import Init_MPC
    import MPC_branch
    from highway_branch_dyn import PredictiveModel, backup_brake, backup_lc, backup_maintain
    from oracle.env import HighwayOvertake
    from utils import Branch_constants
    g = golden("highway_robust_n8_nb2")
    N, n, d, am, rm, dt, NB, N_lane = 8, 4, 2, 6.0, 0.3, 0.1, 2, 4
    xRef = np.array([0.5, 1.8, 15, 0])
    cons = Branch_constants(s1=2, s2=3, c2=0.5, tran_diag=0.3, alpha=1, R=1.2, am=am, rm=rm, J_c=20, s_c=1,
                            ylb=0., yub=7.2, L=4, W=2.5, col_alpha=5, Kpsi=0.1)
    backupcons = [lambda x: backup_maintain(x, cons), lambda x: backup_brake(x, cons), lambda x: backup_lc(x, xRef)]
    model = PredictiveModel(n, d, N, backupcons, dt, cons)
    mpc = MPC_branch.robustMPC(Init_MPC.initBranchMPC(n, d, N, NB, xRef, am, rm, N_lane, cons.W), model)

    class Backups:   # the scene re-targets the lane-change backup (Highway_env_branch.py:117)
        def zpred_eval(self, z):
            return model.zpred_eval(z)

        def update_backup(self, _oracle_policies):
            tgt = env.lc_target.copy()
            model.update_backup([lambda x: backup_maintain(x, cons), lambda x: backup_brake(x, cons),
                                 lambda x: backup_lc(x, tgt)])

    env = HighwayOvertake(mpc, Backups(), N_lane=N_lane, L=cons.L, W=cons.W, Kpsi=cons.Kpsi, lc_target0=xRef,
                          dt=dt)
    for t in range(10):
        rec = env.step(t)
        np.testing.assert_allclose(rec["x"], g["traj_x"][t], atol=1e-6, err_msg=f"ego state, step {t}")
        np.testing.assert_allclose(mpc.uPred, g["traj_uPred"][t], atol=1e-6, err_msg=f"uPred, step {t}")
        assert mpc.feasible == 1
    xs, zs, us, ws = mpc.BT2array()
    assert len(xs) == 1 and xs[0].shape == (N * NB + 2, n) and ws == []
    assert len(zs) == 3 + 9 and zs[0].shape == (N + 1, n)
