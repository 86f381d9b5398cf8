"""The reference's own entry scripts run unchanged against the drop-in modules.

``main_quadruped.py`` and ``main_branch.py`` are executed from ``/root/reference`` (this
container only; skipped where the reference is absent, e.g. on the GPU box) with
``belief-planning_amd`` first on ``sys.path``, so every ``import`` in them resolves to the
build's modules.  Only the device calls are replaced: ``bmpc.plan.BatchPlan`` and
``bmpc.plan.model_eval`` are swapped for the test-only host build of the same kernels
(tests/hostsim), so the scripts run their full controller path on CPU.
"""
import os
import runpy

import numpy as np
import pytest

REF = "/root/reference"
pytestmark = pytest.mark.skipif(not os.path.isdir(REF), reason="reference checkout not present")


class _HostPlan:
    """BatchPlan stand-in over the host build (same methods the compat classes call)."""

    solves = 0

    def __init__(self, desc, batch, device=0):
        import hostsim_lib
        self.desc, self.batch = desc, batch
        self._hs = hostsim_lib.HostSim(desc, batch)
        self.T, self.U, self.bdim, self.nbranch = self._hs.T, self._hs.U, self._hs.bdim, self._hs.nbranch

    def set_policies(self, rows, mask=None):
        self._hs.set_policies(rows)

    def solve(self, x, z, xref):
        type(self).solves += 1
        return self._hs.solve(x, z, xref)

    def tree(self):
        return self._hs.tree()

    def set_transform(self, S=None, bx=None, s_on=None, mask=None):
        self._hs.set_transform(S, bx, s_on)

    def set_fx(self, Fx, mask=None):
        self._hs.set_fx(Fx)

    def branch_dp(self):
        return self._hs.branch_dp()

    def set_lane_ref(self, grid, values):
        self._hs.set_lane_ref(grid, values)


@pytest.fixture
def host_device(monkeypatch):
    import hostsim_lib
    from bmpc import plan
    monkeypatch.setattr(plan, "BatchPlan", _HostPlan)
    monkeypatch.setattr(plan, "model_eval", lambda desc, rows, x, u, z, device=0, lane_ref=None:
                        hostsim_lib.model_eval(desc, rows, x, u, z, lane_ref=lane_ref))
    _HostPlan.solves = 0
    yield


def test_reference_main_quadruped_runs_unchanged(host_device, monkeypatch):
    """main_quadruped.py (reference :1-48): Quad_constants from the star import (:31),
    BranchMPCProx, quadruped_env.sim(mpc) (:43) -- the scene loop is shortened to 2 s."""
    import quadruped_env
    full = quadruped_env.sim
    recs = []
    monkeypatch.setattr(quadruped_env, "sim", lambda mpc: recs.append(full(mpc, T=2.0)))
    ns = runpy.run_path(os.path.join(REF, "main_quadruped.py"), run_name="ref_main_quadruped")
    ns["main"]()
    assert _HostPlan.solves == 10
    state_rec, input_rec, backup_rec, choice_rec, xPred_rec, zPred_rec = recs[0]
    assert np.all(np.isfinite(state_rec)) and np.all(np.isfinite(input_rec))
    # the ego moves under the MPC's inputs, bounded by Fu (vxm 0.2, vym 0.1, rm 0.5)
    assert np.all(np.abs(input_rec[0][:, 0]) <= 0.2 + 1e-6) and np.all(np.abs(input_rec[0][:, 2]) <= 0.5 + 1e-6)
    assert len(xPred_rec[0]) == 6        # BT2array over the 2 + 4 non-root branches


def test_reference_main_branch_runs_unchanged(host_device, monkeypatch):
    """main_branch.sim_overtake (reference :20-51): BranchMPC_CVaR with N=8, NB=2 in the
    overtake scene (Highway_env_branch.sim_overtake) -- shortened to 1 s."""
    import Highway_env_branch
    full_sim = Highway_env_branch.Highway_sim
    recs = []

    def short(env, T):
        recs.append(full_sim(env, 1.0))
        return recs[-1]
    monkeypatch.setattr(Highway_env_branch, "Highway_sim", short)
    ns = runpy.run_path(os.path.join(REF, "main_branch.py"), run_name="ref_main_branch")
    ns["sim_overtake"]()
    assert _HostPlan.solves == 10
    state_rec, input_rec = recs[0][0], recs[0][1]
    assert np.all(np.isfinite(state_rec))
    assert np.all(np.abs(input_rec[0][:, 1]) <= 0.3 + 1e-6)     # steering-rate bound rm
    # the scene is the one tools/gen_golden.py recorded through the reference's own controller
    # (highway_n8_nb2): every step exits 0 there, and the closed loop holds to 1e-6
    from common import golden
    g = golden("highway_n8_nb2")
    assert np.all(g["traj_exit"][:10] == 0)
    np.testing.assert_allclose(input_rec[0][:10], g["traj_u"][:10], atol=1e-6)
    np.testing.assert_allclose(state_rec[0][:9], g["traj_x"][1:10], atol=1e-6)


def test_bt_is_live_after_solve(host_device):
    """mpc.BT is populated after every solve (reference keeps a live BranchTree)."""
    import Init_MPC
    import MPC_branch
    from highway_branch_dyn import PredictiveModel, backup_brake, backup_lc, backup_maintain
    from utils import Branch_constants
    cons = Branch_constants(s1=2, s2=3, c2=0.5, tran_diag=0.3, alpha=1, R=1.2, am=6.0, rm=0.3, J_c=20, s_c=1,
                            ylb=0., yub=7.2, L=4, W=2.5, col_alpha=5, Kpsi=0.1)
    xRef = np.array([0.5, 1.8, 15, 0])
    model = PredictiveModel(4, 2, 8, [lambda x: backup_maintain(x, cons), lambda x: backup_brake(x, cons),
                                      lambda x: backup_lc(x, xRef)], 0.1, cons)
    mpc = MPC_branch.BranchMPC_CVaR(Init_MPC.initBranchMPC(4, 2, 8, 2, xRef, 6.0, 0.3, 4, cons.W), model, 0.9)
    assert mpc.BT is None
    mpc.solve(np.array([0, 1.8, 20, 0.]), np.array([5, 5.4, 20, 0.]), xRef)
    bt = mpc.BT
    assert bt is not None and len(bt.children) == 3 and len(bt.children[0].children) == 3
    w = sum(c.w for c in bt.children)
    assert abs(w - 1.0) < 1e-12
    assert bt.children[1].xtraj.shape == (8, 4)
    first = mpc.BT
    mpc.solve(np.array([2, 1.8, 20, 0.]), np.array([7, 5.4, 20, 0.]), xRef)
    assert mpc.BT is not first              # rebuilt for the new solve


def test_reference_sim_merge_runs_unchanged(host_device, monkeypatch):
    """main_branch.sim_merge (reference :53-88): PredictiveModel_merge with linear
    interpolants, BranchMPC_CVaR(ralpha=0.1) taking S / bx every step, Highway_env_merge --
    shortened to 1 s and compared with the reference's own recording of the scene."""
    import Highway_env_branch
    from common import golden
    full_sim = Highway_env_branch.Highway_sim
    recs = []

    def short(env, T):
        recs.append(full_sim(env, 1.0))
        return recs[-1]
    monkeypatch.setattr(Highway_env_branch, "Highway_sim", short)
    ns = runpy.run_path(os.path.join(REF, "main_branch.py"), run_name="ref_main_branch")
    ns["sim_merge"]()
    assert _HostPlan.solves == 10
    g = golden("merge_n40_nb1")
    state_rec, input_rec = recs[0][0], recs[0][1]
    # Highway_sim records the state after each step: row t = traj_x[t+1].  The merge optimum pins
    # J (~3e4) to ECOS's 1e-8 relative gap, ~3e-4, but uPred[0] only to ~1e-2 through R = diag(1,
    # 100): once the closed loop's state differs from the recording's at the rounding floor, the
    # next solve's input moves by up to ~1e3 x that difference (measured on the host build, steps
    # 0-3: |du| 1e-10, 7e-8, 2.5e-5, 2.6e-3).  The replays (test_merge.py) hold every recorded
    # step to 1e-5 on identical problems; here the first two steps are held to 1e-6 and the
    # rest of the 1-s scene to the optimum's 1e-2 precision.  Measured (round 6,
    # tools/optimum_precision.py, profiles/r06/optimum_precision.log): the reference's own recorded
    # problems of this scene solved at ECOS's 1e-8 and again at 1e-10 / 1e-12 move uPred[0] by
    # 2.1e-6, 4.5e-5, 2.6e-5 at steps 0-2 and 7.0e-5 at step 30 -- the recorded inputs are only
    # defined to ~5e-5 by the tolerances the reference runs, so a loop that feeds each solution into
    # the next step cannot be held near 1e-5 by any implementation of the solver.
    np.testing.assert_allclose(state_rec[0][:2], g["traj_x"][1:3], atol=1e-6)
    np.testing.assert_allclose(input_rec[0][:2], g["traj_u"][:2], atol=1e-6)
    np.testing.assert_allclose(state_rec[0][:9], g["traj_x"][1:10], atol=1e-2)
    np.testing.assert_allclose(input_rec[0][:10], g["traj_u"][:10], atol=2e-2)
    np.testing.assert_allclose(state_rec[1][:9], g["traj_z"][1:10], atol=1e-9)
