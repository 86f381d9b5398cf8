"""Highway_env.sim's belief scene (row f4: the ego's PredictiveControllers.MPC and the other
vehicles' backup-CBF QPs) against the reference's own run.

``tests/golden/belief_env_m2.npz`` was recorded by ``tools/gen_golden.py`` from the
reference's ``Highway_env`` (its vehicles, CBF QPs, belief update and ``Highway_sim``) with the
reference's ``PredictiveControllers.MPC`` (:121 fixed) over its HMM model; the QPs (the MPC's
and the CBF filters') went to the oracle QP behind the ``osqp`` stub; ``random`` and
``np.random`` seeded before the env was built.  The compat module consumes random numbers in
the same order, so the seeded replay is the same scene: vehicle placement, lane / speed
draws, backup choices.  Checked on CPU through the host build of the kernels (HMM
linearisation, QP solver) and on the GPU through libbmpc.
"""
import random

import numpy as np
import pytest

from common import golden

NAME = "belief_env_m2"


def run_scene(g):
    import HMM_backup_dyn as HM
    import Highway_env
    import Init_MPC
    import PredictiveControllers
    from utils import Branch_constants
    cons = Branch_constants(s1=2, s2=3, c2=0.5, tran_diag=0.3, alpha=1, R=1.2, am=float(g["am"]), rm=float(g["rm"]),
                            J_c=20, s_c=1, ylb=0., yub=7.2, L=4, W=float(g["W"]), col_alpha=5, Kpsi=0.1)
    M, m, N = int(g["M"]), int(g["m"]), int(g["N"])
    pols = [lambda x: HM.backup_maintain(x, cons), lambda x: HM.backup_brake(x, cons),
            lambda x: np.array([-2.0, -cons.Kpsi * x[3]])][:m]
    model = HM.PredictiveModel(4, 2, M, pols, float(g["dt"]), cons)
    param = Init_MPC.initMPCParams(4, 2, N, M, m, 1.8, Highway_env.v0, cons.am, cons.rm, int(g["N_lane"]), cons.W)
    mpc = PredictiveControllers.MPC(param, model)
    random.seed(int(g["seed"]))
    np.random.seed(int(g["seed"]))
    env = Highway_env.Highway_env(NV=M + 1, mpc=mpc, N_lane=int(g["N_lane"]))
    np.testing.assert_allclose(np.array([v.state for v in env.veh_set]), g["init"], rtol=0, atol=0)
    return Highway_env.Highway_sim(env, float(g["T"]))


def check(recs, g):
    state_rec, input_rec, _, choice_rec, b_rec, xPred_rec, collision = recs
    np.testing.assert_array_equal(np.array(choice_rec, float), g["choice_rec"])
    # the MPC's and the CBF filters' optima agree to ~1e-9; over 30 steps of the closed loop
    np.testing.assert_allclose(input_rec, g["input_rec"], atol=1e-6)
    np.testing.assert_allclose(state_rec, g["state_rec"], atol=1e-6)
    np.testing.assert_allclose(np.array(b_rec), g["b_rec"], atol=1e-6)
    np.testing.assert_allclose(np.array(xPred_rec), g["xPred_rec"], atol=1e-5)
    assert int(collision) == int(g["collision"])


@pytest.fixture
def host_device(monkeypatch):
    from test_predictive_controllers import host_device as fx  # noqa: F401
    import hostsim_lib as H
    from bmpc import plan
    monkeypatch.setattr(plan, "hmm_eval", lambda M, m, hc, xb, u, xbk, device=0: H.hmm_eval(
        M, m, hc, np.atleast_2d(xb), np.broadcast_to(np.atleast_2d(u), (np.atleast_2d(xb).shape[0], 2)),
        np.broadcast_to(np.asarray(xbk, float).reshape(-1, M * m, 4), (np.atleast_2d(xb).shape[0], M * m, 4))))

    def qp(P, q, A, l, u, max_iter=100, eps=1e-10, device=0):
        a = plan.qp_arrays(P, q, A, l, u)
        return H.qp_solve(a["n"], a["m"], a["Pp"], a["Pi"], a["Ap"], a["Ai"], a["Px"], a["q"], a["Ax"], a["l"], a["u"],
                          max_iter, eps)
    monkeypatch.setattr(plan, "qp_solve", qp)
    yield


def test_host_build_replays_reference_scene(host_device):
    g = golden(NAME)
    check(run_scene(g), g)


@pytest.fixture(scope="module")
def gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from bmpc import plan
    plan.context(0)
    return plan


@pytest.mark.gpu
def test_gpu_replays_reference_scene(gpu):
    g = golden(NAME)
    check(run_scene(g), g)
