"""PredictiveControllers.MPC (belief LTV-MPC, reference :56-340) against the reference's run.

``tests/golden/belief_{m1,m2}.npz`` were recorded by ``tools/gen_golden.py`` from the
reference's own ``PredictiveControllers.MPC`` (its ``get_xLin`` :121 TypeError replaced by
the intended flatten, nothing else) over the reference's own HMM model (CasADi shim) with
``Init_MPC.initMPCParams``, the oracle QP interior point behind the ``osqp`` stub: per step
the ego state, the agents' backup rollouts, the beliefs, the warm start carried in, the exact
(P, q, A, l, u) handed to OSQP on kept steps, and the solution.  M = 1 (3 backups) and
M = 2 (2 backups -- the row- vs column-major belief quirk of :208 matters there).

Checked: the compat class's assembly at 1e-9 against the reference's matrices (rows gated
by the belief included), and a closed-loop replay in which the compat MPC carries its own
state from step to step -- on CPU with the host build of the kernels (tests/hostsim), on the
GPU with libbmpc (bmpc_hmm_eval + bmpc_qp_solve).  Parity of the solution is to the exact QP
optimum; OSQP's own iterate is unpinned (OSQP absent).
"""
import numpy as np
import pytest

from common import coo, golden

NAMES = ("belief_m1", "belief_m2")


def make_mpc(g):
    import HMM_backup_dyn as HM
    import Init_MPC
    import PredictiveControllers
    from utils import Branch_constants
    cons = Branch_constants(s1=2, s2=3, c2=0.5, tran_diag=0.3, alpha=1, R=1.2, am=float(g["am"]), rm=float(g["rm"]),
                            J_c=20, s_c=1, ylb=0., yub=7.2, L=4, W=float(g["W"]), col_alpha=5, Kpsi=0.1)
    M, m, N, nx = int(g["M"]), int(g["m"]), int(g["N"]), int(g["nx"])
    pols = [lambda x: HM.backup_maintain(x, cons), lambda x: HM.backup_brake(x, cons),
            lambda x: np.array([-2.0, -cons.Kpsi * x[3]])][:m]
    model = HM.PredictiveModel(nx, 2, M, pols, float(g["dt"]), cons)
    param = Init_MPC.initMPCParams(nx, 2, N, M, m, float(g["ydes"]), float(g["vdes"]), cons.am, cons.rm,
                                   int(g["N_lane"]), cons.W)
    return PredictiveControllers.MPC(param, model), model


def xref(g):
    return np.array([0.0, float(g["ydes"]), float(g["vdes"]), 0.0])


def warm(mpc, g, t):
    u = g["traj_uLin_in"][t]
    mpc.uLin = None if np.isnan(u).all() else u[~np.isnan(u).any(axis=1)].copy()
    mpc.OldInput = g["traj_old_in"][t].copy() if t else np.zeros((1, 2))


def assemble(mpc, g, t):
    """The matrices solve() hands to the QP solver, without solving."""
    x, b, xbk = g["traj_x"][t], g["traj_b"][t], g["traj_xbackup"][t]
    mpc.xRef = np.append(xref(g), np.zeros(mpc.M * mpc.m))
    mpc.get_xLin(x, xbk, b)
    mpc.computeLTVdynamics(xbk)
    mpc.buildIneqConstr()
    mpc.buildCost()
    mpc.buildEqConstr()
    xb0 = np.append(x, np.reshape(b, [-1, 1]))
    mpc.addTerminalComponents(xb0)
    import scipy.sparse as sp
    A = sp.vstack([mpc.F_FTOCP, mpc.G_FTOCP]).toarray()
    beq = mpc.E_FTOCP @ xb0 + mpc.L_FTOCP
    return mpc.H_FTOCP.toarray(), mpc.q_FTOCP, A, np.hstack([np.full(len(mpc.b_FTOCP), -np.inf), beq]), \
        np.hstack([mpc.b_FTOCP, beq])


@pytest.fixture
def host_device(monkeypatch):
    """bmpc.plan's device calls replaced by the host build of the same kernels."""
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


def test_assembly_matches_reference(host_device):
    """buildIneqConstr / buildCost / buildEqConstr over the linearisation of the belief model:
    the reference's (P, q, A, l, u) at 1e-9 (the rollout compounds 1e-16 model differences
    over N stages), belief-gated collision rows identical in number and place."""
    for name in NAMES:
        g = golden(name)
        for t in (int(k) for k in g["keep"]):
            mpc, _ = make_mpc(g)
            warm(mpc, g, t)
            P, q, A, l, u = assemble(mpc, g, t)
            p = f"s{t}_"
            assert mpc.slackdim == int(g["traj_slackdim"][t]), (name, t)
            for mine, ref, what in ((P, coo(g, p + "P").toarray(), "P"), (A, coo(g, p + "A").toarray(), "A"),
                                    (q, g[p + "q"], "q"), (u, g[p + "u"], "u")):
                assert mine.shape == ref.shape, (name, t, what)
                np.testing.assert_allclose(mine, ref, rtol=1e-9, atol=1e-9, err_msg=f"{name} s{t} {what}")
            assert np.array_equal(np.isinf(l), np.isinf(g[p + "l"]))


def replay(g, mpc):
    """The compat MPC stepped through the recorded scene, carrying its own warm start."""
    us, st = [], []
    T = len(g["traj_x"])
    for t in range(T):
        mpc.solve(g["traj_x"][t], g["traj_b"][t], g["traj_xbackup"][t], xref(g))
        us.append(mpc.uPred[0].copy())
        st.append(mpc.feasible)
    return np.array(us), np.array(st)


def check_replay(g, us, st, name):
    assert np.all(st == 1) and np.all(g["traj_status"] == 1), name
    # x* is unique (P > 0 on the inputs, slacks priced linearly); both stop at 1e-10
    np.testing.assert_allclose(us, g["traj_u"], atol=1e-6, err_msg=name)


def test_host_build_replays_belief_scenes(host_device):
    for name in NAMES:
        g = golden(name)
        mpc, _ = make_mpc(g)
        us, st = replay(g, mpc)
        check_replay(g, us, st, name)
        assert mpc.timeStep == len(g["traj_x"])
        assert mpc.xPred.shape == (int(g["N"]) + 1, mpc.n) and mpc.uLin.shape == (int(g["N"]), 2)


def test_reference_quirks_kept(host_device):
    """:121 fixed (b0 flattened), :208 row-major gating, timeVarying False keeps growing uLin."""
    g = golden("belief_m2")
    mpc, _ = make_mpc(g)
    mpc.timeVarying = False
    mpc.A, mpc.B = np.eye(mpc.n), np.zeros((mpc.n, 2))
    x, b, xbk = g["traj_x"][0], g["traj_b"][0], g["traj_xbackup"][0]
    mpc.get_xLin(x, xbk, b)
    np.testing.assert_allclose(mpc.xLin[0], np.append(x, np.reshape(b, -1)))
    n0 = len(mpc.uLin)
    mpc.uLin = np.vstack((mpc.uLin, mpc.uLin[-1]))
    mpc.get_xLin(x, xbk, b)
    assert len(mpc.uLin) == n0 + 2


# ---- GPU -------------------------------------------------------------------------------------
@pytest.fixture(scope="module")
def gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from bmpc import plan
    plan.context(0)
    return plan


@pytest.mark.gpu
def test_gpu_replays_belief_scenes(gpu):
    for name in NAMES:
        g = golden(name)
        mpc, _ = make_mpc(g)
        us, st = replay(g, mpc)
        check_replay(g, us, st, name)
