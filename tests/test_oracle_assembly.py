"""Pin the oracle's tree/assembly restatement to the reference's own code.

tests/golden/*.npz were produced by running the reference's MPC_branch.BranchMPC_CVaR
(imported with solver stubs, tools/gen_golden.py) through the sim_overtake closed loop;
they hold the exact (c, G, h, dims, A, b) it handed to ecos.solve.  The oracle restatement
must rebuild the same matrices from the same state (<= 1e-12)."""
import numpy as np
import pytest

from common import coo, golden
from oracle.ecos_ipm import ecos_solve, kkt_residuals
from oracle.model import HighwayModel, highway_policies
from oracle.tree import CVaRController, TreeState

CASES = [("highway_n20_nb1", [0, 1, 2]), ("highway_n8_nb2", [0, 1, 2]), ("highway_n10_nb1", [0, 1]),
         ("highway_n30_nb2", [0, 1])]


def controller(g, t):
    mdl = HighwayModel(int(g["N"]), float(g["dt"]), highway_policies(float(g["Kpsi"]), g["traj_lc_target"][t]),
                       L=float(g["L"]), W=float(g["W"]), s1=float(g["s1"]))
    return CVaRController(mdl, int(g["N"]), int(g["NB"]), g["Q"], g["R"], g["Fx"], g["bx"], g["Fu"], g["bu"],
                          g["Qslack"], g["xRef0"], float(g["ralpha"]), solver=ecos_solve)


def inject_previous(c, g, t):
    """Warm-start state after the reference's step t-1: uLin from its solution, p from its
    branch weights, Jcons from the first solve's x_ref."""
    prev = g[f"s{t - 1}_sol"]
    topo = c.topo
    n, d = c.n, c.d
    uP = prev[topo.T * n: topo.T * n + topo.U * d].reshape(topo.U, d)
    c.uLin = np.vstack((uP, uP[-1]))
    c.tree = TreeState(topo, n, d)
    w = np.concatenate([[1.0], g[f"s{t - 1}_bt_w"]])
    for b in range(topo.nbranch):
        if not topo.is_leaf(b):
            c.tree.p[b] = np.array([w[ch] / w[b] for ch in topo.children[b]])
    xr0 = g["traj_xRef"][0]
    c.Jcons = float(xr0 @ c.Q @ xr0)


@pytest.mark.parametrize("name,steps", CASES)
def test_assembly_matches_reference(name, steps):
    g = golden(name)
    for t in steps:
        c = controller(g, t)
        if t > 0:
            inject_previous(c, g, t)
        prob = c.setup_problem(g["traj_x"][t], g["traj_z"][t], g["traj_xRef"][t])
        p = f"s{t}_"
        assert prob.dims["l"] == int(g[p + "dims_l"])
        assert list(prob.dims["q"]) == [int(v) for v in g[p + "dims_q"]]
        np.testing.assert_array_equal(prob.c, g[p + "c"])
        for mine, key in ((prob.G, "G"), (prob.A, "A")):
            ref = coo(g, p + key)
            assert mine.shape == ref.shape
            diff = abs(mine - ref)
            assert diff.max() <= 1e-12 * max(1.0, abs(ref).max()), (name, t, key, diff.max())
            assert (mine != 0).sum() == (ref != 0).sum()
        np.testing.assert_allclose(prob.h, g[p + "h"], rtol=1e-12, atol=1e-12)
        np.testing.assert_allclose(prob.b, g[p + "b"], rtol=1e-12, atol=1e-12)
        np.testing.assert_allclose(prob.cone_boost, g[p + "cone_boost"], rtol=1e-12, atol=1e-12)
        # BT2array of the reference tree vs the oracle tree
        xs, zs, us, ws = c.tree.bt2array()
        np.testing.assert_allclose(np.array(xs), g[p + "bt_x"], atol=1e-11)
        np.testing.assert_allclose(np.array(zs), g[p + "bt_z"], atol=1e-11)
        np.testing.assert_allclose(np.array(ws), g[p + "bt_w"], atol=1e-14)


@pytest.mark.parametrize("name", ["highway_n20_nb1", "highway_n8_nb2"])
def test_oracle_ipm_certifies_reference_problems(name):
    """The ECOS-algorithm restatement returns certified optima of the reference problems."""
    from common import cone_problem
    g = golden(name)
    for t in [int(v) for v in g["keep"]][:3]:
        prob = cone_problem(g, t)
        x, info = ecos_solve(prob)
        assert info["exitFlag"] in (0, 10)
        r = kkt_residuals(prob, info["x"], info["y"], info["z"], info["s"])
        if info["exitFlag"] == 0:      # ECOS full accuracy (feastol = abstol = reltol = 1e-8)
            assert r["eq"] < 1e-9 and r["ineq"] < 1e-7 and r["dual"] < 1e-5 and r["cone"] > -1e-6
            assert abs(r["pcost"] - r["dcost"]) <= 1e-6 * max(1.0, abs(r["pcost"]))
        else:                          # ECOS "inaccurate" (feastol 1e-4, abstol / reltol 5e-5)
            assert r["eq"] < 1e-9 and r["ineq"] < 1e-5 and r["dual"] < 1e-4 and r["cone"] > -1e-5
            assert abs(r["pcost"] - r["dcost"]) <= 5e-5 * max(1.0, abs(r["pcost"]))
        assert abs(x[-1] - g[f"s{t}_sol"][-1]) <= 1e-9 * max(1, abs(x[-1]))


def _inject_ws(c, g, t):
    """The warm start the reference controller carried into step t (recorded per step)."""
    topo = c.topo
    c.uLin = g["traj_ws_uLin"][t].copy()
    c.tree = TreeState(topo, c.n, c.d)
    ps = iter(g["traj_ws_p"][t])
    for b in range(topo.nbranch):
        if not topo.is_leaf(b):
            c.tree.p[b] = next(ps).copy()
    c.OldInput = g["traj_ws_old"][t].copy()


def _check_qp(prob, g, t, label):
    p = f"s{t}_"
    for mine, key in ((prob.P, "P"), (prob.A, "A")):
        ref = coo(g, p + key)
        assert mine.shape == ref.shape, (label, t, key)
        diff = abs(mine - ref)
        assert diff.max() <= 1e-12 * max(1.0, abs(ref).max()), (label, t, key, diff.max())
    np.testing.assert_allclose(prob.q, g[p + "q"], rtol=1e-12, atol=1e-12)
    np.testing.assert_array_equal(np.isfinite(prob.l), np.isfinite(g[p + "l"]))
    fin = np.isfinite(g[p + "l"])
    np.testing.assert_allclose(prob.l[fin], g[p + "l"][fin], rtol=1e-12, atol=1e-12)
    np.testing.assert_allclose(prob.u, g[p + "u"], rtol=1e-12, atol=1e-12)


def test_prox_assembly_matches_reference():
    """BranchMPCProx (quadruped): the reference's OSQP (P, q, A, l, u) rebuilt by the oracle."""
    from oracle.model import QuadrupedModel, quadruped_policies
    from oracle.qp_ipm import osqp_like_solve
    from oracle.tree import ProxController
    g = golden("quadruped_n25_nb2")
    for t in (int(k) for k in g["keep"]):
        mdl = QuadrupedModel(int(g["N"]), float(g["dt"]), quadruped_policies(float(g["v0"])), L1=float(g["L1"]),
                             W1=float(g["W1"]), L2=float(g["L2"]), W2=float(g["W2"]), col_tol=float(g["col_tol"]))
        c = ProxController(mdl, int(g["N"]), int(g["NB"]), g["Q"], g["R"], g["dR"], np.zeros((0, 3)), [],
                           g["Fu"], g["bu"], g["Qslack"], g["xRef0"], solver=osqp_like_solve)
        if t > 0:
            _inject_ws(c, g, t)
        prob = c.setup_problem(g["traj_x"][t], g["traj_z"][t], g["traj_xRef"][t])
        _check_qp(prob, g, t, "prox")


def test_branch_qp_assembly_matches_reference():
    """BranchMPC (MPC_branch.py:881, highway): the reference's OSQP problem rebuilt by the oracle."""
    from oracle.qp_ipm import osqp_like_solve
    from oracle.tree import BranchQPController
    g = golden("highway_qp_n8_nb2")
    for t in (int(k) for k in g["keep"]):
        mdl = HighwayModel(int(g["N"]), float(g["dt"]), highway_policies(float(g["Kpsi"]), g["traj_lc_target"][t]),
                           L=float(g["L"]), W=float(g["W"]), s1=float(g["s1"]))
        c = BranchQPController(mdl, int(g["N"]), int(g["NB"]), g["Q"], g["R"], g["dR"], g["Fx"], g["bx"], g["Fu"],
                               g["bu"], g["Qslack"], g["xRef0"], solver=osqp_like_solve)
        if t > 0:
            _inject_ws(c, g, t)
        prob = c.setup_problem(g["traj_x"][t], g["traj_z"][t], g["traj_xRef"][t])
        _check_qp(prob, g, t, "branch-qp")


def _robust(g, t):
    from oracle.qp_ipm import osqp_like_solve
    from oracle.tree import RobustController
    mdl = HighwayModel(int(g["N"]), float(g["dt"]), highway_policies(float(g["Kpsi"]), g["traj_lc_target"][t]),
                       L=float(g["L"]), W=float(g["W"]), s1=float(g["s1"]))
    return RobustController(mdl, int(g["N"]), int(g["NB"]), g["Q"], g["R"], g["dR"], g["Fx"], g["bx"], g["Fu"],
                            g["bu"], g["Qslack"], g["xRef0"], Qf=g["Qf"], solver=osqp_like_solve)


@pytest.mark.parametrize("name", ["highway_robust_n20_nb1", "highway_robust_n8_nb2"])
def test_robust_assembly_matches_reference(name):
    """robustMPC (MPC_branch.py:1275): the reference's OSQP problem rebuilt by the oracle from
    the warm start it carried (shifted prediction, OldInput), and its obstacle tree."""
    g = golden(name)
    for t in (int(k) for k in g["keep"]):
        c = _robust(g, t)
        if t > 0:
            c.xLin = g["traj_ws_xLin"][t].copy()
            c.uLin = g["traj_ws_uLin"][t].copy()
            c.OldInput = g["traj_ws_old"][t].copy()
        prob = c.setup_problem(g["traj_x"][t], g["traj_z"][t], g["traj_xRef"][t])
        _check_qp(prob, g, t, name)
        np.testing.assert_allclose(np.array(c.ztraj), g[f"s{t}_bt_z"], rtol=0, atol=1e-12)


def test_robust_closed_loop_replay():
    """The oracle robustMPC driven through the recorded loop: its warm start after each step
    equals the reference's (shifted prediction to 1e-7, the OSQP stand-in's tolerance)."""
    g = golden("highway_robust_n8_nb2")
    c = _robust(g, 0)
    for t in range(6):
        c.model.update_backup(highway_policies(float(g["Kpsi"]), g["traj_lc_target"][t]))
        c.solve(g["traj_x"][t], g["traj_z"][t], g["traj_xRef"][t])
        np.testing.assert_allclose(c.uPred, g["traj_uPred"][t], atol=1e-7)
        np.testing.assert_allclose(c.xPred, g["traj_xPred"][t], atol=1e-7)
        assert c.feasible == 1 and g["traj_status"][t] == 1
