"""Drop-in Python surface, host-side parts: Init_MPC numbers (against the values the
reference's own Init_MPC produced, recorded in the golden fixtures), backup-lambda tracing
into policy descriptors, and the plan description the controller hands to the C ABI."""
import numpy as np

from common import golden


def test_init_branch_mpc_matches_reference_values():
    import Init_MPC
    for name in ("highway_n20_nb1", "highway_n8_nb2"):
        g = golden(name)
        p = Init_MPC.initBranchMPC(4, 2, int(g["N"]), int(g["NB"]), g["xRef0"], float(g["am"]), float(g["rm"]),
                                   int(g["N_lane"]), float(g["W"]))
        np.testing.assert_array_equal(p.Q, g["Q"])
        np.testing.assert_array_equal(p.R, g["R"])
        np.testing.assert_array_equal(p.Fx, g["Fx"])
        np.testing.assert_array_equal(np.asarray(p.bx, float).reshape(-1), g["bx"])
        assert isinstance(p.bx, tuple) and len(p.bx) == 1        # trailing-comma quirk (Init_MPC.py:48-51)
        np.testing.assert_array_equal(p.Fu, g["Fu"])
        np.testing.assert_array_equal(np.asarray(p.bu, float).reshape(-1), g["bu"])
        np.testing.assert_array_equal(p.Qslack, g["Qslack"])


def test_init_quad_branch_mpc_matches_reference_values():
    import Init_MPC
    g = golden("quadruped_n25_nb2")
    p = Init_MPC.initquadBranchMPC(3, 3, int(g["N"]), int(g["NB"]), g["xRef0"], float(g["vxm"]), float(g["vym"]),
                                   float(g["rm"]))
    np.testing.assert_array_equal(p.Q, g["Q"])
    np.testing.assert_array_equal(p.R, g["R"])
    np.testing.assert_array_equal(p.dR, g["dR"])
    np.testing.assert_array_equal(p.Fu, g["Fu"])
    np.testing.assert_array_equal(np.asarray(p.bu, float).reshape(-1), g["bu"])


def test_backup_lambdas_trace_to_descriptors():
    from bmpc import abi
    from bmpc.tracing import trace
    from highway_branch_dyn import backup_brake, backup_lc, backup_maintain
    from utils import Branch_constants
    cons = Branch_constants(s1=2, s2=3, c2=0.5, tran_diag=0.3, alpha=1, R=1.2, am=6.0, rm=0.3, J_c=20, s_c=1,
                            ylb=0., yub=7.2, L=4, W=2.5, col_alpha=5, Kpsi=0.1)
    xRef = np.array([0.5, 1.8, 15, 0])
    pols = trace([lambda x: backup_maintain(x, cons), lambda x: backup_brake(x, cons), lambda x: backup_lc(x, xRef)])
    rows = [p.as_row() for p in pols]
    assert rows[0][0] == abi.POL_MAINTAIN and rows[0][1][0] == 0.1
    assert rows[1][0] == abi.POL_BRAKE and rows[1][1][0] == 0.1
    assert rows[2][0] == abi.POL_LC and tuple(rows[2][1]) == tuple(xRef)
    # the numpy path of the traced functions still works for the env (Highway_env_branch :137-149)
    u = backup_lc(np.array([0, 1.8, 18, 0.1]), xRef)
    np.testing.assert_allclose(u, [-0.8558 * (18 - 15), -0.3162 * (1.8 - 1.8) - 3.9889 * (0.1 - 0)])


def test_cvar_controller_plan_description():
    """BranchMPC_CVaR builds the same plan description as the test helper (no GPU touched)."""
    import Init_MPC
    import MPC_branch
    from highway_branch_dyn import PredictiveModel, backup_brake, backup_lc, backup_maintain
    from utils import Branch_constants
    from common import highway_desc
    cons = Branch_constants(s1=2, s2=3, c2=0.5, tran_diag=0.3, alpha=1, R=1.2, am=6.0, rm=0.3, J_c=20, s_c=1,
                            ylb=0., yub=7.2, L=4, W=2.5, col_alpha=5, Kpsi=0.1)
    xRef = np.array([0.5, 1.8, 15, 0])
    model = PredictiveModel(4, 2, 20, [lambda x: backup_maintain(x, cons), lambda x: backup_brake(x, cons),
                                       lambda x: backup_lc(x, xRef)], 0.1, cons)
    param = Init_MPC.initBranchMPC(4, 2, 20, 1, xRef, 6.0, 0.3, 4, cons.W)
    mpc = MPC_branch.BranchMPC_CVaR(param, model, ralpha=0.9)
    d, ref = mpc.plan_desc(), highway_desc(N=20, NB=1)
    for f in ("controller", "model", "n", "d", "N", "NB", "m", "nFx", "nFu"):
        assert getattr(d, f) == getattr(ref, f), f
    for f in ("Q", "R", "Fx", "bx", "Fu", "bu", "Qslack", "mc"):
        np.testing.assert_array_equal(np.array(getattr(d, f)), np.array(getattr(ref, f)), err_msg=f)
    assert d.ralpha == 0.9 and d.dt == 0.1
