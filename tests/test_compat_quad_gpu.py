"""main_quadruped.py's controller through the drop-in surface (Init_MPC.initquadBranchMPC +
quadruped PredictiveModel + BranchMPCProx) in the closed loop the golden fixture recorded
(tools/gen_golden.py: the reference's quadruped_env rules, whose own loop crashes at
quadruped_env.py:120).  uPred[0] to 1e-6 on every one of the 40 steps."""
import numpy as np
import pytest

from common import golden

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")


def test_main_quadruped_loop(gpu):
    import Init_MPC
    import MPC_branch
    from quadruped_branch_dyn import PredictiveModel, backup_forward, backup_stop
    from utils import Quad_constants
    g = golden("quadruped_n25_nb2")
    dt, NB, vxm, vym, rm, v0, n, d, N = 0.2, 2, 0.2, 0.1, 0.5, 0.2, 3, 3, 25
    cons = Quad_constants(s1=2, s2=3, c2=0.5, alpha=1, R=1.2, vxm=vxm, vym=vym, rm=rm, L1=0.5, W1=0.3, L2=1,
                          W2=0.6, col_tol=0.2, col_alpha=5)
    model = PredictiveModel(n, d, N, [lambda x: backup_forward(x, v0), lambda x: backup_stop(x)], dt, cons)
    mpc = MPC_branch.BranchMPCProx(Init_MPC.initquadBranchMPC(n, d, N, NB, np.array([5., 5., 0.]), vxm, vym, rm),
                                   model)
    for t in range(len(g["traj_x"])):
        mpc.solve(g["traj_x"][t], g["traj_z"][t], g["traj_xRef"][t])
        assert mpc.feasible == 1, t
        np.testing.assert_allclose(mpc.uPred[0], g["traj_u"][t], atol=1e-6, err_msg=f"step {t}")
    xs, zs, us, ws = mpc.BT2array()
    assert len(xs) == 6 and xs[0].shape == (N + 1, n)
