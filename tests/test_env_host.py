"""The closed-loop sim_overtake scene (csrc/bmpc_env.h, host build -- TEST-ONLY) against the
reference's recorded closed loop.

tools/gen_golden.py ran the reference's own BranchMPC_CVaR inside the oracle restatement of
Highway_env.step (oracle/env.py; Highway_env_branch.py:83-184) and recorded, per step, the
solve's inputs x, z, x_ref, the lane-change target of update_backup and the control u it
applied.  Driving the scene with the recorded u must reproduce every recorded input of the
next solve: obstacle backup choice (argmax of the clipped NumPy veh_col / lane_bdry_h),
lane bookkeeping, re-targeting, x_ref rule and Euler steps.  Tolerance 1e-9 (transcendentals
of a different libm).
"""
import numpy as np
import pytest

import hostsim_lib as H
from bmpc import abi
from common import golden, highway_desc_from_golden, highway_policy_rows


def scene_for(g, B):
    scene = np.zeros((B, abi.ENV_STRIDE))
    scene[:, abi.ENV_X:abi.ENV_X + 4] = g["traj_x"][0]
    scene[:, abi.ENV_Z:abi.ENV_Z + 4] = g["traj_z"][0]
    return scene


def env_for(g):
    return abi.make_env(n_lane=int(g["N_lane"]), L=float(g["L"]), W=float(g["W"]), Kpsi=float(g["Kpsi"]),
                        target=np.asarray(g["xRef0"], float))


def replay_env(step_fn, g, steps, policies_fn):
    """Drive a scene with the recorded controls; compare every recorded solve input."""
    for t in range(steps):
        u = None if t == 0 else np.asarray(g["traj_u"][t - 1], float)
        x, z, xref = step_fn(t, u)
        np.testing.assert_allclose(x[0], g["traj_x"][t], rtol=0, atol=1e-9, err_msg=f"x step {t}")
        np.testing.assert_allclose(z[0], g["traj_z"][t], rtol=0, atol=1e-9, err_msg=f"z step {t}")
        np.testing.assert_allclose(xref[0], g["traj_xRef"][t], rtol=0, atol=1e-9, err_msg=f"xRef step {t}")
        pol = policies_fn()
        np.testing.assert_allclose(np.array(pol[2].p[:]), g["traj_lc_target"][t], atol=1e-12,
                                   err_msg=f"lc target step {t}")


@pytest.mark.parametrize("name,steps", [("highway_n8_nb2", 40), ("highway_n20_nb1", 100), ("highway_n10_nb1", 20)])
def test_host_env_replays_reference_loop(name, steps):
    g = golden(name)
    steps = min(steps, len(g["traj_x"]))
    hs = H.HostSim(highway_desc_from_golden(g), 1)
    hs.set_policies(highway_policy_rows(np.asarray(g["xRef0"], float)[None], float(g["Kpsi"])))
    scene = scene_for(g, 1)
    env = env_for(g)

    def step(t, u):
        up = None
        if u is not None:
            up = np.zeros((1, hs.U, 2))
            up[0, 0] = u
        return hs.env_step(env, t, scene, up)

    replay_env(step, g, steps, hs.get_policies)
    # Highway_sim's collision flag (recorded after the check of each step)
    assert bool(scene[0, abi.ENV_COLL]) == bool(g["traj_collision"][steps - 1])


def test_host_env_statistics():
    g = golden("highway_n10_nb1")
    B = 3
    hs = H.HostSim(highway_desc_from_golden(g), B)
    hs.set_policies(highway_policy_rows(np.repeat(np.asarray(g["xRef0"], float)[None], B, 0), float(g["Kpsi"])))
    scene = scene_for(g, B)
    stats = np.zeros((B, abi.ENV_NSTAT))
    env = env_for(g)
    up = np.zeros((B, hs.U, 2))
    J = np.array([1.0, 2.0, 3.0])
    st = np.array([0, -1, 10], np.int32)
    it = np.array([20, 21, 22], np.int32)
    hs.env_step(env, 0, scene, None, J, st, it, stats)
    assert not stats.any()                      # t = 0: no solve yet
    hs.env_step(env, 1, scene, up, J, st, it, stats)
    np.testing.assert_array_equal(stats[:, abi.ENVS_J], J)
    np.testing.assert_array_equal(stats[:, abi.ENVS_J2], J * J)
    np.testing.assert_array_equal(stats[:, abi.ENVS_INFEAS], [0, 1, 0])   # ECOS: exitFlag >= 0 feasible
    np.testing.assert_array_equal(stats[:, abi.ENVS_ITERS], it)
    np.testing.assert_array_equal(stats[:, abi.ENVS_SOLVES], 1)
