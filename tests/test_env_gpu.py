"""Device closed-loop scene (bmpc_env_step, k_env) against the reference's recorded loop,
and the fully on-device closed loop (env -> tree -> IPM, no host round trip).

Same replay as tests/test_env_host.py, through the C ABI on the GPU: the recorded controls
drive the scene; every recorded solve input (x, z, x_ref, lane-change target) must come back
to 1e-9.  The closed-loop test then lets the GPU controller drive the scene from the
sim_overtake start and compares the first 20 steps with the recording.  The ego state is
held to 1e-4: the solver reproduces uPred[0] to 1e-4 on exit-0 steps and 5e-3 on "inaccurate"
exit-10 steps (tests/test_kernel_host.py), and the recording has exit-10 steps, so the
SURVEY §8(c) 1e-6 closed-loop figure is not attainable once such a step enters the loop
(observed: 2.4e-6 after 7 steps); the obstacle, whose inputs are discrete backup choices,
must follow to 1e-9."""
import numpy as np
import pytest

from bmpc import abi
from common import golden, highway_desc_from_golden, highway_policy_rows

pytestmark = pytest.mark.gpu


def _torch():
    import torch
    assert torch.cuda.is_available()
    return torch


def _plan(g, B):
    from bmpc import plan
    pl = plan.BatchPlan(highway_desc_from_golden(g), B)
    pl.set_policies(highway_policy_rows(np.repeat(np.asarray(g["xRef0"], float)[None], B, 0), float(g["Kpsi"])))
    return pl


def _env(g):
    return abi.make_env(n_lane=int(g["N_lane"]), L=float(g["L"]), W=float(g["W"]), Kpsi=float(g["Kpsi"]),
                        target=np.asarray(g["xRef0"], float))


@pytest.mark.parametrize("name,steps", [("highway_n8_nb2", 40), ("highway_n20_nb1", 100)])
def test_device_env_replays_reference_loop(name, steps):
    torch = _torch()
    g = golden(name)
    steps = min(steps, len(g["traj_x"]))
    B = 4                                   # identical scenes: every ego must agree
    pl = _plan(g, B)
    env = _env(g)
    dev = torch.device("cuda", 0)
    scene = torch.zeros((B, abi.ENV_STRIDE), dtype=torch.float64, device=dev)
    scene[:, 0:4] = torch.tensor(g["traj_x"][0], dtype=torch.float64)
    scene[:, 4:8] = torch.tensor(g["traj_z"][0], dtype=torch.float64)
    up = torch.zeros((B, pl.U, 2), dtype=torch.float64, device=dev)
    x, z, xr = (torch.zeros((B, 4), dtype=torch.float64, device=dev) for _ in range(3))
    stream = torch.cuda.Stream(dev)       # kernels and torch ops in order on one stream
    torch.cuda.set_stream(stream)
    s = stream.cuda_stream
    for t in range(steps):
        if t > 0:
            up[:, 0, :] = torch.tensor(g["traj_u"][t - 1], dtype=torch.float64)
        pl.env_step_device(env, t, scene.data_ptr(), up.data_ptr(), x.data_ptr(), z.data_ptr(), xr.data_ptr(),
                           stream=s)
        torch.cuda.synchronize()
        for name_, v, key in (("x", x, "traj_x"), ("z", z, "traj_z"), ("xRef", xr, "traj_xRef")):
            np.testing.assert_allclose(v.cpu().numpy(), np.repeat(np.asarray(g[key][t])[None], B, 0),
                                       rtol=0, atol=1e-9, err_msg=f"{name_} step {t}")
    assert bool(scene[0, abi.ENV_COLL].item()) == bool(g["traj_collision"][steps - 1])


def test_device_closed_loop_follows_reference(solver_path):
    """env -> solve on the device for 20 steps from the sim_overtake start (highway_n20_nb1
    recording: N=20, NB=1, the metric configuration)."""
    torch = _torch()
    g = golden("highway_n20_nb1")
    T = 20
    B = 2
    pl = _plan(g, B)
    env = _env(g)
    dev = torch.device("cuda", 0)
    f64 = dict(dtype=torch.float64, device=dev)
    scene = torch.zeros((B, abi.ENV_STRIDE), **f64)
    scene[:, 0:4] = torch.tensor(g["traj_x"][0], dtype=torch.float64)
    scene[:, 4:8] = torch.tensor(g["traj_z"][0], dtype=torch.float64)
    up = torch.zeros((B, pl.U, 2), **f64)
    J = torch.zeros(B, **f64)
    st = torch.zeros(B, dtype=torch.int32, device=dev)
    it = torch.zeros(B, dtype=torch.int32, device=dev)
    stats = torch.zeros((B, abi.ENV_NSTAT), **f64)
    x, z, xr = (torch.zeros((B, 4), **f64) for _ in range(3))
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    s = stream.cuda_stream
    xs, zs = [], []
    for t in range(T):
        pl.env_step_device(env, t, scene.data_ptr(), up.data_ptr(), x.data_ptr(), z.data_ptr(), xr.data_ptr(),
                           J.data_ptr(), st.data_ptr(), it.data_ptr(), stats.data_ptr(), stream=s)
        xs.append(x.cpu().numpy().copy())
        zs.append(z.cpu().numpy().copy())
        pl.solve_device(x.data_ptr(), z.data_ptr(), xr.data_ptr(), up.data_ptr(), None, None, J.data_ptr(),
                        st.data_ptr(), it.data_ptr(), s)
    torch.cuda.synchronize()
    from conftest import assert_solver_path
    assert_solver_path(pl, solver_path)
    for t in range(T):
        # (steps 2-3 of the recording exit 10, "inaccurate": their optimum is defined only to ECOS's
        # reduced 5e-5 gap, and the host build's uPred[0] moves 5e-5 there; the state then differs
        # by 5e-6 and decays to ~1e-6 -- every other step exits 0 on both sides)
        np.testing.assert_allclose(xs[t], np.repeat(np.asarray(g["traj_x"][t])[None], B, 0), rtol=0, atol=2e-5,
                                   err_msg=f"closed-loop x at step {t}")
        np.testing.assert_allclose(zs[t], np.repeat(np.asarray(g["traj_z"][t])[None], B, 0), rtol=0, atol=1e-9,
                                   err_msg=f"closed-loop z at step {t}")
    sh = stats.cpu().numpy()
    assert np.all(sh[:, abi.ENVS_SOLVES] == T - 1) and np.all(sh[:, abi.ENVS_INFEAS] == 0)
