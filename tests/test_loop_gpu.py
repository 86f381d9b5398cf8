"""The fused closed loop (bmpc_loop_device, k_loop): K steps of every ego in one launch give the
same bits as K rounds of bmpc_env_step + bmpc_solve_device (k_env, k_tree, k_ipm launched per
step) -- the scene, the plan's last outputs, the statistics and the warm start carried between
calls -- and a loop split over several calls is the same loop."""
import numpy as np
import pytest

from bmpc import abi
from common import highway_desc, highway_policy_rows, seeded_batch

pytestmark = pytest.mark.gpu

B = 300   # more egos than CUs: the batch takes the one-wave k_ipm, so the loop is fused


def _run(torch, chunks, monkeypatch, fused_env=None):
    from bmpc import plan
    for k in ("BMPC_BLOCK_EGOS", "BMPC_LDS_RICH", "BMPC_LOOP_FUSED"):
        monkeypatch.delenv(k, raising=False)
    if fused_env is not None:
        monkeypatch.setenv("BMPC_LOOP_FUSED", fused_env)
    x, z, xref, tgt = seeded_batch(B, seed=5)
    pl = plan.BatchPlan(highway_desc(N=20, NB=1), B)
    pl.set_policies(highway_policy_rows(tgt))
    dev = torch.device("cuda", 0)
    f64 = dict(dtype=torch.float64, device=dev)
    scene = torch.zeros((B, abi.ENV_STRIDE), **f64)
    scene[:, 0:4] = torch.tensor(x)
    scene[:, 4:8] = torch.tensor(z)
    up = torch.zeros((B, pl.U, 2), **f64)
    J = torch.zeros(B, **f64)
    st = torch.zeros(B, dtype=torch.int32, device=dev)
    it = torch.zeros(B, dtype=torch.int32, device=dev)
    stats = torch.zeros((B, abi.ENV_NSTAT), **f64)
    tx, tz, tr = (torch.zeros((B, 4), **f64) for _ in range(3))
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    s = stream.cuda_stream
    env = abi.make_env()
    t = 0
    kernels = []
    for c in chunks:
        if c == "step":   # one step as its two launches
            pl.env_step_device(env, t, scene.data_ptr(), up.data_ptr(), tx.data_ptr(), tz.data_ptr(), tr.data_ptr(),
                               J.data_ptr(), st.data_ptr(), it.data_ptr(), stats.data_ptr(), stream=s)
            pl.solve_device(tx.data_ptr(), tz.data_ptr(), tr.data_ptr(), up.data_ptr(), None, None, J.data_ptr(),
                            st.data_ptr(), it.data_ptr(), s)
            t += 1
        else:
            pl.loop_device(env, t, c, scene.data_ptr(), up.data_ptr(), tx.data_ptr(), tz.data_ptr(), tr.data_ptr(),
                           J.data_ptr(), st.data_ptr(), it.data_ptr(), stats.data_ptr(), s)
            t += c
        torch.cuda.synchronize()
        kernels.append(pl.last_kernel())
    out = {k: v.cpu().numpy().copy() for k, v in dict(scene=scene, up=up, J=J, st=st, it=it, stats=stats, x=tx, z=tz,
                                                         xref=tr).items()}
    out["ws"] = pl.get_warm_start()
    return out, kernels


def _same(a, b):
    for k in a:
        if k == "ws":
            for kk in a[k]:
                assert np.array_equal(a[k][kk], b[k][kk]), ("warm start", kk)
        else:
            assert np.array_equal(a[k], b[k]), k


def test_fused_loop_equals_per_step_launches(monkeypatch):
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    ref, kr = _run(torch, ["step"] * 5, monkeypatch)
    assert set(kr) == {abi.KERNEL_IPM_RICH}, kr
    fused, kf = _run(torch, [5], monkeypatch)
    assert kf == [abi.KERNEL_LOOP_RICH], kf
    _same(ref, fused)
    split, ks = _run(torch, [2, 3], monkeypatch)          # a loop continued over calls
    assert ks == [abi.KERNEL_LOOP_RICH] * 2, ks
    _same(ref, split)
    mixed, _ = _run(torch, ["step", 4], monkeypatch)        # t0 > 0 after a per-step start
    _same(ref, mixed)
    steps, kp = _run(torch, [5], monkeypatch, fused_env="0")   # the per-step path of the same call
    assert kp == [abi.KERNEL_IPM_RICH], kp
    _same(ref, steps)
    assert np.all(ref["st"] >= 0) and ref["stats"][:, abi.ENVS_SOLVES].min() == 4


def test_loop_rejects_other_plans():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from bmpc import plan
    from bmpc.scenarios import quadruped_desc
    pl = plan.BatchPlan(quadruped_desc(), 4)
    with pytest.raises(RuntimeError, match="overtake scene"):
        pl.loop_device(abi.make_env(), 0, 1, 1, 1, 1, 1, 1, 1, 1, 1)
