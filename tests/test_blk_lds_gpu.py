"""The small-batch kernel's LDS-resident spans (bmpc_hip.hip blk_layouts, bmpc_dev.h k_solve_blk;
DESIGN §2.4): per-ego layouts move spans of the IPM's own arrays from the ego's slab to the
workgroup's LDS.  Only where the values live changes, so a seeded batch on the small-batch path
gives the same bits with and without them (BMPC_BLK_LDS, read on every launch), over closed-loop
steps, on both wave counts' trees -- and on every translation unit that uses the relocated
layouts (bmpc_kb_*.hip): the plain highway model, the highway model's transform plans (per-ego S
/ Fx / bx), the merge model (S and bx from the reference's merge recording) and a quadruped CVaR
plan."""
import numpy as np
import pytest

from common import highway_desc, highway_policy_rows, seeded_batch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from bmpc import plan
    return plan


def _loop(gpu, desc, B, steps, monkeypatch, lds):
    from bmpc import abi
    monkeypatch.setenv("BMPC_BLK_LDS", "1" if lds else "0")
    x, z, xref, tgt = seeded_batch(B, seed=3)
    pl = gpu.BatchPlan(desc, B)
    pl.set_policies(highway_policy_rows(tgt))
    out = []
    for _ in range(steps):
        r = pl.solve(x, z, xref)
        assert pl.last_kernel() in (abi.KERNEL_IPM_BLK4, abi.KERNEL_IPM_BLK8)
        assert (r["status"] >= 0).all(), r["status"]
        out.append({k: np.array(r[k]) for k in ("status", "iters", "J", "upred")})
        u0 = r["upred"][:, 0]
        x = x + 0.1 * np.stack([x[:, 2] * np.cos(x[:, 3]), x[:, 2] * np.sin(x[:, 3]), u0[:, 0], u0[:, 1]], 1)
        z = z + 0.1 * np.stack([z[:, 2], 0 * z[:, 0], 0 * z[:, 0], 0 * z[:, 0]], 1)
    return out


@pytest.mark.parametrize("N,NB,B", [(20, 1, 3), (8, 2, 2), (30, 2, 1)])
def test_blk_lds_spans_bit_identical(gpu, monkeypatch, N, NB, B):
    for k in ("BMPC_BLOCK_EGOS", "BMPC_LDS_RICH", "BMPC_BLOCK_WAVES"):
        monkeypatch.delenv(k, raising=False)
    desc = highway_desc(N, NB)
    a = _loop(gpu, desc, B, 3, monkeypatch, True)
    b = _loop(gpu, desc, B, 3, monkeypatch, False)
    for s, (ra, rb) in enumerate(zip(a, b)):
        for k in ra:
            assert np.array_equal(ra[k], rb[k]), (N, NB, s, k, ra[k], rb[k])


def _loop_generic(gpu, make, steps, monkeypatch, lds):
    """make() -> (plan, x, z, xref, setup): setup(plan) before each solve (transform arguments)."""
    from bmpc import abi
    monkeypatch.setenv("BMPC_BLK_LDS", "1" if lds else "0")
    pl, x, z, xref, setup = make(gpu)
    out = []
    for _ in range(steps):
        setup(pl)
        r = pl.solve(x, z, xref)
        assert pl.last_kernel() in (abi.KERNEL_IPM_BLK4, abi.KERNEL_IPM_BLK8)
        assert (r["status"] >= 0).all(), r["status"]
        out.append({k: np.array(r[k]) for k in ("status", "iters", "J", "upred")})
    return out


def _highway_transform(gpu):
    from bmpc import abi
    B = 2
    x, z, xref, tgt = seeded_batch(B, seed=4)
    desc = highway_desc(8, 2)
    desc.flags = abi.PLAN_TRANSFORM
    pl = gpu.BatchPlan(desc, B)
    pl.set_policies(highway_policy_rows(tgt))
    S = np.repeat(np.array([[1.0, 0, 0, 0], [0, 0.98, 0.01, 0], [0, 0, 1, 0], [0, 0, 0.05, 1]])[None], B, 0)
    Fx = np.repeat((np.diag([1.0, 1.0, 2.0, 2.0]) @ np.array([[0., 1, 0, 0], [0, -1, 0, 0], [0, 0, 0, 1],
                                                               [0, 0, 0, -1]]))[None], B, 0)

    def setup(p):
        p.set_fx(Fx)
        p.set_transform(S, np.repeat(np.array([[4 * 3.6 - 1.0, -1.0, 0.2, 0.2]]), B, 0))
    return pl, x, z, xref, setup


def _merge(gpu):
    from common import golden
    from test_merge import merge_desc, merge_rows, replay_inputs
    g = golden("merge_n40_nb1")
    rb = replay_inputs(g, 2)
    pl = gpu.BatchPlan(merge_desc(g), rb["T"])
    pl.set_policies(merge_rows(g, rb["T"]))

    def setup(p):
        p.set_transform(rb["S"], rb["bx"])
    return pl, rb["x"], rb["z"], rb["xref"], setup


def _quadruped_cvar(gpu):
    from bmpc import abi
    from bmpc.scenarios import quadruped_policy_rows, seeded_quadruped_batch
    B = 2
    Fu = np.kron(np.eye(3), np.array([1, -1])).T
    desc = abi.make_desc(abi.CTRL_CVAR, abi.MODEL_QUADRUPED, 3, 3, 10, 2, 2, 0.2, np.eye(3), np.diag([1., 100., 1.]),
                         np.zeros((0, 3)), [], Fu, [0.2, 0.0, 0.1, 0.1, 0.5, 0.5], [0., 300.],
                         [0.5, 0.3, 1.0, 0.6, 0.2, 2.0], dR=[0.9, 5.0, 1.0])
    x, z, xref = seeded_quadruped_batch(B)
    pl = gpu.BatchPlan(desc, B)
    pl.set_policies(quadruped_policy_rows(B))
    return pl, x, z, xref, lambda p: None


@pytest.mark.parametrize("case", ["highway_transform", "merge", "quadruped_cvar"])
def test_blk_lds_spans_bit_identical_other_units(gpu, monkeypatch, case):
    for k in ("BMPC_BLOCK_EGOS", "BMPC_LDS_RICH", "BMPC_BLOCK_WAVES"):
        monkeypatch.delenv(k, raising=False)
    make = {"highway_transform": _highway_transform, "merge": _merge, "quadruped_cvar": _quadruped_cvar}[case]
    a = _loop_generic(gpu, make, 2, monkeypatch, True)
    b = _loop_generic(gpu, make, 2, monkeypatch, False)
    for s, (ra, rb) in enumerate(zip(a, b)):
        for k in ra:
            assert np.array_equal(ra[k], rb[k]), (case, s, k, ra[k], rb[k])
