"""The small-batch kernel's LDS-resident spans (bmpc_hip.hip blk_layouts, bmpc_dev.h k_solve_blk;
DESIGN §2.4): per-ego layouts move spans of the IPM's own arrays from the ego's slab to the
workgroup's LDS.  Only where the values live changes, so a seeded batch on the small-batch path
gives the same bits with and without them (BMPC_BLK_LDS, read on every launch), over closed-loop
steps, on both wave counts' trees."""
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
