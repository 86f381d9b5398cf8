"""N > 1 path on CPU: two gloo ranks shard a seeded ego population, accumulate closed-loop
statistics, and reduce them exactly as bench.py does over RCCL on GPUs."""
import os
import socket

import numpy as np
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, total, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import torch
    from bmpc import distributed as D
    from bmpc.scenarios import seeded_batch
    r, _, ws = D.init("gloo")
    assert (r, ws) == (rank, world)
    lo, hi = D.shard(total, rank, world)
    x, z, xref, _ = seeded_batch(total, seed=0)
    stats = torch.zeros(D.NSTAT, dtype=torch.float64)
    stats[D.STAT_J] = float(x[lo:hi, 2].sum())            # stand-in per-ego values
    stats[D.STAT_SOLVES] = hi - lo
    stats[D.STAT_COLL] = float((np.abs(x[lo:hi, 0] - z[lo:hi, 0]) < 4).sum())
    D.reduce_stats(stats)
    t = D.max_over_ranks(float(rank + 1))
    out[rank] = (stats.numpy().copy(), t, lo, hi)
    import torch.distributed as dist
    dist.destroy_process_group()


def test_two_rank_shard_and_reduce():
    total, world = 1001, 2
    port = _free_port()
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, port, total, out), nprocs=world, join=True)
    from bmpc import distributed as D
    from bmpc.scenarios import seeded_batch
    x, z, _, _ = seeded_batch(total, seed=0)
    (s0, t0, lo0, hi0), (s1, t1, lo1, hi1) = out[0], out[1]
    assert (lo0, hi0, lo1, hi1) == (0, 501, 501, 1001)
    np.testing.assert_array_equal(s0, s1)                 # every rank holds the reduced vector
    assert s0[D.STAT_SOLVES] == total
    np.testing.assert_allclose(s0[D.STAT_J], x[:, 2].sum(), rtol=1e-12)
    assert s0[D.STAT_COLL] == (np.abs(x[:, 0] - z[:, 0]) < 4).sum()
    assert t0 == t1 == 2.0


def test_shard_covers_population():
    from bmpc.distributed import shard
    for total in (1, 7, 4096, 65536):
        for world in (1, 2, 3, 8):
            spans = [shard(total, r, world) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == total
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
