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
    stats[D.STAT_ANY_COLLIDED] = float(rank == 1)          # a flag only one rank raises
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
    assert s0[D.STAT_ANY_COLLIDED] == 1.0                 # MAX, not the sum over ranks
    assert t0 == t1 == 2.0


def test_shard_covers_population():
    from bmpc.distributed import shard
    for total in (1, 7, 4096, 65536):
        for world in (1, 2, 3, 8):
            spans = [shard(total, r, world) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == total
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))


def _episode(lo, hi, total, steps, N=10, NB=1):
    """The bench's closed loop on the host build for egos [lo, hi) of the seeded population:
    device-scene step (host build of k_env) -> solve, per-ego statistics summed over the shard."""
    import hostsim_lib as H
    from bmpc import abi
    from bmpc.scenarios import highway_desc, highway_policy_rows, seeded_batch
    x, z, xref, tgt = (v[lo:hi] for v in seeded_batch(total, seed=0))
    B = hi - lo
    hs = H.HostSim(highway_desc(N=N, NB=NB), B)
    hs.set_policies(highway_policy_rows(tgt))
    env = abi.make_env()
    scene = np.zeros((B, abi.ENV_STRIDE))
    scene[:, 0:4], scene[:, 4:8] = x, z
    estats = np.zeros((B, abi.ENV_NSTAT))
    r = None
    for t in range(steps + 1):
        if r is None:
            x, z, xref = hs.env_step(env, t, scene)
        else:
            x, z, xref = hs.env_step(env, t, scene, r["upred"], r["J"], r["status"], r["iters"], estats)
        r = hs.solve(x, z, xref)
    from bmpc import distributed as D
    return D.episode_stats(estats)


def _loop_worker(rank, world, port, total, steps, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), OMP_NUM_THREADS="1")
    import torch
    import torch.distributed as dist
    from bmpc import distributed as D
    D.init("gloo")
    lo, hi = D.shard(total, rank, world)
    stats = torch.tensor(_episode(lo, hi, total, steps), dtype=torch.float64)
    D.reduce_stats(stats)                     # the bench's only collective
    out[rank] = stats.numpy().copy()
    dist.destroy_process_group()


def test_two_rank_sharded_closed_loop_matches_single_rank():
    """Two gloo ranks each run the real closed loop (host build of the kernels and the
    device scene) on their contiguous shard; the all-reduced statistics equal one rank
    running the whole population."""
    from bmpc import abi
    total, world, steps = 9, 2, 3
    port = _free_port()
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_loop_worker, args=(world, port, total, steps, out), nprocs=world, join=True)
    ref = _episode(0, total, total, steps)
    np.testing.assert_array_equal(out[0], out[1])
    assert ref[abi.ENVS_SOLVES] == total * steps
    np.testing.assert_allclose(out[0], ref, rtol=1e-12, atol=1e-9)
