"""Headline benchmark: branch-MPC solves/sec, highway N=20, 3 branches, 4096 egos per GPU.

One step = one closed-loop step of every ego: the batched BranchMPC_CVaR solve (tree update,
linearisation, structured IPM) followed by the device-side Euler step of ego and obstacle
and the x_ref rule of Highway_env.step.  Inputs stay in HBM (torch tensors on cuda).
Multi-GPU: one process per GPU, egos sharded (weak scaling), one RCCL all-reduce of the
closed-loop statistics per episode.  Rank 0 prints one JSON line.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
for _p in (REPO, os.path.join(REPO, "belief-planning_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import numpy as np  # noqa: E402

METRIC = "branch-MPC solves/sec (whole node), highway N=20 M=3 branches, batch 4096 egos"
FP64_PEAK_TFLOPS = 78.6     # MI355X FP64 vector (= FP64 matrix) peak, spec
HBM_PEAK_TBPS = 8.0         # MI355X HBM3E peak, spec (MI355X_MICROARCH.md)


def flops_per_iter(T, n, d, Nc, nFu, cone_dims):
    """SURVEY §8(d) F_iter (transcendentals = 1)."""
    per_node = (2 * (2 * n ** 3 + 3 * n ** 2 * d + 2 * n * d ** 2 + d ** 3 / 3.0) + 2 * Nc * n ** 2
                + 4 * 2 * (2 * n ** 2 + 2 * n * d + d ** 2) + 2 * (2 * n ** 2 + 2 * n * d)
                + 10 * (n + d + 2 * Nc + nFu))
    return T * per_node + sum(20 * q for q in cone_dims)


def flops_model(U, Bn, bdim, m, N, n):
    """SURVEY §8(d) F_model."""
    return (U + Bn) * 40 + bdim * (m * N * 60 + (2 * N * m * 50) * (1 + n)) + U * 30


def usable_cores():
    """Host cores this process may use: the affinity mask, capped by the cgroup CPU quota
    and by OMP_NUM_THREADS when set (the GPU box grants a 16-CPU share of a larger host)."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()
        if q != "max":
            quota = max(1, int(int(q) / int(per)))
    except (OSError, ValueError):
        pass
    env = os.environ.get("OMP_NUM_THREADS")
    n = min(v for v in (aff, quota, int(env) if env and env.isdigit() else None) if v)
    return n, aff, quota


def cpu_cxx_baseline(N, NB, egos, warm_steps, threads):
    """SURVEY 8(d) CPU baseline (ii): the kernel algorithm compiled for the host
    (tests/hostsim, g++ -O2 -fopenmp), OpenMP over `threads` cores, steady state: one cold
    closed-loop step (inittree, untimed), then `warm_steps` timed warm steps (updatetree +
    IPM) of `egos` seeded egos, with the same device-scene rules stepped by the host build."""
    os.environ["OMP_NUM_THREADS"] = str(threads)
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import hostsim_lib as H
    from bmpc import abi
    from bmpc.scenarios import highway_desc, highway_policy_rows, seeded_batch
    x, z, xref, tgt = seeded_batch(egos, seed=0)
    hs = H.HostSim(highway_desc(N=N, NB=NB), egos)
    hs.set_policies(highway_policy_rows(tgt))
    env = abi.make_env()
    scene = np.zeros((egos, abi.ENV_STRIDE))
    scene[:, 0:4], scene[:, 4:8] = x, z
    x, z, xref = hs.env_step(env, 0, scene)
    r = hs.solve(x, z, xref)                        # cold solve (untimed)
    t0 = time.time()
    for t in range(1, warm_steps + 1):
        x, z, xref = hs.env_step(env, t, scene, r["upred"], r["J"], r["status"], r["iters"])
        r = hs.solve(x, z, xref)
    dt = time.time() - t0
    return dict(value=round(warm_steps * egos / dt, 2), unit="solves/s", cores=threads, kind="port",
                sample=f"{egos} seeded egos x {warm_steps} warm closed-loop steps after one untimed cold step, "
                       f"N={N} NB={NB}: the kernel algorithm built for the host from the same csrc templates "
                       f"(tests/hostsim, g++ -O2 -fopenmp, {threads} OpenMP threads), {dt:.2f} s wall")


def cpu_oracle_baseline(N, NB, egos, warm_steps, procs):
    """The NumPy oracle (reference-structured: model + tree assembly + ECOS-algorithm IPM),
    one process per core, steady state: per ego one untimed cold solve then `warm_steps`
    timed warm solves along the closed loop."""
    import multiprocessing as mp
    t0 = time.time()
    with mp.get_context("spawn").Pool(procs, initializer=_worker_init) as pool:
        res = pool.map(_oracle_episode, [(i, N, NB, warm_steps) for i in range(egos)])
    wall = time.time() - t0
    per = float(np.mean([r for rs in res for r in rs]))
    return dict(value=round(procs / per, 3), unit="solves/s", cores=procs, kind="port",
                sample=f"{egos} seeded egos x {warm_steps} warm solves (after one untimed cold solve each), N={N} "
                       f"NB={NB}: oracle/ (NumPy model + tree assembly + ECOS-algorithm IPM), {procs} processes x 1 "
                       f"thread; value = procs / mean warm-solve time ({per:.3f} s), {wall:.1f} s wall incl. pool start")


def _worker_init():
    os.environ["OMP_NUM_THREADS"] = "1"
    os.environ["OPENBLAS_NUM_THREADS"] = "1"
    for _p in (REPO, os.path.join(REPO, "belief-planning_amd")):
        if _p not in sys.path:
            sys.path.insert(0, _p)


def _oracle_episode(args):
    i, N, NB, warm = args
    from bmpc.scenarios import seeded_batch
    from oracle.ecos_ipm import ecos_solve
    from oracle.model import HighwayModel, highway_policies
    from oracle.tree import CVaRController
    x, z, xref, tgt = seeded_batch(max(i + 1, 2), seed=0)
    x, z, xr = x[i].copy(), z[i].copy(), xref[i].copy()
    mdl = HighwayModel(N, 0.1, highway_policies(0.1, tgt[i]))
    Fx = np.array([[0., 1, 0, 0], [0, -1, 0, 0], [0, 0, 0, 1], [0, 0, 0, -1]])
    c = CVaRController(mdl, N, NB, np.diag([0., 3, 3, 10]), np.diag([1., 100]), Fx,
                       [4 * 3.6 - 1.25, -1.25, .25, .25], np.kron(np.eye(2), [1, -1]).T,
                       [6., 6., .3, .3], [0, 300], xr, 0.9, solver=ecos_solve)
    times = []
    for k in range(warm + 1):
        t0 = time.time()
        c.solve(x, z, xr)
        if k > 0:
            times.append(time.time() - t0)
        u = c.uPred[0]
        x = x + 0.1 * np.array([x[2] * np.cos(x[3]), x[2] * np.sin(x[3]), u[0], u[1]])
        z = z + 0.1 * np.array([z[2] * np.cos(z[3]), z[2] * np.sin(z[3]), 0.0, 0.0])
    return times


def load_traffic(path, key, src):
    """Per-launch HBM bytes (FETCH_SIZE x2 + WRITE_SIZE, rocprofv3 --pmc passes) of the IPM
    kernel, measured for THIS workload key on THIS source build (profiles/pmc_traffic.json,
    written by tools/prof_summary.py); None when no entry matches."""
    if not path or not os.path.exists(path):
        return None, None
    try:
        with open(path) as f:
            entries = json.load(f)
    except (OSError, ValueError):
        return None, None
    for e in entries:
        if e.get("key") == key and e.get("source_hash") == src:
            return e.get("bytes_per_launch"), e.get("profile")
    return None, None


def algorithmic_bytes(T, U, bdim, nbranch, m, n, d):
    """SURVEY 8(d) compulsory HBM bytes per solve: inputs 3n, warm start read + write
    2[(U+1)d + bdim m + d], outputs U d + T n + Bn + 2 (J, status)."""
    return 8 * (3 * n + 2 * ((U + 1) * d + bdim * m + d) + U * d + T * n + (nbranch - 1) + 2)


def launch_ranks(a):
    """bench.py --gpus N run directly: start N ranks through torchrun (127.0.0.1) as child
    processes before this process touches the GPU, and exit with their status."""
    import socket
    import subprocess
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={a.gpus}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    sys.exit(subprocess.call(cmd, env=dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")))


class _HostSimPlan:
    """TEST-ONLY backend of this script (BMPC_BENCH_BACKEND=hostsim): the host build of the
    kernel templates (tests/hostsim) behind the few BatchPlan calls the closed loop makes, on
    CPU tensors, so that tests/test_bench_launch.py can drive bench.py's N > 1 path -- the
    torchrun self-launch, sharding, the statistics all-reduce and max-over-ranks timing -- over
    gloo without a GPU.  Its numbers are never a measurement: the JSON line names the backend."""

    def __init__(self, desc, B):
        sys.path.insert(0, os.path.join(REPO, "tests"))
        import hostsim_lib as H
        self.hs = H.HostSim(desc, B)
        self.T, self.U, self.bdim, self.nbranch = self.hs.T, self.hs.U, self.hs.bdim, self.hs.nbranch
        self._ms = 0.0

    def set_policies(self, rows):
        self.hs.set_policies(rows)

    def env_step(self, env, t, scene, up, tx, tz, tr, Jv, st, it, estats):
        x, z, xref = self.hs.env_step(env, t, scene.numpy(), up.numpy(), Jv.numpy(), st.numpy(), it.numpy(),
                                      estats.numpy())
        tx.copy_(_torch().from_numpy(x)), tz.copy_(_torch().from_numpy(z)), tr.copy_(_torch().from_numpy(xref))

    def solve(self, tx, tz, tr, up, Jv, st, it):
        t0 = time.perf_counter()
        r = self.hs.solve(tx.numpy(), tz.numpy(), tr.numpy())
        self._ms += 1e3 * (time.perf_counter() - t0)
        T = _torch()
        up.copy_(T.from_numpy(r["upred"])), Jv.copy_(T.from_numpy(r["J"]))
        st.copy_(T.from_numpy(r["status"])), it.copy_(T.from_numpy(r["iters"]))

    def enable_timing(self, on=True):
        self._ms = 0.0

    def timing(self):
        return dict(tree_ms=0.0, ipm_ms=self._ms)


def _torch():
    import torch
    return torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1, help="ranks (one per GPU); run directly with N > 1 it "
                                                        "launches the ranks itself through torchrun")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", choices=("highway", "quadruped", "robust"), default="highway",
                    help="highway = BASELINE metric config; quadruped = BASELINE config 4 (BranchMPCProx)")
    ap.add_argument("--batch", type=int, default=None, help="egos per GPU (highway 4096, quadruped 1024)")
    ap.add_argument("--global-batch", type=int, default=None,
                    help="egos over all ranks, sharded contiguously (BASELINE config 5: 65536 over 8 GPUs)")
    ap.add_argument("--N", type=int, default=None)
    ap.add_argument("--NB", type=int, default=None)
    ap.add_argument("--loop", choices=("fused", "steps"), default="steps",
                    help="highway CVaR closed loop: fused = the K steps of every ego in one k_loop launch "
                         "(bmpc_loop_device: the egos' loops are independent, so no step waits for the slowest "
                         "ego of the previous one); steps = k_env + k_tree + k_ipm launched per step")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-egos", type=int, default=4096, help="egos of the C++ host-build baseline sample")
    ap.add_argument("--oracle-egos", type=int, default=16, help="egos of the NumPy-oracle baseline sample")
    ap.add_argument("--traffic", default=os.path.join(REPO, "profiles", "pmc_traffic.json"))
    a = ap.parse_args()
    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        launch_ranks(a)                 # never returns
    quad = a.workload == "quadruped"
    robust = a.workload == "robust"     # robustMPC (MPC_branch.py:1275) in the same scene
    a.N = a.N or (25 if quad else 20)
    a.NB = a.NB or (2 if quad else 1)

    import torch
    import torch.distributed as dist
    from bmpc import _lib, abi, plan
    from bmpc.scenarios import (highway_desc, highway_policy_rows, quadruped_desc, quadruped_policy_rows,
                                seeded_batch, seeded_quadruped_batch)

    from bmpc import distributed as D
    rank, local, world = D.world()
    if world != a.gpus:
        raise SystemExit(f"bench.py: --gpus {a.gpus} but the launcher started {world} ranks")
    host = os.environ.get("BMPC_BENCH_BACKEND") == "hostsim"   # test-only (see _HostSimPlan)
    if host and quad:
        raise SystemExit("bench.py: the hostsim test backend runs the highway workloads only")
    if host:
        dev = torch.device("cpu")
        D.init("gloo")
    else:   # the hardware-only lines of the N > 1 path: RCCL init with device_id, HIP streams
        dev = torch.device("cuda", local)
        torch.cuda.set_device(dev)
        D.init("nccl", device=dev)
    if world > 1:
        assert dist.get_world_size() == world, (dist.get_world_size(), world)

    def sync():
        if not host:
            torch.cuda.synchronize()
    # one global seeded population; rank r owns a contiguous shard of it
    G = a.global_batch or (a.batch or (1024 if quad else 4096)) * world
    lo, hi = D.shard(G, rank, world)
    B = hi - lo
    if quad:
        x, z, xref = (v[lo:hi] for v in seeded_quadruped_batch(G, seed=1))
        desc = quadruped_desc(N=a.N, NB=a.NB)
        pl = plan.BatchPlan(desc, B, device=local)
        pl.set_policies(quadruped_policy_rows(B))
    else:
        x, z, xref, tgt = (v[lo:hi] for v in seeded_batch(G, seed=0))
        desc = highway_desc(N=a.N, NB=a.NB)
        if robust:
            desc.controller = abi.CTRL_ROBUST
        pl = _HostSimPlan(desc, B) if host else plan.BatchPlan(desc, B, device=local)
        pl.set_policies(highway_policy_rows(tgt))
    tx = torch.tensor(x, device=dev, dtype=torch.float64)
    tz = torch.tensor(z, device=dev, dtype=torch.float64)
    tr = torch.tensor(xref, device=dev, dtype=torch.float64)
    up = torch.zeros((B, pl.U, desc.d), device=dev, dtype=torch.float64)
    Jv = torch.zeros(B, device=dev, dtype=torch.float64)
    st = torch.zeros(B, device=dev, dtype=torch.int32)
    it = torch.zeros(B, device=dev, dtype=torch.int32)
    # one dedicated stream: the library's kernels and torch's ops run in order on it
    if not host:
        stream = torch.cuda.Stream(dev)
        torch.cuda.set_stream(stream)
        sh = stream.cuda_stream
    env = abi.make_env()                       # main_branch.sim_overtake scene constants
    scene = torch.zeros((B, abi.ENV_STRIDE), device=dev, dtype=torch.float64)
    if not quad:
        scene[:, 0:4] = tx
        scene[:, 4:8] = tz
    estats = torch.zeros((B, abi.ENV_NSTAT), device=dev, dtype=torch.float64)
    tstep = [0]

    def env_step():
        """Highway_env.step around the solve, on the device (k_env): Euler steps with
        uPred[0], collision flag, obstacle backup argmax, lane bookkeeping / lane-change
        re-targeting, x_ref rule (Highway_env_branch.py:83-184, :421-429)."""
        if host:
            pl.env_step(env, tstep[0], scene, up, tx, tz, tr, Jv, st, it, estats)
        else:
            pl.env_step_device(env, tstep[0], scene.data_ptr(), up.data_ptr(), tx.data_ptr(), tz.data_ptr(),
                               tr.data_ptr(), Jv.data_ptr(), st.data_ptr(), it.data_ptr(), estats.data_ptr(), sh)
        tstep[0] += 1

    qdt, qv0 = 0.2, 0.2
    xdes = torch.tensor([5.0, -3.0, 0.0], device=dev, dtype=torch.float64)

    def quad_env_step():
        """robot.step of ego (uPred[0]) and obstacle (forward policy), body-frame kinematics
        (quadruped_env.py:34-37), and the reference point towards x_des, on device."""
        u0 = up[:, 0, :]
        c, s_ = torch.cos(tx[:, 2]), torch.sin(tx[:, 2])
        tx.copy_(tx + qdt * torch.stack([u0[:, 0] * c - u0[:, 1] * s_, u0[:, 1] * c + u0[:, 0] * s_, u0[:, 2]], 1))
        tz.copy_(tz + qdt * torch.stack([qv0 * torch.cos(tz[:, 2]), qv0 * torch.sin(tz[:, 2]),
                                          torch.zeros_like(tz[:, 2])], 1))
        dxy = xdes[None, 0:2] - tx[:, 0:2]
        nrm = torch.linalg.norm(dxy, dim=1)
        dxy = dxy / nrm.clamp_min(1e-300)[:, None] * nrm.clamp_max(5.0)[:, None]
        psi = torch.where(torch.linalg.norm(dxy, dim=1) > 0.1, torch.atan2(dxy[:, 1], dxy[:, 0]), tx[:, 2])
        psi = psi - 2 * math.pi * torch.round((psi - xdes[2]) / (2 * math.pi))
        tr[:, 0:2] = tx[:, 0:2] + dxy
        tr[:, 2] = psi
        dis = torch.linalg.norm(tx[:, 0:2] - tz[:, 0:2], dim=1) - 0.75
        estats[:, abi.ENVS_J] += Jv
        estats[:, abi.ENVS_J2] += Jv * Jv
        estats[:, abi.ENVS_INFEAS] += (st != 1).double()
        estats[:, abi.ENVS_ITERS] += it.double()
        estats[:, abi.ENVS_SOLVES] += 1.0
        estats[:, abi.ENVS_COLL_STEPS] += (dis < 0).double()

    fused = a.loop == "fused" and not (quad or robust or host)

    def steps(k):
        """k closed-loop steps of every ego as ONE launch (bmpc_loop_device -> k_loop), the same
        per-ego work and results as k calls of step()"""
        pl.loop_device(env, tstep[0], k, scene.data_ptr(), up.data_ptr(), tx.data_ptr(), tz.data_ptr(), tr.data_ptr(),
                       Jv.data_ptr(), st.data_ptr(), it.data_ptr(), estats.data_ptr(), sh)
        tstep[0] += k

    def step():
        # one closed-loop step: scene update -> solve (inputs / outputs stay in HBM)
        if not quad:
            env_step()
        if host:
            pl.solve(tx, tz, tr, up, Jv, st, it)
        else:
            pl.solve_device(tx.data_ptr(), tz.data_ptr(), tr.data_ptr(), up.data_ptr(), None, None,
                            Jv.data_ptr(), st.data_ptr(), it.data_ptr(), sh)
        if quad:
            quad_env_step()

    it_sum = torch.zeros(B, dtype=torch.float64, device=dev)
    if fused:
        if a.warmup:
            steps(a.warmup)
    else:
        for _ in range(a.warmup):
            step()
            it_sum.add_(it)
    # the timed region's own torch ops once beforehand: their kernels load lazily on first use
    # (~20-60 ms each, measured at one ego: 2.3 ms per step of a 20-step region)
    D.episode_stats(estats)
    sync()
    # per-kernel device timing over the timed steps themselves: HIP events recorded on the
    # launch stream around each kernel, read back after the region (no host synchronisation
    # inside it); the IPM iteration mean comes from the same launches
    it_sum.zero_()
    pl.enable_timing(True)
    estats.zero_()
    if world > 1:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    if fused:
        steps(a.steps)
    else:
        for _ in range(a.steps):
            step()
            it_sum.add_(it)
    stats = D.episode_stats(estats)
    D.reduce_stats(stats)        # the only collective: SUM, MAX for the flag
    sync()
    if world > 1:
        dist.barrier()
    elapsed = D.max_over_ranks(time.perf_counter() - t0, device=dev)
    tm = pl.timing()
    pl.enable_timing(False)
    # per-step kernel time: a fused launch covers a.steps steps (k_env + k_tree + k_ipm work of each)
    ipm_ms = D.max_over_ranks(tm["ipm_ms"] / (a.steps if fused else 1), device=dev)
    if fused:   # the closed-loop statistics count every solve's iterations (k_env's accumulate)
        st_loc = estats.sum(0).cpu().numpy()
        iters_mean = float(st_loc[abi.ENVS_ITERS] / max(st_loc[abi.ENVS_SOLVES], 1))
    else:
        iters_mean = float(it_sum.sum().item()) / (B * max(a.steps, 1))
    total = G * a.steps
    value = total / elapsed
    if rank == 0:
        st_h = stats.cpu().numpy()
        T, U, bdim, nbr = pl.T, pl.U, pl.bdim, pl.nbranch
        if quad:   # same per-node formula, n = d = 3, Nc = 1, nFu = 6, no cones, m = 2
            F_it = flops_per_iter(T, 3, 3, 1, 6, [])
            F_mod = flops_model(U, nbr - 1, bdim, 2, a.N, 3)
        elif robust:   # chain of T nodes, Nc = 4 Fx rows + 3^NB collision rows, no cones
            F_it = flops_per_iter(T, 4, 2, 4 + 3 ** a.NB, 4, [])
            F_mod = flops_model(U, nbr - 1, bdim, 3, a.N, 4)
        else:
            cone_dims = [2 + a.N * 6] * (bdim * 3) + [4]
            F_it = flops_per_iter(T, 4, 2, 5, 4, cone_dims)
            F_mod = flops_model(U, nbr - 1, bdim, 3, a.N, 4)
        kern_s = ipm_ms * 1e-3
        achieved = B * iters_mean * F_it / kern_s / 1e12 if kern_s > 0 else 0.0
        abytes = algorithmic_bytes(T, U, bdim, nbr, desc.m, desc.n, desc.d)
        hbm_alg = B * abytes / kern_s / 1e9 if kern_s > 0 else 0.0
        key = f"{a.workload}:N{a.N}:NB{a.NB}:B{B}" + (":loop" if fused else "")   # traffic per step
        src = _lib.source_hash()
        lib_stamp = None if host else _lib.LOADED_STAMP   # lib() refused the product .so unless == src
        traffic, tsrc = load_traffic(a.traffic, key, src)
        kname = ("k_qp (structured Mehrotra QP IPM)" if (quad or robust) else
                 "k_loop (per ego: k_env scene step + k_tree + k_ipm structured HSDE IPM, fused over the steps)"
                 if fused else "k_ipm (structured HSDE IPM)")
        headline = not (quad or robust) and (a.N, a.NB, B) == (20, 1, 4096)
        out = {
            "metric": (METRIC if headline else
                       f"branch-MPC solves/sec (whole node), quadruped BranchMPCProx N={a.N} NB={a.NB} m=2 "
                       f"({2 ** a.NB} leaves), batch {B} egos" if quad else
                       f"robustMPC solves/sec (whole node), highway N={a.N} NB={a.NB}, {3 ** a.NB} obstacle "
                       f"predictions per slot, batch {B} egos" if robust else
                       f"branch-MPC solves/sec (whole node), highway N={a.N} NB={a.NB} ({3 ** a.NB} leaves), "
                       f"batch {B} egos"),
            "value": round(value, 2), "unit": "solves/s", "n_gpus": world,
            "steps": a.steps, "warmup": a.warmup, "ms_per_step": round(1e3 * elapsed / a.steps, 4),
            "higher_is_better": True, "scaling": "weak" if not a.global_batch else "strong",
            "vs_baseline": None, "dtype": "f64",
            "data": ("synthetic (seeded quadruped egos, seed 1; obstacle on the forward policy)" if quad
                     else "synthetic (seeded SURVEY §8d egos, sim_overtake row 0)"),
            "config": {"workload": (f"quadruped BranchMPCProx closed loop, N={a.N}, NB={a.NB}, m=2 " if quad else
                                    f"highway robustMPC closed loop, N={a.N}, NB={a.NB}, m=3 " if robust else
                                    f"highway BranchMPC_CVaR closed loop, N={a.N}, NB={a.NB}, m=3 ")
                                   + f"(T={T}, U={U}), {B} egos per GPU", "batch_per_gpu": B,
                       "global_batch": G, "world_size": world, "parallelism": f"ego-sharded dp{world}",
                       "loop": ("fused: one k_loop launch per timed region (bmpc_loop_device)" if fused else
                                "per step: k_env + solve launches"),
                       "shards": [list(D.shard(G, r, world)) for r in range(world)]},
            "roofline": {"bound": "fp64-valu", "achieved": round(achieved, 5), "peak": FP64_PEAK_TFLOPS,
                         "unit": "TFLOP/s", "frac": round(achieved / FP64_PEAK_TFLOPS, 7),
                         "traffic": traffic, "traffic_source": tsrc, "traffic_key": key, "source_hash": src,
                         "library_stamp": lib_stamp,
                         "hbm_alg_GBps": round(hbm_alg, 4), "hbm_frac": round(hbm_alg / (HBM_PEAK_TBPS * 1e3), 9),
                         "alg_bytes_per_solve": abytes,
                         "hbm_traffic_frac": (round(traffic / kern_s / (HBM_PEAK_TBPS * 1e12), 4)
                                              if traffic and kern_s > 0 else None),
                         "kernel": kname, "kernel_ms": round(ipm_ms, 4),
                         "tree_kernel_ms": round(tm["tree_ms"], 4),
                         "flop_per_iter": F_it, "iters_mean": round(iters_mean, 2),
                         "flop_model_per_solve": F_mod},
            "closed_loop": {"J_mean": float(st_h[abi.ENVS_J] / max(st_h[abi.ENVS_SOLVES], 1)),
                            "infeasible": int(st_h[abi.ENVS_INFEAS]),
                            "iters_mean": float(st_h[abi.ENVS_ITERS] / max(st_h[abi.ENVS_SOLVES], 1)),
                            "solves": int(st_h[abi.ENVS_SOLVES]),
                            "collision_steps": int(st_h[abi.ENVS_COLL_STEPS]),
                            "collided_egos": int(st_h[D.STAT_COLLIDED]),
                            "any_collided": bool(st_h[D.STAT_ANY_COLLIDED] > 0),
                            "env": "device k_env (sim_overtake scene)" if not quad else "torch ops"},
        }
        if host:
            out["backend"] = "hostsim (TEST-ONLY host build over gloo: not a measurement)"
        if not a.no_cpu_baseline and world == 1 and not (quad or robust) and not host:
            cores, aff, quota = usable_cores()
            try:
                cb = cpu_cxx_baseline(a.N, a.NB, min(a.cpu_egos, G), 3, cores)
            except Exception as exc:
                cb = {"error": str(exc)[:200]}
            cb["affinity_cpus"], cb["cgroup_quota_cpus"] = aff, quota
            out["cpu_baseline"] = cb
            ob = cpu_oracle_baseline(a.N, a.NB, a.oracle_egos, 2, cores)
            out["cpu_oracle_baseline"] = ob
        else:
            out["cpu_baseline"] = None
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
