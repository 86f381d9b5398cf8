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


def flops_per_iter(T, n, d, Nc, nFu, cone_dims):
    """SURVEY §8(d) F_iter (transcendentals = 1)."""
    per_node = (2 * (2 * n ** 3 + 3 * n ** 2 * d + 2 * n * d ** 2 + d ** 3 / 3.0) + 2 * Nc * n ** 2
                + 4 * 2 * (2 * n ** 2 + 2 * n * d + d ** 2) + 2 * (2 * n ** 2 + 2 * n * d)
                + 10 * (n + d + 2 * Nc + nFu))
    return T * per_node + sum(20 * q for q in cone_dims)


def flops_model(U, Bn, bdim, m, N, n):
    """SURVEY §8(d) F_model."""
    return (U + Bn) * 40 + bdim * (m * N * 60 + (2 * N * m * 50) * (1 + n)) + U * 30


def cpu_baseline(N, NB, sample, procs):
    """Oracle (NumPy restatement of the reference + ECOS-algorithm IPM) on host cores."""
    import multiprocessing as mp
    t0 = time.time()
    with mp.get_context("spawn").Pool(procs, initializer=_worker_init) as pool:
        res = pool.map(_cpu_solve, [(i, N, NB) for i in range(sample)])
    dt = time.time() - t0
    return dict(value=sample / dt, unit="solves/s", cores=procs, kind="port",
                sample=f"{sample} first solves of seeded egos (seed 0) at N={N} NB={NB} m=3, "
                       f"oracle/ (NumPy model+tree assembly, ECOS-algorithm IPM with sparse LU), "
                       f"{procs} processes x 1 thread, {dt:.1f} s wall incl. pool start",
                per_solve_s=float(np.mean([r for r in res])))


def cpu_cxx_baseline(N, NB, sample, threads):
    """The kernel's own algorithm compiled for the host (tests/hostsim, g++ -O2 -fopenmp),
    OpenMP over `threads` host cores: SURVEY 8(d) CPU baseline (ii).  Two closed-loop steps
    (cold + warm) of the first `sample` egos of the seeded population."""
    os.environ["OMP_NUM_THREADS"] = str(threads)
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import hostsim_lib as H
    from bmpc.scenarios import highway_desc, highway_policy_rows, seeded_batch
    x, z, xref, tgt = seeded_batch(sample, seed=0)
    hs = H.HostSim(highway_desc(N=N, NB=NB), sample)
    hs.set_policies(highway_policy_rows(tgt))
    t0 = time.time()
    for _ in range(2):
        r = hs.solve(x, z, xref)
        u0 = r["upred"][:, 0]
        x = x + 0.1 * np.stack([x[:, 2] * np.cos(x[:, 3]), x[:, 2] * np.sin(x[:, 3]), u0[:, 0], u0[:, 1]], 1)
        z = z + 0.1 * np.stack([z[:, 2] * np.cos(z[:, 3]), z[:, 2] * np.sin(z[:, 3]), 0 * z[:, 0], 0 * z[:, 0]], 1)
    dt = time.time() - t0
    return dict(value=round(2 * sample / dt, 2), unit="solves/s", cores=threads, kind="port",
                sample=f"{sample} seeded egos x 2 closed-loop steps (cold + warm), the kernel algorithm built "
                       f"for the host (g++ -O2 -fopenmp, {threads} threads), {dt:.1f} s")


def _worker_init():
    os.environ["OMP_NUM_THREADS"] = "1"
    os.environ["OPENBLAS_NUM_THREADS"] = "1"
    for _p in (REPO, os.path.join(REPO, "belief-planning_amd")):
        if _p not in sys.path:
            sys.path.insert(0, _p)


def _cpu_solve(args):
    i, N, NB = args
    from bmpc.scenarios import seeded_batch
    from oracle.ecos_ipm import ecos_solve
    from oracle.model import HighwayModel, highway_policies
    from oracle.tree import CVaRController
    x, z, xref, tgt = seeded_batch(max(i + 1, 2), seed=0)
    mdl = HighwayModel(N, 0.1, highway_policies(0.1, tgt[i]))
    Fx = np.array([[0., 1, 0, 0], [0, -1, 0, 0], [0, 0, 0, 1], [0, 0, 0, -1]])
    c = CVaRController(mdl, N, NB, np.diag([0., 3, 3, 10]), np.diag([1., 100]), Fx,
                       [4 * 3.6 - 1.25, -1.25, .25, .25], np.kron(np.eye(2), [1, -1]).T,
                       [6., 6., .3, .3], [0, 300], xref[i], 0.9, solver=ecos_solve)
    t0 = time.time()
    c.solve(x[i], z[i], xref[i])
    return time.time() - t0


def load_traffic(path):
    """Per-launch HBM bytes of the IPM kernel from a committed rocprofv3 --pmc summary."""
    if not path or not os.path.exists(path):
        return None
    try:
        with open(path) as f:
            d = json.load(f)
        return d.get("k_ipm_bytes_per_launch")
    except Exception:
        return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", choices=("highway", "quadruped", "robust"), default="highway",
                    help="highway = BASELINE metric config; quadruped = BASELINE config 4 (BranchMPCProx)")
    ap.add_argument("--batch", type=int, default=None, help="egos per GPU (highway 4096, quadruped 1024)")
    ap.add_argument("--N", type=int, default=None)
    ap.add_argument("--NB", type=int, default=None)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample", type=int, default=24)
    ap.add_argument("--traffic", default=os.path.join(REPO, "profiles", "r01_pmc_traffic.json"))
    a = ap.parse_args()
    quad = a.workload == "quadruped"
    robust = a.workload == "robust"     # robustMPC (MPC_branch.py:1275) in the same scene
    a.batch = a.batch or (1024 if quad else 4096)
    a.N = a.N or (25 if quad else 20)
    a.NB = a.NB or (2 if quad else 1)

    import torch
    import torch.distributed as dist
    from bmpc import abi, plan
    from bmpc.scenarios import (highway_desc, highway_policy_rows, quadruped_desc, quadruped_policy_rows,
                                seeded_batch, seeded_quadruped_batch)

    from bmpc import distributed as D
    rank, local, world = D.world()
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    D.init("nccl", device=dev)
    B = a.batch
    # one global seeded population of B*world egos; rank r owns a contiguous shard
    lo, hi = D.shard(B * world, rank, world)
    if quad:
        x, z, xref = (v[lo:hi] for v in seeded_quadruped_batch(B * world, seed=1))
        desc = quadruped_desc(N=a.N, NB=a.NB)
        pl = plan.BatchPlan(desc, B, device=local)
        pl.set_policies(quadruped_policy_rows(B))
    else:
        x, z, xref, tgt = (v[lo:hi] for v in seeded_batch(B * world, seed=0))
        desc = highway_desc(N=a.N, NB=a.NB)
        if robust:
            desc.controller = abi.CTRL_ROBUST
        pl = plan.BatchPlan(desc, B, device=local)
        pl.set_policies(highway_policy_rows(tgt))
    tx = torch.tensor(x, device=dev, dtype=torch.float64)
    tz = torch.tensor(z, device=dev, dtype=torch.float64)
    tr = torch.tensor(xref, device=dev, dtype=torch.float64)
    up = torch.zeros((B, pl.U, desc.d), device=dev, dtype=torch.float64)
    Jv = torch.zeros(B, device=dev, dtype=torch.float64)
    st = torch.zeros(B, device=dev, dtype=torch.int32)
    it = torch.zeros(B, device=dev, dtype=torch.int32)
    # one dedicated stream: the library's kernels and torch's ops run in order on it
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

    def step():
        # one closed-loop step: scene update -> solve (inputs / outputs stay in HBM)
        if not quad:
            env_step()
        pl.solve_device(tx.data_ptr(), tz.data_ptr(), tr.data_ptr(), up.data_ptr(), None, None,
                        Jv.data_ptr(), st.data_ptr(), it.data_ptr(), sh)
        if quad:
            quad_env_step()

    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize()
    # per-kernel device timing over the timed steps themselves: HIP events recorded on the
    # launch stream around each kernel, read back after the region (no host synchronisation
    # inside it); the IPM iteration mean comes from the same launches
    it_sum = torch.zeros(B, dtype=torch.float64, device=dev)
    pl.enable_timing(True)
    estats.zero_()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
        it_sum.add_(it)
    stats = estats.sum(0)
    D.reduce_stats(stats)        # the only collective
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = D.max_over_ranks(time.perf_counter() - t0, device=dev)
    tm = pl.timing()
    pl.enable_timing(False)
    iters_mean = float(it_sum.sum().item()) / (B * max(a.steps, 1))
    total = B * world * a.steps
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
        achieved = B * iters_mean * F_it / (tm["ipm_ms"] * 1e-3) / 1e12 if tm["ipm_ms"] > 0 else 0.0
        traffic = None if (quad or robust) else load_traffic(a.traffic)
        out = {
            "metric": (METRIC if not (quad or robust) else
                       "branch-MPC solves/sec (whole node), quadruped BranchMPCProx N=25 NB=2 m=2 (4 leaves), "
                       "batch 1024 egos" if quad else
                       f"robustMPC solves/sec (whole node), highway N={a.N} NB={a.NB}, {3 ** a.NB} obstacle "
                       f"predictions per slot, batch {B} egos"),
            "value": round(value, 2), "unit": "solves/s", "n_gpus": world,
            "steps": a.steps, "warmup": a.warmup, "ms_per_step": round(1e3 * elapsed / a.steps, 4),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f64",
            "data": ("synthetic (seeded quadruped egos, seed 1; obstacle on the forward policy)" if quad
                     else "synthetic (seeded SURVEY §8d egos, sim_overtake row 0)"),
            "config": {"workload": (f"quadruped BranchMPCProx closed loop, N={a.N}, NB={a.NB}, m=2 " if quad else
                                    f"highway robustMPC closed loop, N={a.N}, NB={a.NB}, m=3 " if robust else
                                    f"highway BranchMPC_CVaR closed loop, N={a.N}, NB={a.NB}, m=3 ")
                                   + f"(T={T}, U={U}), {B} egos per GPU", "batch_per_gpu": B,
                       "global_batch": B * world, "parallelism": f"ego-sharded dp{world}"},
            "roofline": {"bound": "mfma", "achieved": round(achieved, 5), "peak": FP64_PEAK_TFLOPS,
                         "unit": "TFLOP/s", "frac": round(achieved / FP64_PEAK_TFLOPS, 7),
                         "traffic": traffic,
                         "kernel": "k_qp (structured Mehrotra QP IPM)" if (quad or robust) else
                                   "k_ipm (structured HSDE IPM)",
                         "kernel_ms": round(tm["ipm_ms"], 4),
                         "tree_kernel_ms": round(tm["tree_ms"], 4),
                         "flop_per_iter": F_it, "iters_mean": round(iters_mean, 2),
                         "flop_model_per_solve": F_mod},
            "closed_loop": {"J_mean": float(st_h[abi.ENVS_J] / max(st_h[abi.ENVS_SOLVES], 1)),
                            "infeasible": int(st_h[abi.ENVS_INFEAS]),
                            "iters_mean": float(st_h[abi.ENVS_ITERS] / max(st_h[abi.ENVS_SOLVES], 1)),
                            "solves": int(st_h[abi.ENVS_SOLVES]),
                            "collision_steps": int(st_h[abi.ENVS_COLL_STEPS]),
                            "env": "device k_env (sim_overtake scene)" if not quad else "torch ops"},
        }
        if not a.no_cpu_baseline and world == 1 and not (quad or robust):
            procs = max(1, min(8, len(os.sched_getaffinity(0))))
            cb = cpu_baseline(a.N, a.NB, a.cpu_sample, procs)
            out["cpu_baseline"] = {k: (round(v, 3) if isinstance(v, float) else v) for k, v in cb.items()}
            try:
                out["cpu_cxx_baseline"] = cpu_cxx_baseline(a.N, a.NB, 1024, max(1, min(16, len(os.sched_getaffinity(0)))))
            except Exception as exc:   # the C++ host build is a secondary figure only
                out["cpu_cxx_baseline"] = {"error": str(exc)[:200]}
        else:
            out["cpu_baseline"] = None
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
