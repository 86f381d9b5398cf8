"""A/B of the rotated-cone row boost (oracle/ecos_ipm.py boost_rows, k_tree's per-cone beta) with
ECOS's equilibration on: boost as shipped through round 5 vs beta = 0 (plain ECOS).  CPU, test tooling.

    python tools/boost_experiment.py [EGOS STEPS] > profiles/r06/boost_ab.log

1. the oracle on every solver problem the six CVaR recordings hold (kept steps, the reference's own
   assembled c, G, h, A, b) with the recorded beta and with beta = 0;
2. the oracle's closed loop of EGOS seeded egos (SURVEY 8(d) batch, seed 0) x STEPS steps at N=20 NB=1,
   each arm carrying its own trajectory;
3. the kernel algorithm (host build, -DBMPC_CONE_BOOST=0/1) on every recorded step of the four highway
   recordings, one ego per step with the reference's warm start.
Reports exit-0 share, mean iterations, and the J difference where both arms exit 0."""
import multiprocessing as mp
import os
import subprocess
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "tests"), REPO, os.path.join(REPO, "belief-planning_amd")]
RECS = ("highway_n10_nb1", "highway_n8_nb2", "highway_n20_nb1", "highway_n30_nb2", "highway_xform_n8_nb2",
        "merge_n40_nb1")


def _solve_kept(args):
    name, t, zero = args
    os.environ["OMP_NUM_THREADS"] = "1"
    from common import cone_problem, golden
    from oracle.ecos_ipm import ecos_solve
    g = golden(name)
    prob = cone_problem(g, t)
    if zero:
        prob.cone_boost = [0.0] * len(prob.cone_boost)
    x, info = ecos_solve(prob)
    return info["exitFlag"], info["iter"], float(x[-1])


def _episode(args):
    i, E, N, NB, steps, zero = args
    os.environ["OMP_NUM_THREADS"] = "1"
    from bmpc.scenarios import seeded_batch
    from oracle.ecos_ipm import ecos_solve
    from oracle.model import HighwayModel, highway_policies
    from oracle.tree import CVaRController
    if zero:
        CVaRController.cone_boost = lambda self: [0.0] * (len(self.topo.children[0]) * self.topo.bdim + 1)
    x, z, xref, tgt = seeded_batch(E, seed=0)
    x, z, xr = x[i].copy(), z[i].copy(), xref[i].copy()
    c = CVaRController(HighwayModel(N, 0.1, highway_policies(0.1, tgt[i])), N, NB, np.diag([0., 3, 3, 10]),
                       np.diag([1., 100]), np.array([[0., 1, 0, 0], [0, -1, 0, 0], [0, 0, 0, 1], [0, 0, 0, -1]]),
                       [4 * 3.6 - 1.25, -1.25, .25, .25], np.kron(np.eye(2), [1, -1]).T, [6., 6., .3, .3], [0, 300],
                       xr, 0.9, solver=ecos_solve)
    out = []
    for _ in range(steps):
        c.solve(x, z, xr)
        inf = c.last_info
        out.append((inf["exitFlag"], inf["iter"], inf["x"][-1]))
        u = c.uPred[0]
        x = x + 0.1 * np.array([x[2] * np.cos(x[3]), x[2] * np.sin(x[3]), u[0], u[1]])
        z = z + 0.1 * np.array([z[2] * np.cos(z[3]), z[2] * np.sin(z[3]), 0.0, 0.0])
    return out


def _report(tag, a, b):
    """a, b: [..., 3] arrays (exit, iters, J) of the boosted / unboosted arm."""
    for lab, r in (("boost", a), ("beta=0", b)):
        ex = r[..., 0].astype(int)
        vals, cnt = np.unique(ex, return_counts=True)
        print(f"  {tag} {lab:7s}: exits {dict(zip(vals.tolist(), cnt.tolist()))}  exit-0 share {np.mean(ex == 0):.4f}"
              f"  iters mean {r[..., 1].mean():.2f}")
    both0 = (a[..., 0] == 0) & (b[..., 0] == 0)
    dJ = np.abs(a[..., 2] - b[..., 2]) / np.maximum(1, np.abs(a[..., 2]))
    print(f"  {tag} exit agreement {np.mean(a[..., 0] == b[..., 0]):.4f}; both exit 0 on {int(both0.sum())}; "
          f"max rel |dJ| there {dJ[both0].max() if both0.any() else float('nan'):.2e}")


_HOST = r"""
import sys, numpy as np
sys.path[:0] = [%r, %r, %r]
import hostsim_lib as H
from common import golden, highway_desc_from_golden, replay_batch
out = {}
for name, steps in (("highway_n10_nb1", 20), ("highway_n8_nb2", 40), ("highway_n20_nb1", 100), ("highway_n30_nb2", 24)):
    g = golden(name); rb = replay_batch(g, steps)
    hs = H.HostSim(highway_desc_from_golden(g), rb["T"]); hs.set_policies(rb["rows"])
    hs.set_warm_start(rb["uLin"], rb["p"], rb["jcons"]); hs.reset_mask(~rb["warm"])
    r = hs.solve(rb["x"], rb["z"], rb["xref"])
    out[name] = np.stack([r["status"], r["iters"], r["J"]], 1)
np.savez(sys.argv[1], **out)
"""


def host_arm(boost, path):
    here = os.path.join(REPO, "tests")
    env = dict(os.environ, BMPC_HOSTSIM_FLAGS=f"-DBMPC_CONE_BOOST={boost}")
    code = _HOST % (here, REPO, os.path.join(REPO, "belief-planning_amd"))
    subprocess.run([sys.executable, "-c", code, path], env=env, check=True, timeout=3000)
    return dict(np.load(path))


def main():
    E, steps = (int(v) for v in sys.argv[1:3]) if len(sys.argv) > 2 else (96, 3)
    from common import golden
    jobs = [(n, int(t)) for n in RECS for t in golden(n)["keep"]]
    ctx = mp.get_context("spawn")
    with ctx.Pool(8) as pool:
        a = np.array(pool.map(_solve_kept, [(n, t, False) for n, t in jobs]))
        b = np.array(pool.map(_solve_kept, [(n, t, True) for n, t in jobs]))
    print(f"1. oracle on the {len(jobs)} recorded solver problems (six CVaR recordings, kept steps)")
    for n in RECS:
        ix = [i for i, (m, _) in enumerate(jobs) if m == n]
        g = golden(n)
        rec = np.array([int(g["traj_exit"][jobs[i][1]]) for i in ix])
        print(f"  {n}: recorded exits {rec.tolist()}  boost {a[ix, 0].astype(int).tolist()} it {a[ix, 1].astype(int).tolist()}"
              f"  beta=0 {b[ix, 0].astype(int).tolist()} it {b[ix, 1].astype(int).tolist()}")
    _report("kept", a, b)
    with ctx.Pool(8) as pool:
        ea = np.array(pool.map(_episode, [(i, E, 20, 1, steps, False) for i in range(E)]))
        eb = np.array(pool.map(_episode, [(i, E, 20, 1, steps, True) for i in range(E)]))
    print(f"2. oracle closed loop, {E} seeded egos x {steps} steps, N=20 NB=1")
    _report("seeded", ea, eb)
    import tempfile
    with tempfile.TemporaryDirectory() as d:
        ha = host_arm(1, os.path.join(d, "a.npz"))
        hb = host_arm(0, os.path.join(d, "b.npz"))
    print("3. kernel algorithm (host build) on every recorded step of the highway recordings")
    for n in ha:
        rec = np.asarray(golden(n)["traj_exit"][:len(ha[n])]).astype(int)
        print(f"  {n}: agreement with the recorded exits boost {np.mean(ha[n][:, 0] == rec):.3f} "
              f"beta=0 {np.mean(hb[n][:, 0] == rec):.3f}")
        _report(n, ha[n], hb[n])


if __name__ == "__main__":
    main()
