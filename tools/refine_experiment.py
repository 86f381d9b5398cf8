"""End-game refinement A/B on the host build of the kernel templates (CPU, test tooling).

Each variant is a host build with extra -D flags, built twice: plain and with FMA contraction
(-mfma -ffp-contract=fast), the latter a stand-in for the GPU's different rounding (the device code
contracts multiply-adds; the plain host build does not).  Per variant: exit agreement with the four
highway recordings, the merge and the S / Fx recordings, and the exit agreement between the plain and
the FMA build on every recorded step and on the seeded 64-ego N=20 batch over 3 closed-loop steps
(tests/test_gpu_parity.py's GPU-vs-host check) -- how stable a variant's 0-vs-10 decisions are under
a rounding change -- with mean iterations.

    python tools/refine_experiment.py "" "-DBMPC_NITREF2=4 -DBMPC_REF_STALL=6" ... > profiles/r06/refine_ab.log"""
import os
import subprocess
import sys
import tempfile
from concurrent.futures import ThreadPoolExecutor

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FMA = "-mfma -ffp-contract=fast"

RUN = r"""
import sys, numpy as np
sys.path[:0] = [%r, %r, %r]
import hostsim_lib as H
from common import golden, highway_desc_from_golden, replay_batch, highway_desc, highway_policy_rows, seeded_batch
out = {}
for name in ("highway_n10_nb1", "highway_n8_nb2", "highway_n20_nb1", "highway_n30_nb2"):
    g = golden(name); rb = replay_batch(g)
    hs = H.HostSim(highway_desc_from_golden(g), rb["T"]); hs.set_policies(rb["rows"])
    hs.set_warm_start(rb["uLin"], rb["p"], rb["jcons"]); hs.reset_mask(~rb["warm"])
    r = hs.solve(rb["x"], rb["z"], rb["xref"])
    out[name] = np.stack([r["status"], r["iters"], r["J"], r["upred"][:, 0, 0], r["upred"][:, 0, 1]], 1)
from test_merge import merge_desc, merge_rows, replay_inputs
g = golden("merge_n40_nb1"); rb = replay_inputs(g)
hs = H.HostSim(merge_desc(g), rb["T"]); hs.set_policies(merge_rows(g, rb["T"]))
hs.set_warm_start(rb["uLin"], rb["p"], rb["jcons"]); hs.reset_mask(~rb["warm"]); hs.set_transform(rb["S"], rb["bx"])
r = hs.solve(rb["x"], rb["z"], rb["xref"])
out["merge_n40_nb1"] = np.stack([r["status"], r["iters"], r["J"], r["upred"][:, 0, 0], r["upred"][:, 0, 1]], 1)
import test_xform as X
g = golden(X.NAME); steps = len(g["traj_x"])
o = X.replay(H.HostSim(X.xform_desc(g), 1), g, steps)
out["highway_xform_n8_nb2"] = np.stack([o["status"], 0 * o["status"], o["J"], o["u0"][:, 0], o["u0"][:, 1]], 1)
B = 64
x, z, xref, tgt = seeded_batch(B, seed=1)
hs = H.HostSim(highway_desc(N=20, NB=1), B); hs.set_policies(highway_policy_rows(tgt))
rows = []
for step in range(3):
    r = hs.solve(x, z, xref)
    rows.append(np.stack([r["status"], r["iters"], r["J"], r["upred"][:, 0, 0], r["upred"][:, 0, 1]], 1))
    u0 = r["upred"][:, 0]
    x = x + 0.1 * np.stack([x[:, 2] * np.cos(x[:, 3]), x[:, 2] * np.sin(x[:, 3]), u0[:, 0], u0[:, 1]], 1)
    z = z + 0.1 * np.stack([z[:, 2] * np.cos(z[:, 3]), z[:, 2] * np.sin(z[:, 3]), 0 * z[:, 0], 0 * z[:, 0]], 1)
out["seeded_n20_b64x3"] = np.concatenate(rows)
np.savez(sys.argv[1], **out)
"""


def run(flags, path):
    env = dict(os.environ, BMPC_HOSTSIM_FLAGS=flags, OMP_NUM_THREADS="2")
    code = RUN % (os.path.join(REPO, "tests"), REPO, os.path.join(REPO, "belief-planning_amd"))
    r = subprocess.run([sys.executable, "-c", code, path], env=env, capture_output=True, text=True, timeout=7200,
                       cwd=os.path.join(REPO, "tests"))
    if r.returncode:
        raise RuntimeError(flags + "\n" + r.stderr[-3000:])
    return dict(np.load(path))


def main():
    sys.path[:0] = [os.path.join(REPO, "tests"), REPO, os.path.join(REPO, "belief-planning_amd")]
    from common import golden
    variants = sys.argv[1:] or [""]
    with tempfile.TemporaryDirectory() as d:
        jobs = [(v, f) for v in variants for f in ("", FMA)]
        with ThreadPoolExecutor(4) as pool:
            res = list(pool.map(lambda a: run((a[0] + " " + a[1]).strip(), os.path.join(d, f"{hash(a)}.npz")), jobs))
    R = {job: r for job, r in zip(jobs, res)}
    for v in variants:
        a, b = R[(v, "")], R[(v, FMA)]
        print(f"== variant [{v or 'shipped'}]")
        tot_a = tot_b = tot = 0
        for name in a:
            ex_a, ex_b = a[name][:, 0].astype(int), b[name][:, 0].astype(int)
            rec = "" if name.startswith("seeded") else "  vs recording: plain %d/%d fma %d/%d" % (
                (ex_a == np.asarray(golden(name)["traj_exit"][:len(ex_a)])).sum(), len(ex_a),
                (ex_b == np.asarray(golden(name)["traj_exit"][:len(ex_b)])).sum(), len(ex_b))
            both0 = (ex_a == 0) & (ex_b == 0)
            du = np.abs(a[name][:, 3:5] - b[name][:, 3:5]).max(axis=1)
            print(f"  {name:22s} plain/fma exits agree {int((ex_a == ex_b).sum())}/{len(ex_a)}  exit10 {int((ex_a == 10).sum())}/"
                  f"{int((ex_b == 10).sum())}  iters {a[name][:, 1].mean():.2f}/{b[name][:, 1].mean():.2f}  both-0 max|du0| "
                  f"{du[both0].max() if both0.any() else 0:.1e}{rec}")
            tot += len(ex_a)
            tot_a += (ex_a == ex_b).sum()
        print(f"  total plain/fma agreement {tot_a}/{tot}")


if __name__ == "__main__":
    main()
