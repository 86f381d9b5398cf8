"""Replay the golden CVaR closed loops on the HOST build of the kernel templates (tests/hostsim)
and print per-scene exit agreement and the exit-0 errors (development helper, CPU; the
BMPC_HOSTSIM_FLAGS environment variable selects a host build with extra -D flags)."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "tests"), REPO, os.path.join(REPO, "belief-planning_amd")]
import hostsim_lib as H  # noqa: E402
from common import golden, highway_desc_from_golden, replay_batch  # noqa: E402


def report(name, r, g, T):
    ex, J, u = (np.asarray(g[k][:T]) for k in ("traj_exit", "traj_J", "traj_u"))
    both0 = (ex == 0) & (r["status"] == 0)
    rel = np.abs(r["J"] - J) / np.maximum(1, np.abs(J))
    du = np.max(np.abs(r["upred"][:, 0] - u), axis=1)
    print(f"{name:22s} T={T:3d} exit agree {int((r['status'] == ex).sum())}/{T}  ref exit10 {int((ex == 10).sum())}  "
          f"got exit10 {int((r['status'] == 10).sum())}  exit-0: max relJ {rel[both0].max() if both0.any() else 0:.1e} "
          f"max|du0| {du[both0].max() if both0.any() else 0:.1e}  all: max|du0| {du.max():.1e}  iters {r['iters'].mean():.2f}",
          flush=True)


for name in sys.argv[1:] or ("highway_n10_nb1", "highway_n8_nb2", "highway_n20_nb1", "highway_n30_nb2", "merge_n40_nb1"):
    g = golden(name)
    if name.startswith("merge"):
        from test_merge import merge_desc, merge_rows, replay_inputs
        rb = replay_inputs(g)
        hs = H.HostSim(merge_desc(g), rb["T"])
        hs.set_policies(merge_rows(g, rb["T"]))
        hs.set_warm_start(rb["uLin"], rb["p"], rb["jcons"])
        hs.reset_mask(~rb["warm"])
        hs.set_transform(rb["S"], rb["bx"])
    else:
        rb = replay_batch(g)
        hs = H.HostSim(highway_desc_from_golden(g), rb["T"])
        hs.set_policies(rb["rows"])
        hs.set_warm_start(rb["uLin"], rb["p"], rb["jcons"])
        hs.reset_mask(~rb["warm"])
    r = hs.solve(rb["x"], rb["z"], rb["xref"])
    report(name, r, g, rb["T"])
