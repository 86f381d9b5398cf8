"""Replay the golden closed loops on the GPU and print per-step exit / J agreement
(development helper; set BMPC_LIBRARY to compare builds)."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "tests"), REPO, os.path.join(REPO, "belief-planning_amd")]
from common import golden, highway_desc_from_golden, replay_batch  # noqa: E402
from bmpc import plan  # noqa: E402

for name in ("highway_n20_nb1", "highway_n8_nb2", "highway_n10_nb1", "highway_n30_nb2"):
    g = golden(name)
    rb = replay_batch(g)
    T = rb["T"]
    pl = plan.BatchPlan(highway_desc_from_golden(g), T)
    pl.set_policies(rb["rows"])
    pl.set_warm_start(rb["uLin"], rb["p"], rb["jcons"], mask=rb["warm"])
    r = pl.solve(rb["x"], rb["z"], rb["xref"])
    ex = np.asarray(g["traj_exit"][:T])
    J = np.asarray(g["traj_J"][:T])
    rel = np.abs(r["J"] - J) / np.maximum(1, np.abs(J))
    print(f"{name}: T={T} exit agree {np.mean(r['status'] == ex):.3f}  ref10 {int((ex == 10).sum())} "
          f"got10 {int((r['status'] == 10).sum())}  max relJ {rel.max():.2e}  iters {r['iters'][:6]}")
    bad = np.nonzero(r["status"] != ex)[0]
    print(f"   kernel {pl.last_kernel()}  steps whose exit differs: {bad.tolist()} (got {r['status'][bad].tolist()})")
    if T <= 5:
        print("   status", r["status"], "ref", ex, "J", r["J"], "refJ", J)
