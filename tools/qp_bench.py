"""bmpc_qp_solve timing on the belief-MPC problems the reference assembled
(tests/golden/belief_m1.npz, step 0): one problem (the drop-in's per-solve latency, host
analysis and transfers included) and a batch of B copies with perturbed q (throughput).
Prints one JSON line."""
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "belief-planning_amd"), os.path.join(REPO, "tests")]
from bmpc import plan  # noqa: E402
from common import coo, golden  # noqa: E402

g = golden("belief_m1")
P, q, A, l, u = coo(g, "s0_P"), g["s0_q"], coo(g, "s0_A"), g["s0_l"], g["s0_u"]
plan.context(0)
r = plan.qp_solve(P, q, A, l, u)
lat = []
for _ in range(5):
    t0 = time.perf_counter()
    r = plan.qp_solve(P, q, A, l, u)
    lat.append(time.perf_counter() - t0)
B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
rng = np.random.default_rng(0)
qs = q[None, :] * (1.0 + 0.01 * rng.standard_normal((B, len(q))))
t0 = time.perf_counter()
rb = plan.qp_solve([P] * B, qs, [A] * B, np.tile(l, (B, 1)), np.tile(u, (B, 1)))
tb = time.perf_counter() - t0
print(json.dumps({"problem": "belief_m1 step 0 (PredictiveControllers.MPC QP)", "n": int(P.shape[0]),
                  "m": int(A.shape[0]), "kkt_dim": int(r["info"][0]), "bandwidth": int(r["info"][1]),
                  "iters": int(r["iters"][0]), "latency_ms_median": 1e3 * float(np.median(lat)),
                  "batch": B, "batch_s": tb, "batch_solves_per_s": B / tb,
                  "batch_solved": int(np.sum(rb["status"] == 1)), "batch_iters_mean": float(rb["iters"].mean())}))
