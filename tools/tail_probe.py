"""Straggler probe (development helper, GPU box): how much of a k_ipm launch is the tail of
egos that need many more IPM iterations than the batch mean.

For the seeded 4096-ego highway batch (N=20, NB=1) over a few closed-loop steps it prints the
iteration distribution and the k_ipm time (HIP events), then the same launch with every ego a
copy of one median-iteration ego (identical work, no tail): the per-iteration time at full load.
    python tools/tail_probe.py [B] [N] [NB]
"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "belief-planning_amd")]
from bmpc import plan  # noqa: E402
from bmpc.scenarios import highway_desc, highway_policy_rows, seeded_batch  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
N = int(sys.argv[2]) if len(sys.argv) > 2 else 20
NB = int(sys.argv[3]) if len(sys.argv) > 3 else 1
x, z, xref, tgt = seeded_batch(B, 0)


def run(x, z, xref, tgt, steps, tag):
    pl = plan.BatchPlan(highway_desc(N, NB), len(x))
    pl.set_policies(highway_policy_rows(tgt))
    pl.enable_timing(True)
    out = []
    for step in range(steps):
        r = pl.solve(x, z, xref)
        tm = pl.timing()
        its = r["iters"]
        pc = np.percentile(its, [50, 90, 99, 100])
        print(f"{tag} step {step}: k_ipm {tm['ipm_ms']:.2f} ms  iters mean {its.mean():.2f}  p50/p90/p99/max "
              f"{pc[0]:.0f}/{pc[1]:.0f}/{pc[2]:.0f}/{pc[3]:.0f}  ms per mean-iter {tm['ipm_ms'] / its.mean():.3f}  "
              f"ms per max-iter {tm['ipm_ms'] / its.max():.3f}", flush=True)
        out.append((tm["ipm_ms"], its.copy()))
        u0 = r["upred"][:, 0]
        x = x + 0.1 * np.stack([x[:, 2] * np.cos(x[:, 3]), x[:, 2] * np.sin(x[:, 3]), u0[:, 0], u0[:, 1]], 1)
        z = z + 0.1 * np.stack([z[:, 2], 0 * z[:, 0], 0 * z[:, 0], 0 * z[:, 0]], 1)
    return out


res = run(x, z, xref, tgt, 4, "seeded")
its = res[-1][1]
e = int(np.argsort(its)[len(its) // 2])   # a median-iteration ego of the last step
rep = lambda a: np.repeat(a[e:e + 1], B, 0)   # noqa: E731
run(rep(x), rep(z), rep(xref), rep(tgt), 2, f"uniform(ego {e})")
for b in (16, 64, 256, 1024):
    run(x[:b], z[:b], xref[:b], tgt[:b], 2, f"B={b}")
