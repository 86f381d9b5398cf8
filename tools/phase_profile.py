"""Per-phase cycle breakdown of the IPM kernel (BMPC_PROFILE build, s_memtime per ego).

usage: BMPC_LIBRARY=belief-planning_amd/libbmpc_prof.so python tools/phase_profile.py [B] [N] [NB]
"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "belief-planning_amd")]
import numpy as np  # noqa: E402

from bmpc import plan  # noqa: E402
from bmpc.scenarios import highway_desc, highway_policy_rows, seeded_batch  # noqa: E402


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    N = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    NB = int(sys.argv[3]) if len(sys.argv) > 3 else 1
    x, z, xref, tgt = seeded_batch(B, seed=0)
    pl = plan.BatchPlan(highway_desc(N=N, NB=NB), B)
    pl.set_policies(highway_policy_rows(tgt))
    pl.enable_timing(True)
    r0 = pl.solve(x, z, xref)
    c0 = pl.counters(32)
    # the profiled solve is the same first solve tools/variant_check.py records (reset: no warm
    # start carried over from the solve above), so its statuses compare with the product's
    pl.reset()
    t0 = time.time()
    r = pl.solve(x, z, xref)
    assert np.array_equal(r0["status"], r["status"]) and np.array_equal(r0["iters"], r["iters"])
    wall = time.time() - t0
    c = pl.counters(32) - c0
    tm = pl.timing()
    it = r["iters"].astype(float)
    print(f"B={B} N={N} NB={NB} wall {wall*1e3:.1f} ms  k_ipm {tm['ipm_ms']:.2f} ms  k_tree {tm['tree_ms']:.3f} ms"
          f"  iters mean {it.mean():.2f}  status {np.unique(r['status'], return_counts=True)}")
    tot = c[:, 10].mean()
    print(f"{'phase':>10s} {'Mcyc/ego':>10s} {'% total':>8s} {'kcyc/iter':>10s}")
    for i, name in enumerate(plan.BatchPlan.PHASES):
        if name == "-" or name.startswith("n"):
            continue
        v = c[:, i].mean()
        print(f"{name:>10s} {v/1e6:10.3f} {100*v/max(tot,1):8.1f} {v/max(it.mean(),1)/1e3:10.1f}")
    print(f"probe: one dependent global load = {c[:, 8].mean() / (it.mean() + 1):.0f} cycles")
    ng = c[:, 18].mean()
    print(f"apply_G calls/iter {ng/it.mean():.2f}: per call total {c[:, 13].mean()/max(ng,1):.0f} "
          f"LP {c[:, 16].mean()/max(ng,1):.0f} cones {c[:, 17].mean()/max(ng,1):.0f} cycles")
    ns, nt = c[:, 11].mean(), c[:, 15].mean()
    print(f"kkt solves/ego {ns:.1f} ({ns/it.mean():.2f}/iter), tree solves/ego {nt:.1f} ({nt/it.mean():.2f}/iter); "
          f"cycles per tree solve {c[:, 6].mean()/max(nt,1):.0f}, per kkt solve {c[:, 5].mean()/max(ns,1):.0f}")


if __name__ == "__main__":
    main()
