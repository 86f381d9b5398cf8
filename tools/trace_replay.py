"""Iteration traces of single recorded closed-loop steps (development helper).

    python tools/trace_replay.py host  NAME STEP [STEP ...]   # host build with -DBMPC_HOST_DEBUG
    python tools/trace_replay.py gpu   NAME STEP [STEP ...]   # BMPC_LIBRARY = a -DBMPC_DEV_DEBUG build

Each step is replayed as a ONE-ego batch (the reference's warm start through the checkpoint ABI) so
that the trace (lane 0 of workgroup 0 on the device) is that ego's; the launch path follows the
environment (BMPC_BLOCK_EGOS=0 forces the one-wave k_ipm).  Every step's trace is preceded by a
line "== NAME STEP status J iters" printed after the solve (stdout is flushed around the solve so
the device printf buffer lands between the markers).  tools/trace_diff.py compares two traces."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "tests"), REPO, os.path.join(REPO, "belief-planning_amd")]


def main():
    mode, name, steps = sys.argv[1], sys.argv[2], [int(v) for v in sys.argv[3:]]
    from common import golden, highway_desc_from_golden, replay_batch
    g = golden(name)
    rb = replay_batch(g)
    for t in steps:
        sel = lambda a: np.ascontiguousarray(np.asarray(a)[t:t + 1])
        print(f"== begin {name} {t}", flush=True)
        if mode == "host":
            import hostsim_lib as H
            assert "HOST_DEBUG" in H.SO, H.SO
            hs = H.HostSim(highway_desc_from_golden(g), 1)
            hs.set_policies([rb["rows"][t]])
            hs.set_warm_start(sel(rb["uLin"]), sel(rb["p"]), sel(rb["jcons"]))
            hs.reset_mask(~sel(rb["warm"]))
            r = hs.solve(sel(rb["x"]), sel(rb["z"]), sel(rb["xref"]))
        else:
            from bmpc import plan
            pl = plan.BatchPlan(highway_desc_from_golden(g), 1)
            pl.set_policies([rb["rows"][t]])
            pl.set_warm_start(sel(rb["uLin"]), sel(rb["p"]), sel(rb["jcons"]), mask=sel(rb["warm"]))
            r = pl.solve(sel(rb["x"]), sel(rb["z"]), sel(rb["xref"]))
            print(f"   kernel {pl.last_kernel()}", flush=True)
        import ctypes
        ctypes.CDLL(None).fflush(None)      # the C stdio buffer of the host / HIP runtime printf
        sys.stdout.flush()
        print(f"== {name} {t} status {int(r['status'][0])} J {float(r['J'][0]):.16e} iters {int(r['iters'][0])} "
              f"recorded exit {int(g['traj_exit'][t])} J {float(g['traj_J'][t]):.16e}", flush=True)


if __name__ == "__main__":
    main()
