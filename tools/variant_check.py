"""Run one seeded batch (and ego 0's iteration count) through the library named by
BMPC_LIBRARY and save the outputs: used to compare experimental builds of the same
sources with the production build (no result of this script is a parity claim)."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "belief-planning_amd")]
from bmpc import _lib, plan  # noqa: E402

if os.environ.get("BMPC_OLD_ABI"):   # an older build: declare only the symbols it exports
    def _tolerant(path=_lib.SO_PATH):
        import ctypes as C
        lib = C.CDLL(path)
        for name, (res, args) in _lib._SIGS.items():
            if hasattr(lib, name):
                getattr(lib, name).restype, getattr(lib, name).argtypes = res, args
        return lib
    _lib.load = _tolerant
from bmpc.scenarios import highway_desc, highway_policy_rows, seeded_batch  # noqa: E402

B = int(sys.argv[2]) if len(sys.argv) > 2 else 256
N = int(sys.argv[3]) if len(sys.argv) > 3 else 20     # the plan the A/B times (tools/ab_pmc.sh QB_ARGS)
NB = int(sys.argv[4]) if len(sys.argv) > 4 else 1
x, z, xref, tgt = seeded_batch(B, seed=0)
pl = plan.BatchPlan(highway_desc(N=N, NB=NB), B)
pl.set_policies(highway_policy_rows(tgt))
r = pl.solve(x, z, xref)
np.savez(sys.argv[1], status=r["status"], iters=r["iters"], J=r["J"], upred=r["upred"])
st, cnt = np.unique(r["status"], return_counts=True)
print(os.environ.get("BMPC_LIBRARY", "libbmpc.so"), f"B={B} N={N} NB={NB}", "status", dict(zip(st.tolist(), cnt.tolist())),
      "iters mean %.2f min %d" % (r["iters"].mean(), r["iters"].min()), flush=True)
