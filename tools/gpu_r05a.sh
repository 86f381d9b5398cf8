#!/bin/bash
# round-5 first GPU pass: parity suite, bench, and the phase profile of the current source from
# a -DBMPC_PROFILE build next to variant_check of the product on the same seeded batch
set -o pipefail
tag=${1:-r05a}
mkdir -p gpurun_out/$tag
o=gpurun_out/$tag
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rA --timeout 180 --timeout-method thread > $o/gpu_tests.log 2>&1 || exit $?
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $o/bench.log 2>&1 || exit $?
timeout -k 10 150 python tools/variant_check.py $o/vc_base.npz 4096 20 1 > $o/vc.log 2>&1 || exit $?
BMPC_LIBRARY=belief-planning_amd/libbmpc_prof.so timeout -k 10 150 python tools/variant_check.py $o/vc_prof.npz 4096 20 1 >> $o/vc.log 2>&1 || exit $?
BMPC_LIBRARY=belief-planning_amd/libbmpc_prof.so timeout -k 10 150 python tools/phase_profile.py 4096 20 1 > $o/phase_profile_4k.log 2>&1 || exit $?
BMPC_LIBRARY=belief-planning_amd/libbmpc_prof.so timeout -k 10 150 python tools/phase_profile.py 4096 30 2 > $o/phase_profile_c3.log 2>&1 || exit $?
python - $o <<'PY'
import sys, numpy as np
o = sys.argv[1]
a, b = np.load(f"{o}/vc_base.npz"), np.load(f"{o}/vc_prof.npz")
print("prof vs base: status identical", bool(np.array_equal(a["status"], b["status"])), "iters identical",
      bool(np.array_equal(a["iters"], b["iters"])), "max |dJ|", float(np.max(np.abs(a["J"] - b["J"]))))
PY
