#!/bin/bash
# GPU A/B of the current build (libbmpc.so) against baseline builds (libbmpc_prev.so, ...):
# one seeded 4096-ego batch through each (outputs compared with prev), interleaved k_ipm
# timings, then the GPU suite on the current build.
mkdir -p gpurun_out
VARS=${VARS:-prev f1 base}
for v in $VARS; do
  lib=belief-planning_amd/libbmpc.so; [ $v != base ] && lib=belief-planning_amd/libbmpc_$v.so
  BMPC_LIBRARY=$lib timeout -k 10 120 python tools/variant_check.py gpurun_out/vc_$v.npz 4096 || exit 1
done
VARS="$VARS" python - <<'PY'
import os
import numpy as np
a = np.load("gpurun_out/vc_prev.npz")
for tag in os.environ["VARS"].split()[1:]:
    b = np.load(f"gpurun_out/vc_{tag}.npz")
    print(tag, "status agree %.4f  #0 %d -> %d  iters mean %.2f -> %.2f  max |dJ|/|J| %.2e  max |du0| %.2e" % (
        np.mean(a["status"] == b["status"]), (a["status"] == 0).sum(), (b["status"] == 0).sum(), a["iters"].mean(),
        b["iters"].mean(), np.max(np.abs(a["J"] - b["J"]) / np.maximum(1, np.abs(a["J"]))),
        np.max(np.abs(a["upred"][:, 0] - b["upred"][:, 0]))))
PY
bash tools/exp_batch.sh "4096" $VARS $VARS || exit 1
[ -n "$SKIP_TESTS" ] && exit 0
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/ab_tests.log 2>&1
tail -5 gpurun_out/ab_tests.log
