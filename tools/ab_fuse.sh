#!/bin/bash
# GPU A/B of the current build (libbmpc.so) against a baseline build (libbmpc_prev.so):
# the GPU suite on the current build, one seeded 4096-ego batch through both (outputs
# compared), then interleaved k_ipm timings.
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ab_tests.log 2>&1 || { tail -30 gpurun_out/ab_tests.log; exit 1; }
tail -2 gpurun_out/ab_tests.log
for v in prev f1 base; do
  lib=belief-planning_amd/libbmpc.so; [ $v != base ] && lib=belief-planning_amd/libbmpc_$v.so
  BMPC_LIBRARY=$lib timeout -k 10 120 python tools/variant_check.py gpurun_out/vc_$v.npz 4096 || exit 1
done
python - <<'PY'
import numpy as np
import sys
for tag in ("f1", "base"):
  a, b = np.load("gpurun_out/vc_prev.npz"), np.load(f"gpurun_out/vc_{tag}.npz")
  print(tag, "status agree %.4f  iters mean %.2f -> %.2f  max |dJ|/|J| %.2e  max |du0| %.2e" % (
      np.mean(a["status"] == b["status"]), a["iters"].mean(), b["iters"].mean(),
    np.max(np.abs(a["J"] - b["J"]) / np.maximum(1, np.abs(a["J"]))), np.max(np.abs(a["upred"][:, 0] - b["upred"][:, 0]))))
PY
bash tools/exp_batch.sh "4096" prev f1 base prev f1 base
