#!/bin/bash
# round-3 GPU pass l: small-batch multi-wave solver (k_solve_blk) vs one wave per ego; GPU suite; phase profiles
set -o pipefail
mkdir -p gpurun_out/r03l
for be in 0 4096; do
  BMPC_BLOCK_EGOS=$be timeout -k 10 150 python tools/variant_check.py gpurun_out/r03l/vc_blk$be.npz 64 || exit $?
done
python - <<'PY' || exit $?
import numpy as np
a, b = np.load("gpurun_out/r03l/vc_blk0.npz"), np.load("gpurun_out/r03l/vc_blk4096.npz")
print("block vs wave (64 egos):", {k: bool(np.array_equal(a[k], b[k])) for k in a.files},
      "max |dJ|/|J| %.3e" % np.max(np.abs(a["J"] - b["J"]) / np.maximum(1, np.abs(a["J"]))),
      "status agree %.4f" % np.mean(a["status"] == b["status"]), "iters", a["iters"].mean(), b["iters"].mean())
PY
for cfg in "1 8 2" "1 20 1" "1 30 2" "64 8 2" "256 8 2"; do
  for be in 0 4096; do
    echo "== blk=$be $cfg" >> gpurun_out/r03l/lat.log
    BMPC_BLOCK_EGOS=$be timeout -k 10 200 python tools/quick_bench.py $cfg 2>&1 | grep "^step [123]" | cut -c1-110 >> gpurun_out/r03l/lat.log || exit $?
  done
done
grep -A3 "==" gpurun_out/r03l/lat.log | grep -v "^--"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rA --timeout 300 --timeout-method thread > gpurun_out/r03l/gpu_tests.log 2>&1 || exit $?
tail -n 2 gpurun_out/r03l/gpu_tests.log
P=belief-planning_amd/libbmpc_prof.so
for cfg in "4096 20 1" "4096 30 2"; do
  echo "== $cfg" >> gpurun_out/r03l/phase.log
  BMPC_LIBRARY=$P timeout -k 10 300 python tools/phase_profile.py $cfg >> gpurun_out/r03l/phase.log 2>&1 || exit $?
done
cat gpurun_out/r03l/phase.log
