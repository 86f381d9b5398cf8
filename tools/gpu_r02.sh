#!/bin/bash
# round-2 GPU pass: parity tests, default bench (CPU baselines), config-5 shard size, profile
tag=${1:-r02}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rA --timeout 120 --timeout-method thread > gpurun_out/${tag}_gpu_tests.log 2>&1 || exit $?
timeout -k 10 400 python bench.py > gpurun_out/${tag}_bench.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --gpus 1 --global-batch 8192 --no-cpu-baseline > gpurun_out/${tag}_bench_gb8192.log 2>&1 || exit $?
PROF_KEY=highway:N20:NB1:B4096 bash tools/gpu_prof.sh ${tag} --steps 5 --warmup 2 > gpurun_out/${tag}_prof.log 2>&1 || exit $?
tail -1 gpurun_out/${tag}_bench.log
