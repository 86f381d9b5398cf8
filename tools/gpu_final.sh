#!/bin/bash
# round-end GPU pass: parity tests, smoke(), default bench (CPU baselines), config-5 shard size, the
# BASELINE config sweep, the QP-solver timing, rocprofv3 stats + PMC passes of the bench
# usage: bash tools/gpu_final.sh TAG
set -o pipefail
tag=${1:-r02}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rA --timeout 180 --timeout-method thread > gpurun_out/${tag}_gpu_tests.log 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${tag}_smoke.log 2>&1 || exit $?
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${tag}_bench.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --gpus 1 --global-batch 8192 --no-cpu-baseline > gpurun_out/${tag}_bench_gb8192.log 2>&1 || exit $?
out=gpurun_out/${tag}_config_sweep.jsonl
: > $out
run() { timeout -k 10 300 python bench.py --no-cpu-baseline "$@" 2>/dev/null | tail -n 1 >> $out || exit $?; }
run --N 20 --NB 1 --batch 1024 --steps 10 --warmup 2
run --N 30 --NB 2 --batch 4096 --steps 3 --warmup 1
run --workload quadruped --steps 10 --warmup 2
run --workload robust --steps 10 --warmup 2
run --N 8 --NB 2 --batch 1 --steps 10 --warmup 2
timeout -k 10 200 python tools/qp_bench.py 4096 > gpurun_out/${tag}_qp_bench.log 2>&1 || exit $?
PROF_KEY=highway:N20:NB1:B4096 bash tools/gpu_prof.sh ${tag} --gpus 1 --steps 20 --warmup 5 > gpurun_out/${tag}_prof.log 2>&1 || exit $?
tail -n 1 gpurun_out/${tag}_bench.log | cut -c1-300
