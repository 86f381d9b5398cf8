#!/bin/bash
# round-3 pass y: the BASELINE config sweep beside the headline (one bench.py line each), config 5's
# 8192-ego shard on one GPU, band-QP timing
set -o pipefail
tag=${1:-r03y}
mkdir -p gpurun_out
out=gpurun_out/${tag}_config_sweep.jsonl
: > $out
run() { timeout -k 10 300 python bench.py --no-cpu-baseline "$@" 2>/dev/null | tail -n 1 >> $out || exit $?; }
run --N 20 --NB 1 --batch 1024 --steps 10 --warmup 2
run --N 30 --NB 2 --batch 4096 --steps 3 --warmup 1
run --workload quadruped --steps 10 --warmup 2
run --workload robust --steps 10 --warmup 2
run --N 8 --NB 2 --batch 1 --steps 20 --warmup 2
run --N 30 --NB 2 --batch 1 --steps 10 --warmup 2
cut -c1-260 $out
timeout -k 10 300 python bench.py --gpus 1 --global-batch 8192 --no-cpu-baseline > gpurun_out/${tag}_bench_gb8192.log 2>&1 || exit $?
tail -n 1 gpurun_out/${tag}_bench_gb8192.log | cut -c1-200
timeout -k 10 200 python tools/qp_bench.py 4096 > gpurun_out/${tag}_qp_bench.log 2>&1 || exit $?
cat gpurun_out/${tag}_qp_bench.log
