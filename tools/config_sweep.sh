#!/bin/bash
# BASELINE.json configs beside the headline (GPU box): one bench.py line each, no CPU leg.
#   cfg2: highway N=20 NB=1, 1024 egos   cfg3: highway N=30 NB=2 (9 leaves), 4096 egos
#   cfg4: quadruped BranchMPCProx N=25 NB=2 (4 leaves), 1024 egos
#   cfg1: main_branch as shipped, N=8 NB=2, 1 ego (plumbing scale)
out=gpurun_out/config_sweep.jsonl
mkdir -p gpurun_out
: > $out
run() { timeout -k 10 300 python bench.py --no-cpu-baseline "$@" 2>/dev/null | tail -1 >> $out || exit $?; }
run --N 20 --NB 1 --batch 1024 --steps 10 --warmup 2
run --N 30 --NB 2 --batch 4096 --steps 5 --warmup 2
run --workload quadruped --steps 10 --warmup 2
run --N 8 --NB 2 --batch 1 --steps 20 --warmup 2
