#!/bin/bash
# round-3 pass x: one-ego latency of the multi-wave small-batch kernel at 4 / 8 / 16 waves per ego
# (BMPC_BLOCK_EGOS forces it for every tree) against the single-wave kernel
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/r03x_blk_waves.log
: > $out
for cfg in "1 8 2" "1 20 1" "1 30 2"; do
  echo "== single-wave $cfg" >> $out
  timeout -k 10 120 python tools/quick_bench.py $cfg 2>&1 | grep "^step [123]" | cut -c1-120 >> $out || exit 1
  for w in w4 w8; do
    echo "== $w $cfg" >> $out
    BMPC_LIBRARY=belief-planning_amd/libbmpc_$w.so BMPC_BLOCK_EGOS=4096 timeout -k 10 120 python tools/quick_bench.py $cfg 2>&1 | grep "^step [123]" | cut -c1-120 >> $out || exit 1
  done
  echo "== w16 $cfg" >> $out
  BMPC_BLOCK_EGOS=4096 timeout -k 10 120 python tools/quick_bench.py $cfg 2>&1 | grep "^step [123]" | cut -c1-120 >> $out || exit 1
done
cat $out
