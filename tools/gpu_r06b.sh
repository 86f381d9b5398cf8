#!/bin/bash
# round 6, pass b: iteration traces of N=10 steps 2-4 (one-ego batches, -DBMPC_DEV_DEBUG build) on
# the three launch paths; the recorded replays on every path with the product build and a build
# without FMA contraction (-ffp-contract=off)
set -o pipefail
tag=${1:-r06b}
o=gpurun_out/$tag
mkdir -p $o
for p in wave lean blk; do
  case $p in
    wave) E="BMPC_BLOCK_EGOS=0 BMPC_LDS_RICH=1";;
    lean) E="BMPC_BLOCK_EGOS=0 BMPC_LDS_RICH=0";;
    blk) E="BMPC_UNUSED=0";;
  esac
  env $E BMPC_LIBRARY=belief-planning_amd/libbmpc_dbg.so timeout -k 10 120 python -u tools/trace_replay.py gpu highway_n10_nb1 2 3 4 > $o/trace_${p}_n10.log 2>&1 || exit $?
  for L in libbmpc libbmpc_nofma; do
    echo "== $p $L" >> $o/replay_paths.log
    env $E BMPC_LIBRARY=belief-planning_amd/$L.so timeout -k 10 200 python -u tools/replay_diag.py >> $o/replay_paths.log 2>&1 || exit $?
  done
done
