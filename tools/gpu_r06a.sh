#!/bin/bash
# round 6, pass a: the GPU suite at the round-5 bars with every replay's exit agreement printed;
# iteration traces of the N=10 recorded steps 2-4 (one-ego batches) on the three launch paths from
# the -DBMPC_DEV_DEBUG build (host-build traces: profiles/r06/trace_host_n10.log); the replays on
# every path with a build without FMA contraction (-ffp-contract=off); smoke; bench.
set -o pipefail
tag=${1:-r06a}
o=gpurun_out/$tag
mkdir -p $o
timeout -k 10 900 python -u -m pytest tests -m gpu --maxfail=20 -q -rA --timeout 300 --timeout-method thread > $o/gpu_tests.log 2>&1
rc=$?; [ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc   # assertion failures (1) go on; faults / timeouts stop here
for p in wave lean blk; do
  case $p in
    wave) E="BMPC_BLOCK_EGOS=0 BMPC_LDS_RICH=1";;
    lean) E="BMPC_BLOCK_EGOS=0 BMPC_LDS_RICH=0";;
    blk) E="";;
  esac
  env $E BMPC_LIBRARY=belief-planning_amd/libbmpc_dbg.so timeout -k 10 120 python -u tools/trace_replay.py gpu highway_n10_nb1 2 3 4 > $o/trace_${p}_n10.log 2>&1 || exit $?
  for L in libbmpc libbmpc_nofma; do
    echo "== $p $L" >> $o/replay_paths.log
    env $E BMPC_LIBRARY=belief-planning_amd/$L.so timeout -k 10 200 python -u tools/replay_diag.py >> $o/replay_paths.log 2>&1 || exit $?
  done
done
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 || exit $?
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $o/bench.log 2>&1 || exit $?
tail -n 1 $o/bench.log | cut -c1-300
