#!/bin/bash
# round 5, ECOS equilibration pass: parity suite on the regenerated fixtures, the seeded headline /
# config-3 batches with and without equilibration (libbmpc_noeq.so = -DBMPC_EQUIL=0: statuses,
# iterations, k_ipm time), the bench, the config sweep.
set -o pipefail
tag=${1:-r05d}
o=gpurun_out/$tag
mkdir -p $o
timeout -k 10 900 python -u -m pytest tests -m gpu --maxfail=10 -q -rA --timeout 300 --timeout-method thread > $o/gpu_tests.log 2>&1
rc=$?; [ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc   # assertion failures (1) go on to the measurements; faults / timeouts stop here
for v in base noeq; do
  L=belief-planning_amd/libbmpc.so; [ $v = noeq ] && L=belief-planning_amd/libbmpc_noeq.so
  BMPC_LIBRARY=$L timeout -k 10 150 python tools/variant_check.py $o/vc_${v}_h.npz 4096 20 1 >> $o/equil_ab.log 2>&1 || exit $?
  BMPC_LIBRARY=$L timeout -k 10 300 python tools/variant_check.py $o/vc_${v}_c3.npz 4096 30 2 >> $o/equil_ab.log 2>&1 || exit $?
  echo "== $v headline" >> $o/equil_ab.log
  BMPC_LIBRARY=$L timeout -k 10 150 python tools/quick_bench.py 4096 20 1 2>&1 | grep "^step" | cut -c1-150 >> $o/equil_ab.log || exit $?
  echo "== $v config3" >> $o/equil_ab.log
  BMPC_LIBRARY=$L timeout -k 10 300 python tools/quick_bench.py 4096 30 2 2>&1 | grep "^step" | cut -c1-150 >> $o/equil_ab.log || exit $?
done
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $o/bench.log 2>&1 || exit $?
BMPC_LIBRARY=belief-planning_amd/libbmpc_noeq.so timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $o/bench_noeq.log 2>&1 || exit $?
tail -n 1 $o/bench.log | cut -c1-400
# per-phase bytes: the phase-per-kernel tools build (same arithmetic as the product kernel, bit for
# bit on the host build: tests/test_phased_host.py), its outputs against the monolithic mode
BMPC_LIBRARY=$PWD/belief-planning_amd/libbmpc_ph.so TAG=${tag}_ph MODES="0 1" PMC="0 1" timeout -k 10 900 bash tools/ab_phased.sh > $o/phased.log 2>&1 || exit $?
