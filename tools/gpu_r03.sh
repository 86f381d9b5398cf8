#!/bin/bash
# Round-3 GPU pass on one box: parity tests, the driver's exact bench command, then rocprofv3 of
# that same command (kernel trace + stats, separate FETCH_SIZE / WRITE_SIZE / SQ passes).
# usage: bash tools/gpu_r03.sh TAG [tests|notests] [pcs]
set -o pipefail
tag=${1:-r03}
mode=${2:-tests}
mkdir -p gpurun_out
if [ "$mode" = tests ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -rA --timeout 300 --timeout-method thread \
    > gpurun_out/${tag}_gpu_tests.log 2>&1 || exit $?
fi
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${tag}_bench.log 2>&1 || exit $?
tail -n 1 gpurun_out/${tag}_bench.log | cut -c1-400
PROF_KEY=highway:N20:NB1:B4096 bash tools/gpu_prof.sh ${tag} --gpus 1 --steps 20 --warmup 5 \
  > gpurun_out/${tag}_prof.log 2>&1 || exit $?
if [ "${3:-}" = pcs ]; then
  out=$PWD/gpurun_out/pcs_${tag}
  mkdir -p $out
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 240 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method host_trap \
     --pc-sampling-unit time --pc-sampling-interval 100 -d $out -o run --output-format csv -- \
     python3 $GRAFT_REPO_ROOT/bench.py --gpus 1 --steps 3 --warmup 1 --no-cpu-baseline > $out/pcs.log 2>&1) || exit $?
fi
echo done
