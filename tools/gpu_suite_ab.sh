# GPU suite on the production build, then once on an experimental build of the same sources
# (BMPC_LIBRARY), then a short bench of the production build
set -o pipefail
mkdir -p gpurun_out
tag=${1:-r02d}
alt=${2:-libbmpc_w8.so}
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -rA --timeout 120 --timeout-method thread > gpurun_out/${tag}_gpu_tests.log 2>&1 || exit $?
BMPC_LIBRARY=$PWD/belief-planning_amd/$alt timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${tag}_gpu_tests_${alt%.so}.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/${tag}_bench_quick.log 2>&1 || exit $?
tail -2 gpurun_out/${tag}_gpu_tests.log gpurun_out/${tag}_gpu_tests_${alt%.so}.log; tail -1 gpurun_out/${tag}_bench_quick.log | cut -c1-600
