set -o pipefail
mkdir -p gpurun_out
bash tools/gpu_calib.sh r03e_calib > gpurun_out/r03e_calib.log 2>&1 || exit $?
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r03e_bench.log 2>&1 || exit $?
tail -n 1 gpurun_out/r03e_bench.log | cut -c1-300
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rA --timeout 300 --timeout-method thread > gpurun_out/r03e_gpu_tests.log 2>&1 || exit $?
tail -n 2 gpurun_out/r03e_gpu_tests.log
