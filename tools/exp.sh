set -e
timeout -k 10 200 python tools/replay_diag.py > gpurun_out/diag.log 2>&1
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/gpu_tests.log 2>&1
timeout -k 10 200 python tools/quick_bench.py 4096 2>&1 | grep "^step" > gpurun_out/qb.log
BMPC_LIBRARY=belief-planning_amd/libbmpc_prof.so timeout -k 10 200 python tools/phase_profile.py 4096 > gpurun_out/ph.log 2>&1
