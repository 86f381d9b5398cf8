# development experiment driver (GPU box): A/B of the LDS-staged tree sweeps
set -e
mkdir -p gpurun_out
timeout -k 10 200 python tools/quick_bench.py 4096 > gpurun_out/qb.log 2>&1
BMPC_NO_STAGE=1 timeout -k 10 200 python tools/quick_bench.py 4096 > gpurun_out/qb_nostage.log 2>&1
timeout -k 10 200 python tools/quick_bench.py 4096 > gpurun_out/qb2.log 2>&1
