# development experiment driver (GPU box): A/B timings of library variants (quick_bench)
set -e
mkdir -p gpurun_out
for v in B inl; do
  lib=belief-planning_amd/libbmpc${v:+_$v}.so
  BMPC_LIBRARY=$lib timeout -k 10 200 python tools/quick_bench.py 4096 > gpurun_out/qb_${v:-base}.log 2>&1
done
