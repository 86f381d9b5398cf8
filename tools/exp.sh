# development experiment driver (GPU box): interleaved A/B timings of two library variants
set -e
mkdir -p gpurun_out
: > gpurun_out/ab.log
for r in 1 2 3; do
  for v in "" prev; do
    lib=belief-planning_amd/libbmpc${v:+_$v}.so
    echo "== ${v:-base} run $r" >> gpurun_out/ab.log
    BMPC_LIBRARY=$lib timeout -k 10 200 python tools/quick_bench.py 4096 2>&1 | grep "^step [123]" | cut -c1-58 >> gpurun_out/ab.log
  done
done
