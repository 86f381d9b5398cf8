mkdir -p gpurun_out
: > gpurun_out/sweep.log
for b in 1 16 64 256 1024 4096; do
  echo "== B $b" >> gpurun_out/sweep.log
  timeout -k 10 100 python tools/quick_bench.py $b 2>&1 | grep "^step [123]" | cut -c1-120 >> gpurun_out/sweep.log || exit 1
done
for b in 64 256 4096; do
  BMPC_LIBRARY=belief-planning_amd/libbmpc_prof.so timeout -k 10 100 python tools/phase_profile.py $b >> gpurun_out/sweep.log 2>&1 || exit 1
done
