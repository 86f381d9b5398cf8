# batch-size sweep of one solve (development helper): latency- vs bandwidth-bound check
mkdir -p gpurun_out
for b in 256 1024 2048 4096 8192; do
  echo "== B $b" >> gpurun_out/occ.log
  timeout -k 10 100 python tools/quick_bench.py $b 2>&1 | grep "^step" >> gpurun_out/occ.log || exit 1
done
