#!/bin/bash
# round-3 pass z: medium batches (512 / 1024 egos) on the single-wave kernel vs the 4-wave
# small-batch kernel (BMPC_BLOCK_EGOS raises its batch limit), then smoke()
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/r03z_blk_medium.log
: > $out
for cfg in "1024 20 1" "512 20 1" "1024 8 2"; do
  echo "== single-wave $cfg" >> $out
  BMPC_BLOCK_EGOS=0 timeout -k 10 120 python tools/quick_bench.py $cfg 2>&1 | grep "^step [123]" | cut -c1-120 >> $out || exit 1
  echo "== blk4 $cfg" >> $out
  BMPC_BLOCK_EGOS=4096 BMPC_BLOCK_WAVES=4 timeout -k 10 120 python tools/quick_bench.py $cfg 2>&1 | grep "^step [123]" | cut -c1-120 >> $out || exit 1
done
cat $out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03z_smoke.log 2>&1 || { tail -n 20 gpurun_out/r03z_smoke.log; exit 1; }
tail -n 5 gpurun_out/r03z_smoke.log
