#!/bin/bash
# round 5: where the one-ego step's time outside k_ipm goes with LDS-resident spans (kernel +
# HIP runtime API trace of the bench's one-ego N=20 NB=1 line)
set -o pipefail
o=$PWD/gpurun_out/${1:-r05r}
mkdir -p $o
R=$PWD
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace --stats -d $o/tr -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --N 20 --NB 1 --batch 1 --steps 20 --warmup 3 > $o/tr.log 2>&1 || exit $?
for f in $(find $o/tr -name "*stats.csv"); do echo "== $f"; head -25 $f; done > $o/stats.txt
find $o/tr -name "*.csv" ! -name "*stats.csv" -size +1M -delete
cat $o/stats.txt | cut -c1-200
