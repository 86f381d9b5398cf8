#!/bin/bash
# round 5: the small-batch kernel with LDS-resident spans (BMPC_BLK_LDS=1, default) vs the slab
# only (BMPC_BLK_LDS=0): seeded outputs compared (one ego and 64 egos, N=20 NB=1 and N=8 NB=2),
# one-ego latency interleaved, then the GPU tests of the small-batch path
set -o pipefail
o=gpurun_out/${1:-r05l}
mkdir -p $o
for cfg in "1 20 1" "64 20 1" "1 8 2" "32 8 2"; do
  set -- $cfg
  for v in 0 1; do
    BMPC_BLK_LDS=$v timeout -k 10 120 python tools/variant_check.py $o/vc_${v}_$1_$2_$3.npz $1 $2 $3 >> $o/vc.log 2>&1 || exit $?
  done
done
python - $o <<'PY' >> $o/vc.log
import sys, glob, numpy as np
o = sys.argv[1]
for f in sorted(glob.glob(f"{o}/vc_0_*.npz")):
    a, b = np.load(f), np.load(f.replace("vc_0_", "vc_1_"))
    same = all(np.array_equal(a[k], b[k]) for k in ("status", "iters", "J", "upred"))
    print(f.split("/")[-1][5:-4], "LDS vs slab bit-identical", same, "status", a["status"][:8], b["status"][:8],
          "max|dJ|", float(np.max(np.abs(a["J"] - b["J"]))))
PY
: > $o/lat.log
for rep in 1 2; do
  for cfg in "1 20 1" "1 8 2"; do
    for v in 0 1; do
      echo "== BMPC_BLK_LDS=$v B N NB = $cfg rep $rep" >> $o/lat.log
      BMPC_BLK_LDS=$v timeout -k 10 120 python tools/quick_bench.py $cfg 2>&1 | grep "^step" | cut -c1-120 >> $o/lat.log || exit $?
    done
  done
done
cat $o/vc.log; cat $o/lat.log
timeout -k 10 900 python -u -m pytest tests -m gpu -v -rA --timeout 600 --timeout-method thread -k "blk or compat or dropin or latency or xform or env" > $o/gpu_tests_blk.log 2>&1
tail -n 3 $o/gpu_tests_blk.log
