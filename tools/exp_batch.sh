#!/bin/bash
# development: k_ipm time of library variants at several batch sizes (GPU box)
#   bash tools/exp_batch.sh "256 1024 4096" base wpe1 ...   (base = libbmpc.so)
mkdir -p gpurun_out
bs=$1; shift
: > gpurun_out/expb.log
for v in "$@"; do
  lib=belief-planning_amd/libbmpc.so
  [ "$v" != base ] && lib=belief-planning_amd/libbmpc_$v.so
  for b in $bs; do
    echo "== $v B=$b" >> gpurun_out/expb.log
    BMPC_LIBRARY=$lib timeout -k 10 120 python tools/quick_bench.py $b 2>&1 | grep "^step [123]" | cut -c1-100 >> gpurun_out/expb.log || exit 1
  done
done
python - <<'PY'
import re
cur=None; out={}
for ln in open("gpurun_out/expb.log"):
    m = re.match(r"== (\S+ B=\d+)", ln)
    if m: cur = m.group(1); out[cur] = []; continue
    m = re.search(r"ipm ([\d.]+) ms", ln)
    if m: out[cur].append(float(m.group(1)))
with open("gpurun_out/expb.log", "a") as f:
    for k, v in out.items():
        f.write(f"MEAN {k}: {sum(v)/max(len(v),1):.2f} ms\n")
PY
grep MEAN gpurun_out/expb.log
