#!/bin/bash
# round 5: one-ego closed-loop steps (bench.py config lines) after caching the small-batch
# kernel's LDS opt-in
set -o pipefail
o=gpurun_out/${1:-r05q}
mkdir -p $o
: > $o/b1.jsonl
for cfg in "--N 20 --NB 1" "--N 8 --NB 2"; do
  for v in 1 0; do
    BMPC_BLK_LDS=$v timeout -k 10 300 python bench.py --no-cpu-baseline $cfg --batch 1 --steps 20 --warmup 3 2>/dev/null | tail -n 1 | sed "s/^{/{\"blk_lds\": $v, /" >> $o/b1.jsonl || exit $?
  done
done
python - $o/b1.jsonl <<'PY'
import json, sys
for ln in open(sys.argv[1]):
    d = json.loads(ln); r = d["roofline"]
    print("blk_lds", d["blk_lds"], d["config"]["workload"][:60], "ms/step", d["ms_per_step"], "k_ipm", r["kernel_ms"], "k_tree", r["tree_kernel_ms"], "iters", d["closed_loop"]["iters_mean"])
PY
