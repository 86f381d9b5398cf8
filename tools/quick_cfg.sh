# headline and config 3 bench lines (no CPU leg), for A/B of a build
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/${1:-qc}.jsonl
: > $out
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 --warmup 2 2>/dev/null | tail -n 1 >> $out || exit $?
timeout -k 10 300 python bench.py --no-cpu-baseline --N 30 --NB 2 --batch 4096 --steps 3 --warmup 1 2>/dev/null | tail -n 1 >> $out || exit $?
OUT=$out python - <<'PY'
import json, os
for l in open(os.environ["OUT"]):
    d = json.loads(l); r = d["roofline"]
    print(d["config"]["workload"][:60], d["value"], d["ms_per_step"], r.get("kernel_ms"), r.get("iters_mean"))
PY
