# topology tables in LDS vs global memory (BMPC_LDS_RICH) on the deep-tree configs, after the GPU suite
set -o pipefail
mkdir -p gpurun_out
tag=${1:-r02e}
out=gpurun_out/${tag}_topo_ab.jsonl
: > $out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${tag}_gpu_tests.log 2>&1 || exit $?
run() { timeout -k 10 300 python bench.py --no-cpu-baseline "$@" 2>/dev/null | tail -n 1 >> $out || exit $?; }
run --N 30 --NB 2 --batch 4096 --steps 3 --warmup 1
BMPC_LDS_RICH=1 run --N 30 --NB 2 --batch 4096 --steps 3 --warmup 1
run --N 8 --NB 2 --batch 4096 --steps 5 --warmup 2
BMPC_LDS_RICH=1 run --N 8 --NB 2 --batch 4096 --steps 5 --warmup 2
run --steps 10 --warmup 2
BMPC_LDS_RICH=0 run --steps 10 --warmup 2
tail -n 3 gpurun_out/${tag}_gpu_tests.log
OUT=$out python - <<'PY'
import json, os
for l in open(os.environ["OUT"]):
    d = json.loads(l); r = d["roofline"]
    print(d["config"]["workload"][:60], d["value"], d["ms_per_step"], r.get("kernel_ms"), r.get("iters_mean"))
PY
