#!/bin/bash
# round 5 measurement pass on the current source: the BASELINE config sweep, config-5 shard size,
# the band-QP bench, rocprofv3 kernel stats + PMC passes of the default bench (traffic entry keyed
# to this source hash)
set -o pipefail
tag=${1:-r05h}
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --gpus 1 --global-batch 8192 --no-cpu-baseline > gpurun_out/${tag}_bench_gb8192.log 2>&1 || exit $?
out=gpurun_out/${tag}_config_sweep.jsonl
: > $out
run() { timeout -k 10 300 python bench.py --no-cpu-baseline "$@" 2>/dev/null | tail -n 1 >> $out || exit $?; }
run --N 20 --NB 1 --batch 1024 --steps 10 --warmup 2
run --N 30 --NB 2 --batch 4096 --steps 3 --warmup 1
run --workload quadruped --steps 10 --warmup 2
run --workload robust --steps 10 --warmup 2
run --N 8 --NB 2 --batch 1 --steps 10 --warmup 2
run --N 20 --NB 1 --batch 1 --steps 10 --warmup 2
timeout -k 10 200 python tools/qp_bench.py 4096 > gpurun_out/${tag}_qp_bench.log 2>&1 || exit $?
PROF_KEY=highway:N20:NB1:B4096 bash tools/gpu_prof.sh ${tag} --gpus 1 --steps 20 --warmup 5 > gpurun_out/${tag}_prof.log 2>&1 || exit $?
python - gpurun_out/prof_${tag}/pmc_entry.json <<'PY' || exit $?
import json, sys
e = json.load(open(sys.argv[1])); p = "profiles/pmc_traffic.json"; d = json.load(open(p))
d = [x for x in d if not (x["key"] == e["key"] and x["source_hash"] == e["source_hash"])] + [e]
json.dump(d, open(p, "w"), indent=1)
PY
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${tag}_bench.log 2>&1 || exit $?
cut -c1-200 $out; tail -n 1 gpurun_out/${tag}_bench.log | cut -c1-300
