#!/bin/bash
# round 6 final-source pass: GPU parity suite, smoke(), rocprofv3 stats + PMC traffic keyed to this
# source hash, the bench (carrying that traffic entry), the config sweep
set -o pipefail
tag=${1:-r06z}
o=gpurun_out/$tag
mkdir -p $o
timeout -k 10 1200 python -u -m pytest tests -m gpu -v -rA --timeout 600 --timeout-method thread > $o/gpu_tests.log 2>&1
rc=$?; [ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 || exit $?
PROF_KEY=highway:N20:NB1:B4096 bash tools/gpu_prof.sh ${tag} --gpus 1 --steps 20 --warmup 5 > $o/prof.log 2>&1 || exit $?
python - gpurun_out/prof_${tag}/pmc_entry.json <<'PY' || exit $?
import json, sys
e = json.load(open(sys.argv[1])); p = "profiles/pmc_traffic.json"; d = json.load(open(p))
d = [x for x in d if not (x["key"] == e["key"] and x["source_hash"] == e["source_hash"])] + [e]
json.dump(d, open(p, "w"), indent=1)
PY
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $o/bench.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --gpus 1 --global-batch 8192 --no-cpu-baseline > $o/bench_gb8192.log 2>&1 || exit $?
out=$o/config_sweep.jsonl
: > $out
run() { timeout -k 10 300 python bench.py --no-cpu-baseline "$@" 2>/dev/null | tail -n 1 >> $out || exit $?; }
run --N 20 --NB 1 --batch 1024 --steps 10 --warmup 2
run --N 30 --NB 2 --batch 4096 --steps 3 --warmup 1
run --N 30 --NB 2 --batch 4096 --steps 3 --warmup 1 --loop fused
run --N 20 --NB 1 --batch 4096 --steps 20 --warmup 5 --loop fused
run --workload quadruped --steps 10 --warmup 2
run --workload robust --steps 10 --warmup 2
run --N 8 --NB 2 --batch 1 --steps 10 --warmup 2
run --N 20 --NB 1 --batch 1 --steps 10 --warmup 2
tail -n 3 $o/gpu_tests.log; tail -n 1 $o/bench.log | cut -c1-300
