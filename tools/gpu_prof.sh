#!/bin/bash
# GPU-box profile pass: rocprofv3 kernel stats of the bench + separate PMC passes.
# usage: tools/gpu_prof.sh TAG [bench args...]
tag=${1:-r01}; shift
out=$PWD/gpurun_out/prof_${tag}
mkdir -p $out
cd /tmp && export TMPDIR=/tmp
B="$GRAFT_REPO_ROOT/bench.py"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/stats -o run --output-format csv -- python3 $B --no-cpu-baseline "$@" > $out/stats.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $out/fetch -o run --output-format csv -- python3 $B --no-cpu-baseline "$@" > $out/fetch.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $out/write -o run --output-format csv -- python3 $B --no-cpu-baseline "$@" > $out/write.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE --kernel-trace -d $out/sq -o run --output-format csv -- python3 $B --no-cpu-baseline "$@" > $out/sq.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace -d $out/tcc -o run --output-format csv -- python3 $B --no-cpu-baseline "$@" > $out/tcc.log 2>&1 || exit $?
python3 $GRAFT_REPO_ROOT/tools/prof_summary.py $out "${PROF_KEY:-highway:N20:NB1:B4096}"
