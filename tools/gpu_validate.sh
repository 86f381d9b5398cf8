mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > gpurun_out/r01h_smoke.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --workload quadruped --no-cpu-baseline > gpurun_out/r01h_quad.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --workload robust --no-cpu-baseline > gpurun_out/r01h_robust.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --batch 1024 --no-cpu-baseline > gpurun_out/r01h_cfg2.log 2>&1 || exit $?
tail -1 gpurun_out/r01h_smoke.log
