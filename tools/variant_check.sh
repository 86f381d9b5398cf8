# experimental builds of the same sources vs the production build (tools/variant_check.py)
set -o pipefail
mkdir -p gpurun_out
L=$PWD/belief-planning_amd
: > gpurun_out/vc.log
for v in oldA oldB oldC; do
  BMPC_OLD_ABI=1 BMPC_LIBRARY=$L/libbmpc_$v.so timeout -k 10 120 python tools/variant_check.py gpurun_out/vc_$v.npz 64 >> gpurun_out/vc.log 2>&1 || exit $?
done
cat gpurun_out/vc.log
