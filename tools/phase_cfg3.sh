# phase profile (BMPC_PROFILE build) of config 3 (N=30, NB=2) at full and small batch
set -o pipefail
mkdir -p gpurun_out
export BMPC_LIBRARY=$PWD/belief-planning_amd/libbmpc_prof.so
timeout -k 10 200 python tools/phase_profile.py 4096 30 2 > gpurun_out/r02_phase_cfg3.log 2>&1 || exit $?
timeout -k 10 200 python tools/phase_profile.py 256 30 2 >> gpurun_out/r02_phase_cfg3.log 2>&1 || exit $?
cat gpurun_out/r02_phase_cfg3.log
