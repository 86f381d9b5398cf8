#!/bin/bash
# compiler's per-kernel resource report (VGPRs, spills, scratch, LDS, occupancy) of k_ipm<Highway>
# usage: tools/resource_usage.sh [-DFLAG ...]
cd "$(dirname "$0")/.."
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 --cuda-device-only -c -o /tmp/ru_$$.o \
  -Wno-unused-value -Wno-unused-result -Wno-pass-failed -Rpass-analysis=kernel-resource-usage "$@" \
  -Iinclude -Ibelief-planning_amd/csrc belief-planning_amd/csrc/bmpc_hip.hip > /tmp/ru_$$.log 2>&1
grep -A11 "Function Name: _ZN12_GLOBAL__N_15k_ipmIN4bmpc7Highway" /tmp/ru_$$.log | sed 's/.*remark: //'
rm -f /tmp/ru_$$.o /tmp/ru_$$.log
