#!/bin/bash
# compiler's per-kernel / per-function resource report (VGPRs, spills, scratch, LDS, occupancy)
# of the highway model's solver translation unit (k_tree, k_ipm, k_qp and the out-of-line
# device functions they call).
# usage: tools/resource_usage.sh [-DFLAG ...]   (MODEL=merge|quadruped|highway_t picks another TU; TU=bmpc_kp_highway.hip names one)
cd "$(dirname "$0")/.."
tu=belief-planning_amd/csrc/${TU:-bmpc_k_${MODEL:-highway}.hip}
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 --cuda-device-only -c -o /tmp/ru_$$.o \
  -Wno-unused-value -Wno-unused-result -Wno-pass-failed -Rpass-analysis=kernel-resource-usage "$@" \
  -Iinclude -Ibelief-planning_amd/csrc "$tu" > /tmp/ru_$$.log 2>&1
python3 - /tmp/ru_$$.log <<'EOF'
import re, subprocess, sys
blocks, cur = [], None
for line in open(sys.argv[1]):
    m = re.search(r"remark: (.*)", line)
    if not m:
        continue
    s = m.group(1)
    if s.startswith("Function Name:"):
        cur = {"name": s.split(":", 1)[1].strip()}
        blocks.append(cur)
    elif cur is not None and ":" in s:
        k, v = s.split(":", 1)
        cur[k.strip()] = re.sub(r" \[-Rpass.*", "", v.strip())
names = [b["name"] for b in blocks]
dem = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True,
                     text=True).stdout.split("\n") if names else []
cols = ["VGPRs", "AGPRs", "SGPRs", "VGPRs Spill", "SGPRs Spill", "ScratchSize [bytes/lane]",
        "LDS Size [bytes/block]", "Occupancy [waves/SIMD]"]
print("%-60s " % "function" + " ".join("%8s" % c.split()[0][:8] + ("" if " " not in c else "") for c in cols))
for b, d in zip(blocks, dem):
    d = re.sub(r"\(.*", "", d.replace("(anonymous namespace)::", ""))[-60:]
    print("%-60s " % d + " ".join("%8s" % b.get(c, "-") for c in cols))
EOF
rm -f /tmp/ru_$$.o /tmp/ru_$$.log
