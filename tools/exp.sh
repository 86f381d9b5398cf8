# development experiment driver (GPU box): interleaved timings of library variants
#   bash tools/exp.sh [variant ...]   (default: "" prev; "" is libbmpc.so, X is libbmpc_X.so)
set -e
mkdir -p gpurun_out
: > gpurun_out/ab.log
vs=("$@")
[ ${#vs[@]} -eq 0 ] && vs=("" prev)
for r in 1 2 3; do
  for v in "${vs[@]}"; do
    lib=belief-planning_amd/libbmpc${v:+_$v}.so
    echo "== ${v:-base} run $r" >> gpurun_out/ab.log
    BMPC_LIBRARY=$lib timeout -k 10 200 python tools/quick_bench.py 4096 2>&1 | grep "^step [123]" | cut -c1-130 >> gpurun_out/ab.log
  done
done
python - <<'PY'
import re, collections
d = collections.defaultdict(list); cur = None
for ln in open("gpurun_out/ab.log"):
    m = re.match(r"== (\S+) run", ln)
    if m: cur = m.group(1); continue
    m = re.search(r"ipm ([\d.]+) ms", ln)
    if m: d[cur].append(float(m.group(1)))
with open("gpurun_out/ab.log", "a") as f:
    for k, v in d.items():
        f.write(f"MEAN {k}: {sum(v)/len(v):.3f} ms over {len(v)}\n")
PY
