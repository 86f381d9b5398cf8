#!/bin/bash
# build libbmpc.so of git revision REV (default HEAD) into belief-planning_amd/libbmpc_prev.so
# (GPU A/B of the working tree against a committed state; dev helper)
set -e
rev=${1:-HEAD}
repo=$(cd "$(dirname "$0")/.." && pwd)
tmp=$(mktemp -d /tmp/bmpc_prev_XXXX)
git -C "$repo" archive "$rev" belief-planning_amd include | tar -x -C "$tmp"
python3 - "$tmp" <<'PY'
import sys
sys.path.insert(0, sys.argv[1] + "/belief-planning_amd")
from bmpc import _lib
print(_lib.build(force=True))
PY
cp "$tmp/belief-planning_amd/libbmpc.so" "$repo/belief-planning_amd/libbmpc_prev.so"
rm -rf "$tmp"
echo "built $rev -> belief-planning_amd/libbmpc_prev.so"
