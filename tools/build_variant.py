"""Build an experimental variant of libbmpc.so with extra -D flags (development helper).

    python tools/build_variant.py TAG -DBMPC_WPE=3 ...  ->  belief-planning_amd/libbmpc_TAG.so
Run it with BMPC_LIBRARY=belief-planning_amd/libbmpc_TAG.so."""
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "belief-planning_amd"))
from bmpc import _lib  # noqa: E402

tag, flags = sys.argv[1], sys.argv[2:]
out = os.path.join(os.path.dirname(_lib.SO_PATH), f"libbmpc_{tag}.so")
_lib.EXTRA_FLAGS[:] = flags
_lib.SO_PATH = out
print(_lib.build(force=True))
