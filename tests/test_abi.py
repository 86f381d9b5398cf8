"""The C ABI library loads and exports every entry point include/bmpc.h declares (no device
access), and the ctypes mirror matches the header's struct layout."""
import ctypes as C
import os
import re

from common import REPO


def header_functions():
    src = open(os.path.join(REPO, "include", "bmpc.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(bmpc_[a-z_]+)\s*\(", src)))


def test_library_exports_all_header_symbols():
    from bmpc import _lib
    _lib.build()
    lib = C.CDLL(_lib.SO_PATH)
    names = header_functions()
    assert len(names) >= 15
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing
    assert set(names) == set(_lib.EXPORTED)


def test_library_is_gfx950_code_object():
    from bmpc import _lib
    _lib.build()
    blob = open(_lib.SO_PATH, "rb").read()
    assert b"gfx950" in blob


def test_abi_version_without_device():
    from bmpc import _lib
    lib = _lib.load()
    assert lib.bmpc_abi_version() == 2


def test_desc_struct_layout_matches_header():
    """sizeof(bmpc_plan_desc) from the header, computed by the host compiler."""
    import subprocess
    import tempfile
    from bmpc import abi
    code = ('#include <stdio.h>\n#include <stddef.h>\n#include "bmpc.h"\n'
            'int main(){printf("%zu %zu %zu %zu %zu\\n", sizeof(bmpc_plan_desc), offsetof(bmpc_plan_desc, Q),'
            ' offsetof(bmpc_plan_desc, mc), sizeof(bmpc_policy), offsetof(bmpc_plan_desc, flags));return 0;}\n')
    with tempfile.TemporaryDirectory() as d:
        c = os.path.join(d, "t.c")
        open(c, "w").write(code)
        exe = os.path.join(d, "t")
        subprocess.check_call(["gcc", "-I" + os.path.join(REPO, "include"), c, "-o", exe])
        out = subprocess.check_output([exe]).decode().split()
    size, offQ, offmc, psize, offfl = map(int, out)
    assert size == C.sizeof(abi.PlanDesc)
    assert offQ == abi.PlanDesc.Q.offset
    assert offmc == abi.PlanDesc.mc.offset
    assert psize == C.sizeof(abi.Policy)
    assert offfl == abi.PlanDesc.flags.offset


def test_alternate_builds_load_non_strictly(tmp_path):
    """The product library binds every entry point or fails; another build named by
    BMPC_LIBRARY (an older source in an A/B) loads without the ones it lacks, which then
    raise BmpcUnavailable when called."""
    import subprocess
    import pytest
    from bmpc import _lib
    src = tmp_path / "old.c"
    src.write_text("int bmpc_abi_version(void) { return 2; }\n")
    so = tmp_path / "libold.so"
    subprocess.check_call(["gcc", "-shared", "-fPIC", str(src), "-o", str(so)])
    with pytest.raises(AttributeError):
        _lib.load(str(so))
    lib = _lib.load(str(so), strict=False)
    assert lib.bmpc_abi_version() == 2
    with pytest.raises(_lib.BmpcUnavailable):
        lib.bmpc_set_lane_ref(None, 0, None, None)


def test_lib_refuses_a_stale_product_library(tmp_path, monkeypatch):
    """lib() loads the product libbmpc.so only when its <so>.srchash stamp equals the hash of the
    sources in the tree (a stale prebuilt binary would otherwise be measured and reported under
    the current source's hash); another build named by BMPC_LIBRARY is exempt."""
    import shutil
    import pytest
    from bmpc import _lib
    _lib.build()
    so = tmp_path / "libbmpc.so"
    shutil.copy(_lib.SO_PATH, so)
    (tmp_path / "libbmpc.so.srchash").write_text("0123456789abcdef\n")
    monkeypatch.setattr(_lib, "SO_PATH", str(so))
    monkeypatch.setattr(_lib, "_LIB", None)
    monkeypatch.delenv("BMPC_LIBRARY", raising=False)
    with pytest.raises(_lib.BmpcUnavailable, match="stale"):
        _lib.lib()
    (tmp_path / "libbmpc.so.srchash").unlink()
    with pytest.raises(_lib.BmpcUnavailable, match="no stamp"):
        _lib.lib()
    (tmp_path / "libbmpc.so.srchash").write_text(_lib.source_hash() + "\n")
    assert _lib.lib() is not None and _lib.LOADED_STAMP == _lib.source_hash()
    # an A/B build named by BMPC_LIBRARY loads whatever its stamp says
    monkeypatch.setattr(_lib, "_LIB", None)
    other = tmp_path / "libother.so"
    shutil.copy(_lib.SO_PATH, other)
    (tmp_path / "libother.so.srchash").write_text("feedfeedfeedfeed\n")
    monkeypatch.setenv("BMPC_LIBRARY", str(other))
    _lib.lib()
    assert _lib.LOADED_STAMP == "feedfeedfeedfeed"
    monkeypatch.setattr(_lib, "_LIB", None)
