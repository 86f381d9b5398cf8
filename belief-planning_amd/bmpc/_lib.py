"""Loader of the HIP library ``libbmpc.so`` (the product path; there is no CPU fallback).

``build()`` compiles it in-tree for gfx950 with hipcc; ``lib()`` loads it and raises
``BmpcUnavailable`` when it is missing or no HIP device is usable.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REPO = os.path.dirname(PKG_DIR)
CSRC = os.path.join(PKG_DIR, "csrc")
INCLUDE = os.path.join(REPO, "include")
SO_PATH = os.path.join(PKG_DIR, "libbmpc.so")
PROF_SO_PATH = os.path.join(PKG_DIR, "libbmpc_prof.so")   # -DBMPC_PROFILE variant (tools only)
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
EXTRA_FLAGS = []      # experiment builds (tools/build_variant.py) append -D flags here
ARCH = os.environ.get("BMPC_OFFLOAD_ARCH", "gfx950")


class BmpcUnavailable(RuntimeError):
    """libbmpc.so (the MI355X kernels) cannot be loaded or has no usable HIP device."""


EXPERIMENTAL = os.path.join(CSRC, "experimental")


def _phased() -> bool:
    """Tools-only builds with -DBMPC_WITH_PHASED add the phase-per-kernel IPM (csrc/experimental)."""
    return "-DBMPC_WITH_PHASED" in EXTRA_FLAGS


def sources():
    """Translation units of libbmpc.so: the C ABI + small kernels, one unit per predictive model's
    solver kernels (compiled in parallel), the host-side plan builders."""
    srcs = [os.path.join(CSRC, f) for f in ("bmpc_hip.hip", "bmpc_k_highway.hip", "bmpc_k_highway_t.hip",
                                            "bmpc_k_merge.hip", "bmpc_k_quadruped.hip", "bmpc_kb_highway.hip",
                                            "bmpc_kb_highway_t.hip", "bmpc_kb_merge.hip", "bmpc_kb_quadruped.hip",
                                            "bmpc_plan.cpp", "bmpc_qpplan.cpp")]
    if _phased():
        srcs += [os.path.join(EXPERIMENTAL, f) for f in ("bmpc_kp_highway.hip", "bmpc_kp_highway_t.hip",
                                                         "bmpc_kp_merge.hip")]
    return srcs


def headers():
    hs = [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".h")]
    if _phased():
        hs += [os.path.join(EXPERIMENTAL, f) for f in os.listdir(EXPERIMENTAL) if f.endswith(".h")]
    return hs + [os.path.join(INCLUDE, "bmpc.h")]


def build(force: bool = False, verbose: bool = False, profile: bool = False) -> str:
    """Compile libbmpc.so (or the phase-counter variant libbmpc_prof.so) for gfx950 in-tree
    unless a build of exactly these sources exists: the sidecar ``<so>.srchash`` records the
    source_hash() a library was compiled from (an mtime check would accept a stale binary
    that merely carries a newer timestamp)."""
    out = PROF_SO_PATH if profile else SO_PATH
    stamp = out + ".srchash"
    want = source_hash()
    if not force and os.path.exists(out) and os.path.exists(stamp):
        with open(stamp) as f:
            if f.read().strip() == want:
                return out
    import tempfile
    from concurrent.futures import ThreadPoolExecutor
    flags = [f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC",
             "-Wno-unused-value", "-Wno-unused-result", "-Wno-pass-failed",
             *(["-DBMPC_PROFILE"] if profile else []), *EXTRA_FLAGS, "-I" + INCLUDE, "-I" + CSRC,
             *(["-I" + EXPERIMENTAL] if _phased() else [])]
    with tempfile.TemporaryDirectory(prefix="bmpc_build_") as tmp:
        objs = [os.path.join(tmp, os.path.basename(src) + ".o") for src in sources()]
        cmds = [[HIPCC, *flags, "-c", src, "-o", obj] for src, obj in zip(sources(), objs)]
        if verbose:
            for c in cmds:
                print(" ".join(c))
        jobs = int(os.environ.get("MAX_JOBS", "0")) or min(len(cmds), os.cpu_count() or 1)
        with ThreadPoolExecutor(jobs) as pool:
            for f in [pool.submit(subprocess.check_call, c) for c in cmds]:
                f.result()
        link = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", *objs, "-o", out + ".tmp"]
        if verbose:
            print(" ".join(link))
        subprocess.check_call(link)
    os.replace(out + ".tmp", out)
    with open(stamp, "w") as f:
        f.write(want + "\n")
    return out


_LIB = None

_SIGS = {
    "bmpc_last_error": (C.c_char_p, []),
    "bmpc_abi_version": (C.c_int, []),
    "bmpc_open": (C.c_int, [C.c_int, C.c_void_p]),
    "bmpc_close": (C.c_int, [C.c_void_p]),
    "bmpc_plan_create": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int, C.c_void_p]),
    "bmpc_plan_destroy": (C.c_int, [C.c_void_p]),
    "bmpc_plan_info": (C.c_int, [C.c_void_p, C.c_void_p]),
    "bmpc_set_policies": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p]),
    "bmpc_reset": (C.c_int, [C.c_void_p, C.c_void_p]),
    "bmpc_get_policies": (C.c_int, [C.c_void_p, C.c_void_p]),
    "bmpc_solve": (C.c_int, [C.c_void_p] + [C.c_void_p] * 9),
    "bmpc_solve_device": (C.c_int, [C.c_void_p] + [C.c_void_p] * 10),
    "bmpc_get_tree": (C.c_int, [C.c_void_p] + [C.c_void_p] * 6),
    "bmpc_get_warm_start": (C.c_int, [C.c_void_p] * 4),
    "bmpc_get_counters": (C.c_int, [C.c_void_p] * 2),
    "bmpc_set_warm_start": (C.c_int, [C.c_void_p] * 5),
    "bmpc_get_robust_warm_start": (C.c_int, [C.c_void_p] * 4),
    "bmpc_set_robust_warm_start": (C.c_int, [C.c_void_p] * 5),
    "bmpc_set_transform": (C.c_int, [C.c_void_p] * 5),
    "bmpc_set_fx": (C.c_int, [C.c_void_p] * 3),
    "bmpc_get_branch_dp": (C.c_int, [C.c_void_p] * 2),
    "bmpc_enable_timing": (C.c_int, [C.c_void_p, C.c_int]),
    "bmpc_timing": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p]),
    "bmpc_model_eval": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int] + [C.c_void_p] * 12),
    "bmpc_model_eval_ref": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_int]
                            + [C.c_void_p] * 12),
    "bmpc_set_lane_ref": (C.c_int, [C.c_void_p, C.c_int, C.c_void_p, C.c_void_p]),
    "bmpc_hmm_eval": (C.c_int, [C.c_void_p, C.c_int, C.c_int, C.c_void_p, C.c_int] + [C.c_void_p] * 9),
    "bmpc_env_step": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int] + [C.c_void_p] * 10),
    "bmpc_loop_device": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int, C.c_int] + [C.c_void_p] * 10),
    "bmpc_qp_solve": (C.c_int, [C.c_void_p, C.c_int, C.c_int] + [C.c_void_p] * 4 + [C.c_int] + [C.c_void_p] * 5
                      + [C.c_int, C.c_double] + [C.c_void_p] * 5),
}

EXPORTED = tuple(_SIGS)


def load(path: str = SO_PATH, strict: bool = True):
    """Load a libbmpc.so and declare the C ABI (no device access).  strict=False (another
    build named by BMPC_LIBRARY, e.g. an older source for an A/B) tolerates entry points the
    build lacks: calling one raises BmpcUnavailable."""
    if not os.path.exists(path):
        raise BmpcUnavailable(f"{path} not built; run __graft_entry__.build() (hipcc --offload-arch=gfx950)")
    lib = C.CDLL(path)
    for name, (res, args) in _SIGS.items():
        if not strict and not hasattr(lib, name):
            def missing(*a, _n=name):
                raise BmpcUnavailable(f"{path} has no {_n}")
            setattr(lib, name, missing)
            continue
        f = getattr(lib, name)
        f.restype = res
        f.argtypes = args
    return lib


def stamp(path: str = SO_PATH):
    """The source hash a library was compiled from (its ``<so>.srchash`` sidecar), or None."""
    try:
        with open(path + ".srchash") as f:
            return f.read().strip() or None
    except OSError:
        return None


def check_stamp(path: str = SO_PATH) -> str:
    """Refuse a product library that was not compiled from the sources in this tree: its stamp
    must equal source_hash().  Returns the stamp."""
    have, want = stamp(path), source_hash()
    if have != want:
        raise BmpcUnavailable(f"{path} is stale: built from sources {have or '<no stamp>'}, the tree's sources "
                              f"hash to {want}; rebuild with __graft_entry__.build()")
    return have


LOADED_STAMP = None     # stamp of the library lib() loaded (bench.py reports it)


def lib():
    """The product library, refused when its stamp does not match the tree's sources;
    BMPC_LIBRARY may name another in-tree build (e.g. libbmpc_prof.so for phase counters,
    an older source for an A/B), which is loaded without the check."""
    global _LIB, LOADED_STAMP
    if _LIB is None:
        path = os.environ.get("BMPC_LIBRARY", SO_PATH)
        product = os.path.abspath(path) == os.path.abspath(SO_PATH)
        LOADED_STAMP = check_stamp(path) if product else stamp(path)
        _LIB = load(path, strict=product)
    return _LIB


def check(rc: int, what: str):
    if rc != 0:
        msg = lib().bmpc_last_error().decode(errors="replace")
        raise BmpcUnavailable(f"{what} failed ({rc}): {msg}") if rc in (-19, -5, -12) else RuntimeError(
            f"{what} failed ({rc}): {msg}")


def source_hash() -> str:
    """sha1 over the kernel sources and the ABI header: ties a profile (e.g. the PMC traffic
    bench.py reports) to the build it was measured on."""
    import hashlib
    h = hashlib.sha1()
    for p in sorted(sources() + headers()):
        with open(p, "rb") as f:
            h.update(os.path.basename(p).encode())
            h.update(f.read())
    return h.hexdigest()[:16]
