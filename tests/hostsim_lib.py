"""ctypes wrapper of the TEST-ONLY host build (tests/hostsim/libbmpc_hostsim.so).

Builds the shared object on first use with g++ from the same csrc templates the HIP
kernels instantiate, so CPU tests can check the kernel algorithm against the oracle.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
PKG = os.path.join(REPO, "belief-planning_amd")
if PKG not in sys.path:
    sys.path.insert(0, PKG)

from bmpc import abi  # noqa: E402

# BMPC_HOSTSIM_FLAGS: extra -D flags for algorithm experiments (a separate .so per flag set)
FLAGS = os.environ.get("BMPC_HOSTSIM_FLAGS", "").split()
SO = os.path.join(HERE, "hostsim", "libbmpc_hostsim%s.so" % (
    "" if not FLAGS else "_" + "".join(c if c.isalnum() else "_" for c in "".join(FLAGS))[:80]))
SRCS = [os.path.join(HERE, "hostsim", "hostsim.cpp"), os.path.join(PKG, "csrc", "bmpc_plan.cpp"),
        os.path.join(PKG, "csrc", "bmpc_qpplan.cpp")]
EXP = os.path.join(PKG, "csrc", "experimental")   # the phase sequence of the experimental phased IPM
HDRS = [os.path.join(PKG, "csrc", f) for f in os.listdir(os.path.join(PKG, "csrc")) if f.endswith(".h")] + \
    [os.path.join(EXP, f) for f in os.listdir(EXP) if f.endswith(".h")]


def source_hash():
    """Hash of the sources, headers and flag set a host build is compiled from (the sidecar
    ``<so>.srchash`` records it: an mtime check would accept a stale binary)."""
    import hashlib
    h = hashlib.sha256()
    for p in sorted(SRCS + HDRS + [os.path.join(REPO, "include", "bmpc.h")]):
        with open(p, "rb") as f:
            h.update(os.path.basename(p).encode() + b"\0" + f.read())
    h.update(" ".join(FLAGS).encode())
    return h.hexdigest()[:16]


def build(force=False):
    stamp = SO + ".srchash"
    want = source_hash()
    have = open(stamp).read().strip() if os.path.exists(stamp) and os.path.exists(SO) else None
    if force or have != want:
        tmp = SO + f".{os.getpid()}.tmp"
        cmd = ["g++", "-O2", "-std=c++17", "-shared", "-fPIC", "-fopenmp", "-Wno-unknown-pragmas",
               *FLAGS, "-I" + os.path.join(REPO, "include"), "-I" + os.path.join(PKG, "csrc"), "-I" + EXP, *SRCS,
               "-o", tmp]
        subprocess.check_call(cmd)
        os.replace(tmp, SO)                      # atomic: concurrent test workers each build their own
        with open(stamp + f".{os.getpid()}", "w") as f:
            f.write(want + "\n")
        os.replace(stamp + f".{os.getpid()}", stamp)
    return SO


_lib = None


def lib():
    global _lib
    if _lib is None:
        _lib = C.CDLL(build())
        _lib.hs_last_error.restype = C.c_char_p
    return _lib


def _p(a):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


class HostSim:
    def __init__(self, desc, batch):
        self.desc = desc
        self.batch = batch
        h = C.c_void_p()
        rc = lib().hs_create(C.byref(desc), batch, C.byref(h))
        if rc != 0:
            raise RuntimeError(lib().hs_last_error().decode())
        self.h = h
        info = np.zeros(abi.INFO_COUNT, np.int32)
        lib().hs_info(h, _p(info))
        self.T, self.U, self.bdim, self.nbranch, self.nv = (int(info[i]) for i in range(5))
        self.info = info

    def __del__(self):
        try:
            lib().hs_destroy(self.h)
        except Exception:
            pass

    def set_policies(self, pol_rows):
        arr = abi.policy_array(pol_rows)
        lib().hs_set_policies(self.h, arr)

    def set_lane_ref(self, grid, values):
        self._lref = [np.ascontiguousarray(np.asarray(v, float).reshape(-1)) for v in (grid, values)]
        lib().hs_set_lane_ref(self.h, self._lref[0].size, _p(self._lref[0]), _p(self._lref[1]))

    def solve(self, x, z, xref):
        B, n, d = self.batch, self.desc.n, self.desc.d
        x, z, xref = (np.ascontiguousarray(np.asarray(v, float).reshape(B, n)) for v in (x, z, xref))
        up = np.zeros((B, self.U, d))
        xp = np.zeros((B, self.T, n))
        bw = np.zeros((B, self.nbranch - 1))
        J = np.zeros(B)
        st = np.zeros(B, np.int32)
        it = np.zeros(B, np.int32)
        lib().hs_solve(self.h, _p(x), _p(z), _p(xref), _p(up), _p(xp), _p(bw), _p(J), _p(st), _p(it))
        return dict(upred=up, xpred=xp, branch_w=bw, J=J, status=st, iters=it)

    def env_step(self, env, t, scene, upred=None, J=None, status=None, iters=None, stats=None):
        """Host build of bmpc_env_step: advances `scene` [B][16] in place, returns x, z, xref."""
        B = self.batch
        x, z, xref = np.zeros((B, 4)), np.zeros((B, 4)), np.zeros((B, 4))
        up = None if upred is None else np.ascontiguousarray(np.asarray(upred, float).reshape(B, self.U, self.desc.d))
        lib().hs_env_step(self.h, C.byref(env), int(t), _p(scene), _p(up), _p(J), _p(status), _p(iters),
                          _p(x), _p(z), _p(xref), _p(stats))
        return x, z, xref

    def get_policies(self):
        arr = (abi.Policy * (self.batch * self.desc.m))()
        lib().hs_get_policies(self.h, arr)
        return arr

    def set_warm_start(self, uLin, pprev, jcons=None, oldu=None):
        B = self.batch
        uLin = np.ascontiguousarray(np.asarray(uLin, float).reshape(B, self.U + 1, self.desc.d))
        pprev = np.ascontiguousarray(np.asarray(pprev, float).reshape(B, self.bdim, self.desc.m))
        jcons = None if jcons is None else np.ascontiguousarray(np.asarray(jcons, float).reshape(B))
        oldu = None if oldu is None else np.ascontiguousarray(np.asarray(oldu, float).reshape(B, self.desc.d))
        lib().hs_set_warm_start(self.h, _p(uLin), _p(pprev), _p(jcons), _p(oldu))

    def set_transform(self, S=None, bx=None, s_on=None):
        B, n = self.batch, self.desc.n
        S = None if S is None else np.ascontiguousarray(np.asarray(S, float).reshape(B, n, n))
        bx = None if bx is None else np.ascontiguousarray(np.asarray(bx, float).reshape(B, self.desc.nFx))
        on = None if s_on is None else np.ascontiguousarray(s_on, np.uint8)
        lib().hs_set_transform(self.h, _p(S), _p(on), _p(bx))

    def set_fx(self, Fx):
        """Per-ego Fx [B,nFx,n] of the next solves (solve's Fx argument)."""
        Fx = np.ascontiguousarray(np.asarray(Fx, float).reshape(self.batch, self.desc.nFx, self.desc.n))
        lib().hs_set_fx(self.h, _p(Fx))

    def branch_dp(self):
        """BranchTree.dp of every non-leaf branch [B, bdim, m, n] of the last solve."""
        out = np.zeros((self.batch, self.bdim, self.desc.m, self.desc.n))
        lib().hs_get_branch_dp(self.h, _p(out))
        return out

    def set_robust_warm_start(self, xlin, ulin, oldu):
        xlin, ulin, oldu = (np.ascontiguousarray(a, dtype=np.float64) for a in (xlin, ulin, oldu))
        lib().hs_set_robust_warm_start(self.h, _p(xlin), _p(ulin), _p(oldu))

    def reset_mask(self, mask=None):
        m = None if mask is None else np.ascontiguousarray(mask, np.uint8)
        lib().hs_reset(self.h, _p(m))

    def layout(self):
        """Layout offsets by field name (parsed from csrc/bmpc_core.h, declaration order)."""
        import re
        src = open(os.path.join(PKG, "csrc", "bmpc_core.h")).read()
        body = src[src.index("struct Layout {"):src.index("};", src.index("struct Layout {"))]
        names = [n for line in body.splitlines() if line.strip().startswith("size_t")
                 for n in re.findall(r"(\w+)\s*[,;]", line.split("//", 1)[0].split("size_t", 1)[1])]
        out = np.zeros(256, np.uint64)
        cnt = lib().hs_layout(self.h, _p(out))
        assert cnt == len(names), (cnt, names)
        return dict(zip(names, (int(v) for v in out[:cnt])))

    def workspace(self, e=0):
        lib().hs_ws_ptr.restype = C.POINTER(C.c_double)
        ptr = lib().hs_ws_ptr(self.h, e)
        return np.ctypeslib.as_array(ptr, shape=(self.layout()["stride"],))

    def tree(self):
        B, n, d = self.batch, self.desc.n, self.desc.d
        out = dict(xbar=np.zeros((B, self.T, n)), ubar=np.zeros((B, self.U, d)),
                   zbar=np.zeros((B, self.T, n)), w=np.zeros((B, self.nbranch)),
                   p=np.zeros((B, self.bdim, self.desc.m)), sol=np.zeros((B, self.nv)))
        lib().hs_get_tree(self.h, *(_p(out[k]) for k in ("xbar", "ubar", "zbar", "w", "p", "sol")))
        return out


def model_eval(desc, pol_rows, x, u, z, lane_ref=None):
    """Host build of bmpc_model_eval(_ref); lane_ref = (grid, values) of psiref policies."""
    x, u, z = (np.ascontiguousarray(np.atleast_2d(np.asarray(v, float))) for v in (x, u, z))
    B, n, d, m, N = x.shape[0], desc.n, desc.d, desc.m, desc.N
    out = dict(A=np.zeros((B, n, n)), B=np.zeros((B, n, d)), C=np.zeros((B, n)), xp=np.zeros((B, n)),
               p=np.zeros((B, m)), dp=np.zeros((B, m, n)), zpred=np.zeros((B, N, m * n)),
               h0=np.zeros(B), dh=np.zeros((B, n)))
    arr = abi.policy_array(pol_rows)
    g, v = (None, None) if lane_ref is None else (np.ascontiguousarray(np.asarray(a, float).reshape(-1))
                                                  for a in lane_ref)
    lib().hs_model_eval_ref(C.byref(desc), arr, 0 if g is None else g.size, _p(g), _p(v), B, _p(x), _p(u), _p(z),
                            *(_p(out[k]) for k in ("A", "B", "C", "xp", "p", "dp", "zpred", "h0", "dh")))
    return out


def hmm_eval(M, m, consts, xb, u, xbackup):
    xb = np.ascontiguousarray(np.atleast_2d(np.asarray(xb, float)))
    B, nb = xb.shape[0], 4 + M * m
    u = np.ascontiguousarray(np.broadcast_to(np.atleast_2d(np.asarray(u, float)), (B, 2)))
    xbk = np.ascontiguousarray(np.broadcast_to(np.asarray(xbackup, float).reshape(-1, M * m, 4), (B, M * m, 4)))
    hc = np.ascontiguousarray(np.asarray(consts, float).reshape(8))
    out = dict(xbp=np.zeros((B, nb)), A=np.zeros((B, nb, nb)), B=np.zeros((B, nb, 2)), C=np.zeros((B, nb)),
               h0=np.zeros((B, M, m)), Jh=np.zeros((B, M, m, nb)))
    lib().hs_hmm_eval(M, m, _p(hc), B, _p(xb), _p(u), _p(xbk), *(_p(out[k]) for k in ("xbp", "A", "B", "C", "h0", "Jh")))
    return out


def qp_solve(n, m, Pp, Pi, Ap, Ai, Px, q, Ax, l, u, max_iter=100, eps=1e-10):
    """Host build of bmpc_qp_solve (batched arrays: Px [B][nnzP], q [B][n], ...)."""
    i32 = lambda a: np.ascontiguousarray(a, np.int32)
    f64 = lambda a: np.ascontiguousarray(a, float)
    Pp, Pi, Ap, Ai = i32(Pp), i32(Pi), i32(Ap), i32(Ai)
    q = f64(q).reshape(-1, n)
    B = q.shape[0]
    Px, Ax = f64(Px).reshape(B, -1), f64(Ax).reshape(B, -1)
    l, u = f64(l).reshape(B, m), f64(u).reshape(B, m)
    x, y = np.zeros((B, n)), np.zeros((B, m))
    st, it, info = np.zeros(B, np.int32), np.zeros(B, np.int32), np.zeros(4, np.int32)
    rc = lib().hs_qp_solve(n, m, _p(Pp), _p(Pi), _p(Ap), _p(Ai), B, _p(Px), _p(q), _p(Ax), _p(l), _p(u),
                           int(max_iter), C.c_double(eps), _p(x), _p(y), _p(st), _p(it), _p(info))
    if rc != 0:
        raise RuntimeError(lib().hs_last_error().decode())
    return dict(x=x, y=y, status=st, iters=it, info=info)
