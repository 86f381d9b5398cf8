"""Model functions vs vectors produced by the REFERENCE's own model code.

``tests/golden/model_{highway,quadruped,hmm}.npz`` were written by ``tools/gen_golden_model.py``,
which runs ``highway_branch_dyn.py`` / ``quadruped_branch_dyn.py`` / ``HMM_backup_dyn.py`` from
the reference unchanged over a CasADi-API stand-in (``tools/casadi_shim``).  Checked here,
all at 1e-12 (relative to max(1, |ref|)):

* the oracle's NumPy restatement (``oracle/model.py``, ``oracle/hmm.py``) -- CPU;
* the host build of the kernels' model templates (tests/hostsim) -- CPU;
* ``libbmpc.so`` through the C ABI (``bmpc_model_eval`` / ``bmpc_hmm_eval``) -- GPU.
"""
import numpy as np
import pytest

from common import golden
from bmpc import abi
from bmpc.scenarios import highway_desc, highway_policy_rows, quadruped_desc, quadruped_policy_rows

TOL = 1e-12
KEYS = ("A", "B", "C", "xp", "p", "dp", "zpred", "h0", "dh")


def close(got, ref, what):
    got, ref = np.asarray(got, float), np.asarray(ref, float)
    assert got.shape == ref.shape, (what, got.shape, ref.shape)
    err = np.max(np.abs(got - ref)) / max(1.0, float(np.max(np.abs(ref))))
    assert err <= TOL, f"{what}: rel err {err:.3e}"


def highway_cases():
    g = golden("model_highway")
    for c in range(int(g["ncases"])):
        yield g, f"c{c}_"


def quadruped_cases():
    g = golden("model_quadruped")
    for c in range(int(g["ncases"])):
        yield g, f"c{c}_"


def hmm_cases():
    g = golden("model_hmm")
    for c in range(int(g["ncases"])):
        yield g, f"c{c}_"


def _quad_desc(g, p):
    L1, W1, L2, W2, tol, s1 = (float(v) for v in g[p + "consts"])
    return quadruped_desc(N=int(g[p + "N"]), dt=float(g[p + "dt"]), L1=L1, W1=W1, L2=L2, W2=W2, col_tol=tol, s1=s1)


def _check_batch(out, g, p, what):
    for k in KEYS:
        close(out[k], g[p + k], f"{what} {p}{k}")


# ---- oracle (CPU) -----------------------------------------------------------------------------
def test_oracle_highway_model_matches_reference_code():
    from oracle.model import HighwayModel, highway_policies
    for g, p in highway_cases():
        mdl = HighwayModel(int(g[p + "N"]), float(g["dt"]), highway_policies(float(g["Kpsi"]), g[p + "lc_target"]),
                           L=float(g["L"]), W=float(g["W"]), s1=float(g["s1"]))
        for k in range(g[p + "x"].shape[0]):
            x, z, u = g[p + "x"][k], g[p + "z"][k], g[p + "u"][k]
            got = dict(zip(("A", "B", "C", "xp"), mdl.dyn_linearization(x, u)))
            got["p"], got["dp"] = mdl.branch_eval(x, z)
            got["zpred"] = mdl.zpred_eval(z)
            got["h0"], got["dh"] = mdl.col_eval(x, z)
            for key in KEYS:
                close(got[key], g[p + key][k], f"oracle highway {p}{key}[{k}]")


def test_oracle_quadruped_model_matches_reference_code():
    from oracle.model import QuadrupedModel, quadruped_policies
    for g, p in quadruped_cases():
        L1, W1, L2, W2, tol, s1 = (float(v) for v in g[p + "consts"])
        mdl = QuadrupedModel(int(g[p + "N"]), float(g[p + "dt"]), quadruped_policies(float(g[p + "v0"])),
                             L1=L1, W1=W1, L2=L2, W2=W2, col_tol=tol, s1=s1)
        for k in range(g[p + "x"].shape[0]):
            x, z, u = g[p + "x"][k], g[p + "z"][k], g[p + "u"][k]
            got = dict(zip(("A", "B", "C", "xp"), mdl.dyn_linearization(x, u)))
            got["p"], got["dp"] = mdl.branch_eval(x, z)
            got["zpred"] = mdl.zpred_eval(z)
            got["h0"], got["dh"] = mdl.col_eval(x, z)
            for key in KEYS:
                close(got[key], g[p + key][k], f"oracle quadruped {p}{key}[{k}]")


def test_oracle_hmm_model_matches_reference_code():
    from oracle.hmm import HMMModel
    dt, L, W, ylb, yub, ca, s1, tau = (float(v) for v in golden("model_hmm")["consts"])
    for g, p in hmm_cases():
        M, m = int(g[p + "M"]), int(g[p + "m"])
        mdl = HMMModel(M, m, dt, L=L, W=W, ylb=ylb, yub=yub, col_alpha=ca, s1=s1, tran_diag=tau)
        for k in range(g[p + "xb"].shape[0]):
            A, B, C, h0, Jh, _ = mdl.linearize(g[p + "xb"][k], g[p + "u"][k], g[p + "xbackup"][k])
            close(A, g[p + "A"][k], f"oracle hmm {p}A[{k}]")
            close(B, g[p + "B"][k], f"oracle hmm {p}B[{k}]")
            close(C, g[p + "C"][k], f"oracle hmm {p}C[{k}]")
            close(np.reshape(h0, (M, m)), g[p + "h0"][k], f"oracle hmm {p}h0[{k}]")
            close(np.reshape(Jh, (M, m, -1)), g[p + "Jh"][k], f"oracle hmm {p}Jh[{k}]")


# ---- host build of the kernel templates (CPU) ---------------------------------------------------
def test_host_build_model_eval_matches_reference_code():
    import hostsim_lib as H
    for g, p in highway_cases():
        B = g[p + "x"].shape[0]
        out = H.model_eval(highway_desc(N=int(g[p + "N"])), highway_policy_rows(np.tile(g[p + "lc_target"], (B, 1))),
                           g[p + "x"], g[p + "u"], g[p + "z"])
        _check_batch(out, g, p, "hostsim highway")
    for g, p in quadruped_cases():
        B = g[p + "x"].shape[0]
        out = H.model_eval(_quad_desc(g, p), quadruped_policy_rows(B, float(g[p + "v0"])), g[p + "x"], g[p + "u"],
                           g[p + "z"])
        _check_batch(out, g, p, "hostsim quadruped")


def test_host_build_hmm_eval_matches_reference_code():
    import hostsim_lib as H
    hc = golden("model_hmm")["consts"]
    for g, p in hmm_cases():
        M, m = int(g[p + "M"]), int(g[p + "m"])
        out = H.hmm_eval(M, m, hc, g[p + "xb"], g[p + "u"], g[p + "xbackup"])
        for k in ("A", "B", "C", "h0", "Jh"):
            close(out[k], g[p + k], f"hostsim hmm {p}{k}")


# ---- libbmpc.so on the GPU -------------------------------------------------------------------------
@pytest.fixture(scope="module")
def gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from bmpc import plan
    plan.context(0)
    return plan


@pytest.mark.gpu
def test_gpu_model_eval_matches_reference_code(gpu):
    for g, p in highway_cases():
        B = g[p + "x"].shape[0]
        out = gpu.model_eval(highway_desc(N=int(g[p + "N"])), highway_policy_rows(np.tile(g[p + "lc_target"], (B, 1))),
                             g[p + "x"], g[p + "u"], g[p + "z"])
        _check_batch(out, g, p, "gpu highway")
    for g, p in quadruped_cases():
        B = g[p + "x"].shape[0]
        out = gpu.model_eval(_quad_desc(g, p), quadruped_policy_rows(B, float(g[p + "v0"])), g[p + "x"], g[p + "u"],
                             g[p + "z"])
        _check_batch(out, g, p, "gpu quadruped")


@pytest.mark.gpu
def test_gpu_hmm_eval_matches_reference_code(gpu):
    hc = golden("model_hmm")["consts"]
    for g, p in hmm_cases():
        M, m = int(g[p + "M"]), int(g[p + "m"])
        out = gpu.hmm_eval(M, m, hc, g[p + "xb"], g[p + "u"], g[p + "xbackup"])
        for k in ("A", "B", "C", "h0", "Jh"):
            close(out[k], g[p + k], f"gpu hmm {p}{k}")


def test_fixture_provenance():
    """The vectors are data written by tools/gen_golden_model.py (no reference text)."""
    for name in ("model_highway", "model_quadruped", "model_hmm"):
        g = golden(name)
        assert all(g[k].dtype.kind in "fiu" for k in g.files), name
    assert abi.MODEL_HIGHWAY != abi.MODEL_QUADRUPED
