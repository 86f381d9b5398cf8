"""GPU parity tests: libbmpc.so (gfx950 kernels, through the C ABI) vs the oracle.

Tolerances (stated per check):
* model functions: 1e-12 relative -- same closed-form expressions, fp64;
* solver: the reference solves with ECOS to feastol=abstol=reltol=1e-8 (MPC_branch.py:2136),
  so a solution is only defined to that precision.  J must agree to 1e-6 relative and the
  applied input uPred[0] to 1e-6 absolute on steps both sides end optimal (exit 0; 1e-4 against
  the oracle's independent solves of the seeded batch, 5e-3 on "inaccurate" steps); the unique part of the primal vector
  (everything except the cost-free leaf-terminal slacks) to 1e-3 absolute.  GPU vs the
  host build of the same algorithm is compared tighter (J 1e-7 rel, uPred 1e-5 abs).
"""
import numpy as np
import pytest

from common import golden, highway_desc, highway_desc_from_golden, highway_policy_rows, replay_batch, seeded_batch
from conftest import assert_solver_path

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from bmpc import plan
    plan.context(0)
    return plan


def test_library_is_native(gpu):
    from bmpc import _lib
    assert _lib.lib().bmpc_abi_version() == 2


def test_model_eval_matches_oracle(gpu):
    from oracle.model import HighwayModel, highway_policies
    rng = np.random.default_rng(3)
    B = 256
    desc = highway_desc(N=20, NB=1)
    x = np.stack([rng.uniform(-5, 5, B), rng.uniform(0, 13, B), rng.uniform(10, 30, B), rng.normal(0, .1, B)], 1)
    u = np.stack([rng.uniform(-6, 6, B), rng.uniform(-.3, .3, B)], 1)
    z = x + np.stack([rng.uniform(-10, 30, B), rng.uniform(-6, 6, B), rng.uniform(-5, 5, B), np.zeros(B)], 1)
    tg = np.stack([np.zeros(B), rng.choice([1.8, 5.4, 9.0], B), np.full(B, 20.0), np.zeros(B)], 1)
    out = gpu.model_eval(desc, highway_policy_rows(tg), x, u, z)
    for b in range(0, B, 17):
        mdl = HighwayModel(20, 0.1, highway_policies(0.1, tg[b]))
        A, Bm, C, xp = mdl.dyn_linearization(x[b], u[b])
        p, dp = mdl.branch_eval(x[b], z[b])
        h0, dh = mdl.col_eval(x[b], z[b])
        zp = mdl.zpred_eval(z[b])
        for got, ref in ((out["A"][b], A), (out["B"][b], Bm), (out["C"][b], C), (out["xp"][b], xp),
                         (out["p"][b], p), (out["dp"][b], dp), (out["zpred"][b], zp),
                         (out["h0"][b], h0), (out["dh"][b], dh)):
            np.testing.assert_allclose(got, ref, rtol=1e-12, atol=1e-12)


@pytest.mark.parametrize("name,steps", [("highway_n20_nb1", 100), ("highway_n8_nb2", 40), ("highway_n10_nb1", 20),
                                        ("highway_n30_nb2", 24)])
def test_replay_matches_reference(gpu, name, steps, solver_path):
    """Every step of the reference's recorded closed loop, one ego per step, each with the
    warm start the reference carried into it (set through the checkpoint ABI), in ONE
    batched launch; exit codes, J and uPred[0] must reproduce the recording -- through each
    launch path: the small-batch kernel these batch sizes take by default, and the one-wave
    k_ipm (LDS-rich and lean) that serves the 4096-ego batches."""
    from test_kernel_host import check_replay
    g = golden(name)
    rb = replay_batch(g, steps)
    pl = gpu.BatchPlan(highway_desc_from_golden(g), rb["T"])
    pl.set_policies(rb["rows"])
    pl.set_warm_start(rb["uLin"], rb["p"], rb["jcons"], mask=rb["warm"])
    r = pl.solve(rb["x"], rb["z"], rb["xref"])
    assert_solver_path(pl, solver_path)
    check_replay(r, g, rb["T"], pl.tree())
    ws = pl.get_warm_start()
    np.testing.assert_allclose(ws["jcons"], rb["jcons"])


def test_replay_exit_agreement_pooled(gpu, solver_path):
    """Exit codes of all 184 recorded highway steps (the four loops above) on one launch path:
    >= 97% agree with the recording.  0 vs 10 is decided at the 1e-8 margin, where the GPU's
    rounding (FMA contraction, 64-lane reduction trees) and the host build's differ: the traces of
    the N=10 loop (profiles/r06/trace_*) diverge from 2.6e-13 at iteration 0 and the final primal
    residual of a step lands anywhere in 1e-10 .. 1.5e-8; the host build with FMA contraction
    flips 9 of 454 recorded / seeded step decisions the same way (profiles/r06/refine_ab.log)."""
    agree, total = 0, 0
    for name, steps in (("highway_n20_nb1", 100), ("highway_n8_nb2", 40), ("highway_n10_nb1", 20),
                        ("highway_n30_nb2", 24)):
        g = golden(name)
        rb = replay_batch(g, steps)
        pl = gpu.BatchPlan(highway_desc_from_golden(g), rb["T"])
        pl.set_policies(rb["rows"])
        pl.set_warm_start(rb["uLin"], rb["p"], rb["jcons"], mask=rb["warm"])
        r = pl.solve(rb["x"], rb["z"], rb["xref"])
        assert_solver_path(pl, solver_path)
        agree += int(np.sum(r["status"] == np.asarray(g["traj_exit"][:rb["T"]])))
        total += rb["T"]
    print(f"pooled replay [{solver_path[0]}]: exit codes agree on {agree} of {total} recorded steps")
    assert total == 184 and agree >= 0.97 * total, (agree, total)


def test_batch_matches_host_build(gpu):
    """Seeded batch: every GPU ego equals the host build of the same algorithm."""
    import hostsim_lib as H
    B = 64
    x, z, xref, tgt = seeded_batch(B, seed=1)
    desc = highway_desc(N=20, NB=1)
    pl = gpu.BatchPlan(desc, B)
    pl.set_policies(highway_policy_rows(tgt))
    hs = H.HostSim(desc, B)
    hs.set_policies(highway_policy_rows(tgt))
    agree = []
    for step in range(3):
        r = pl.solve(x, z, xref)
        h = hs.solve(x, z, xref)
        assert np.all(r["status"] >= 0) and np.all(h["status"] >= 0)
        # both exit 0 (certified to 1e-8): tight -- the J tolerance of the reference parity tests
        # (1e-6; the two builds sum in different orders, observed up to 2e-7); otherwise ECOS
        # "inaccurate" class (1e-4 gap)
        tight = (r["status"] == 0) & (h["status"] == 0)
        # 0 vs 10 is decided at the rounding floor: which of the egos that stall near 1e-8 make it
        # moves with the summation order (two GPU builds of one algorithm that sum cone rows in
        # different orders agree on 97.4% of a 4096-ego batch with the same 0/10 split; the host
        # build with and without FMA contraction on 186 of these 192 ego-steps, profiles/r06/
        # refine_ab.log), so the bar is on the 192 ego-steps of the run (>= 95%; round 6: 188), with
        # a per-step floor of 90% (round 6: 64, 63, 61 of 64)
        agree.append(np.mean(r["status"] == h["status"]))
        print(f"GPU vs host build, step {step}: exit codes agree on {int(np.sum(r['status'] == h['status']))} of {B}; "
              f"both exit 0 on {int(tight.sum())}, max |du0| there "
              f"{np.abs(r['upred'][tight, 0] - h['upred'][tight, 0]).max() if tight.any() else 0:.1e}")
        assert agree[-1] >= 0.9, (step, agree)
        np.testing.assert_allclose(r["J"][tight], h["J"][tight], rtol=1e-6)
        np.testing.assert_allclose(r["upred"][tight, 0], h["upred"][tight, 0], atol=1e-5)
        np.testing.assert_allclose(r["J"], h["J"], rtol=1e-4)
        np.testing.assert_allclose(r["upred"][:, 0], h["upred"][:, 0], atol=5e-3)
        u0 = r["upred"][:, 0]
        x = x + 0.1 * np.stack([x[:, 2] * np.cos(x[:, 3]), x[:, 2] * np.sin(x[:, 3]), u0[:, 0], u0[:, 1]], 1)
        z = z + 0.1 * np.stack([z[:, 2] * np.cos(z[:, 3]), z[:, 2] * np.sin(z[:, 3]), 0 * z[:, 0], 0 * z[:, 0]], 1)
    assert np.mean(agree) >= 0.95, agree


def _check_sample_against_oracle(r, N, NB, x, z, xref, tgt, egos, workers=None):
    """Each sampled ego re-solved by the CPU oracle (the ECOS-algorithm restatement on the
    reference's assembly, tests/oracle_pool.py): J to 1e-6 relative; uPred[0] to 1e-6 where
    both exit 0 (certified to the 1e-8 tolerances), else 5e-3 (ECOS's reduced
    "inaccurate" tolerances); exit codes agree on >= 90% of the sample (0 vs 10 is decided at
    the rounding floor).  Returns the number of egos both sides solved to exit 0."""
    from oracle_pool import solve_many
    res = solve_many([(N, NB, tgt[e], xref[e], x[e], z[e]) for e in egos], workers=workers)
    agree, tight = 0, 0
    for e, (st, J, u0) in zip(egos, res):
        assert abs(r["J"][e] - J) <= 1e-6 * max(1, abs(r["J"][e])), (e, r["J"][e], J)
        both0 = st == 0 and r["status"][e] == 0
        np.testing.assert_allclose(r["upred"][e, 0], u0, atol=1e-6 if both0 else 5e-3, err_msg=f"ego {e}")
        agree += st == r["status"][e]
        tight += both0
    print(f"oracle re-solves (N={N} NB={NB}): exit codes agree on {agree} of {len(egos)} sampled egos, both exit 0 on {tight}")
    assert agree >= 0.9 * len(egos), (agree, len(egos))
    return tight


@pytest.mark.timeout(300)
def test_full_batch_certified(gpu):
    """B=4096 (the metric batch, the one-wave LDS-rich k_ipm the bench runs): every ego returns
    a feasible ECOS-class status and a finite plan; 32 sampled egos are re-solved by the CPU
    oracle (tolerances in _check_sample_against_oracle)."""
    from bmpc import abi
    B = 4096
    x, z, xref, tgt = seeded_batch(B, seed=0)
    desc = highway_desc(N=20, NB=1)
    pl = gpu.BatchPlan(desc, B)
    pl.set_policies(highway_policy_rows(tgt))
    r = pl.solve(x, z, xref)
    assert pl.last_kernel() == abi.KERNEL_IPM_RICH
    assert np.all(r["status"] >= 0), np.unique(r["status"], return_counts=True)
    assert np.all(np.isfinite(r["J"])) and np.all(np.isfinite(r["upred"]))
    egos = np.unique(np.concatenate([[0, 1, 777, 4095], np.random.default_rng(11).choice(B, 28, replace=False)]))
    assert len(egos) >= 32
    tight = _check_sample_against_oracle(r, 20, 1, x, z, xref, tgt, egos)
    # with ECOS's equilibration 4009 of the 4096 seeded egos exit 0 (3739 without it, round 4)
    assert tight >= 0.9 * len(egos)


@pytest.mark.timeout(900)
def test_config3_full_batch_lean(gpu):
    """BASELINE config 3 (N=30, NB=2: 9 leaves, 13 cones, a 50 x 50 coupling system) at 4096
    egos: the launch takes the lean k_ipm (coupling system in the slab, 16 egos per CU); every
    ego returns a feasible ECOS-class status and a finite plan, and 32 sampled egos agree with
    the CPU oracle (~45 s of oracle per ego, 12 worker processes)."""
    from bmpc import abi
    B = 4096
    x, z, xref, tgt = seeded_batch(B, seed=3)
    pl = gpu.BatchPlan(highway_desc(N=30, NB=2), B)
    pl.set_policies(highway_policy_rows(tgt))
    r = pl.solve(x, z, xref)
    assert pl.last_kernel() == abi.KERNEL_IPM_LEAN
    assert np.all(r["status"] >= 0), np.unique(r["status"], return_counts=True)
    assert np.all(np.isfinite(r["J"])) and np.all(np.isfinite(r["upred"]))
    egos = np.unique(np.concatenate([[0, 4095], np.random.default_rng(12).choice(B, 30, replace=False)]))
    assert len(egos) >= 32
    _check_sample_against_oracle(r, 30, 2, x, z, xref, tgt, egos, workers=12)


def test_quadruped_prox_replay_gpu(gpu, qp_path):
    """BranchMPCProx (BASELINE config 4): every recorded step of the reference quadruped loop
    as one ego of one batched launch, with its warm start (uLin, p, OldInput); status_val 1
    and uPred[0] to 1e-6 (the oracle QP optimum is exact to ~1e-10)."""
    from common import quad_replay_batch, quadruped_desc_from_golden, quadruped_policy_rows
    g = golden("quadruped_n25_nb2")
    rb = quad_replay_batch(g)
    pl = gpu.BatchPlan(quadruped_desc_from_golden(g), rb["T"])
    pl.set_policies(quadruped_policy_rows(rb["T"]))
    pl.set_warm_start(rb["uLin"], rb["p"], None, rb["old"], mask=rb["warm"])
    r = pl.solve(rb["x"], rb["z"], rb["xref"])
    assert_solver_path(pl, qp_path)
    np.testing.assert_array_equal(r["status"], np.ones(rb["T"]))
    np.testing.assert_allclose(r["upred"][:, 0], g["traj_u"][:rb["T"]], atol=1e-6)
    sol = pl.tree()["sol"]
    for t in (int(k) for k in g["keep"]):
        ref = g[f"s{t}_sol"]
        np.testing.assert_allclose(sol[t], ref, atol=1e-6 * max(1.0, np.abs(ref).max()), err_msg=f"step {t}")


def test_quadruped_model_eval_matches_oracle(gpu):
    from oracle.model import QuadrupedModel, quadruped_policies
    from common import quadruped_desc, quadruped_policy_rows
    rng = np.random.default_rng(5)
    B = 128
    desc = quadruped_desc()
    x = np.stack([rng.uniform(-2, 6, B), rng.uniform(-4, 4, B), rng.uniform(-np.pi, np.pi, B)], 1)
    u = np.stack([rng.uniform(0, .2, B), rng.uniform(-.1, .1, B), rng.uniform(-.5, .5, B)], 1)
    z = x + np.stack([rng.uniform(-3, 3, B), rng.uniform(-3, 3, B), rng.uniform(-1, 1, B)], 1)
    out = gpu.model_eval(desc, quadruped_policy_rows(B), x, u, z)
    mdl = QuadrupedModel(25, 0.2, quadruped_policies(0.2))
    for b in range(0, B, 7):
        A, Bm, C, xp = mdl.dyn_linearization(x[b], u[b])
        p, dp = mdl.branch_eval(x[b], z[b])
        h0, dh = mdl.col_eval(x[b], z[b])
        zp = mdl.zpred_eval(z[b])
        for got, ref in ((out["A"][b], A), (out["B"][b], Bm), (out["C"][b], C), (out["xp"][b], xp),
                         (out["p"][b], p), (out["dp"][b], dp), (out["zpred"][b], zp),
                         (out["h0"][b], h0), (out["dh"][b], dh)):
            np.testing.assert_allclose(got, ref, rtol=1e-12, atol=1e-12)


def test_branch_mpc_qp_replay_gpu(gpu, qp_path):
    """BranchMPC (MPC_branch.py:881) highway scene, every recorded step in one launch."""
    from bmpc import abi
    g = golden("highway_qp_n8_nb2")
    T = len(g["traj_x"])
    desc = highway_desc_from_golden(g)
    desc.controller = abi.CTRL_QP
    pl = gpu.BatchPlan(desc, T)
    pl.set_policies(highway_policy_rows(g["traj_lc_target"], float(g["Kpsi"])))
    ws_u = np.asarray(g["traj_ws_uLin"], float)
    warm = ~np.isnan(ws_u).any(axis=(1, 2))
    pl.set_warm_start(np.nan_to_num(ws_u), np.nan_to_num(g["traj_ws_p"]), None, g["traj_ws_old"], mask=warm)
    r = pl.solve(g["traj_x"], g["traj_z"], g["traj_xRef"])
    assert_solver_path(pl, qp_path)
    np.testing.assert_array_equal(r["status"], g["traj_status"])
    np.testing.assert_allclose(r["upred"][:, 0], g["traj_u"], atol=1e-6)


def test_hmm_eval_matches_oracle(gpu):
    """HMM belief linearisation (HMM_backup_dyn.py:216-276) on the GPU vs the oracle, 1e-12."""
    from test_oracle_hmm import HC, _hmm_case, check_hmm_against_oracle
    for M, m in ((1, 3), (2, 3), (4, 4)):
        xb, u, xbk = _hmm_case(M * 10 + m, M, m, 64)
        check_hmm_against_oracle(gpu.hmm_eval(M, m, HC, xb, u, xbk), M, m, xb, u, xbk)


def test_kernel_timing_ring(gpu):
    """bmpc_enable_timing / bmpc_timing: 40 timed solves (more than the 32-slot event ring, so the
    ring is read back once inside a solve and once by bmpc_timing) are all counted, with positive
    per-kernel averages; the timed solves' results equal untimed ones."""
    B = 8
    x, z, xref, tgt = seeded_batch(B, seed=2)
    desc = highway_desc(N=10, NB=1)
    ref = gpu.BatchPlan(desc, B)
    ref.set_policies(highway_policy_rows(tgt))
    pl = gpu.BatchPlan(desc, B)
    pl.set_policies(highway_policy_rows(tgt))
    pl.enable_timing(True)
    for _ in range(40):
        r = pl.solve(x, z, xref)
        q = ref.solve(x, z, xref)
        np.testing.assert_array_equal(r["upred"], q["upred"])
    tm = pl.timing()
    assert tm["count"] == 40
    assert tm["tree_ms"] > 0 and tm["ipm_ms"] > 0
    assert pl.timing()["count"] == 0      # reading resets the accumulators
    pl.enable_timing(False)
