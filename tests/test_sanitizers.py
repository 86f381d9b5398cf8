"""AddressSanitizer + UndefinedBehaviorSanitizer over the host build of the kernel templates
("ASan/UBSan on the C++ host lib").

The host build (tests/hostsim) instantiates every solver template the HIP kernels use -- the
slab Layout offsets, the LDS spans of the plan, the tree / cone / coupling index arithmetic of
the IPM, the band-QP analysis and factorisation -- with a 1-lane executor, so an out-of-bounds
index or an undefined operation in that arithmetic shows up here on CPU.  The sanitized build is
a separate .so (hostsim_lib names it by its flags); the replays of the reference's recorded closed
loops run over it in a child pytest with the ASan runtime preloaded (Python itself is not
instrumented), and any report aborts the child.  Host code only: GPU sanitizers are not used."""
import os
import subprocess
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))

SAN_FLAGS = "-fsanitize=address,undefined -fno-sanitize-recover=undefined -fno-omit-frame-pointer -g"
# the host replays of every solver family: CVaR IPM (N=10 NB=1, N=8 NB=2, N=30 NB=2, merge with S / bx,
# per-step Fx and S), the OSQP controllers' QP IPM (quadruped Prox, BranchMPC, robustMPC), the band QP
# of the belief MPC, the device-scene env step
CASES = [
    "test_kernel_host.py::test_host_build_replays_reference",
    "test_kernel_host.py::test_lean_lds_path_matches",
    "test_merge.py::test_host_build_replays_merge_scene",
    "test_merge.py::test_host_build_tree_with_psiref_policies",
    "test_xform.py::test_host_build_replays_xform_scene",
    "test_qp_host.py::test_quadruped_prox_replay",
    "test_qp_host.py::test_branch_mpc_qp_replay",
    "test_qp_host.py::test_robust_mpc_replay",
    "test_bandqp.py::test_host_build_matches_oracle_on_random_qps",
    "test_bandqp.py::test_host_build_window_and_in_lds_factorisations_agree",
    "test_bandqp.py::test_host_build_solves_reference_belief_problems",
    "test_bandqp.py::test_analysis_rejects_bad_input",
    "test_env_host.py::test_host_env_replays_reference_loop",
    "test_model_golden.py",
]


def _runtime(name):
    p = subprocess.run(["g++", f"-print-file-name={name}"], capture_output=True, text=True).stdout.strip()
    return p if os.path.isabs(p) and os.path.exists(p) else None


@pytest.mark.slow
def test_host_build_is_clean_under_asan_and_ubsan():
    asan = _runtime("libasan.so")
    if asan is None:
        pytest.skip("no libasan in this toolchain")
    env = dict(os.environ, BMPC_HOSTSIM_FLAGS=SAN_FLAGS, OMP_NUM_THREADS="4",
               ASAN_OPTIONS="detect_leaks=0:abort_on_error=1:halt_on_error=1:detect_stack_use_after_return=0",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    # build the sanitized library first, without the runtime preloaded (g++ itself is not instrumented)
    subprocess.run([sys.executable, "-c", "import hostsim_lib; print(hostsim_lib.build())"], env=env, cwd=HERE,
                   check=True, timeout=1800)
    env["LD_PRELOAD"] = ":".join(p for p in (asan, os.environ.get("LD_PRELOAD", "")) if p)
    r = subprocess.run([sys.executable, "-m", "pytest", "-x", "-q", "-p", "no:cacheprovider", "-m", "not gpu",
                        *CASES], env=env, cwd=HERE, capture_output=True, text=True, timeout=5400)
    out = r.stdout[-4000:] + r.stderr[-4000:]
    assert r.returncode == 0, out
    assert "ERROR: AddressSanitizer" not in out and "runtime error:" not in out, out
    assert "passed" in r.stdout, out
