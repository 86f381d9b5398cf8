import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
for p in (HERE, REPO, os.path.join(REPO, "belief-planning_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device) and libbmpc.so")
    config.addinivalue_line("markers", "slow: long CPU test")


# Launch paths of the CVaR IPM (bmpc_hip.hip launch_solve; read from the environment on every
# launch): a batch of at most one ego per CU takes the multi-wave small-batch kernel by default;
# BMPC_BLOCK_EGOS=0 forces the one-wave-per-ego k_ipm that serves large batches (the bench's
# kernel), BMPC_LDS_RICH=0/1 its lean / LDS-rich instantiation.  The GPU replays of the
# reference's recorded loops run through every path; each test asserts the path was taken
# (BMPC_INFO_SOLVER).
SOLVER_PATHS = {
    "blk": ({}, None),
    "wave": ({"BMPC_BLOCK_EGOS": "0", "BMPC_LDS_RICH": "1"}, "IPM_RICH"),
    "lean": ({"BMPC_BLOCK_EGOS": "0", "BMPC_LDS_RICH": "0"}, "IPM_LEAN"),
}
QP_PATHS = {
    "rich": ({"BMPC_LDS_RICH": "1"}, "QP_RICH"),
    "lean": ({"BMPC_LDS_RICH": "0"}, "QP_LEAN"),
}


def _set_path(monkeypatch, table, name):
    import pytest  # noqa: F401
    for k in ("BMPC_BLOCK_EGOS", "BMPC_LDS_RICH", "BMPC_BLOCK_WAVES"):
        monkeypatch.delenv(k, raising=False)
    env, kern = table[name]
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    return name, kern


import pytest  # noqa: E402


@pytest.fixture(params=list(SOLVER_PATHS))
def solver_path(request, monkeypatch):
    """(name, expected BMPC_KERNEL_* name or None for the small-batch kernel)."""
    return _set_path(monkeypatch, SOLVER_PATHS, request.param)


@pytest.fixture(params=list(QP_PATHS))
def qp_path(request, monkeypatch):
    return _set_path(monkeypatch, QP_PATHS, request.param)


def assert_solver_path(pl, path):
    """The plan's last solve ran the kernel the path names (blk: one of the small-batch kernels)."""
    from bmpc import abi
    name, kern = path
    got = pl.last_kernel()
    if kern is None:
        assert got in (abi.KERNEL_IPM_BLK4, abi.KERNEL_IPM_BLK8), (name, got)
    else:
        assert got == getattr(abi, "KERNEL_" + kern), (name, got)
