"""The phase-per-kernel IPM (csrc/bmpc_ipm_ph.h) on the host build: the GPU's phase sequence
(each phase's LDS contents scrambled, as a new kernel's are) must give exactly the monolithic
ipm_solve's results over closed-loop steps -- bit for bit, statuses and iteration counts
included."""
import os

import numpy as np
import pytest

import hostsim_lib as H
from bmpc import abi
from common import highway_desc, highway_policy_rows, seeded_batch


def _loop(N, NB, egos, steps, phased, monkeypatch):
    monkeypatch.setenv("BMPC_HOST_PHASED", "1" if phased else "0")
    x, z, xref, tgt = seeded_batch(egos, 0)
    hs = H.HostSim(highway_desc(N, NB), egos)
    hs.set_policies(highway_policy_rows(tgt))
    env = abi.make_env()
    scene = np.zeros((egos, abi.ENV_STRIDE))
    scene[:, 0:4], scene[:, 4:8] = x, z
    x, z, xref = hs.env_step(env, 0, scene)
    r = hs.solve(x, z, xref)
    out = [r]
    for t in range(1, steps):
        x, z, xref = hs.env_step(env, t, scene, r["upred"], r["J"], r["status"], r["iters"])
        r = hs.solve(x, z, xref)
        out.append(r)
    return out


@pytest.mark.parametrize("N,NB,egos", [(10, 1, 48), (8, 2, 16)])
def test_phased_equals_monolithic(N, NB, egos, monkeypatch):
    mono = _loop(N, NB, egos, 3, False, monkeypatch)
    ph = _loop(N, NB, egos, 3, True, monkeypatch)
    for a, b in zip(mono, ph):
        assert np.all(b["status"] >= 0)
        for k in ("upred", "J", "status", "iters"):
            assert np.array_equal(a[k], b[k]), k
