"""bench.py's N > 1 path on CPU: `bench.py --gpus 2` run directly launches its own two ranks
through torchrun (127.0.0.1), each rank runs the closed loop on its contiguous shard, the
statistics are all-reduced (SUM, MAX for the flag) and the time is the max over ranks.  The
test-only backend switch BMPC_BENCH_BACKEND=hostsim puts the host build of the kernels and
gloo under the same code (bench.py _HostSimPlan); what stays hardware-only is named in
DESIGN.md §7 (RCCL init with device_id, the HIP stream, torch.cuda synchronisation)."""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(*args):
    env = dict(os.environ, BMPC_BENCH_BACKEND="hostsim", OMP_NUM_THREADS="1")
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), *args], env=env, capture_output=True,
                       text=True, timeout=600, cwd=REPO)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-3000:]      # rank 0 alone prints the line
    return json.loads(lines[0])


@pytest.mark.timeout(900)
def test_bench_two_ranks_self_launch_matches_one_rank():
    common = ["--N", "10", "--NB", "1", "--steps", "2", "--warmup", "1", "--no-cpu-baseline"]
    two = _bench("--gpus", "2", "--batch", "5", *common)
    one = _bench("--gpus", "1", "--global-batch", "10", *common)
    assert two["backend"].startswith("hostsim") and one["backend"].startswith("hostsim")
    assert two["n_gpus"] == 2 and two["config"]["world_size"] == 2
    assert two["config"]["global_batch"] == 10 and two["config"]["batch_per_gpu"] == 5
    assert two["config"]["shards"] == [[0, 5], [5, 10]]
    assert one["config"]["shards"] == [[0, 10]]
    # whole-job throughput: all ranks' solves over the max-over-ranks time
    assert abs(two["value"] - 10 * 2 / (two["ms_per_step"] * 2 / 1e3)) <= 1e-3 * two["value"] + 0.02
    c2, c1 = two["closed_loop"], one["closed_loop"]
    assert c2["solves"] == c1["solves"] == 10 * 2
    for k in ("J_mean", "iters_mean"):
        assert abs(c2[k] - c1[k]) <= 1e-9 * max(1.0, abs(c1[k])), (k, c2[k], c1[k])
    for k in ("infeasible", "collision_steps", "collided_egos", "any_collided"):
        assert c2[k] == c1[k], (k, c2[k], c1[k])
