"""bench.py's launch contract: `--gpus N` runs N ranks from one command."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_launch_cmd_starts_n_ranks_on_loopback():
    sys.path.insert(0, ROOT)
    import bench
    cmd = bench.launch_cmd(4, ["--gpus", "4", "--steps", "7"], 29511)
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=4" in cmd and "--nnodes=1" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[cmd.index("--master-port") + 1] == "29511"
    assert cmd[-4:] == ["--gpus", "4", "--steps", "7"] and cmd[-5].endswith("bench.py")


def test_gpus_must_match_the_launchers_world_size():
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "3"], env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode != 0 and "WORLD_SIZE=2" in r.stderr


def test_amortized_density_update():
    """One partial device update per 16 steps (nerf/utils.py:
    update_extra_interval) added to the step; None when it was not measured."""
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    r = bench.amortized_density(0.2, {"fused_partial": 0.48}, 4096)
    assert r["ms_per_step"] == 0.23 and abs(r["rays_per_s"] - 4096 / 0.23e-3) < 1
    assert bench.amortized_density(0.2, {}, 4096) is None
    assert bench.amortized_density(0.2, None, 4096) is None


@pytest.mark.gpu
def test_bench_gpus2_gloo_runs_two_ranks():
    """`bench.py --gpus 2 --backend gloo` on the one-GPU box: both ranks run the
    data-parallel step and rank 0 reports n_gpus 2 and the 2 ranks gloo joined."""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--backend", "gloo",
                        "--steps", "3", "--warmup", "2", "--kernel-steps", "1", "--no-cpu", "--no-graph",
                        "--settle-steps", "2"],
                       capture_output=True, text=True, timeout=600, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["config"]["parallelism"] == "dp2"
    assert out["config"]["collective"] == {"backend": "gloo", "world_size": 2}
    assert out["value"] > 0 and out["config"]["global_batch_rays"] == 2 * out["config"]["num_rays_per_gpu"]
