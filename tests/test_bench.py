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


def test_algorithmic_bytes_of_the_step_launches():
    """SURVEY §8(d) per-unit bytes: Adam 28 B per table value (world 1, no fp16
    table copy) and 30 B per MLP weight; march 48 B/ray + 32 B/sample; grid
    forward 588 and backward 1,100 B/sample; composite 84 B/ray + 64 B/sample."""
    import types
    import torch
    sys.path.insert(0, ROOT)
    import bench
    ft = types.SimpleNamespace(params=[torch.zeros(6119864, 2), torch.zeros(7168), torch.zeros(11264)],
                               table32=True, dp=False)
    assert bench.adam_bytes(ft) == 28 * 12239728 + 30 * 18432
    b = bench.launch_bytes(ft, 80000, 4096)
    assert b["march_rays_train+adam"] == bench.adam_bytes(ft) + 48 * 4096 + 32 * 80000
    assert b["grid_encode_backward"] == 1100 * 80000 and b["grid_encode_forward"] == 588 * 80000
    assert b["composite_loss"] == 84 * 4096 + 64 * 80000 and b["ffmlp_backward"] is None
    dp = types.SimpleNamespace(params=ft.params, table32=False, dp=True, chunk=1532288)
    assert bench.adam_bytes(dp) == 30 * 1532288
    # the table groups the sweep leaves unchanged (reads only, 16 B) or does not clear (26 B)
    idle, zg = 1000000, 2000000
    assert bench.adam_bytes(ft, (idle, zg, 12239728 // 4)) == (16 * 4 * idle + 26 * 4 * zg
                                                               + 28 * (12239728 - 4 * (idle + zg)) + 30 * 18432)
    assert bench.adam_bytes(ft, (0, 0, 12239728 // 4)) == bench.adam_bytes(ft)


def test_flat_buffer_sizes_of_configs_4_and_5():
    """The data-parallel collectives move the flat fp16 gradient / forward copy:
    table + both MLPs, 8-aligned (12,239,728 table values at log2T
    19, 39,625,280 entries x 2 at log2T 22)."""
    sys.path.insert(0, ROOT)
    import bench
    assert bench._flat_total(19) == 12239728 + 7168 + 11264
    assert bench._flat_total(22) == 2 * 39625280 + 7168 + 11264


def test_fox_leg_occupancy_is_not_degenerate():
    """The Config-3 leg's Fox-shaped occupancy gives >= 20 samples per ray at
    dt_gamma 1/128 from the bench's cameras (the Lego boxes at bound 2 gave
    2.7), counted by the oracle's march_rays_train on two poses."""
    import numpy as np
    import torch
    sys.path[:0] = [ROOT, os.path.join(ROOT, "torch-ngp_amd")]
    import oracle
    from nerf.provider import SyntheticLego, fox_bitfield
    from nerf.utils import get_rays
    bits = fox_bitfield()
    data = SyntheticLego("cpu", num_rays=2048)
    total = 0
    for k in (10, 60):
        torch.manual_seed(k)
        r = get_rays(data.poses[k:k + 1], data.intrinsics, 800, 800, 2048)
        ro, rd = (r[n][0].numpy().astype(np.float32) for n in ("rays_o", "rays_d"))
        nears, fars = oracle.near_far_from_aabb(ro, rd, np.array([-2.0] * 3 + [2.0] * 3, np.float32), 0.2)
        out = oracle.march_rays_train(ro, rd, 2.0, bits, 2, 128, nears, fars, np.zeros(2048, np.float32),
                                      M=2048 * 1024, dt_gamma=1 / 128)
        total += int(out[4][0])
    assert total / (2 * 2048) >= 20, total / 4096


@pytest.mark.gpu
@pytest.mark.parametrize("exchange", ["zero1", "sparse"])
def test_bench_gpus2_gloo_runs_two_ranks(exchange):
    """`bench.py --gpus 2 --backend gloo` on the one-GPU box: both ranks run the
    data-parallel step (ZeRO-1, or the replicated step with the touched-entry
    exchange) and rank 0 reports n_gpus 2 and the 2 ranks gloo joined."""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--backend", "gloo",
                        "--steps", "3", "--warmup", "2", "--kernel-steps", "1", "--no-cpu", "--no-graph",
                        "--settle-steps", "2", "--exchange", exchange],
                       capture_output=True, text=True, timeout=600, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["config"]["parallelism"] == "dp2"
    assert out["config"]["collective"] == {"backend": "gloo", "world_size": 2, "exchange": exchange}
    assert out["value"] > 0 and out["config"]["global_batch_rays"] == 2 * out["config"]["num_rays_per_gpu"]
