"""The fused density-grid update (FusedTrainer.update_density) on its own, for
rocprofv3 kernel traces: 16 full updates (iter_density < 16), then `n` timed
partial updates, each after a few training steps.
    rocprofv3 --kernel-trace --stats -d OUT -o run -- python3 tools/density_fused_probe.py [n]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "torch-ngp_amd")]
import torch  # noqa: E402

import bench  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    argv, sys.argv = sys.argv, sys.argv[:1]
    args = bench.parse()
    sys.argv = argv
    dev = torch.device("cuda:0")
    model, data, bits, *_, dt_gamma = bench.make_workload("lego", dev, 1, 4096)
    ft, _ = bench.make_trainer(args, model, data, 1, dev, dt_gamma, grid_timing=False)
    for _ in range(16):
        ft.update_density()
    torch.cuda.synchronize()
    out = []
    for _ in range(n):
        for _ in range(16):
            ft.step()
        ft.flush()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        ft.update_density()
        e.record()
        torch.cuda.synchronize()
        out.append(round(s.elapsed_time(e), 4))
    print(json.dumps({"partial_update_ms": out, "iter_density": int(model.iter_density)}))


if __name__ == "__main__":
    main()
