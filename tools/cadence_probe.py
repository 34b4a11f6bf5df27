"""Where the density-update cadence's time goes (bench.py `with_density_update`):
the Lego bench trainer timed as run(96) alone, update_density alone, flush +
run(16) cycles, and the full [update + fixture restore + run(16)] cycles.

    python tools/cadence_probe.py
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "torch-ngp_amd")]
import torch  # noqa: E402

import bench  # noqa: E402


def wall(fn):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) * 1e3


def main():
    args = bench.parse()
    dev = torch.device("cuda:0")
    model, data, bits, *_ , dt_gamma = bench.make_workload("lego", dev, 1, 4096)
    ft, _ = bench.make_trainer(args, model, data, 1, dev, dt_gamma, grid_timing=False)
    bench.timed_run(args, ft, 1, dev, 20, 5, 300, 10)
    C, E = 6, 16
    out = {}
    out["run96_ms_per_step"] = wall(lambda: ft.run(C * E)) / (C * E)

    def updates():
        for _ in range(C):
            model.iter_density = 16
            ft.update_density()
    out["update_density_ms"] = wall(updates) / C
    ft._dens_sorted = False  # partial queries in draw order (A/B of the brick sort)
    out["update_density_unsorted_ms"] = wall(updates) / C
    ft._dens_sorted = True
    out["update_density_sorted_ms"] = wall(updates) / C
    model.density_bitfield.copy_(bits)
    ft.refresh_occupancy()
    ft.run(E)

    def flush_cycles():
        for _ in range(C):
            ft.flush()
            ft.run(E)
    out["flush_run16_ms_per_step"] = wall(flush_cycles) / (C * E)

    def restore_cycles():
        for _ in range(C):
            model.density_bitfield.copy_(bits)
            ft.refresh_occupancy()
            ft.run(E)
    out["restore_run16_ms_per_step"] = wall(restore_cycles) / (C * E)

    def full_cycles():
        for _ in range(C):
            model.iter_density = 16
            ft.update_density()
            model.density_bitfield.copy_(bits)
            ft.refresh_occupancy()
            ft.run(E)
    out["cycle_ms_per_step"] = wall(full_cycles) / (C * E)
    out["samples_after"] = ft.sample_count()

    def sync_cycles():
        for _ in range(C):
            ft.run(E)
            torch.cuda.synchronize()
    out["run16_sync_ms_per_step"] = wall(sync_cycles) / (C * E)
    print(json.dumps({k: round(v, 4) if isinstance(v, float) else v for k, v in out.items()}))


if __name__ == "__main__":
    main()
