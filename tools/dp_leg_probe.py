"""Runs legs of bench.py's dp_path probe in order in ONE process on a one-rank
RCCL group, keeping every trainer alive like bench.py does (debug aid):
zero1 | three | sparse | exact. Prints each leg's ms/step.
    python tools/dp_leg_probe.py LEG [LEG...]"""
import os
import socket
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "torch-ngp_amd")]
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import bench  # noqa: E402


def main():
    legs = sys.argv[1:]
    argv, sys.argv = sys.argv, sys.argv[:1]
    args = bench.parse()
    sys.argv = argv
    dev = torch.device("cuda:0")
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ["MASTER_PORT"] = str(s.getsockname()[1])
    s.close()
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    try:
        keep = []
        for leg in legs:
            m, d, _, _, _, _, dtg = bench.make_workload(args.workload, dev, 1, args.num_rays)
            opts = {"zero1": None, "three": dict(dp_graph=False), "sparse": dict(sparse_exchange=True),
                    "exact": dict(exact_reduce=True)}[leg]
            ft, _ = bench.make_trainer(args, m, d, 1, dev, dtg, distributed=True, options=opts)
            gs = 1 if leg in ("three", "sparse") else args.graph_steps
            e, g, _ = bench.timed_run(args, ft, 1, dev, 20, 5, 300, gs)
            if leg == "zero1":
                print("phases", ft.timed_steps(args.kernel_steps), flush=True)
                keep.append(ft)
            if leg == "sparse":
                print("touched", bench.touched_pairs(ft), flush=True)
            print(leg, "ms/step", round(e / 20 * 1e3, 4), "graphs", g, flush=True)
            del ft, m
    finally:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
