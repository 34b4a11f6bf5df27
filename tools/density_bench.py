"""Times NeRFNetwork.update_extra_state (full and partial updates) on the GPU:
wall time per call after warm-up, for rocprofv3 kernel traces of the update.
usage: python tools/density_bench.py [--iters N] [--bound B]"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "torch-ngp_amd")]

import json  # noqa: E402

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--bound", type=float, default=1.0)
    args = ap.parse_args()
    from nerf.network_ff import NeRFNetwork
    from nerf.provider import lego_bitfield
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    m = NeRFNetwork(bound=args.bound, cuda_ray=True, density_thresh=10).to(dev)
    with torch.no_grad():
        m.encoder.embeddings.normal_(0, 0.3)
    m.density_bitfield.copy_(torch.from_numpy(lego_bitfield(cascade=m.cascade, bound=args.bound)).to(dev))
    out = {}
    for mode, it0 in (("full", 0), ("partial", 16)):
        ts = []
        for i in range(args.iters + 2):
            m.iter_density = it0
            torch.cuda.synchronize()
            t = time.perf_counter()
            with torch.autocast("cuda", dtype=torch.float16):
                m.update_extra_state()
            torch.cuda.synchronize()
            ts.append((time.perf_counter() - t) * 1e3)
        ts = sorted(ts[2:])
        out[mode + "_ms_median"] = round(ts[len(ts) // 2], 3)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
