"""Fused grid backward on a real step's samples: runs a few fused train steps,
then times ngp_grid_encode_backward_fused alone (HIP events, back to back)
and dumps the step's samples / output grads to gpurun_out/grid_step.npz for
CPU-side analysis (item counts per bin after merging)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "torch-ngp_amd")]
import numpy as np
import torch

import _ngp_native as nat
from nerf.fused import FusedTrainer
from nerf.network_ff import NeRFNetwork
from nerf.provider import SyntheticLego, lego_bitfield

KNOBS = {k: os.environ.pop(k) for k in ("NGP_DBG_ACCUM",) if k in os.environ}  # experiment knobs, if a build reads any
dev = torch.device("cuda:0")
torch.manual_seed(0)
model = NeRFNetwork(bound=1, cuda_ray=True).to(dev)
model.density_bitfield.copy_(torch.from_numpy(lego_bitfield()).to(dev))
data = SyntheticLego(dev, num_rays=4096)
ft = FusedTrainer(model, data, M=101762)
for _ in range(20):
    ft.step()
torch.cuda.synchronize()
e, m = ft.enc, ft.model
n = ft.sample_count()
lib, P = nat.lib(), nat.ptr
s = nat.stream_of(ft.xyzs)


def call():
    nat.check(lib.ngp_grid_encode_backward_fused(
        P(ft.g_enc), P(ft.xyzs), float(m.bound), P(e.offsets), P(ft.grads[0]), ft.M, P(ft.counter),
        e.input_dim, e.level_dim, e.num_levels, ft.S, e.base_resolution, e.gridtype_id, int(e.align_corners),
        e.interp_id, ft._offsets_host, P(ft.grid_ws), ft.grid_ws.numel(), 0, None, s), "grid_bwd")


os.environ.update(KNOBS)  # debug knobs only for the timed calls (training above runs the product path)
for _ in range(3):
    call()
torch.cuda.synchronize()
reps = int(os.environ.get("REPS", "50"))
a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
a.record()
for _ in range(reps):
    call()
b.record()
b.synchronize()
print({"samples": n, "grid_bwd_us": round(a.elapsed_time(b) / reps * 1e3, 2)})
out = os.path.join(ROOT, "gpurun_out", "grid_step.npz")
np.savez_compressed(out, xyzs=ft.xyzs[:n].cpu().numpy(), g_enc=ft.g_enc[:n].cpu().numpy(),
                    offsets=e.offsets.cpu().numpy(), S=np.float32(ft.S), H=e.base_resolution)
