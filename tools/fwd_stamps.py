"""Phase clocks of the one-launch NeRF forward (k_nerf_fwd), diagnostic build
with -DNGP_STAMPS (SRCS=ffmlp bash tools/variants.sh stamps "-DNGP_STAMPS"):
per wave, s_memtime after each phase (each stamp first waits for the wave's
outstanding memory operations), plus chip-wide realtime at entry / exit.
    NGP_HIP_LIB=torch-ngp_amd/variants/stamps/libngp_hip.so python tools/fwd_stamps.py"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "torch-ngp_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import _ngp_native as nat  # noqa: E402
from nerf.fused import FusedTrainer  # noqa: E402
from nerf.network_ff import NeRFNetwork  # noqa: E402
from nerf.provider import SyntheticLego, lego_bitfield  # noqa: E402

dev = torch.device("cuda:0")
torch.manual_seed(0)
model = NeRFNetwork(bound=1, cuda_ray=True).to(dev)
model.density_bitfield.copy_(torch.from_numpy(lego_bitfield()).to(dev))
ft = FusedTrainer(model, SyntheticLego(dev, num_rays=4096), M=101762)
assert ft._one_fwd
base = 2 * 2048 * 16
ms = torch.zeros(base + 4096 * 16, dtype=torch.int64, device=dev)
lib = nat.lib()
assert lib.ngp_debug_mlp_stamps(ctypes.c_void_p(nat.ptr(ms))) == 0
for _ in range(200):
    ft.step()
torch.cuda.synchronize()
ms.zero_()
ft.step()
torch.cuda.synchronize()
f = ms[base:].view(-1, 16).cpu().numpy().astype(np.int64)
f = f[f[:, 0] > 0]
names = ["frag_copy", "x_load", "sigma_mlp", "epilogue", "color_mlp", "store"]
work = f[f[:, 6] > 0]  # waves that ran a chunk
d = np.diff(work[:, :7], axis=1)
rt = f[:, 8:10]
out = {"waves": int(len(f)), "waves_with_chunk": int(len(work)),
       "phase_cycles_med": dict(zip(names, [int(x) for x in np.median(d, axis=0)])),
       "phase_cycles_p90": dict(zip(names, [int(x) for x in np.percentile(d, 90, axis=0)])),
       "wave_total_med": int(np.median(work[:, 6] - work[:, 0])),
       # inside the epilogue, first 16 rows: shuffles | h/sigma/color_in stores | SH + its store
       "epilogue_nb0_med": [int(np.median(work[:, 10] - work[:, 3])), int(np.median(work[:, 11] - work[:, 10])),
                            int(np.median(work[:, 12] - work[:, 11]))],
       "realtime_entry_spread_us": float((rt[:, 0].max() - rt[:, 0].min()) / 100.0),
       "realtime_span_us": float((rt[:, 1].max() - rt[:, 0].min()) / 100.0),
       "realtime_wave_med_us": float(np.median(rt[:, 1] - rt[:, 0]) / 100.0)}
print(json.dumps(out, indent=1))
