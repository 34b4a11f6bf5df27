"""Canonical instant-ngp NeRF on the fused MLP (reference nerf/network_ff.py):
hashgrid(L16, C2, 2048*bound) -> FFMLP 32->64->64->16 -> trunc_exp(sigma) +
15 geometry features; SH(deg 4) ++ geo ++ 1 pad -> FFMLP 32->64->64->64->16
-> sigmoid(rgb[:3]). Constructor keywords of the renderer pass through
(fixes fork break §1.3.4: extra kwargs no longer crash construction)."""
import numpy as np
import torch

from activation import trunc_exp
from encoding import get_encoder
from ffmlp import FFMLP

from .renderer import NeRFRenderer


class NeRFNetwork(NeRFRenderer):
    def __init__(self, encoding="hashgrid", encoding_dir="sphere_harmonics", num_layers=2,
                 hidden_dim=64, geo_feat_dim=15, num_layers_color=3, hidden_dim_color=64, bound=1,
                 log2_hashmap_size=19, **kwargs):
        super().__init__(bound, **kwargs)
        self.num_layers = num_layers
        self.hidden_dim = hidden_dim
        self.geo_feat_dim = geo_feat_dim
        self.encoder, self.in_dim = get_encoder(encoding, desired_resolution=2048 * bound,
                                                log2_hashmap_size=log2_hashmap_size)
        self.sigma_net = FFMLP(input_dim=self.in_dim, output_dim=1 + self.geo_feat_dim,
                               hidden_dim=self.hidden_dim, num_layers=self.num_layers)
        self.num_layers_color = num_layers_color
        self.hidden_dim_color = hidden_dim_color
        self.encoder_dir, self.in_dim_color = get_encoder(encoding_dir)
        self.in_dim_color += self.geo_feat_dim + 1  # pad to 32 (nerf_network.h#178)
        self.color_net = FFMLP(input_dim=self.in_dim_color, output_dim=3,
                               hidden_dim=self.hidden_dim_color, num_layers=self.num_layers_color)

    def forward(self, x, d):
        x = self.encoder(x, bound=self.bound)
        h = self.sigma_net(x)
        sigma = trunc_exp(h[..., 0])
        geo_feat = h[..., 1:]
        d = self.encoder_dir(d)
        p = torch.zeros_like(geo_feat[..., :1])
        h = torch.cat([d, geo_feat, p], dim=-1)
        h = self.color_net(h)
        return sigma, torch.sigmoid(h)

    def density(self, x):
        x = self.encoder(x, bound=self.bound)
        h = self.sigma_net(x)
        return {"sigma": trunc_exp(h[..., 0]), "geo_feat": h[..., 1:]}

    def color(self, x, d, mask=None, geo_feat=None, **kwargs):
        if mask is not None:
            rgbs = torch.zeros(mask.shape[0], 3, dtype=x.dtype, device=x.device)
            if not mask.any():
                return rgbs
            x, d, geo_feat = x[mask], d[mask], geo_feat[mask]
        d = self.encoder_dir(d)
        p = torch.zeros_like(geo_feat[..., :1])
        h = torch.sigmoid(self.color_net(torch.cat([d, geo_feat, p], dim=-1)))
        if mask is not None:
            rgbs[mask] = h.to(rgbs.dtype)
            return rgbs
        return h

    def _query_density(self, xyzs, indices, tmp_grid):
        """Density-grid query of update_extra_state under autocast (the
        reference trainer updates inside autocast, nerf/utils.py): the fused
        grid forward (fp32 table rounded to half on load, as autocast's cast
        does) and the sigma network with its density-scatter epilogue."""
        if not (torch.is_autocast_enabled() and self.encoder.level_dim == 2):
            return super()._query_density(xyzs, indices, tmp_grid)
        import _ngp_native as nat
        e, P = self.encoder, xyzs.shape[0]
        enc = torch.empty(e.num_levels, P, e.level_dim, dtype=torch.float16, device=xyzs.device)
        st, lib, ptr = nat.stream_of(xyzs), nat.lib(), nat.ptr
        # autocast's half table (grid.py:52-56): a 2 MiB fp16 slice per hashed
        # level stays resident in an XCD's 4 MiB L2 (4 MiB in fp32 does not)
        emb = e.embeddings.detach().half()
        emb_dt = nat.DTYPE_CODE[emb.dtype]
        nat.check(lib.ngp_grid_encode_forward_fused(
            ptr(xyzs), float(self.bound), ptr(emb), emb_dt, ptr(e.offsets), ptr(enc), P, None, e.input_dim,
            e.level_dim, e.num_levels, float(np.log2(e.per_level_scale)), e.base_resolution, e.gridtype_id,
            int(e.align_corners), e.interp_id, 0, st), "grid_encode_fused")
        sn = self.sigma_net
        w = sn.weights.detach().half()
        nat.check(lib.ngp_nerf_density_forward(ptr(enc), ptr(w), None, P, sn.input_dim, sn.hidden_dim,
                                               sn.num_layers, float(self.density_scale), ptr(indices),
                                               ptr(tmp_grid), st), "nerf_density_forward")

    def get_params(self, lr):
        return [{"params": self.encoder.parameters(), "lr": lr},
                {"params": self.sigma_net.parameters(), "lr": lr},
                {"params": self.encoder_dir.parameters(), "lr": lr},
                {"params": self.color_net.parameters(), "lr": lr}]
