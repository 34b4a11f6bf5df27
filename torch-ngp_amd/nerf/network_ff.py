"""Canonical instant-ngp NeRF on the fused MLP (reference nerf/network_ff.py):
hashgrid(L16, C2, 2048*bound) -> FFMLP 32->64->64->16 -> trunc_exp(sigma) +
15 geometry features; SH(deg 4) ++ geo ++ 1 pad -> FFMLP 32->64->64->64->16
-> sigmoid(rgb[:3]). Constructor keywords of the renderer pass through
(fixes fork break §1.3.4: extra kwargs no longer crash construction)."""
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

    def get_params(self, lr):
        return [{"params": self.encoder.parameters(), "lr": lr},
                {"params": self.sigma_net.parameters(), "lr": lr},
                {"params": self.encoder_dir.parameters(), "lr": lr},
                {"params": self.color_net.parameters(), "lr": lr}]
