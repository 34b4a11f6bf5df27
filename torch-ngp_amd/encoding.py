"""Encoder factory (mirror of the reference encoding.py:45-103 hot branches).

`get_encoder(name, ...) -> (module, output_dim)` with the reference's keyword
names. 'hashgrid' / 'tiledgrid' -> gridencoder.GridEncoder, 'sphere_harmonics'
-> shencoder.SHEncoder, 'frequency' -> freqencoder.FreqEncoder (the gfx950
kernels, as the reference's :66-69 picks its CUDA extension; the pure-torch
FreqEncoder below is the reference's own restatement, :5-43), 'None' ->
identity. The fork's Minkowski encoders are out of scope.
"""
import torch
import torch.nn as nn


class FreqEncoder(nn.Module):
    """NeRF positional encoding in plain torch (reference encoding.py:5-43)."""

    def __init__(self, input_dim, max_freq_log2, N_freqs, log_sampling=True, include_input=True,
                 periodic_fns=(torch.sin, torch.cos)):
        super().__init__()
        self.input_dim = input_dim
        self.include_input = include_input
        self.periodic_fns = periodic_fns
        self.output_dim = (input_dim if include_input else 0) + input_dim * N_freqs * len(periodic_fns)
        if log_sampling:
            self.freq_bands = (2.0 ** torch.linspace(0.0, max_freq_log2, N_freqs)).tolist()
        else:
            self.freq_bands = torch.linspace(2.0 ** 0.0, 2.0 ** max_freq_log2, N_freqs).tolist()

    def forward(self, input, **kwargs):
        out = [input] if self.include_input else []
        for freq in self.freq_bands:
            for p_fn in self.periodic_fns:
                out.append(p_fn(input * freq))
        return torch.cat(out, dim=-1)


def get_encoder(encoding, input_dim=3, multires=6, degree=4, num_levels=16, level_dim=2,
                base_resolution=16, log2_hashmap_size=19, desired_resolution=2048,
                align_corners=False, **kwargs):
    if encoding == "None":
        return lambda x, **kw: x, input_dim
    if encoding == "frequency":
        from freqencoder import FreqEncoder as _FreqEncoderHIP
        encoder = _FreqEncoderHIP(input_dim=input_dim, degree=multires)
    elif encoding == "sphere_harmonics":
        from shencoder import SHEncoder
        encoder = SHEncoder(input_dim=input_dim, degree=degree)
    elif encoding in ("hashgrid", "tiledgrid"):
        from gridencoder import GridEncoder
        encoder = GridEncoder(input_dim=input_dim, num_levels=num_levels, level_dim=level_dim,
                              base_resolution=base_resolution, log2_hashmap_size=log2_hashmap_size,
                              desired_resolution=desired_resolution,
                              gridtype="hash" if encoding == "hashgrid" else "tiled",
                              align_corners=align_corners)
    else:
        raise NotImplementedError(
            "Unknown encoding mode, choose from [None, frequency, sphere_harmonics, hashgrid, tiledgrid]")
    return encoder, encoder.output_dim
