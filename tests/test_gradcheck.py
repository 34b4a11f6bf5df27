"""The reference's own known-answer test for the hash-grid gradient,
testing/test_hashgrid_grad.py:11-16,25-34,51-61: `torch.autograd.gradcheck`
of `_grid_encode` in float64 at D=3, L=4, C=2, H=4, log2T=8,
per_level_scale=2, with the level offsets NOT rounded to a multiple of 8
(:31 is commented out there), eps=1e-2, atol=1e-3, rtol=0.01, fast_mode=False.

* GPU: the HIP `_grid_encode` (gridencoder/grid.py, fp64 table path) with the
  reference's exact argument tuple (float64 inputs, which the wrapper reads
  as float32 coordinates; the reference kernel rejected them);
* CPU: the C oracle's forward / backward (oracle/ngp_oracle.c) wrapped in an
  autograd Function, so the oracle the GPU parity tests use is pinned by the
  same gradcheck.
The grid is linear in the table, so the finite differences are exact up to
rounding and the check is a strict test of the backward scatter.
"""
import numpy as np
import pytest
import torch
from torch.autograd import gradcheck

import oracle

D, L, C, PER_LEVEL_SCALE, H, LOG2T = 3, 4, 2, 2, 4, 8


def _offsets():
    """testing/test_hashgrid_grad.py:25-34: no rounding to 8."""
    offsets, off = [], 0
    for i in range(L):
        res = int(np.ceil(H * PER_LEVEL_SCALE ** i))
        n = min(2 ** LOG2T, (res + 1) ** D)
        offsets.append(off)
        off += n
    offsets.append(off)
    return np.array(offsets, dtype=np.int32)


def test_reference_offsets_are_unrounded():
    off = _offsets()
    assert off.tolist() == [0, 125, 381, 637, 893]  # level 0 dense (5^3), levels 1-3 hashed (2^8)
    assert off.tolist() != oracle.grid_offsets(D, L, C, H, PER_LEVEL_SCALE, LOG2T).tolist()


class _OracleGridEncode(torch.autograd.Function):
    """The C oracle as an autograd op (float64 table, float32 coordinates)."""

    @staticmethod
    def forward(ctx, inputs, embeddings, offsets, per_level_scale, base_resolution, calc_grad_inputs=False):
        x = inputs.detach().cpu().numpy().astype(np.float32)
        off = offsets.cpu().numpy()
        out, _ = oracle.grid_encode_forward(x, embeddings.detach().cpu().numpy(), off, per_level_scale,
                                            base_resolution)
        ctx.save_for_backward(inputs, offsets)
        ctx.cfg = (per_level_scale, base_resolution, embeddings.shape[1])
        return torch.from_numpy(out)

    @staticmethod
    def backward(ctx, grad):
        inputs, offsets = ctx.saved_tensors
        s, res, c = ctx.cfg
        g = oracle.grid_encode_backward(grad.detach().cpu().numpy().astype(np.float64),
                                        inputs.detach().cpu().numpy().astype(np.float32), offsets.cpu().numpy(),
                                        c, s, res)
        return None, torch.from_numpy(g), None, None, None, None


@pytest.mark.parametrize("B,seed", [(1, 42), (1, 7), (16, 3)])
def test_oracle_gradcheck(B, seed):
    torch.manual_seed(seed)
    inputs = torch.rand(B, D, dtype=torch.float64)
    offsets = torch.from_numpy(_offsets())
    emb = (torch.randn(int(offsets[-1]), C, dtype=torch.float64) * 0.1).requires_grad_(True)
    assert gradcheck(_OracleGridEncode.apply, (inputs, emb, offsets, PER_LEVEL_SCALE, H, False),
                     eps=1e-2, atol=1e-3, rtol=0.01, fast_mode=False)


@pytest.mark.gpu
@pytest.mark.parametrize("B,seed", [(1, 42), (1, 7), (16, 3)])
def test_hip_grid_encode_gradcheck(cuda, parity_report, B, seed):
    """testing/test_hashgrid_grad.py:51-61 on the HIP path, argument tuple as there."""
    from gridencoder.grid import _grid_encode
    torch.manual_seed(seed)
    inputs = torch.rand(B, D, dtype=torch.float64, requires_grad=False).to(cuda)
    offsets = torch.from_numpy(_offsets()).to(cuda)
    embeddings = torch.randn(int(offsets[-1]), C, dtype=torch.float64, requires_grad=True).to(cuda) * 0.1
    Inputs = (inputs, embeddings, offsets, PER_LEVEL_SCALE, H, inputs.requires_grad)
    assert gradcheck(_grid_encode.apply, Inputs, eps=1e-2, atol=1e-3, rtol=0.01, fast_mode=False)
    # and the HIP forward equals the oracle's on the same table, bit for bit
    out = _grid_encode.apply(*Inputs).detach().cpu().numpy()
    ref, _ = oracle.grid_encode_forward(inputs.cpu().numpy().astype(np.float32),
                                        embeddings.detach().cpu().numpy(), offsets.cpu().numpy(),
                                        PER_LEVEL_SCALE, H)
    assert np.array_equal(out.view(np.uint64), ref.view(np.uint64))
    parity_report(f"reference gradcheck (test_hashgrid_grad.py) B {B} seed {seed}: passed, fp64 forward bit-exact")
