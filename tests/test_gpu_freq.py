"""freqencoder (csrc/freqencoder.hip) through the C ABI / _backend shim
against the oracle (freqencoder.cu:30-94 restated) and the reference's
pure-torch FreqEncoder fixture (tests/golden/freq_reference.npz).

Forward: the identity columns bit-exact; the sine columns within the
hardware sine's bound (test_golden_reference.freq_forward_tol: 2^-22 +
2^-22 |arg| absolute -- the reference's __sinf is an approximation as well).
Backward: against the oracle's float64 sum over the kernel's own saved
outputs within float32 summation rounding, and against the reference's
autograd gradient within the forward bound carried through the sum.
"""
import os

import numpy as np
import pytest
import torch

import oracle
from test_golden_reference import freq_backward_tol, freq_forward_tol

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.mark.parametrize("B,D,deg,scale", [(4096, 3, 4, 1.0), (1000, 3, 10, 1.0), (513, 2, 6, 4.0),
                                           (77, 1, 1, 1.0), (1, 3, 12, 2.0)])
def test_freq_forward_backward_vs_oracle(cuda, B, D, deg, scale):
    from freqencoder import FreqEncoder
    g = torch.Generator().manual_seed(B + deg)
    x = ((torch.rand(B, D, generator=g) * 2 - 1) * scale)
    enc = FreqEncoder(input_dim=D, degree=deg)
    assert enc.output_dim == D * (1 + 2 * deg)
    xd = x.to(cuda).requires_grad_(True)
    y = enc(xd)
    assert y.dtype == torch.float32 and y.shape == (B, enc.output_dim)
    ref, args = oracle.freq_encode_forward(x.numpy(), deg)
    got = y.detach().cpu().numpy()
    assert np.array_equal(got[:, :D], x.numpy())
    tol = freq_forward_tol(args)
    assert (np.abs(got - ref) <= tol).all(), float((np.abs(got - ref) / tol).max())
    gy = torch.randn(B, enc.output_dim, generator=g)
    y.backward(gy.to(cuda))
    gi = xd.grad.cpu().numpy().astype(np.float64)
    exact = oracle.freq_encode_backward(gy.numpy(), got, D, deg)
    # float32 rounding of the kernel's sum: 2^-21 of the sum of |terms|
    ga, oa = np.abs(gy.numpy()).astype(np.float64), np.abs(got)
    mag = ga[:, :D].copy()
    for f in range(deg):
        s = D + 2 * D * f
        mag += 2.0 ** f * (ga[:, s:s + D] * oa[:, s + D:s + 2 * D] + ga[:, s + D:s + 2 * D] * oa[:, s:s + D])
    assert (np.abs(gi - exact) <= mag * 2.0 ** -21).all(), float((np.abs(gi - exact) / mag).max())


@pytest.mark.parametrize("deg", [4, 10])
def test_freq_vs_reference_torch_encoder(cuda, deg):
    """The HIP op against the reference's own encoding.FreqEncoder outputs
    and autograd input grads (make_golden.py freq_fixture)."""
    from freqencoder import freq_encode
    f = dict(np.load(os.path.join(GOLDEN, "freq_reference.npz")))
    x, y, gy, gx = f[f"x{deg}"], f[f"y{deg}"], f[f"gy{deg}"], f[f"gx{deg}"]
    xd = torch.from_numpy(x).to(cuda).requires_grad_(True)
    out = freq_encode(xd, deg, 3 * (1 + 2 * deg))
    out.backward(torch.from_numpy(gy).to(cuda))
    _, args = oracle.freq_encode_forward(x, deg)
    tol = freq_forward_tol(args)
    got = out.detach().cpu().numpy().astype(np.float64)
    assert (np.abs(got - y) <= 2 * tol).all(), float((np.abs(got - y) / tol).max())
    btol = freq_backward_tol(gy, args, 3, deg, 2 * tol)
    gi = xd.grad.cpu().numpy().astype(np.float64)
    assert (np.abs(gi - gx) <= btol).all(), float((np.abs(gi - gx) / btol).max())


def test_freq_autocast_unaligned_and_errors(cuda):
    """custom_fwd casts half inputs to float32 (freq.py:17); an output view
    that is not 16-byte aligned takes the scalar store path; a wrong
    output_dim raises, B = 0 returns an empty tensor."""
    from freqencoder import FreqEncoder, freq_encode
    from freqencoder.backend import _backend
    enc = FreqEncoder(3, 4)
    x = torch.rand(64, 3, device=cuda).half()
    with torch.autocast("cuda", dtype=torch.float16):
        y = enc(x)
    assert y.dtype == torch.float32
    ref, _ = oracle.freq_encode_forward(x.float().cpu().numpy(), 4)
    assert np.allclose(y.cpu().numpy(), ref, atol=1e-5)
    buf = torch.empty(64 * 27 + 1, device=cuda)
    out = buf[1:].view(64, 27)
    _backend.freq_encode_forward(x.float().contiguous(), 64, 3, 4, 27, out)
    torch.cuda.synchronize()
    assert torch.equal(out, y)
    with pytest.raises(RuntimeError, match="output_dim"):
        _backend.freq_encode_forward(x.float().contiguous(), 64, 3, 4, 26, out)
    e = freq_encode(torch.empty(0, 3, device=cuda), 4, 27)
    assert e.shape == (0, 27)
