"""`_backend` for shencoder (reference shencoder/src/bindings.cpp:5-8,
shencoder.h:9-10) bound to libngp_hip.so via ctypes."""
import types

import torch

import _ngp_native as nat

_F = (torch.float32, torch.float64)


def sh_encode_forward(inputs, outputs, B, D, C, dy_dx):
    nat.check_tensor(inputs, "inputs", _F, "float32/float64")
    nat.check_tensor(outputs, "outputs", _F, "float32/float64")
    if dy_dx is not None:
        nat.check_tensor(dy_dx, "dy_dx", _F, "float32/float64")
    nat.check(nat.lib().ngp_sh_encode_forward(nat.ptr(inputs), nat.ptr(outputs), B, D, C,
                                              nat.ptr(dy_dx), nat.DTYPE_CODE[inputs.dtype],
                                              nat.stream_of(inputs)), "sh_encode_forward")


def sh_encode_backward(grad, inputs, B, D, C, dy_dx, grad_inputs):
    for t, n in ((grad, "grad"), (inputs, "inputs"), (dy_dx, "dy_dx"), (grad_inputs, "grad_inputs")):
        nat.check_tensor(t, n, _F, "float32/float64")
    nat.check(nat.lib().ngp_sh_encode_backward(nat.ptr(grad), nat.ptr(inputs), B, D, C,
                                               nat.ptr(dy_dx), nat.ptr(grad_inputs),
                                               nat.DTYPE_CODE[grad.dtype], nat.stream_of(grad)),
              "sh_encode_backward")


_backend = types.SimpleNamespace(sh_encode_forward=sh_encode_forward,
                                 sh_encode_backward=sh_encode_backward)

__all__ = ["_backend"]
