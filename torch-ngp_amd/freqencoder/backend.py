"""`_backend` for freqencoder (reference freqencoder/src/bindings.cpp:5-8,
freqencoder.h:7,10) bound to libngp_hip.so via ctypes."""
import types

import torch

import _ngp_native as nat

_F32 = (torch.float32,)


def freq_encode_forward(inputs, B, D, deg, C, outputs):
    nat.check_tensor(inputs, "inputs", _F32, "float32")
    nat.check_tensor(outputs, "outputs", _F32, "float32")
    nat.check(nat.lib().ngp_freq_encode_forward(nat.ptr(inputs), B, D, deg, C, nat.ptr(outputs),
                                                nat.stream_of(inputs)), "freq_encode_forward")


def freq_encode_backward(grad, outputs, B, D, deg, C, grad_inputs):
    for t, n in ((grad, "grad"), (outputs, "outputs"), (grad_inputs, "grad_inputs")):
        nat.check_tensor(t, n, _F32, "float32")
    nat.check(nat.lib().ngp_freq_encode_backward(nat.ptr(grad), nat.ptr(outputs), B, D, deg, C,
                                                 nat.ptr(grad_inputs), nat.stream_of(grad)),
              "freq_encode_backward")


_backend = types.SimpleNamespace(freq_encode_forward=freq_encode_forward,
                                 freq_encode_backward=freq_encode_backward)

__all__ = ["_backend"]
