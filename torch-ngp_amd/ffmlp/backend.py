"""`_backend` for ffmlp (reference ffmlp/src/bindings.cpp:5-11, ffmlp.h:8-14)
bound to libngp_hip.so via ctypes. Same names / positional arguments; the
backward's dW workspace is allocated here from torch's caching allocator."""
import types

import torch

import _ngp_native as nat

_H = (torch.float16,)


def ffmlp_forward(inputs, weights, B, input_dim, output_dim, hidden_dim, num_layers, activation,
                  output_activation, forward_buffer, outputs):
    nat.check_tensor(inputs, "inputs", _H, "Half")
    nat.check_tensor(weights, "weights", _H, "Half")
    nat.check_tensor(outputs, "outputs", _H, "Half")
    if forward_buffer is not None:
        nat.check_tensor(forward_buffer, "forward_buffer", _H, "Half")
    nat.check(nat.lib().ngp_ffmlp_forward(
        nat.ptr(inputs), nat.ptr(weights), B, input_dim, output_dim, hidden_dim, num_layers,
        activation, output_activation, nat.ptr(forward_buffer), nat.ptr(outputs),
        nat.stream_of(inputs)), "ffmlp_forward")


def ffmlp_inference(inputs, weights, B, input_dim, output_dim, hidden_dim, num_layers, activation,
                    output_activation, inference_buffer, outputs):
    nat.check_tensor(inputs, "inputs", _H, "Half")
    nat.check_tensor(weights, "weights", _H, "Half")
    nat.check_tensor(outputs, "outputs", _H, "Half")
    nat.check(nat.lib().ngp_ffmlp_inference(
        nat.ptr(inputs), nat.ptr(weights), B, input_dim, output_dim, hidden_dim, num_layers,
        activation, output_activation, nat.ptr(inference_buffer), nat.ptr(outputs),
        nat.stream_of(inputs)), "ffmlp_inference")


def ffmlp_backward(grad, inputs, weights, forward_buffer, B, input_dim, output_dim, hidden_dim,
                   num_layers, activation, output_activation, calc_grad_inputs, backward_buffer,
                   grad_inputs, grad_weights):
    nat.check_tensor(grad, "grad", _H, "Half")
    nat.check_tensor(inputs, "inputs", _H, "Half")
    nat.check_tensor(weights, "weights", _H, "Half")
    nat.check_tensor(grad_inputs, "grad_inputs", _H, "Half")
    nat.check_tensor(grad_weights, "grad_weights", (torch.float16, torch.float32), "Half/Float")
    ws_bytes = nat.lib().ngp_ffmlp_backward_workspace_bytes(B, input_dim, output_dim, hidden_dim,
                                                            num_layers)
    workspace = torch.empty(max(ws_bytes, 4), dtype=torch.uint8, device=grad.device)
    nat.check(nat.lib().ngp_ffmlp_backward(
        nat.ptr(grad), nat.ptr(inputs), nat.ptr(weights), nat.ptr(forward_buffer), B, input_dim,
        output_dim, hidden_dim, num_layers, activation, output_activation, int(bool(calc_grad_inputs)),
        nat.ptr(backward_buffer), nat.ptr(grad_inputs), nat.ptr(grad_weights),
        nat.DTYPE_CODE[grad_weights.dtype], nat.ptr(workspace), ws_bytes, nat.stream_of(grad)),
        "ffmlp_backward")


def allocate_splitk(size):
    nat.check(nat.lib().ngp_ffmlp_allocate_splitk(size), "allocate_splitk")


def free_splitk():
    nat.check(nat.lib().ngp_ffmlp_free_splitk(), "free_splitk")


_backend = types.SimpleNamespace(ffmlp_forward=ffmlp_forward, ffmlp_inference=ffmlp_inference,
                                 ffmlp_backward=ffmlp_backward, allocate_splitk=allocate_splitk,
                                 free_splitk=free_splitk)

__all__ = ["_backend"]
