"""Fully-fused MLP module (mirror of reference ffmlp/ffmlp.py:15-169).

Same constructor, flat weight Parameter (`weights`, per-layer row-major
[out, in], init manual_seed(42) + U(+-sqrt(3/hidden))), output padding to 16
and fp16 autocast contract. Differences: no batch padding copy (the kernels
take any batch size), and no forward activation buffer (the HIP backward
recomputes activations on chip instead of streaming them through HBM).
"""
import math

import torch
import torch.nn as nn
from torch.autograd import Function

from .backend import _backend


class _ffmlp_forward(Function):
    @staticmethod
    @torch.amp.custom_fwd(device_type="cuda", cast_inputs=torch.half)
    def forward(ctx, inputs, weights, input_dim, output_dim, hidden_dim, num_layers, activation,
                output_activation, inference=False, calc_grad_inputs=False):
        B = inputs.shape[0]
        inputs = inputs.contiguous()
        weights = weights.contiguous()
        outputs = torch.empty(B, output_dim, device=inputs.device, dtype=inputs.dtype)
        if not inference:
            _backend.ffmlp_forward(inputs, weights, B, input_dim, output_dim, hidden_dim, num_layers,
                                   activation, output_activation, None, outputs)
            ctx.save_for_backward(inputs, weights)
            ctx.dims = (input_dim, output_dim, hidden_dim, num_layers, activation, output_activation,
                        calc_grad_inputs)
        else:
            _backend.ffmlp_inference(inputs, weights, B, input_dim, output_dim, hidden_dim,
                                     num_layers, activation, output_activation, None, outputs)
        return outputs

    @staticmethod
    @torch.amp.custom_bwd(device_type="cuda")
    def backward(ctx, grad):
        B = grad.shape[0]
        grad = grad.contiguous()
        if grad.dtype != torch.half:
            grad = grad.half()
        inputs, weights = ctx.saved_tensors
        (input_dim, output_dim, hidden_dim, num_layers, activation, output_activation,
         calc_grad_inputs) = ctx.dims
        grad_inputs = (torch.empty_like(inputs) if calc_grad_inputs
                       else torch.zeros(1, device=grad.device, dtype=grad.dtype))
        grad_weights = torch.empty_like(weights)
        _backend.ffmlp_backward(grad, inputs, weights, None, B, input_dim, output_dim, hidden_dim,
                                num_layers, activation, output_activation, calc_grad_inputs, None,
                                grad_inputs, grad_weights)
        if calc_grad_inputs:
            return grad_inputs, grad_weights, None, None, None, None, None, None, None, None
        return None, grad_weights, None, None, None, None, None, None, None, None


ffmlp_forward = _ffmlp_forward.apply


def convert_activation(act):
    return {"relu": 0, "exponential": 1, "sine": 2, "sigmoid": 3, "squareplus": 4,
            "softplus": 5}.get(act, 6)


class FFMLP(nn.Module):
    def __init__(self, input_dim, output_dim, hidden_dim, num_layers, activation="relu"):
        super().__init__()
        self.input_dim = input_dim
        self.output_dim = output_dim
        self.hidden_dim = hidden_dim
        self.num_layers = num_layers
        self.activation = convert_activation(activation)
        self.output_activation = convert_activation("none")
        self.tensorcore_width = 16

        assert hidden_dim in [32, 64], \
            f"FFMLP on gfx950 supports hidden_dim in [32, 64], but got {hidden_dim}"
        assert input_dim > 0 and input_dim % 16 == 0 and input_dim <= 64, \
            f"FFMLP input_dim should be 16 * m (0 < m <= 4), but got {input_dim}"
        assert output_dim <= 16, f"FFMLP current only supports output dim <= 16, but got {output_dim}"
        assert 2 <= num_layers <= 4, f"FFMLP num_layers should be in [2, 4], but got {num_layers}"

        self.padded_output_dim = int(math.ceil(output_dim / 16)) * 16
        self.num_parameters = hidden_dim * (input_dim + hidden_dim * (num_layers - 1) + self.padded_output_dim)
        self.weights = nn.Parameter(torch.zeros(self.num_parameters))
        self.reset_parameters()
        _backend.allocate_splitk(self.num_layers + 1)

    def cleanup(self):
        _backend.free_splitk()

    def __repr__(self):
        return (f"FFMLP: input_dim={self.input_dim} output_dim={self.output_dim} "
                f"hidden_dim={self.hidden_dim} num_layers={self.num_layers} activation={self.activation}")

    def reset_parameters(self):
        torch.manual_seed(42)
        std = math.sqrt(3 / self.hidden_dim)
        self.weights.data.uniform_(-std, std)

    def forward(self, inputs):
        # inputs: [B, input_dim] -> [B, output_dim]
        outputs = ffmlp_forward(inputs, self.weights, self.input_dim, self.padded_output_dim,
                                self.hidden_dim, self.num_layers, self.activation,
                                self.output_activation, not self.training, inputs.requires_grad)
        if self.padded_output_dim != self.output_dim:
            outputs = outputs[:, :self.output_dim]
        return outputs
