"""`_backend` for gridencoder: the reference's pybind11 module surface
(gridencoder/src/bindings.cpp:5-9) bound to libngp_hip.so via ctypes.

Same function names, positional arguments and in-place output semantics as
the reference (gridencoder/src/gridencoder.h:12-15); argument checks raise
RuntimeError with the reference's TORCH_CHECK wording (gridencoder.cu:15-18).
Extra entries (`*_bm`) take/produce the [B, L*C] layout directly.
"""
import types

import torch

import _ngp_native as nat

_INT = (torch.int32,)


def _dtype(t):
    return nat.DTYPE_CODE[t.dtype]


def _fwd(inputs, embeddings, offsets, outputs, B, D, C, L, S, H, dy_dx, gridtype, align_corners,
         interp, layout):
    nat.check_tensor(inputs, "inputs")
    nat.check_tensor(embeddings, "embeddings")
    nat.check_tensor(offsets, "offsets", _INT, "int")
    nat.check_tensor(outputs, "outputs")
    if inputs.dtype != torch.float32:
        raise RuntimeError("inputs must be a float32 tensor (the kernel reads float coordinates)")
    if outputs.dtype != embeddings.dtype or (dy_dx is not None and dy_dx.dtype != embeddings.dtype):
        raise RuntimeError("outputs and dy_dx must have the embeddings' dtype")
    rc = nat.lib().ngp_grid_encode_forward(
        nat.ptr(inputs), nat.ptr(embeddings), nat.ptr(offsets), nat.ptr(outputs), B, D, C, L,
        float(S), H, nat.ptr(dy_dx), gridtype, int(bool(align_corners)), interp, _dtype(embeddings),
        layout, nat.stream_of(inputs))
    nat.check(rc, "grid_encode_forward")


def _bwd(grad, inputs, embeddings, offsets, grad_embeddings, B, D, C, L, S, H, dy_dx, grad_inputs,
         gridtype, align_corners, interp, layout):
    nat.check_tensor(grad, "grad")
    nat.check_tensor(inputs, "inputs")
    nat.check_tensor(embeddings, "embeddings")
    nat.check_tensor(offsets, "offsets", _INT, "int")
    nat.check_tensor(grad_embeddings, "grad_embeddings")
    if grad.dtype != grad_embeddings.dtype:
        raise RuntimeError("grad and grad_embeddings must have the same dtype")
    rc = nat.lib().ngp_grid_encode_backward(
        nat.ptr(grad), nat.ptr(inputs), nat.ptr(embeddings), nat.ptr(offsets),
        nat.ptr(grad_embeddings), B, D, C, L, float(S), H, nat.ptr(dy_dx), nat.ptr(grad_inputs),
        gridtype, int(bool(align_corners)), interp, _dtype(grad), layout, nat.stream_of(grad))
    nat.check(rc, "grid_encode_backward")


def grid_encode_forward(inputs, embeddings, offsets, outputs, B, D, C, L, S, H, dy_dx, gridtype,
                        align_corners, interp):
    """outputs: [L, B, C] (reference layout, gridencoder.cu:385)."""
    _fwd(inputs, embeddings, offsets, outputs, B, D, C, L, S, H, dy_dx, gridtype, align_corners,
         interp, 0)


def grid_encode_backward(grad, inputs, embeddings, offsets, grad_embeddings, B, D, C, L, S, H,
                         dy_dx, grad_inputs, gridtype, align_corners, interp):
    """grad: [L, B, C] (reference layout)."""
    _bwd(grad, inputs, embeddings, offsets, grad_embeddings, B, D, C, L, S, H, dy_dx, grad_inputs,
         gridtype, align_corners, interp, 0)


def grid_encode_forward_bm(inputs, embeddings, offsets, outputs, B, D, C, L, S, H, dy_dx, gridtype,
                           align_corners, interp):
    """outputs: [B, L*C] written directly (no permute copy)."""
    _fwd(inputs, embeddings, offsets, outputs, B, D, C, L, S, H, dy_dx, gridtype, align_corners,
         interp, 1)


def grid_encode_backward_bm(grad, inputs, embeddings, offsets, grad_embeddings, B, D, C, L, S, H,
                            dy_dx, grad_inputs, gridtype, align_corners, interp):
    """grad: [B, L*C]."""
    _bwd(grad, inputs, embeddings, offsets, grad_embeddings, B, D, C, L, S, H, dy_dx, grad_inputs,
         gridtype, align_corners, interp, 1)


def grad_total_variation(inputs, embeddings, grad, offsets, weight, B, D, C, L, S, H, gridtype,
                         align_corners):
    nat.check_tensor(inputs, "inputs")
    nat.check_tensor(embeddings, "embeddings")
    nat.check_tensor(grad, "grad")
    nat.check_tensor(offsets, "offsets", _INT, "int")
    if inputs.dtype != embeddings.dtype or grad.dtype != embeddings.dtype:
        raise RuntimeError("inputs, embeddings and grad must share a dtype")
    rc = nat.lib().ngp_grad_total_variation(
        nat.ptr(inputs), nat.ptr(embeddings), nat.ptr(grad), nat.ptr(offsets), float(weight), B, D,
        C, L, float(S), H, gridtype, int(bool(align_corners)), _dtype(embeddings),
        nat.stream_of(inputs))
    nat.check(rc, "grad_total_variation")


_backend = types.SimpleNamespace(
    grid_encode_forward=grid_encode_forward,
    grid_encode_backward=grid_encode_backward,
    grid_encode_forward_bm=grid_encode_forward_bm,
    grid_encode_backward_bm=grid_encode_backward_bm,
    grad_total_variation=grad_total_variation,
)

__all__ = ["_backend"]
