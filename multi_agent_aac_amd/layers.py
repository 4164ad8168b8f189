"""Fused linear layers for the learner (forward + hand-written backward).

``fused_linear(x, W, b, act, slot)`` computes ``act(x W^T + b)`` like ``nn.Linear`` followed by
ReLU / Tanh / nothing (ATT/nets:180-184, :699-701), with:
  forward   one GEMM with the bias (and ReLU) fused into the hipBLASLt epilogue;
  backward  one HIP kernel for the activation derivative + bias gradient (aac_act_bgrad), the
            weight gradient as a rocBLAS split-K GEMM written straight into the network's flat
            gradient buffer (no autograd accumulate kernels), and the data-gradient GEMM.
Weight / bias gradients are written, not accumulated: every parameter is used by exactly one
layer call per backward in update_myown, and ``slot.enabled`` switches the writes off for the
backward passes that must not touch a network's grads (the critic during the actor loss).
"""
import contextlib

import torch

from . import ops

IDENTITY, RELU, TANH = 0, 1, 2

_FWD_BLAS = "cublaslt"   # hipBLASLt: fused bias/ReLU epilogues for the M-large forward GEMMs
_BWD_BLAS = "cublas"     # rocBLAS: split-K for dW = G^T X over 5k-20k rows


@contextlib.contextmanager
def blas(name):
    prev = torch.backends.cuda.preferred_blas_library()
    torch.backends.cuda.preferred_blas_library(name)
    try:
        yield
    finally:
        torch.backends.cuda.preferred_blas_library(prev)


def set_blas(fwd, bwd):
    global _FWD_BLAS, _BWD_BLAS
    _FWD_BLAS, _BWD_BLAS = fwd, bwd


class GradSlot:
    """Where a network's weight gradients go, and whether to produce them."""

    def __init__(self):
        self.enabled = True


class _FusedLinear(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, W, b, act, slot):
        with blas(_FWD_BLAS):
            if b is not None and act == RELU:
                y = torch._addmm_activation(b, x, W.t())
            elif b is not None:
                y = torch.addmm(b, x, W.t())
            else:
                y = torch.mm(x, W.t())
                if act == RELU:
                    y = torch.relu_(y)
        if act == TANH:
            y = torch.tanh_(y)
        ctx.save_for_backward(x, W, y)
        ctx.act, ctx.slot, ctx.has_b = act, slot, b is not None
        ctx.b = b
        return y

    @staticmethod
    def backward(ctx, gy):
        x, W, y = ctx.saved_tensors
        act, slot = ctx.act, ctx.slot
        gy = gy.contiguous()
        M, O = gy.shape
        want_w = slot.enabled
        db = ctx.b.grad if (want_w and ctx.has_b) else None
        if act == IDENTITY:
            gm = gy
            if db is not None:
                ops.act_bgrad(gy, None, None, db, IDENTITY)
        else:
            gm = torch.empty_like(gy)
            ops.act_bgrad(gy, y, gm, db, act)
        with blas(_BWD_BLAS):
            if want_w:
                torch.mm(gm.t(), x, out=W.grad)
            dx = torch.mm(gm, W) if ctx.needs_input_grad[0] else None
        return dx, None, None, None, None


def fused_linear(x, W, b, act, slot):
    return _FusedLinear.apply(x, W, b, act, slot)


class _StackedLinearReLU(torch.autograd.Function):
    """Per-agent encoders of the critic: y[b, n, :] = relu(x[b, n, :] W_n^T + b_n), all N agents in
    one strided-batched GEMM; output laid out (B, N*H) so the combine layer reads it directly."""

    @staticmethod
    def forward(ctx, x, W, b, slot):
        B, N, D = x.shape
        H = W.shape[1]
        y = torch.empty(B, N, H, device=x.device, dtype=x.dtype)
        with blas(_BWD_BLAS):
            torch.bmm(x.transpose(0, 1), W.transpose(1, 2), out=y.transpose(0, 1))
        y = y.view(B, N * H)
        ops.bias_act(y, b.view(-1), RELU)
        ctx.save_for_backward(x, W, y)
        ctx.slot, ctx.b = slot, b
        return y

    @staticmethod
    def backward(ctx, gy):
        x, W, y = ctx.saved_tensors
        B, N, D = x.shape
        H = W.shape[1]
        gy = gy.contiguous()
        gm = torch.empty_like(gy)
        db = ctx.b.grad.view(-1) if ctx.slot.enabled else None
        ops.act_bgrad(gy, y, gm, db, RELU)
        g3 = gm.view(B, N, H).transpose(0, 1)                # (N, B, H)
        with blas(_BWD_BLAS):
            if ctx.slot.enabled:
                torch.bmm(g3.transpose(1, 2), x.transpose(0, 1), out=W.grad)
            dx = None
            if ctx.needs_input_grad[0]:
                dx = torch.empty_like(x)
                torch.bmm(g3, W, out=dx.transpose(0, 1))
        return dx, None, None, None


def stacked_linear_relu(x, W, b, slot):
    return _StackedLinearReLU.apply(x, W, b, slot)
