"""Autograd for the forward-backward op (training-mode HMMLayer / compute_loss).

The reference differentiates through its Python loop with plain autograd
(hmm_layer.py:144-173, test_hmm.py:189-208).  Here the gradient is the analytic adjoint
of the two recursions, computed by HIP kernels (csrc/fb_grad.hip).
"""
import torch


def needs_grad(*tensors) -> bool:
    return torch.is_grad_enabled() and any(t is not None and t.requires_grad for t in tensors)


def forward_backward_with_grad(obs, log_P, log_p0):
    raise NotImplementedError(
        "differentiable forward-backward (analytic adjoint kernels) is not built yet; "
        "call under torch.no_grad() for inference")
