"""Shared helpers of the GAR modules (parameter checks, influence bookkeeping)."""
from __future__ import annotations

import torch


def n_of(gradients) -> int:
    if isinstance(gradients, torch.Tensor):
        return gradients.shape[0] if gradients.dim() == 2 else 1
    return len(gradients)


def check_gradients(gradients):
    if isinstance(gradients, torch.Tensor):
        if gradients.dim() != 2 or gradients.shape[0] < 1:
            return f"Expected an [n, d] tensor with n >= 1, got shape {tuple(gradients.shape)}"
        return None
    if not isinstance(gradients, list) or len(gradients) < 1:
        return f"Expected a list of at least one gradient to aggregate, got {gradients!r}"
    return None


def check_f(f, n: int, min_n, bound_text: str):
    """f must be an int >= 1 with n >= min_n(f)."""
    if not isinstance(f, int) or isinstance(f, bool) or f < 1 or n < min_n(f):
        return f"Invalid number of Byzantine gradients to tolerate, got f = {f!r}, expected {bound_text}"
    return None


def accepted_ratio(weights: torch.Tensor, n_honest: int) -> float:
    """Ratio of accepted Byzantine gradients (ids >= n_honest) among the selected ones."""
    w = weights.detach().float().cpu()
    sel = (w != 0).nonzero().flatten().tolist()
    if not sel:
        return 0.0
    return sum(1 for i in sel if i >= n_honest) / len(sel)


def stack_for_influence(honests, attacks):
    return list(honests) + list(attacks), len(honests)
