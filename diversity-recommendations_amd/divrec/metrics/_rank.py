"""Shared host plumbing of the accuracy metrics: positives CSR + one kernel call."""
from __future__ import annotations

import contextlib
from typing import Tuple

import torch

from divrec import _backend, ops


def positives_csr(interactions: torch.Tensor, n_users: int, device) -> Tuple[torch.Tensor, torch.Tensor]:
    """Per-user item ids of ``interactions`` [N, 2] as CSR sorted by item
    (duplicates kept: the reference's recall divides by the raw count)."""
    inter = interactions.to(device=device, dtype=torch.int64)
    inter = inter[(inter[:, 0] >= 0) & (inter[:, 0] < n_users)]
    key = inter[:, 0] * (int(inter[:, 1].max()) + 1 if inter.numel() else 1) + inter[:, 1]
    order = torch.argsort(key)
    users, items = inter[order, 0], inter[order, 1]
    counts = torch.bincount(users, minlength=n_users)
    rowptr = torch.zeros(n_users + 1, dtype=torch.int64, device=device)
    rowptr[1:] = torch.cumsum(counts, 0)
    return rowptr, items.to(torch.int32).contiguous()


_SHARED = None  # [(interactions, recommendations, result)] inside shared_rank_metrics()


@contextlib.contextmanager
def shared_rank_metrics():
    """Inside the block, rank_metrics computes once per (interactions,
    recommendations) pair of tensor OBJECTS and hands the same four per-row
    arrays to every caller: train.recommendations_score_loop evaluates
    P@k, R@k, MAP@k and NDCG@k on one pair, and dr_rank_metrics computes all
    four in one launch. The pair cannot change inside the loop."""
    global _SHARED
    prev, _SHARED = _SHARED, []
    try:
        yield
    finally:
        _SHARED = prev


def rank_metrics(interactions: torch.Tensor, recommendations: torch.Tensor):
    """(precision, recall, AP, NDCG) per recommendation row, on the
    recommendations' device (computed by dr_rank_metrics)."""
    if _SHARED is not None:
        for inter, recs, res in _SHARED:
            if inter is interactions and recs is recommendations:
                return res
    dev = recommendations.device if recommendations.is_cuda else _backend.default_device()
    recs = recommendations.to(dev)
    rowptr, items = positives_csr(interactions, recs.size(0), dev)
    out = ops.rank_metrics(recs, rowptr, items)
    res = tuple(o.to(recommendations.device) for o in out)
    if _SHARED is not None:
        _SHARED.append((interactions, recommendations, res))
    return res
