"""Shared host plumbing of the accuracy metrics: positives CSR + one kernel call."""
from __future__ import annotations

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


def rank_metrics(interactions: torch.Tensor, recommendations: torch.Tensor):
    """(precision, recall, AP, NDCG) per recommendation row, on the
    recommendations' device (computed by dr_rank_metrics)."""
    dev = recommendations.device if recommendations.is_cuda else _backend.default_device()
    recs = recommendations.to(dev)
    rowptr, items = positives_csr(interactions, recs.size(0), dev)
    out = ops.rank_metrics(recs, rowptr, items)
    return tuple(o.to(recommendations.device) for o in out)
