"""Interaction / feature containers (host side).

Mirrors reference divrec/datasets/storages.py:7-110: the same dataclass
fields, derived counts and validation asserts. These are plain host data
structures (the index streams the GPU kernels consume); nothing here computes
on the hot path. Divergence (documented in INTEGRATION.md): derived
``number_of_users`` / ``number_of_items`` are Python ints, where the reference
leaves a 0-d tensor when it derives them from the data (storages.py:63-64).
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import List, Optional, Tuple

import torch


@dataclass
class Features:
    """Table with named columns (reference storages.py:7-30)."""

    features: torch.Tensor = None
    feature_names: List[str] = field(default_factory=list)
    number_of_features: int = 0

    def __post_init__(self):
        self.number_of_features = max(self.number_of_features, self.features.size(1))
        assert len(self.feature_names) == self.number_of_features

    def __len__(self) -> int:
        return self.features.size(0)

    def __getitem__(self, name: str) -> torch.Tensor:
        return self.features[:, self.feature_names.index(name)]

    def __contains__(self, name: str) -> bool:
        return name in self.feature_names


@dataclass
class UserItemInteractionsDataset:
    """User-item interactions with optional scores and features
    (reference storages.py:33-94)."""

    interactions: Optional[torch.LongTensor] = None
    interaction_scores: Optional[torch.Tensor] = None
    user_features: Optional[Features] = None
    item_features: Optional[Features] = None

    number_of_interactions: int = 0
    number_of_users: int = 0
    number_of_items: int = 0

    def __post_init__(self):
        if self.interactions is not None:
            n, cols = self.interactions.size()
            self.number_of_interactions = n
            assert cols == 2
            if self.interaction_scores is None:
                self.interaction_scores = torch.ones(n)
            assert self.interaction_scores.size(0) == n
            users = torch.unique(self.interactions[:, 0])
            items = torch.unique(self.interactions[:, 1])
            self.number_of_users = max(int(self.number_of_users), int(users.max()) + 1)
            self.number_of_items = max(int(self.number_of_items), int(items.max()) + 1)
            assert bool(torch.all((users >= 0) & (users < self.number_of_users)))
            assert bool(torch.all((items >= 0) & (items < self.number_of_items)))
        if self.interaction_scores is not None:
            assert self.interactions is not None
            assert self.interaction_scores.size(0) == self.number_of_interactions
        if self.user_features is not None:
            if self.number_of_users == 0:
                self.number_of_users = len(self.user_features)
            assert self.number_of_users == len(self.user_features)
        if self.item_features is not None:
            if self.number_of_items == 0:
                self.number_of_items = len(self.item_features)
            assert self.number_of_items == len(self.item_features)

    def has_interactions(self) -> bool:
        return self.interactions is not None

    def has_user_features(self) -> bool:
        return self.user_features is not None

    def has_item_features(self) -> bool:
        return self.item_features is not None

    def user_item_csr(self, n_users: Optional[int] = None) -> Tuple[torch.Tensor, torch.Tensor]:
        """Per-user sorted, de-duplicated item ids as CSR (rowptr int64
        [n_users+1], items int32): the exclusion lists / positives the GPU
        kernels consume in place of the reference's per-user Python set ops.

        The CSR is kept between calls (an evaluation loop asks for the same
        exclusions every epoch) and rebuilt when the interactions change: the
        key is the tensor's storage, shape, version and two O(N) checksums of
        its values, so in-place writes torch does not record (``.data``, numpy
        views) are seen too. Treat the returned tensors as read-only."""
        n_users = self.number_of_users if n_users is None else n_users
        if self.interactions is None or self.interactions.numel() == 0:
            return torch.zeros(n_users + 1, dtype=torch.int64), torch.zeros(0, dtype=torch.int32)
        key = _csr_key(self.interactions, n_users)
        cached = getattr(self, "_csr_cache", None)
        if cached is not None and cached[0] == key:
            return cached[1]
        out = self._build_user_item_csr(n_users)
        self._csr_cache = (key, out)
        return out

    def _build_user_item_csr(self, n_users: int) -> Tuple[torch.Tensor, torch.Tensor]:
        inter = self.interactions.to(torch.int64)
        inter = inter[inter[:, 0] < n_users]
        # one sorted, de-duplicated 1-D key per (user, item): the same order as
        # torch.unique(dim=0) and ~20x faster on the host
        span = int(inter[:, 1].max()) + 1 if inter.numel() else 1
        key = torch.unique(inter[:, 0] * span + inter[:, 1])
        users, items = key // span, key % span
        counts = torch.bincount(users, minlength=n_users)
        rowptr = torch.zeros(n_users + 1, dtype=torch.int64)
        rowptr[1:] = torch.cumsum(counts, 0)
        return rowptr, items.to(torch.int32).contiguous()


def _csr_key(inter: torch.Tensor, n_users: int):
    """Identity of an interactions tensor's values for user_item_csr's cache."""
    x = inter.to(torch.int64)
    h1 = int(x.sum())
    h2 = int((x[:, 0] * 1000003 + x[:, 1] * 7919 + 1).mul_(
        torch.arange(1, x.size(0) + 1, dtype=torch.int64)).sum())  # order-sensitive
    return (n_users, inter.data_ptr(), tuple(inter.shape), inter.dtype, inter._version, h1, h2)


def get_user_features(data: UserItemInteractionsDataset, user_id: int) -> Optional[torch.Tensor]:
    if data.user_features is None:
        return None
    return data.user_features.features[user_id]


def get_item_features(data: UserItemInteractionsDataset, item_id: int) -> Optional[torch.Tensor]:
    if data.item_features is None:
        return None
    return data.item_features.features[item_id]
