"""Sample / candidate streams of the reference (host side).

Mirrors reference divrec/datasets/base_datasets.py: PointWiseDataset (:41-56),
PairWiseDataset (:59-110) and RankingDataset (:113-171). They are host-side
index streams; the GPU paths consume them as CSR (``exclusion_csr``).

PairWiseDataset draws its samples with Python ``random.choices`` over the same
populations, in the same order, as the reference, so a seeded ``random``
yields the same (user, positive, negative) triples.

Divergences: RankingDataset accepts ``frozen=None`` (every
item is a candidate) where the reference raises TypeError (:151,168).
"""
from __future__ import annotations

import random
from typing import Iterator, Optional, Tuple

import torch
from torch.utils.data import DataLoader, Dataset, IterableDataset

from .storages import UserItemInteractionsDataset, get_item_features, get_user_features

PointWiseRow = Tuple[int, int, Optional[torch.Tensor], Optional[torch.Tensor], float]
PairWiseRow = Tuple[int, int, int, Optional[torch.Tensor], Optional[torch.Tensor],
                    Optional[torch.Tensor]]
RankingRow = Tuple[torch.LongTensor, torch.LongTensor, torch.LongTensor,
                   Optional[torch.Tensor], Optional[torch.Tensor]]


def _user_items(data: UserItemInteractionsDataset, user_id: int) -> torch.Tensor:
    inter = data.interactions
    return inter[inter[:, 0] == user_id, 1]


class PointWiseDataset(Dataset):
    """(user, item, user features, item features, score) per interaction."""

    def __init__(self, data: UserItemInteractionsDataset):
        self.data = data

    def __len__(self) -> int:
        return self.data.number_of_interactions

    def __getitem__(self, index: int) -> PointWiseRow:
        user_id, item_id = self.data.interactions[index]
        # the reference indexes the scores by item id, not by row (:52)
        score = self.data.interaction_scores[item_id]
        return (user_id, item_id, get_user_features(self.data, user_id),
                get_item_features(self.data, item_id), score)

    def loader(self, **loader_params) -> DataLoader:
        return DataLoader(self, **loader_params)


class PairWiseDataset(IterableDataset):
    """Per user: positives x negatives (the Cartesian product of two samples
    with replacement of ``max_sampled`` items each, pos-major)."""

    def __init__(self, data: UserItemInteractionsDataset,
                 frozen: Optional[UserItemInteractionsDataset] = None, max_sampled: int = 100):
        self.data = data
        self.frozen = frozen
        self.max_sampled = max_sampled

    def __iter__(self) -> Iterator[PairWiseRow]:
        catalog = frozenset(range(self.data.number_of_items))
        for user_id in range(self.data.number_of_users):
            ufeat = get_user_features(self.data, user_id)
            pos = frozenset(_user_items(self.data, user_id).tolist())
            neg = catalog - pos
            if self.frozen is not None:
                neg = neg - frozenset(_user_items(self.frozen, user_id).tolist())
            if self.max_sampled > 0:
                pos = random.choices(list(pos), k=self.max_sampled)
                neg = random.choices(list(neg), k=self.max_sampled)
            for p in pos:
                pfeat = get_item_features(self.data, p)
                for n in neg:
                    yield user_id, p, n, ufeat, pfeat, get_item_features(self.data, n)

    def loader(self, **loader_params) -> DataLoader:
        return DataLoader(self, **loader_params)


class RankingDataset(IterableDataset):
    """One row per user: the user id repeated over its candidates, its
    positives, and the candidates = every item except the user's ``frozen``
    interactions, in ascending item id."""

    def __init__(self, data: UserItemInteractionsDataset,
                 frozen: Optional[UserItemInteractionsDataset] = None):
        self.data = data
        self.frozen = frozen

    def candidates(self, user_id: int) -> torch.LongTensor:
        n = self.data.number_of_items
        if self.frozen is None:
            return torch.arange(n, dtype=torch.long)
        keep = torch.ones(n, dtype=torch.bool)
        f = _user_items(self.frozen, user_id)
        keep[f[f < n]] = False
        return torch.nonzero(keep).flatten()

    def __iter__(self) -> Iterator[RankingRow]:
        for user_id in range(self.data.number_of_users):
            positives = _user_items(self.data, user_id)
            cands = self.candidates(user_id)
            ufeat = ifeat = None
            if self.data.has_user_features():
                # as the reference (:153-163): the whole user table per candidate,
                # and item features gated on has_user_features()
                ufeat = torch.concatenate([self.data.user_features.features for _ in cands])
                ifeat = torch.concatenate([get_item_features(self.data, int(i)) for i in cands])
            yield torch.full((len(cands),), user_id), positives, cands, ufeat, ifeat

    def exclusion_csr(self) -> Optional[Tuple[torch.Tensor, torch.Tensor]]:
        """Frozen items per user as CSR (rowptr int64 [U+1], items int32), or
        None without ``frozen`` — what dr_score_topk excludes."""
        if self.frozen is None or not self.frozen.has_interactions():
            return None
        return self.frozen.user_item_csr(self.data.number_of_users)
