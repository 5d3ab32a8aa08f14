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


def _device_csr(data: UserItemInteractionsDataset, n_users: int, n_items: int, device):
    """Unique (user, item) pairs of ``data`` as a CSR on ``device``: rowptr
    int64 [n_users + 1], items int32 sorted per user (frozenset semantics)."""
    inter = data.interactions.to(device=device, dtype=torch.int64)
    key = torch.unique(inter[:, 0] * n_items + inter[:, 1])  # sorted, unique
    users, items = key // n_items, key % n_items
    counts = torch.bincount(users, minlength=n_users)
    rowptr = torch.zeros(n_users + 1, dtype=torch.int64, device=device)
    rowptr[1:] = torch.cumsum(counts, 0)
    return rowptr, items.to(torch.int32).contiguous()


class DevicePairWiseDataset:
    """PairWiseDataset with the sampling on the GPU.

    Same populations, layout and order as the reference's PairWiseDataset
    (base_datasets.py:70-107): users 0..U-1, per user m positives drawn with
    replacement from its unique positives and m negatives from
    items - positives - frozen, yielded as the m x m product (positive-major).
    The draws come from dr_sample_pairwise's counter-based generator instead of
    Python's ``random`` (parity is distributional; each ``loader()`` call is a
    new epoch with fresh draws). ``loader(batch_size=B)`` yields batches of B
    consecutive triples as device tensors ``(user, positive, negative, None,
    None, None)`` (features are not gathered: the MF fast path ignores them).
    Requires ``max_sampled > 0``. A user without positives raises IndexError,
    as the reference does, when its chunk is sampled."""

    def __init__(self, data: UserItemInteractionsDataset,
                 frozen: Optional[UserItemInteractionsDataset] = None, max_sampled: int = 100,
                 device="cuda", seed: int = 0, triples_per_chunk: int = 1 << 22):
        if max_sampled <= 0:
            raise ValueError("DevicePairWiseDataset samples: max_sampled must be > 0")
        self.data = data
        self.frozen = frozen
        self.max_sampled = int(max_sampled)
        self.device = torch.device(device)
        self.seed = int(seed)
        self.epoch = 0
        self.n_users = int(data.number_of_users)
        self.n_items = int(data.number_of_items)
        self.pos_csr = _device_csr(data, self.n_users, self.n_items, self.device)
        self.excl_csr = None
        if frozen is not None:
            self.excl_csr = _device_csr(frozen, self.n_users, self.n_items, self.device)
        self.users_per_chunk = max(1, triples_per_chunk // (self.max_sampled ** 2))

    def __len__(self) -> int:
        return self.n_users * self.max_sampled ** 2

    def loader(self, batch_size: int = 1, **_unused) -> Iterator[PairWiseRow]:
        from .. import ops  # device path only

        seed = (self.seed * 0x9E3779B97F4A7C15 + self.epoch) & ((1 << 64) - 1)
        self.epoch += 1
        carry = None
        for u0 in range(0, self.n_users, self.users_per_chunk):
            users = torch.arange(u0, min(u0 + self.users_per_chunk, self.n_users),
                                 dtype=torch.int64, device=self.device)
            _, _, trip = ops.sample_pairwise(users, *self.pos_csr, self.n_items, self.max_sampled,
                                             seed, exclude=self.excl_csr)
            if carry is not None:
                trip = tuple(torch.cat([c, t]) for c, t in zip(carry, trip))
            n_full = trip[0].numel() // batch_size * batch_size
            for b0 in range(0, n_full, batch_size):
                yield (trip[0][b0:b0 + batch_size], trip[1][b0:b0 + batch_size],
                       trip[2][b0:b0 + batch_size], None, None, None)
            carry = tuple(t[n_full:] for t in trip)
        if carry is not None and carry[0].numel() > 0:
            yield carry[0], carry[1], carry[2], None, None, None
