from .base_datasets import (
    PairWiseDataset,
    PairWiseRow,
    PointWiseDataset,
    PointWiseRow,
    RankingDataset,
    RankingRow,
)
from .storages import Features, UserItemInteractionsDataset

__all__ = [
    "Features",
    "UserItemInteractionsDataset",
    "PairWiseRow",
    "PairWiseDataset",
    "PointWiseRow",
    "PointWiseDataset",
    "RankingDataset",
    "RankingRow",
]
