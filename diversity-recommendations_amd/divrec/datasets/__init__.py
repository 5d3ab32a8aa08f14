from .base_datasets import (
    DevicePairWiseDataset,
    PairWiseDataset,
    PairWiseRow,
    PointWiseDataset,
    PointWiseRow,
    RankingDataset,
    RankingRow,
)
from .storages import Features, UserItemInteractionsDataset

__all__ = [
    "DevicePairWiseDataset",
    "Features",
    "UserItemInteractionsDataset",
    "PairWiseRow",
    "PairWiseDataset",
    "PointWiseRow",
    "PointWiseDataset",
    "RankingDataset",
    "RankingRow",
]
