from divrec.losses.intra_list_diversity_score import IntraListDiversityScore

from .auc_score import AUCScore
from .average_precision_at_k import (
    AveragePrecisionAtKScore,
    MeanAveragePrecisionAtKScore,
    average_precision_at_k,
)
from .entropy_diversity_score import EntropyDiversityScore
from .normalized_discounted_cumulative_gain import NDCGScore, normalized_discounted_cumulative_gain
from .popularity_rank_correlation_for_items import PRI, avg_rank, rank
from .precision_at_k import HitRateScore, PrecisionAtKScore, precision_at_k
from .recall_at_k import RecallAtKScore, recall_at_k

__all__ = [
    "AUCScore",
    "AveragePrecisionAtKScore",
    "EntropyDiversityScore",
    "HitRateScore",
    "IntraListDiversityScore",
    "MeanAveragePrecisionAtKScore",
    "NDCGScore",
    "avg_rank",
    "rank",
    "PRI",
    "PrecisionAtKScore",
    "RecallAtKScore",
    "average_precision_at_k",
    "normalized_discounted_cumulative_gain",
    "precision_at_k",
    "recall_at_k",
]
