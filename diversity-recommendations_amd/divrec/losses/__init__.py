from .base_losses import (
    DatasetAwareLoss,
    PairWiseLoss,
    PointWiseLoss,
    RecommendationsAwareLoss,
    ScoreWithReduction,
)
from .intra_list_diversity_score import (
    EmbeddingDistance,
    IntraListBinaryUnfairnessScore,
    IntraListDiversityScore,
    LabelEquality,
)
from .log_sigmoid_difference_loss import LogSigmoidDifferenceLoss
from .mse_loss import MSELoss

__all__ = [
    "LogSigmoidDifferenceLoss",
    "IntraListDiversityScore",
    "IntraListBinaryUnfairnessScore",
    "EmbeddingDistance",
    "LabelEquality",
    "PointWiseLoss",
    "PairWiseLoss",
    "RecommendationsAwareLoss",
    "DatasetAwareLoss",
    "MSELoss",
    "ScoreWithReduction",
]
