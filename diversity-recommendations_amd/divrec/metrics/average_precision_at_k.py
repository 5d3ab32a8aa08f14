"""AP@k / MAP@k (reference divrec/metrics/average_precision_at_k.py:6-38) with
the reference's formula: sum over ALL k positions of cumhits(p) / (p+1),
divided by k."""
import torch

from divrec.losses.base_losses import RecommendationsAwareLoss

from ._rank import rank_metrics


def average_precision_at_k(interactions: torch.LongTensor, recommendations: torch.LongTensor):
    return rank_metrics(interactions, recommendations)[2]


class AveragePrecisionAtKScore(RecommendationsAwareLoss):
    def recommendations_loss(self, interactions, recommendations) -> torch.Tensor:
        return average_precision_at_k(interactions, recommendations)


class MeanAveragePrecisionAtKScore(AveragePrecisionAtKScore):
    def forward(self, interactions, recommendations):
        return torch.mean(average_precision_at_k(interactions, recommendations))
