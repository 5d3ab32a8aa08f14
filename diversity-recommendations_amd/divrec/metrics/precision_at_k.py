"""Precision@k (reference divrec/metrics/precision_at_k.py:6-32), computed by
dr_rank_metrics: hits among the k recommendations / k, per user."""
import torch

from divrec.losses.base_losses import RecommendationsAwareLoss

from ._rank import rank_metrics


def precision_at_k(interactions: torch.LongTensor, recommendations: torch.LongTensor):
    return rank_metrics(interactions, recommendations)[0]


class PrecisionAtKScore(RecommendationsAwareLoss):
    def recommendations_loss(self, interactions, recommendations) -> torch.Tensor:
        return precision_at_k(interactions, recommendations)


HitRateScore = PrecisionAtKScore
