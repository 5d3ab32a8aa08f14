"""NDCG@k (reference divrec/metrics/normalized_discounted_cumulative_gain.py:6-30):
sum_p rel(p) / log2(p+2), normalised by sum_p 1 / log2(p+2)."""
import torch

from divrec.losses.base_losses import RecommendationsAwareLoss

from ._rank import rank_metrics


def normalized_discounted_cumulative_gain(interactions: torch.LongTensor,
                                          recommendations: torch.LongTensor):
    return rank_metrics(interactions, recommendations)[3]


class NDCGScore(RecommendationsAwareLoss):
    def recommendations_loss(self, interactions, recommendations) -> torch.Tensor:
        return normalized_discounted_cumulative_gain(interactions, recommendations)
