"""Recall@k (reference divrec/metrics/recall_at_k.py:6-29): hits / number of
the user's test interactions (NaN for a user without any; the reference
raises ZeroDivisionError there)."""
import torch

from divrec.losses.base_losses import RecommendationsAwareLoss

from ._rank import rank_metrics


def recall_at_k(interactions: torch.LongTensor, recommendations: torch.LongTensor):
    return rank_metrics(interactions, recommendations)[1]


class RecallAtKScore(RecommendationsAwareLoss):
    def recommendations_loss(self, interactions, recommendations) -> torch.Tensor:
        return recall_at_k(interactions, recommendations)
