"""Pointwise squared error (reference divrec/losses/mse_loss.py:6-10)."""
import torch

from .base_losses import PointWiseLoss


class MSELoss(PointWiseLoss):
    def point_wise(self, true_relevance: torch.Tensor, predicted_relevance: torch.Tensor):
        return (true_relevance - predicted_relevance) ** 2
