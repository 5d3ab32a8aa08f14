"""Entropy diversity of the recommended items (reference
divrec/metrics/entropy_diversity_score.py:8-26): normalised Shannon entropy of
the recommendation histogram between log(k) and log(#items). Catalog-level
statistic: the histogram is one HIP kernel
(dr_catalog_histogram, integer atomics); the entropy of the non-zero counts
follows the reference's own tensor expression."""
import math

import torch

from divrec import _backend, ops
from divrec.losses.base_losses import DatasetAwareLoss, RecommendationsAwareLoss


class EntropyDiversityScore(RecommendationsAwareLoss, DatasetAwareLoss):
    def __init__(self, *args, **kwargs):
        DatasetAwareLoss.__init__(self, *args, **kwargs)
        RecommendationsAwareLoss.__init__(self, *args, **kwargs)
        self.max_entropy = math.log(self.dataset.number_of_items)

    def forward(self, interactions, recommendations):
        return self.recommendations_loss(interactions, recommendations)

    def recommendations_loss(self, interactions, recommendations) -> torch.Tensor:
        dev = recommendations.device if recommendations.is_cuda else _backend.default_device()
        n_items = int(self.dataset.number_of_items)
        hist, _ = ops.catalog_histogram(recommendations.to(dev), n_items)
        counts = hist[hist > 0].to(torch.int64)  # torch.unique's counts: ascending item order
        p = counts / counts.sum()
        actual = -torch.sum(p * torch.log(p))
        min_entropy = math.log(recommendations.size(1))
        return (actual - min_entropy) / (self.max_entropy - min_entropy)
