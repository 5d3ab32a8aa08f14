"""Popularity-rank correlation PRI (reference
divrec/metrics/popularity_rank_correlation_for_items.py:6-63): Pearson
correlation between an item's popularity rank and its average position in the
recommendation lists. Catalog-level statistic: the
per-item counts and position sums come from one HIP kernel
(dr_catalog_histogram, exact integer atomics) instead of the reference's
Python dict loop; the correlation is the reference's tensor expression."""
import torch

from divrec import _backend, ops
from divrec.losses.base_losses import DatasetAwareLoss, RecommendationsAwareLoss


def rank(a: torch.Tensor, dim=-1, descending=False, stable=False):
    return torch.argsort(torch.argsort(a, dim=dim, descending=descending, stable=stable),
                         dim=dim, stable=stable)


def spearman_rank_correlation(a: torch.Tensor, b: torch.Tensor, evaluate_rank: bool = True):
    assert a.size(0) == b.size(0)
    n = a.size(0)
    if evaluate_rank:
        d = rank(a) - rank(b)
        return 1 - 6 * torch.sum(d ** 2) / n / (n ** 2 - 1)
    a_std, a_mean = torch.std_mean(a)
    b_std, b_mean = torch.std_mean(b)
    return torch.mean((a - a_mean) * (b - b_mean)) / a_std / b_std


def avg_rank(recommendations: torch.LongTensor, n_items=None):
    """(items ascending, mean 0-based position of each item over all lists):
    the reference's sum(r) / len(r) per item (exact integer sums, divided in
    float64, stored as float32 like its FloatTensor)."""
    dev = recommendations.device if recommendations.is_cuda else _backend.default_device()
    recs = recommendations.to(dev)
    if n_items is None:
        n_items = int(recs.max()) + 1 if recs.numel() else 1
    counts, pos_sum = ops.catalog_histogram(recs, int(n_items))
    items = torch.nonzero(counts > 0).flatten()
    avg = (pos_sum[items].to(torch.float64) / counts[items].to(torch.float64)).to(torch.float32)
    return items, avg


class PRI(RecommendationsAwareLoss, DatasetAwareLoss):
    def __init__(self, *args, **kwargs):
        DatasetAwareLoss.__init__(self, *args, **kwargs)
        RecommendationsAwareLoss.__init__(self, *args, **kwargs)
        items, counts = torch.unique(self.dataset.interactions[:, 1], return_counts=True)
        self.popularity = torch.zeros(self.dataset.number_of_items, dtype=torch.float)
        self.popularity[items] = counts.float()
        self.popularity_rank = rank(self.popularity, descending=True).float()

    def forward(self, interactions, recommendations):
        return self.recommendations_loss(interactions, recommendations)

    def recommendations_loss(self, interactions, recommendations) -> torch.Tensor:
        items, ranks = avg_rank(recommendations, int(self.dataset.number_of_items))
        pr = self.popularity_rank.to(items.device)[items]
        return spearman_rank_correlation(pr, ranks, evaluate_rank=False)
