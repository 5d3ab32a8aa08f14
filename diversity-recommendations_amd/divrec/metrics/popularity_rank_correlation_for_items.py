"""Popularity-rank correlation PRI (reference
divrec/metrics/popularity_rank_correlation_for_items.py:6-63): Pearson
correlation between an item's popularity rank and its average position in the
recommendation lists. Catalog-level statistic (SURVEY.md §8f rank 2, next
tier): tensor ops, the per-item average position by a scatter instead of the
reference's Python dict loop."""
import torch

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


def avg_rank(recommendations: torch.LongTensor):
    """(items ascending, mean position of each item over all lists)."""
    n, k = recommendations.shape
    flat = recommendations.reshape(-1)
    pos = torch.arange(k, device=recommendations.device).repeat(n).to(torch.float64)
    items, inv = torch.unique(flat, return_inverse=True)
    total = torch.zeros(items.numel(), dtype=torch.float64, device=flat.device).index_add_(0, inv, pos)
    cnt = torch.bincount(inv, minlength=items.numel()).to(torch.float64)
    return items, (total / cnt).to(torch.float32)


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
        items, ranks = avg_rank(recommendations)
        pr = self.popularity_rank.to(items.device)[items]
        return spearman_rank_correlation(pr, ranks, evaluate_rank=False)
