"""Pairwise AUC hit (reference divrec/metrics/auc_score.py:6-10): pos >= neg
(ties count); averaged by the reduction. The fused BPR step produces the same
flags in dr_bpr_fwd_bwd."""
import torch

from divrec.losses.base_losses import PairWiseLoss


class AUCScore(PairWiseLoss):
    def pair_wise(self, positives: torch.Tensor, negatives: torch.Tensor) -> torch.Tensor:
        return (positives >= negatives).int()
