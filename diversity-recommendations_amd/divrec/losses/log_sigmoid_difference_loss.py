"""BPR loss -logsigmoid(pos - neg) (reference log_sigmoid_difference_loss.py:6-14).

As in the reference, keyword arguments do not reach ScoreWithReduction (the
reference forwards ``*kwargs``), so the reduction is always 'mean'. The fused
training path (divrec.train.pair_wise_train_loop with a MatrixFactorization)
computes this loss and its gradients inside dr_bpr_fwd_bwd."""
import torch

from .base_losses import PairWiseLoss


class LogSigmoidDifferenceLoss(PairWiseLoss):
    def __init__(self, *args, **kwargs):
        PairWiseLoss.__init__(self, *args)  # keyword arguments ignored, as the reference

    def pair_wise(self, positives: torch.Tensor, negatives: torch.Tensor) -> torch.Tensor:
        return -torch.nn.functional.logsigmoid(positives - negatives)
