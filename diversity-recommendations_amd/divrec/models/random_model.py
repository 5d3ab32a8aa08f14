"""RandomModel (reference divrec/models/random_model.py:8-21): N(0,1) scores of
the ids' shape, generated on the CPU as the reference does (no value parity:
it is an RNG baseline)."""
from typing import Optional

import torch

from .base_models import RankingModel


class RandomModel(RankingModel):
    def __init__(self, no_users: int, no_items: int):
        torch.nn.Module.__init__(self)
        self.no_users = no_users
        self.no_items = no_items

    def forward(
        self,
        user_id: torch.LongTensor,
        item_id: torch.LongTensor,
        user_features: Optional[torch.Tensor] = None,
        item_features: Optional[torch.Tensor] = None,
    ) -> torch.Tensor:
        return torch.randn(user_id.size())
