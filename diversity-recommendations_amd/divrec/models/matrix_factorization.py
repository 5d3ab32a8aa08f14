"""MatrixFactorization on the HIP path (reference divrec/models/matrix_factorization.py:8-28).

Same constructor, attributes and state-dict keys (``user_embeddings.weight``,
``item_embeddings.weight``: fp32 nn.Embedding, N(0,1) init, dense gradients),
so reference checkpoints load unchanged. ``forward`` is the fused embedding
gather + row dot of libdivrec_hip (dr_gather_dot) with its backward
(dr_gather_dot_backward) into dense fp32 gradients; parameters must live on a
ROCm device (``model.to("cuda")``) — there is no CPU path.

New, non-breaking: ``score_topk`` — full-catalog bf16 MFMA scoring with a
fused top-k (dr_score_topk), the hot path of get_model_recommendations.
"""
from __future__ import annotations

from typing import Optional, Tuple

import torch

from divrec import ops

from .base_models import RankingModel


class _GatherDot(torch.autograd.Function):
    @staticmethod
    def forward(ctx, user_table, item_table, user_id, item_id):
        ctx.save_for_backward(user_table, item_table, user_id, item_id)
        return ops.gather_dot(user_table, item_table, user_id, item_id)

    @staticmethod
    def backward(ctx, grad_out):
        user_table, item_table, user_id, item_id = ctx.saved_tensors
        gu = torch.zeros_like(user_table) if ctx.needs_input_grad[0] else None
        gi = torch.zeros_like(item_table) if ctx.needs_input_grad[1] else None
        ops.gather_dot_backward(user_table, item_table, user_id, item_id, grad_out, gu, gi)
        return gu, gi, None, None


def _on_device(model_device: torch.device, ids: torch.Tensor) -> torch.Tensor:
    ids = torch.as_tensor(ids)
    if ids.dtype != torch.int64:
        ids = ids.to(torch.int64)
    return ids.to(model_device, non_blocking=True)


class MatrixFactorization(RankingModel):
    def __init__(self, no_users: int, no_items: int, embedding_dim: int):
        torch.nn.Module.__init__(self)
        self.no_users = no_users
        self.no_items = no_items
        self.embedding_dim = embedding_dim
        self.user_embeddings = torch.nn.Embedding(no_users, embedding_dim)
        self.item_embeddings = torch.nn.Embedding(no_items, embedding_dim)
        self._bf16 = None  # (key, user_bf16, item_bf16) cache for score_topk

    def _device(self) -> torch.device:
        dev = self.user_embeddings.weight.device
        if dev.type != "cuda":
            raise RuntimeError(
                "MatrixFactorization runs on the divrec HIP backend: move the model to a "
                "ROCm device first (model.to('cuda')); there is no CPU path"
            )
        return dev

    def forward(
        self,
        user_id: torch.LongTensor,
        item_id: torch.LongTensor,
        user_features: Optional[torch.Tensor] = None,
        item_features: Optional[torch.Tensor] = None,
    ) -> torch.Tensor:
        dev = self._device()
        uid = _on_device(dev, user_id)
        iid = _on_device(dev, item_id)
        return _GatherDot.apply(self.user_embeddings.weight, self.item_embeddings.weight, uid, iid)

    def bf16_tables(self) -> Tuple[torch.Tensor, torch.Tensor]:
        """bf16 copies of both tables (re-made only when a parameter changed)."""
        self._device()
        U, I = self.user_embeddings.weight, self.item_embeddings.weight
        key = (U.data_ptr(), U._version, I.data_ptr(), I._version)
        if self._bf16 is None or self._bf16[0] != key:
            with torch.no_grad():
                self._bf16 = (key, U.detach().to(torch.bfloat16).contiguous(),
                              I.detach().to(torch.bfloat16).contiguous())
        return self._bf16[1], self._bf16[2]

    @torch.no_grad()
    def score_topk(
        self,
        k: int,
        user_ids: Optional[torch.Tensor] = None,
        exclude: Optional[Tuple[torch.Tensor, torch.Tensor]] = None,
    ) -> Tuple[torch.Tensor, torch.Tensor]:
        """Top-k items of each user (all users, or ``user_ids``) over the whole
        catalog: (items int64 [n, k], scores fp32 [n, k]) on the model's
        device, ordered by score desc then item id asc. ``exclude`` =
        (rowptr int64 [n+1], items int32) CSR of items never to return."""
        dev = self._device()
        U, I = self.bf16_tables()
        uids = None if user_ids is None else _on_device(dev, user_ids)
        ex = None
        if exclude is not None:
            ex = (exclude[0].to(dev, torch.int64), exclude[1].to(dev, torch.int32))
        scores, items = ops.score_topk(U, I, int(k), user_ids=uids, exclude=ex)
        return items.to(torch.int64), scores
