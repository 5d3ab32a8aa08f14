"""MatrixFactorization on the HIP path (reference divrec/models/matrix_factorization.py:8-28).

Same constructor, attributes and state-dict keys (``user_embeddings.weight``,
``item_embeddings.weight``: fp32 nn.Embedding, N(0,1) init, dense gradients),
so reference checkpoints load unchanged. ``forward`` is the fused embedding
gather + row dot of libdivrec_hip (dr_gather_dot) with its backward
(dr_gather_dot_backward) into dense fp32 gradients; parameters must live on a
ROCm device (``model.to("cuda")``) — there is no CPU path.

New, non-breaking: ``score_topk`` — full-catalog MFMA scoring with a fused
top-k (dr_score_topk), the hot path of get_model_recommendations. Two
precisions:
  * ``"fp32"`` (default): the fp32 parameters themselves, scored on
    v_mfma_f32_32x32x2_f32 — each score an exact fp32 fmaf chain, i.e. the
    reference's fp32 arithmetic (matrix_factorization.py:26-28) up to the
    summation order;
  * ``"bf16"``: bf16 copies of the tables on the bf16 MFMA (16x the rate),
    ranking the tables' bf16 rounding — the explicit fast mode.
Any ``embedding_dim`` works: widths without a scan instance (e.g. the
reference experiments' 100) are zero-padded per call (a copy of O((U + I) d)
bytes, small beside the O(U I d) scan; no cache, so writes through ``.data``
or raw pointers, which bump no autograd version, are always seen).
"""
from __future__ import annotations

from typing import Optional, Tuple

import torch

from divrec import ops

from .base_models import RankingModel

PRECISIONS = {"fp32": torch.float32, "bf16": torch.bfloat16}


class _GatherDot(torch.autograd.Function):
    @staticmethod
    def forward(ctx, user_table, item_table, user_id, item_id, checked):
        ctx.save_for_backward(user_table, item_table, user_id, item_id)
        # ids validated on the host need no device read-back of the counter
        return ops.gather_dot(user_table, item_table, user_id, item_id, check=not checked)

    @staticmethod
    def backward(ctx, grad_out):
        user_table, item_table, user_id, item_id = ctx.saved_tensors
        gu = torch.zeros_like(user_table) if ctx.needs_input_grad[0] else None
        gi = torch.zeros_like(item_table) if ctx.needs_input_grad[1] else None
        ops.gather_dot_backward(user_table, item_table, user_id, item_id, grad_out, gu, gi)
        return gu, gi, None, None, None


def _on_device(model_device: torch.device, ids: torch.Tensor) -> torch.Tensor:
    ids = torch.as_tensor(ids)
    if ids.dtype != torch.int64:
        ids = ids.to(torch.int64)
    return ids.to(model_device, non_blocking=True)


def _ids_for(model_device: torch.device, ids, n_rows: int, what: str):
    """(device ids, validated on the host?): host ids are range-checked before
    the upload (IndexError, as nn.Embedding raises), device ids in the kernel."""
    ids = torch.as_tensor(ids)
    host = ids.device.type == "cpu"
    if host:
        from divrec import _backend
        _backend.host_ids_in_range(ids, n_rows, what)
    return _on_device(model_device, ids), host


class MatrixFactorization(RankingModel):
    def __init__(self, no_users: int, no_items: int, embedding_dim: int):
        torch.nn.Module.__init__(self)
        self.no_users = no_users
        self.no_items = no_items
        self.embedding_dim = embedding_dim
        self.user_embeddings = torch.nn.Embedding(no_users, embedding_dim)
        self.item_embeddings = torch.nn.Embedding(no_items, embedding_dim)

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
        uid, hu = _ids_for(dev, user_id, self.user_embeddings.num_embeddings, "user_id")
        iid, hi = _ids_for(dev, item_id, self.item_embeddings.num_embeddings, "item_id")
        return _GatherDot.apply(self.user_embeddings.weight, self.item_embeddings.weight, uid, iid,
                                hu and hi)

    def scoring_tables(self, precision: str = "fp32") -> Tuple[torch.Tensor, torch.Tensor]:
        """The (user, item) tables score_topk scans at ``precision``: the
        parameters themselves when their dtype and width already have a scan
        instance, else a converted / zero-padded copy made by this call (never
        cached: an update through ``weight.data`` or a raw-pointer optimizer
        bumps no version a cache could key on)."""
        if precision not in PRECISIONS:
            raise ValueError(f"precision must be one of {sorted(PRECISIONS)}")
        self._device()
        U, I = self.user_embeddings.weight, self.item_embeddings.weight
        dt = PRECISIONS[precision]
        w = ops.score_width(dt, U.size(1))
        if dt == U.dtype and w == U.size(1) and U.is_contiguous() and I.is_contiguous():
            return U.detach(), I.detach()
        with torch.no_grad():
            return (ops.pad_columns(U.detach().to(dt).contiguous(), w),
                    ops.pad_columns(I.detach().to(dt).contiguous(), w))

    def bf16_tables(self) -> Tuple[torch.Tensor, torch.Tensor]:
        """bf16 copies of both tables (the fast scoring mode's operands)."""
        return self.scoring_tables("bf16")

    @torch.no_grad()
    def score_topk(
        self,
        k: int,
        user_ids: Optional[torch.Tensor] = None,
        exclude: Optional[Tuple[torch.Tensor, torch.Tensor]] = None,
        precision: str = "fp32",
        n_items: Optional[int] = None,
    ) -> Tuple[torch.Tensor, torch.Tensor]:
        """Top-k items of each user (all users, or ``user_ids``) over the
        catalog (the first ``n_items`` item rows; default all): (items int64
        [n, k], scores fp32 [n, k]) on the model's device, ordered by score
        desc then item id asc. ``exclude`` = (rowptr int64 [n+1], items int32)
        CSR of items never to return. ``precision`` "fp32" (default, the
        reference's arithmetic) or "bf16" (fast mode)."""
        dev = self._device()
        U, I = self.scoring_tables(precision)
        if n_items is not None:
            I = I[: int(n_items)]
        uids = None if user_ids is None else _on_device(dev, user_ids)
        ex = None
        if exclude is not None:
            ex = (exclude[0].to(dev, torch.int64), exclude[1].to(dev, torch.int32))
        scores, items = ops.score_topk(U, I, int(k), user_ids=uids, exclude=ex)
        return items.to(torch.int64), scores
