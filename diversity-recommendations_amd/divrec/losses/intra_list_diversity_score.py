"""Intra-list diversity on the HIP path
(reference divrec/losses/intra_list_diversity_score.py:8-63).

``IntraListDiversityScore(distance_matrix=D)`` with D one of
  * a dense [I, I] tensor (float32/float64/int32/int64) — dr_ild_dense, which
    accumulates fp32 D in itertools.combinations order exactly like the
    reference's Python sum (bit-identical values);
  * ``EmbeddingDistance(item_table, kind)`` — D computed on the fly from item
    embeddings ('cosine', 'dot', 'euclidean'; dr_ild_embedding, bf16 MFMA Gram
    tiles) for catalogs where an I x I matrix cannot exist;
  * ``LabelEquality(labels)`` — D[i,j] = (labels[i] == labels[j]) on the fly
    (dr_ild_labels), what IntraListBinaryUnfairnessScore builds densely.

Values are (sum over pairs p < q of D[r_p, r_q]) / (k (k - 1)) per user, on
the recommendations' device. Divergence: ``forward`` reduces
once; the reference reduces twice and raises IndexError for 'mean'
(:34 + base_losses.py:76); 'sum' and 'none' agree.
"""
from __future__ import annotations

from typing import Optional, Union

import torch

from divrec import _backend, ops

from .base_losses import DatasetAwareLoss, RecommendationsAwareLoss


class EmbeddingDistance:
    """Lazy D from item embeddings (computed per pair inside the kernel).

    The kernel reads a bf16 table; a float table is rounded to bf16, and a
    width without a kernel instance (e.g. the reference experiments' 100) is
    zero-padded. That device copy is kept between calls and rebuilt whenever
    the source table changes in a way torch records: another tensor assigned
    to ``item_table``, a new storage (data_ptr), shape or device, or an
    in-place update through autograd-visible ops (its ``_version``, e.g. an
    optimizer step). Writes torch cannot see (``.data`` views of another
    tensor, raw pointers, a kernel writing the storage) need ``refresh()``."""

    KINDS = ("cosine", "dot", "euclidean")

    def __init__(self, item_table: torch.Tensor, kind: str = "cosine"):
        if kind not in self.KINDS:
            raise ValueError(f"kind must be one of {self.KINDS}")
        self.kind = kind
        self.item_table = item_table
        self._dev_table = None
        self._key = None

    def refresh(self) -> None:
        """Drop the device copy: the next call rebuilds it from item_table."""
        self._dev_table = None
        self._key = None

    def _source_key(self, device: torch.device):
        t = self.item_table
        return (str(device), t.data_ptr(), tuple(t.shape), t.dtype, t.device, t._version)

    def table(self, device: torch.device) -> torch.Tensor:
        key = self._source_key(device)
        if self._dev_table is None or key != self._key:
            t = self.item_table.detach().to(device=device, dtype=torch.bfloat16).contiguous()
            # widths without a kernel instance: zero columns change no distance
            t = ops.pad_columns(t, ops._width_of(ops.ILD_WIDTHS, t.size(1), "embedding ILD"))
            self._dev_table, self._key = t, key
        return self._dev_table


class LabelEquality:
    """Lazy D[i, j] = (labels[i] == labels[j])."""

    def __init__(self, labels: torch.Tensor):
        self.labels = labels
        self._dev = None

    def device_labels(self, device: torch.device) -> torch.Tensor:
        if self._dev is None or self._dev.device != device:
            self._dev = self.labels.to(device=device, dtype=torch.int64).contiguous()
        return self._dev


DistanceLike = Union[torch.Tensor, EmbeddingDistance, LabelEquality]


class IntraListDiversityScore(RecommendationsAwareLoss):
    """Diversity metric of Wasilewski & Hurley, "Incorporating Diversity in a
    Learning to Rank Recommender System"."""

    def __init__(self, *args, distance_matrix: DistanceLike, **kwargs):
        RecommendationsAwareLoss.__init__(self, *args, **kwargs)
        self.distance_matrix = distance_matrix
        self._dense_dev = None

    def _dense_on(self, device: torch.device) -> torch.Tensor:
        D = self.distance_matrix
        if D.device == device:
            return D
        if self._dense_dev is None or self._dense_dev.device != device:
            self._dense_dev = D.to(device).contiguous()
        return self._dense_dev

    def per_user(self, recommendations: torch.Tensor) -> torch.Tensor:
        """ILD per user on the device (no reduction)."""
        dev = recommendations.device if recommendations.is_cuda else _backend.default_device()
        recs = recommendations.to(dev)
        D = self.distance_matrix
        if isinstance(D, EmbeddingDistance):
            return ops.ild_embedding(recs, D.table(dev), D.kind)
        if isinstance(D, LabelEquality):
            return ops.ild_labels(recs, D.device_labels(dev))
        return ops.ild_dense(recs, self._dense_on(dev))

    def recommendations_loss(
        self, interactions: torch.LongTensor, recommendations: torch.LongTensor
    ) -> torch.Tensor:
        values = self.per_user(recommendations).to(recommendations.device)
        return self.reduce_loss_values(values)

    def forward(self, interactions: torch.LongTensor, recommendations: torch.LongTensor):
        return self.recommendations_loss(interactions, recommendations)

    @staticmethod
    def user_ild(user_recommendations: torch.Tensor, distance_matrix: torch.Tensor):
        """Un-normalised pair sum of one list (reference :36-42): Python's
        sum over itertools.combinations of 0-d tensors of D's dtype, i.e. a
        0-d tensor of that dtype accumulated in order (int 0 for fewer than
        two items). Computed by dr_ild_dense_pair_sum in D's own precision, so
        a float D's value is bit-identical; an integer D is summed exactly in
        int64 and stored through a double, so it is exact while |sum| < 2^53
        and, for int32 D, while the sum fits int32 (the reference's int32 sum
        would wrap there; label matrices of 0/1 never come near either bound).
        Returned on D's device."""
        recs = user_recommendations.reshape(1, -1)
        if recs.size(1) < 2:
            return 0  # sum() of no pairs
        dev = _backend.default_device()
        val = ops.ild_dense_pair_sum(recs.to(dev), distance_matrix.to(dev))
        return val[0].to(distance_matrix.dtype).to(distance_matrix.device)


class IntraListBinaryUnfairnessScore(IntraListDiversityScore, DatasetAwareLoss):
    """ILD with the item-partition equality matrix (Abdollahpouri, Burke et al.,
    "Controlling Popularity Bias in Learning to Rank Recommendation"), computed
    on the fly from the labels instead of an I x I matrix."""

    def __init__(self, *args, items_partition_feature: str = "partition", **kwargs):
        DatasetAwareLoss.__init__(self, *args, **kwargs)
        self.items_partition_feature = items_partition_feature
        assert items_partition_feature in self.dataset.item_features
        labels = self.dataset.item_features[items_partition_feature]
        IntraListDiversityScore.__init__(self, *args, distance_matrix=LabelEquality(labels),
                                         **kwargs)

    def get_distance_matrix(self) -> torch.Tensor:
        """The dense int matrix the reference builds (:60-63); not used here."""
        labels = self.dataset.item_features[self.items_partition_feature]
        return (labels.unsqueeze(0) == labels.unsqueeze(1)).int()
