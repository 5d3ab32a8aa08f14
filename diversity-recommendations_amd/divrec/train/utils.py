"""Training / scoring loops (reference divrec/train/utils.py:10-216).

Same functions, arguments and return values as the reference. On the hot path:

* ``get_model_recommendations`` with a MatrixFactorization model runs ONE
  dr_score_topk over all users (fp32 MFMA scores by default, fused top-k,
  frozen items excluded through a CSR) instead of the reference's per-user
  loop of set differences, full-catalog forward and full argsort (:58-77).
  Ties are broken by item id ascending (the reference's argsort is unstable
  there, :73).
* ``pair_wise_train_loop`` with MatrixFactorization + LogSigmoidDifferenceLoss
  runs each batch as ONE dr_bpr_fwd_bwd (gather, loss, AUC flags and dense
  embedding gradients fused) followed by dr_adam_dense when the optimizer is a
  plain torch.optim.Adam (its state tensors are used and kept up to date, so
  the optimizer stays usable). Other combinations take the generic path: the
  model's HIP forward/backward under autograd and ``optimizer.step()``.
"""
from __future__ import annotations

from typing import List, Optional, Tuple

import torch

from torch.autograd.graph import increment_version

from divrec import _backend, ops
from divrec.datasets import PairWiseDataset, PointWiseDataset, RankingDataset
from divrec.losses import (
    LogSigmoidDifferenceLoss,
    PairWiseLoss,
    PointWiseLoss,
    RecommendationsAwareLoss,
)
from divrec.metrics import AUCScore
from divrec.metrics import _rank
from divrec.models import MatrixFactorization, RankingModel


def _model_device(model: torch.nn.Module) -> Optional[torch.device]:
    for p in model.parameters():
        return p.device
    return None


def _to(t, device):
    return t.to(device, non_blocking=True) if isinstance(t, torch.Tensor) and device else t


# --------------------------------------------------------------------------- scoring
def point_wise_score_loop(dataset: PointWiseDataset, model: RankingModel,
                          losses: List[PointWiseLoss], **loader_params):
    model.eval()
    dev = _model_device(model)
    values = {loss.__class__.__name__: [] for loss in losses}
    with torch.no_grad():
        for user_id, item_id, uf, itf, true_rel in dataset.loader(**loader_params):
            pred = model(user_id, item_id, uf, itf)
            for loss in losses:
                values[loss.__class__.__name__].append(loss.point_wise(_to(true_rel, pred.device), pred))
    return [loss.reduce_loss_values(torch.concatenate(values[loss.__class__.__name__]))
            for loss in losses]


def pair_wise_score_loop(dataset: PairWiseDataset, model: RankingModel,
                         losses: List[PairWiseLoss], **loader_params):
    model.eval()
    values = {loss.__class__.__name__: [] for loss in losses}
    with torch.no_grad():
        for user_id, pos, neg, uf, pf, nf in dataset.loader(**loader_params):
            positives = model(user_id, pos, uf, pf)
            negatives = model(user_id, neg, uf, nf)
            for loss in losses:
                values[loss.__class__.__name__].append(loss.pair_wise(positives, negatives))
    return [loss.reduce_loss_values(torch.concatenate(values[loss.__class__.__name__]))
            for loss in losses]


def _mf_scoring(model: RankingModel) -> bool:
    """The MF fast path applies only to MatrixFactorization's own forward: a
    subclass that overrides forward is scored through its forward."""
    return (isinstance(model, MatrixFactorization)
            and type(model).forward is MatrixFactorization.forward)


def _list_length(dataset: RankingDataset, excl, n_users: int, n_items: int, k: int) -> int:
    """Length of the reference's recommendation lists: min(k, candidates),
    where the candidates of a user are the catalog minus its frozen items.
    Lists of different lengths make the reference's torch.LongTensor(...)
    raise (utils.py:77); so does this."""
    if excl is None:
        return min(k, n_items)
    rowptr, cols = excl
    inside = (cols.to(torch.int64) < n_items).to(torch.int64)
    csum = torch.zeros(cols.numel() + 1, dtype=torch.int64)
    csum[1:] = torch.cumsum(inside, 0)
    n_cands = n_items - (csum[rowptr[1:]] - csum[rowptr[:-1]])
    lengths = torch.clamp(n_cands, max=k)
    lo, hi = int(lengths.min()), int(lengths.max())
    if lo != hi:
        raise ValueError(f"expected sequence of length {hi} at dim 1 (got {lo}): a user has "
                         f"fewer than {k} candidates, so the recommendation lists are ragged")
    return lo


MAX_SCAN_K = 1024  # dr_score_topk's largest k (include/divrec_hip.h)


def get_model_recommendations(dataset: RankingDataset, model: RankingModel,
                              number_of_recommendations: int) -> torch.LongTensor:
    """Top-``number_of_recommendations`` candidates of every user of
    ``dataset`` (LongTensor [U, k] on the CPU, like the reference), scored in
    fp32 (MatrixFactorization.score_topk's faithful mode)."""
    k = int(number_of_recommendations)
    n_users = int(dataset.data.number_of_users)
    n_items = int(dataset.data.number_of_items)
    if _mf_scoring(model) and n_users <= model.no_users and n_items <= model.no_items:
        if n_users == 0:
            return torch.LongTensor([])
        excl = dataset.exclusion_csr()
        k_len = _list_length(dataset, excl, n_users, n_items, k)
        if k_len == 0:
            return torch.zeros((n_users, 0), dtype=torch.int64)
        if k_len <= MAX_SCAN_K:
            user_ids = None if n_users == model.no_users else torch.arange(n_users)
            items, _ = model.score_topk(k_len, user_ids=user_ids, exclude=excl, n_items=n_items)
            return items.cpu()
        # lists longer than the scan's top-k bound: the loop below (the model's
        # HIP forward per user, full sort), as the reference returns any length
    # Generic RankingModel: the reference loop (model scores per user), with
    # the deterministic tie-break. Outside the MF hot path.
    recs = []
    with torch.no_grad():
        for rep_user, _, cands, uf, itf in dataset:
            scores = model(rep_user, cands, uf, itf).to("cpu")
            order = torch.sort(scores, descending=True, stable=True).indices
            recs.append(cands[order][:k].tolist())
    return torch.LongTensor(recs)


def recommendations_score_loop(dataset: RankingDataset, model: RankingModel,
                               losses: List[RecommendationsAwareLoss],
                               number_of_recommendations: int):
    model.eval()
    interactions = dataset.data.interactions
    recommendations = get_model_recommendations(dataset, model, number_of_recommendations)
    # P@k / R@k / MAP@k / NDCG@k of one (interactions, recommendations) pair
    # come from one dr_rank_metrics launch
    with _rank.shared_rank_metrics():
        return [loss(interactions, recommendations) for loss in losses]


# --------------------------------------------------------------------------- training
def point_wise_train_loop(dataset: PointWiseDataset, model: RankingModel, loss: PointWiseLoss,
                          optimizer: torch.optim.Optimizer,
                          scores: Optional[List[PointWiseLoss]] = None,
                          **loader_params) -> Tuple[float, List[float]]:
    assert scores is None or all(score.reduce for score in scores)
    model.train()
    batch_count, mean_loss = 0, 0.0
    mean_scores = [0.0] * (len(scores) if scores is not None else 0)
    for user_id, item_id, uf, itf, true_rel in dataset.loader(**loader_params):
        pred = model(user_id, item_id, uf, itf)
        true_rel = _to(true_rel, pred.device)
        loss_value = loss(true_rel, pred)
        loss_value.backward()
        optimizer.step()
        optimizer.zero_grad()
        batch_count += 1
        mean_loss += loss_value.item()
        if scores is not None:
            for i, score in enumerate(scores):
                mean_scores[i] += score(true_rel, pred).item()
    return mean_loss / batch_count, [s / batch_count for s in mean_scores]


def _plain_adam(optimizer: torch.optim.Optimizer) -> bool:
    if type(optimizer) is not torch.optim.Adam:
        return False
    for g in optimizer.param_groups:
        if g.get("amsgrad") or g.get("maximize") or g.get("capturable") or g.get("differentiable"):
            return False
        if g.get("decoupled_weight_decay", False):
            return False
    return True


def fused_adam_step(optimizer: torch.optim.Adam) -> None:
    """optimizer.step() of a plain torch.optim.Adam done by dr_adam_dense, on
    the optimizer's own state (step / exp_avg / exp_avg_sq), so torch's
    optimizer remains consistent and resumable."""
    for group in optimizer.param_groups:
        beta1, beta2 = group["betas"]
        for p in group["params"]:
            if p.grad is None:
                continue
            st = optimizer.state[p]
            if len(st) == 0:
                st["step"] = torch.tensor(0.0, dtype=torch.float32)
                st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
            st["step"] += 1
            ops.adam_dense(p.data, p.grad, st["exp_avg"], st["exp_avg_sq"], group["lr"], beta1,
                           beta2, group["eps"], group["weight_decay"], int(st["step"].item()))
            # the kernel wrote p through a raw pointer: bump its autograd
            # version, as a torch in-place update would
            increment_version(p)


def _plain_sparse_adam(optimizer: torch.optim.Optimizer) -> bool:
    return type(optimizer) is torch.optim.SparseAdam and not any(
        g.get("maximize") for g in optimizer.param_groups)


def lazy_adam_step(optimizer: torch.optim.SparseAdam, rows: dict) -> None:
    """optimizer.step() of torch.optim.SparseAdam done by dr_adam_rows on the
    optimizer's own state: for each parameter p, ``rows[p]`` holds the unique
    rows the batch touched (the indices a sparse embedding gradient would
    carry). The reference's embeddings are dense (sparse=False), so plain
    torch cannot run SparseAdam on them; this is the opt-in row-sparse
    ("lazy") alternative to dense Adam. The touched
    gradient rows are zeroed, so the dense gradient tables stay allocated and
    all-zero between batches (no full memset, no re-allocation)."""
    for group in optimizer.param_groups:
        beta1, beta2 = group["betas"]
        for p in group["params"]:
            if p.grad is None or p not in rows:
                continue
            st = optimizer.state[p]
            if len(st) == 0:
                st["step"] = 0
                st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
            st["step"] += 1
            ops.adam_rows(p.data, p.grad, st["exp_avg"], st["exp_avg_sq"], rows[p],
                          group["lr"], beta1, beta2, group["eps"], st["step"])
            increment_version(p)  # raw-pointer update, as in fused_adam_step


def _bpr_fast_path(model, loss, scores) -> bool:
    return (isinstance(model, MatrixFactorization) and type(loss) is LogSigmoidDifferenceLoss
            and (scores is None or all(type(s) is AUCScore for s in scores)))


def pair_wise_train_loop(dataset: PairWiseDataset, model: RankingModel, loss: PairWiseLoss,
                         optimizer: torch.optim.Optimizer,
                         scores: Optional[List[PairWiseLoss]] = None,
                         **loader_params) -> Tuple[float, List[float]]:
    """One epoch of pairwise training; returns (mean batch loss, [mean score])."""
    assert scores is None or all(score.reduce for score in scores)
    model.train()
    n_scores = len(scores) if scores is not None else 0
    batch_losses, batch_scores = [], []
    fused = _bpr_fast_path(model, loss, scores)
    adam = _plain_adam(optimizer)
    lazy = fused and _plain_sparse_adam(optimizer)
    epoch_err = None  # id range errors of the fused kernel on device batches
    for user_id, pos, neg, uf, pf, nf in dataset.loader(**loader_params):
        if fused:
            dev = model._device()
            U, I = model.user_embeddings.weight, model.item_embeddings.weight
            host = user_id.device.type == "cpu"
            if host:  # host batches: raise before any compute
                _backend.host_ids_in_range(user_id, U.size(0), "user_id")
                _backend.host_ids_in_range(pos, I.size(0), "positive item_id")
                _backend.host_ids_in_range(neg, I.size(0), "negative item_id")
            uid, pid, nid = (t.to(dev, torch.int64, non_blocking=True) for t in (user_id, pos, neg))
            if not host and uid.numel():
                # device batches: one min/max reduction read back (one sync)
                # BEFORE the kernel, so a bad batch raises IndexError with the
                # weights, the optimizer state and the gradient tables as they
                # were (the reference's nn.Embedding fails before any backward;
                # the lazy path's all-zero gradient invariant holds)
                mm = torch.stack([uid.min(), uid.max(), torch.minimum(pid.min(), nid.min()),
                                  torch.maximum(pid.max(), nid.max())]).cpu().tolist()
                if mm[0] < 0 or mm[1] >= U.size(0):
                    raise IndexError("index out of range in self (user_id)")
                if mm[2] < 0 or mm[3] >= I.size(0):
                    raise IndexError("index out of range in self (item_id)")
            if U.grad is None:
                U.grad = torch.zeros_like(U)
            if I.grad is None:
                I.grad = torch.zeros_like(I)
            if epoch_err is None:
                epoch_err = _backend.error_counter(dev)
            B = uid.numel()
            losses_b, hits = ops.bpr_fwd_bwd(U.data, I.data, uid, pid, nid, 1.0 / B, U.grad, I.grad,
                                             err=epoch_err, check=False)
            loss_value = torch.sum(losses_b, dim=0) / B
            if lazy:  # touched rows only; the kernel zeroes those gradient rows
                lazy_adam_step(optimizer, {U: torch.unique(uid),
                                           I: torch.unique(torch.cat([pid, nid]))})
            elif adam:
                fused_adam_step(optimizer)
                optimizer.zero_grad()
            else:
                optimizer.step()
                optimizer.zero_grad()
            batch_losses.append(loss_value.detach())
            if n_scores:  # AUCScore.pair_wise = the hit flags, reduced as each score says
                batch_scores.append(torch.stack(
                    [s.reduce_loss_values(hits).double() for s in scores]))
        else:
            positives = model(user_id, pos, uf, pf)
            negatives = model(user_id, neg, uf, nf)
            loss_value = loss(positives, negatives)
            loss_value.backward()
            optimizer.step()
            optimizer.zero_grad()
            batch_losses.append(loss_value.detach())
            if n_scores:
                batch_scores.append(torch.stack(
                    [s(positives.detach(), negatives.detach()).double() for s in scores]))
    _backend.raise_if_out_of_range(epoch_err, "pair_wise_train_loop")
    count = len(batch_losses)
    # per-batch values summed as Python floats in batch order, like the reference
    mean_loss = sum(float(v) for v in torch.stack(batch_losses).double().cpu().tolist()) / count
    means = [0.0] * n_scores
    if n_scores:
        rows = torch.stack(batch_scores).double().cpu().tolist()
        means = [sum(r[i] for r in rows) / count for i in range(n_scores)]
    return mean_loss, means


def recommendations_train_loop(dataset: RankingDataset, model: RankingModel,
                               loss: RecommendationsAwareLoss, number_of_recommendations: int,
                               optimizer: torch.optim.Optimizer,
                               scores: Optional[List[RecommendationsAwareLoss]] = None
                               ) -> Tuple[float, List[float]]:
    """The reference's listwise loop (:167-216), kept for API completeness: it
    ranks ASCENDING and back-propagates through integer recommendations, so
    with the shipped losses it fails at backward() exactly as the reference."""
    assert scores is None or all(score.reduce for score in scores)
    model.train()
    batch_count, mean_loss = 0, 0.0
    mean_scores = [0.0] * (len(scores) if scores is not None else 0)
    for rep_user, _, cands, uf, itf in dataset:
        model_scores = model(rep_user, cands, uf, itf)
        inter = dataset.data.interactions
        interactions = inter[inter[:, 0] == rep_user[0]]
        recommendations = cands[torch.argsort(model_scores.cpu())][:number_of_recommendations]
        loss_value = loss(interactions, recommendations)
        loss_value.backward()
        optimizer.step()
        optimizer.zero_grad()
        batch_count += 1
        mean_loss += loss_value.item()
        if scores is not None:
            for i, score in enumerate(scores):
                mean_scores[i] += score(interactions, recommendations).item()
    return mean_loss / batch_count, [s / batch_count for s in mean_scores]
