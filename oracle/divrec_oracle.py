"""CPU restatement of the reference hot path (TEST INFRASTRUCTURE ONLY).

See oracle/__init__.py for the import rule. Reference paths are relative to
the reference tree (amtsyplov/diversity-recommendations).
"""
from __future__ import annotations

import math
from itertools import combinations
from typing import List, Optional, Sequence, Tuple

import numpy as np

__all__ = [
    "as_bf16_f32",
    "mf_forward",
    "candidates_for_user",
    "recommend_topk",
    "reference_loop_topk",
    "reference_mf_forward",
    "reference_bpr_steps",
    "mmr_greedy_torch",
    "topk_order",
    "topk_merge",
    "ild_sequential",
    "ild_pair_sums",
    "ild_labels",
    "ild_embedding_f64",
    "embedding_distance_matrix",
    "reduce_values",
    "bpr_forward_backward",
    "sparse_adam_rows",
    "adam_step",
    "mmr_greedy",
    "mmr_check",
    "exclusion_csr",
]


def as_bf16_f32(x: np.ndarray) -> np.ndarray:
    """Round fp32 to bf16 (round-to-nearest-even) and widen back to fp32 —
    the values the bf16 MFMA path sees (the oracle runs on the
    bf16-quantised weights)."""
    u = np.ascontiguousarray(x, dtype=np.float32).view(np.uint32).astype(np.uint64)
    r = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16) << 16
    return r.astype(np.uint32).view(np.float32)


def mf_forward(U: np.ndarray, I: np.ndarray, uid: np.ndarray, iid: np.ndarray) -> np.ndarray:
    """MatrixFactorization.forward (divrec/models/matrix_factorization.py:26-28):
    gather both rows, multiply elementwise in fp32, sum over d."""
    u = U[uid].astype(np.float32)
    i = I[iid].astype(np.float32)
    return np.sum(u * i, axis=1, dtype=np.float32)


def candidates_for_user(n_items: int, frozen: Optional[Sequence[int]]) -> np.ndarray:
    """RankingDataset.__iter__ candidates (divrec/datasets/base_datasets.py:143-151):
    list(frozenset(range(I)) - frozen) — ascending item ids (CPython int-set
    order); all items when frozen is None."""
    if frozen is None or len(frozen) == 0:
        return np.arange(n_items, dtype=np.int64)
    mask = np.ones(n_items, dtype=bool)
    mask[np.asarray(list(frozen), dtype=np.int64)] = False
    return np.nonzero(mask)[0].astype(np.int64)


def topk_order(scores: np.ndarray, k: int) -> np.ndarray:
    """Positions of the top-k scores with the build's deterministic tie-break:
    score descending, then position (= item id, candidates are ascending)
    ascending. Equals torch.sort(stable=True, descending=True); on tie-free
    input it equals the reference's argsort (divrec/train/utils.py:73)."""
    s = scores.astype(np.float32)
    order = np.argsort(-s, kind="stable")
    return order[:k]


def recommend_topk(
    U: np.ndarray,
    I: np.ndarray,
    k: int,
    users: Optional[Sequence[int]] = None,
    frozen: Optional[List[Sequence[int]]] = None,
    return_scores: bool = False,
    block: int = 1 << 18,
):
    """get_model_recommendations (divrec/train/utils.py:53-77) with
    MatrixFactorization scores: per user, score every candidate with
    sum(u * i) in fp32 (products rounded to fp32, summed over d) and keep
    candidates[order][:k]. Candidates are scored in blocks of ``block`` rows
    only to bound memory; the arithmetic per (user, item) is unchanged."""
    users = range(U.shape[0]) if users is None else users
    recs, scs = [], []
    I32 = I if I.dtype == np.float32 else I.astype(np.float32)
    for n, u in enumerate(users):
        fz = None if frozen is None else frozen[n]
        cands = candidates_for_user(I.shape[0], fz)
        dense = fz is None or len(fz) == 0  # candidates are arange(I): slice, don't gather
        uu = U[u].astype(np.float32)[None, :]
        s = np.empty(len(cands), dtype=np.float32)
        for b0 in range(0, len(cands), block):
            c = cands[b0 : b0 + block]
            rows = I32[b0 : b0 + len(c)] if dense else I32[c]
            s[b0 : b0 + len(c)] = np.sum(uu * rows, axis=1, dtype=np.float32)
        o = topk_order(s, k)
        recs.append(cands[o])
        scs.append(s[o])
    recs = np.stack(recs).astype(np.int64) if recs else np.zeros((0, k), np.int64)
    if return_scores:
        return recs, np.stack(scs).astype(np.float32) if scs else np.zeros((0, k), np.float32)
    return recs


def reference_loop_topk(U, I, k: int, users: Sequence[int], frozen=None):
    """get_model_recommendations (divrec/train/utils.py:53-77) over
    RankingDataset (divrec/datasets/base_datasets.py:136-171), restated op for
    op in torch for the CPU baseline (bench.py): per user the frozenset
    difference of the catalog, torch.LongTensor of the candidate list,
    torch.full of the user id, MatrixFactorization.forward (embedding gathers
    + sum(u * i, dim=1), matrix_factorization.py:26-28), argsort descending and
    the first k ids as a list. U, I: fp32 torch tables. Intra-op parallel on
    torch's threads like the reference. Returns LongTensor [len(users), k]."""
    import torch

    items = frozenset(range(I.shape[0]))
    recs = []
    with torch.no_grad():
        for n, u in enumerate(users):
            fz = frozenset() if frozen is None else frozenset(frozen[n])
            negatives = torch.LongTensor(list(items - fz))
            rep = torch.full((len(negatives),), int(u))
            scores = torch.sum(torch.nn.functional.embedding(rep, U) *
                               torch.nn.functional.embedding(negatives, I), dim=1)
            recs.append(negatives[torch.argsort(scores, descending=True)][:k].tolist())
    return torch.LongTensor(recs)


def reference_mf_forward(U, I, uid, iid):
    """MatrixFactorization.forward (divrec/models/matrix_factorization.py:26-28)
    restated in torch for the CPU baseline: two embedding gathers and
    torch.sum(u * i, dim=1), intra-op parallel on torch's threads like the
    reference. U, I fp32 torch tables; uid, iid LongTensors."""
    import torch

    with torch.no_grad():
        return torch.sum(torch.nn.functional.embedding(uid, U) *
                         torch.nn.functional.embedding(iid, I), dim=1)


def reference_bpr_steps(U, I, batches, lr=1e-3):
    """pair_wise_train_loop (divrec/train/utils.py:130-164) restated in torch
    for the CPU baseline: per batch (u, p, n) the reference's two
    MatrixFactorization forwards, LogSigmoidDifferenceLoss
    (-logsigmoid(pos - neg), mean; log_sigmoid_difference_loss.py:11-14),
    backward through dense nn.Embedding gradients and torch.optim.Adam.step
    + zero_grad over both tables. U, I: fp32 torch tables (trained on
    copies). Returns (per-batch losses, final U, final I)."""
    import torch

    ue = torch.nn.Embedding.from_pretrained(U.clone(), freeze=False)
    ie = torch.nn.Embedding.from_pretrained(I.clone(), freeze=False)
    opt = torch.optim.Adam(list(ue.parameters()) + list(ie.parameters()), lr=lr)
    losses = []
    for uid, pid, nid in batches:
        pos = torch.sum(ue(uid) * ie(pid), dim=1)
        neg = torch.sum(ue(uid) * ie(nid), dim=1)
        per = -torch.nn.functional.logsigmoid(pos - neg)
        loss = torch.sum(per, 0) / per.size(0)  # ScoreWithReduction 'mean' (base_losses.py:22-27)
        loss.backward()
        opt.step()
        opt.zero_grad()
        losses.append(float(loss.detach()))
    return losses, ue.weight.detach(), ie.weight.detach()


def mmr_greedy_torch(cand_items, cand_scores, E, k_out, lam):
    """The build's MMR spec (mmr_greedy) restated as the eager per-user greedy
    in torch fp32 for the CPU baseline: per user the C x C cosine matrix of
    the candidates (one GEMM), then k_out argmax rounds over
    lam * s - (1 - lam) * max_picked cos. cand_items int [n, C], cand_scores
    fp32 [n, C], E fp32 torch table. Returns LongTensor [n, k_out]."""
    import torch

    out = []
    with torch.no_grad():
        for u in range(cand_items.shape[0]):
            X = E[cand_items[u].long()]
            Xn = X / X.norm(dim=1, keepdim=True)
            S = Xn @ Xn.T
            s = cand_scores[u]
            pen = torch.zeros_like(s)
            alive = torch.ones_like(s, dtype=torch.bool)
            picks = []
            for t in range(k_out):
                val = lam * s - (1 - lam) * pen if t else lam * s
                val = torch.where(alive, val, torch.full_like(val, -float("inf")))
                j = int(torch.argmax(val))
                picks.append(int(cand_items[u, j]))
                alive[j] = False
                pen = S[:, j] if t == 0 else torch.maximum(pen, S[:, j])
            out.append(picks)
    return torch.LongTensor(out)


def topk_merge(scores: np.ndarray, items: np.ndarray, k: int) -> Tuple[np.ndarray, np.ndarray]:
    """Merge per-part top-k lists [P, n, k_in] under (score desc, item asc)."""
    P, n, kin = scores.shape
    out_s = np.empty((n, k), np.float32)
    out_i = np.empty((n, k), np.int64)
    for u in range(n):
        s = scores[:, u, :].reshape(-1)
        it = items[:, u, :].reshape(-1).astype(np.int64)
        keep = it >= 0
        s, it = s[keep], it[keep]
        o = np.lexsort((it, -s.astype(np.float64)))[:k]
        out_s[u, : len(o)] = s[o]
        out_i[u, : len(o)] = it[o]
        out_s[u, len(o):] = -np.inf
        out_i[u, len(o):] = -1
    return out_s, out_i


def ild_pair_sums(recs: np.ndarray, D: np.ndarray) -> np.ndarray:
    """IntraListDiversityScore.user_ild per list
    (divrec/losses/intra_list_diversity_score.py:36-42): Python sum over
    itertools.combinations of positions, accumulated in D's dtype (fp32 for
    fp32 D, exact for integer D); 0 for fewer than two items. float64 [n]."""
    n, k = recs.shape
    out = np.empty(n, dtype=np.float64)
    is_int = np.issubdtype(D.dtype, np.integer)
    for u in range(n):
        acc = 0
        row = recs[u]
        for i, j in combinations(range(k), 2):
            v = D[row[i], row[j]]
            acc = acc + (int(v) if is_int else v)  # 0 + v == v exactly, then D-dtype adds
        out[u] = acc
    return out


def ild_sequential(recs: np.ndarray, D: np.ndarray) -> np.ndarray:
    """IntraListDiversityScore.recommendations_loss, reduction 'none'
    (divrec/losses/intra_list_diversity_score.py:20-34): the user_ild pair
    sums (ild_pair_sums) converted to fp32 by torch.Tensor, divided by
    k*(k-1) in fp32."""
    k = recs.shape[1]
    out = ild_pair_sums(recs, D).astype(np.float32)
    with np.errstate(invalid="ignore", divide="ignore"):
        return (out / np.float32(k * (k - 1))).astype(np.float32)


def ild_labels(recs: np.ndarray, labels: np.ndarray) -> np.ndarray:
    """ILD with the label-equality matrix of IntraListBinaryUnfairnessScore
    (divrec/losses/intra_list_diversity_score.py:60-63), counted exactly."""
    n, k = recs.shape
    lab = labels[recs]
    cnt = np.zeros(n, dtype=np.int64)
    for i in range(k):
        cnt += (lab[:, i : i + 1] == lab[:, i + 1 :]).sum(axis=1)
    with np.errstate(invalid="ignore", divide="ignore"):
        return (cnt.astype(np.float32) / np.float32(k * (k - 1))).astype(np.float32)


def embedding_distance_matrix(E: np.ndarray, kind: str = "cosine") -> np.ndarray:
    """Dense D from item embeddings in float64 (what a user of the reference
    would pass as ``distance_matrix`` for an embedding-based ILD)."""
    E = E.astype(np.float64)
    G = E @ E.T
    nsq = np.diag(G)
    if kind == "cosine":
        return 1.0 - G / np.sqrt(np.outer(nsq, nsq))
    if kind == "dot":
        return G
    if kind == "euclidean":
        return np.sqrt(np.maximum(nsq[:, None] + nsq[None, :] - 2.0 * G, 0.0))
    raise ValueError(kind)


def ild_embedding_f64(recs: np.ndarray, E: np.ndarray, kind: str = "cosine") -> np.ndarray:
    """Float64 ILD from embeddings (ground truth for the fp32 GPU value)."""
    n, k = recs.shape
    out = np.empty(n, dtype=np.float64)
    for u in range(n):
        X = E[recs[u]].astype(np.float64)
        G = X @ X.T
        nsq = np.diag(G)
        iu = np.triu_indices(k, 1)
        if kind == "cosine":
            d = 1.0 - G[iu] / np.sqrt(nsq[iu[0]] * nsq[iu[1]])
        elif kind == "dot":
            d = G[iu]
        else:
            d = np.sqrt(np.maximum(nsq[iu[0]] + nsq[iu[1]] - 2 * G[iu], 0.0))
        out[u] = d.sum() / (k * (k - 1)) if k > 1 else np.nan
    return out


def reduce_values(x: np.ndarray, reduction: str = "mean") -> np.ndarray:
    """ScoreWithReduction.reduce_loss_values (divrec/losses/base_losses.py:22-27):
    'none' identity, 'mean' = sum / size(0), 'sum' = sum."""
    if reduction == "none":
        return x
    s = np.sum(x.astype(np.float64))
    return np.float32(s / x.shape[0]) if reduction == "mean" else np.float32(s)


def bpr_forward_backward(U, I, uid, pid, nid):
    """One BPR batch of pair_wise_train_loop (divrec/train/utils.py:145-149)
    with LogSigmoidDifferenceLoss (log_sigmoid_difference_loss.py:11-14) and
    the 'mean' reduction: returns (loss, auc, grad_U, grad_I) in float64."""
    U = U.astype(np.float64)
    I = I.astype(np.float64)
    u, p, n = U[uid], I[pid], I[nid]
    sp, sn = (u * p).sum(1), (u * n).sum(1)
    x = sp - sn
    B = len(uid)
    loss = np.mean(np.maximum(-x, 0) + np.log1p(np.exp(-np.abs(x))))
    auc = np.mean((sp >= sn).astype(np.float64))
    g = -1.0 / (1.0 + np.exp(x)) / B  # d mean(-logsigmoid(x)) / dx
    gU = np.zeros_like(U)
    gI = np.zeros_like(I)
    np.add.at(gU, uid, g[:, None] * (p - n))
    np.add.at(gI, pid, g[:, None] * u)
    np.add.at(gI, nid, -g[:, None] * u)
    return loss, auc, gU, gI


def adam_step(param, grad, m, v, step, lr=1e-3, beta1=0.9, beta2=0.999, eps=1e-8, wd=0.0):
    """torch.optim.Adam single-tensor update (amsgrad=False), float64."""
    param, grad, m, v = (np.asarray(a, np.float64) for a in (param, grad, m, v))
    if wd:
        grad = grad + wd * param
    m = beta1 * m + (1 - beta1) * grad
    v = beta2 * v + (1 - beta2) * grad * grad
    bc1 = 1 - beta1 ** step
    bc2 = 1 - beta2 ** step
    denom = np.sqrt(v) / math.sqrt(bc2) + eps
    return param - (lr / bc1) * m / denom, m, v


def sparse_adam_rows(param, m, v, rows, grad_values, step, lr=1e-3, beta1=0.9, beta2=0.999,
                     eps=1e-8):
    """torch.optim.SparseAdam (torch/optim/_functional.py, sparse_adam) on a
    coalesced gradient with unique ``rows`` and ``grad_values`` [len(rows), d]:
    the same fp32 op sequence with IEEE correctly rounded sqrt and division
    (torch's CPU sqrt is a 0.5-ulp-bound vector sqrt that differs in the last
    bit for ~0.7 % of inputs). In place on fp32 param / m / v."""
    f = np.float32
    g = np.asarray(grad_values, f)
    mo, vo = m[rows].copy(), v[rows].copy()
    u1 = (g - mo) * f(1 - beta1)
    u2 = (g * g - vo) * f(1 - beta2)
    m[rows] = mo + u1
    v[rows] = vo + u2
    denom = np.sqrt((u2 + vo).astype(np.float64)).astype(f) + f(eps)
    q = (u1 + mo) / denom
    step_size = lr * math.sqrt(1 - beta2 ** step) / (1 - beta1 ** step)
    param[rows] = param[rows] + f(-step_size) * q


def _mmr_values(scores, sims, picked, lam):
    pen = np.max(sims[:, picked], axis=1) if picked else np.zeros(len(scores))
    return lam * scores - (1 - lam) * pen


def mmr_greedy(cand_items, cand_scores, E, k_out, lam):
    """Build-defined MMR spec (no reference symbol):
    greedy argmax of lam*s_i - (1-lam)*max_{j picked} cos(e_i, e_j), ties to
    the lowest candidate position; float64."""
    n, C = cand_items.shape
    out = np.full((n, k_out), -1, dtype=np.int64)
    for u in range(n):
        X = E[cand_items[u]].astype(np.float64)
        Xn = X / np.linalg.norm(X, axis=1, keepdims=True)
        sims = Xn @ Xn.T
        s = cand_scores[u].astype(np.float64)
        picked: List[int] = []
        alive = np.ones(C, dtype=bool)
        for t in range(k_out):
            val = _mmr_values(s, sims, picked, lam)
            val[~alive] = -np.inf
            j = int(np.argmax(val))  # first max = lowest position
            picked.append(j)
            alive[j] = False
            out[u, t] = cand_items[u, j]
    return out


def mmr_check(picks, cand_items, cand_scores, E, lam, tol=1e-4):
    """Replay a pick sequence and check each pick is a valid greedy MMR choice
    (its value within ``tol`` of the step's maximum, float64). Returns the
    number of invalid steps over all users."""
    n, C = cand_items.shape
    bad = 0
    for u in range(n):
        X = E[cand_items[u]].astype(np.float64)
        Xn = X / np.linalg.norm(X, axis=1, keepdims=True)
        sims = Xn @ Xn.T
        s = cand_scores[u].astype(np.float64)
        pos = {int(it): c for c, it in enumerate(cand_items[u])}
        picked: List[int] = []
        alive = np.ones(C, dtype=bool)
        for it in picks[u]:
            val = _mmr_values(s, sims, picked, lam)
            val[~alive] = -np.inf
            j = pos[int(it)]
            if not alive[j] or val[j] < val.max() - tol:
                bad += 1
            picked.append(j)
            alive[j] = False
    return bad


def exclusion_csr(frozen: List[Sequence[int]]) -> Tuple[np.ndarray, np.ndarray]:
    """Per-user sorted exclusion lists -> (rowptr int64, items int32)."""
    rowptr = np.zeros(len(frozen) + 1, dtype=np.int64)
    cols = []
    for i, f in enumerate(frozen):
        s = np.unique(np.asarray(list(f), dtype=np.int64))
        cols.append(s)
        rowptr[i + 1] = rowptr[i] + len(s)
    items = np.concatenate(cols).astype(np.int32) if cols else np.zeros(0, np.int32)
    return rowptr, items
