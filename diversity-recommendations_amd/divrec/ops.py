"""Tensor-level entry points of the HIP hot path (one function per C-ABI call).

Every function takes device tensors, validates dtype / shape / contiguity on
the host, and enqueues the HIP kernel on the current stream of the tensors'
device. Outputs are freshly allocated by the PyTorch caching allocator; the
native library never allocates. There is no CPU implementation here.
"""
from __future__ import annotations

from typing import Optional, Tuple

import torch

from divrec import _backend as B


def _contig(t: torch.Tensor, name: str) -> torch.Tensor:
    if not t.is_contiguous():
        raise ValueError(f"{name} must be contiguous")
    return t


def _need(cond: bool, msg: str) -> None:
    if not cond:
        raise ValueError(msg)


# --------------------------------------------------------------------------- MF forward
def gather_dot(
    user_table: torch.Tensor,
    item_table: torch.Tensor,
    user_id: torch.Tensor,
    item_id: torch.Tensor,
    err: Optional[torch.Tensor] = None,
    check: bool = True,
) -> torch.Tensor:
    """s[n] = <U[user_id[n]], I[item_id[n]]> (MatrixFactorization.forward,
    reference divrec/models/matrix_factorization.py:26-28). fp32 or bf16 tables,
    int64 ids, fp32 output. Ids are range-checked on the device (an invalid
    pair reads nothing and gives NaN): with ``check`` and no ``err`` this call
    reads the count (one sync) and raises IndexError like nn.Embedding;
    otherwise the count goes to the caller's ``err`` (may be None), which the
    caller reads when it chooses (divrec._backend.raise_if_out_of_range)."""
    dev = B.require_device(user_table, item_table, user_id, item_id)
    _need(user_table.dim() == 2 and item_table.dim() == 2, "tables must be 2-D")
    _need(user_table.size(1) == item_table.size(1), "tables must share embedding_dim")
    _need(user_table.dtype == item_table.dtype, "tables must share dtype")
    _need(user_table.dtype in (torch.float32, torch.bfloat16), "tables must be fp32 or bf16")
    _need(user_id.dtype == torch.int64 and item_id.dtype == torch.int64, "ids must be int64")
    _need(user_id.dim() == 1 and user_id.shape == item_id.shape, "ids must be 1-D, same length")
    _contig(user_table, "user_table"), _contig(item_table, "item_table")
    user_id, item_id = user_id.contiguous(), item_id.contiguous()
    out = torch.empty(user_id.numel(), dtype=torch.float32, device=dev)
    own = err is None and check
    if own:
        err = B.error_counter(dev)
    rc = B.lib().dr_gather_dot(
        user_table.data_ptr(), user_table.size(0), item_table.data_ptr(), item_table.size(0),
        B.dtype_code(user_table.dtype), user_table.size(1), user_id.data_ptr(), item_id.data_ptr(),
        user_id.numel(), out.data_ptr(), B.ptr(err), B.stream(dev),
    )
    B.check(rc, "dr_gather_dot")
    if own:
        B.raise_if_out_of_range(err, "dr_gather_dot")
    return out


def gather_dot_backward(
    user_table: torch.Tensor,
    item_table: torch.Tensor,
    user_id: torch.Tensor,
    item_id: torch.Tensor,
    grad_out: torch.Tensor,
    grad_user: Optional[torch.Tensor],
    grad_item: Optional[torch.Tensor],
    err: Optional[torch.Tensor] = None,
) -> None:
    """Accumulate dense fp32 embedding gradients of gather_dot in place.
    Out-of-range pairs add nothing and count in ``err`` (if given)."""
    dev = B.require_device(user_table, item_table, user_id, item_id, grad_out, grad_user, grad_item)
    _need(user_table.dtype == torch.float32 and item_table.dtype == torch.float32,
          "backward needs fp32 tables")
    for g, t, nm in ((grad_user, user_table, "grad_user"), (grad_item, item_table, "grad_item")):
        if g is not None:
            _need(g.shape == t.shape and g.dtype == torch.float32 and g.is_contiguous(),
                  f"{nm} must be a contiguous fp32 tensor shaped like its table")
    grad_out = grad_out.to(torch.float32).contiguous()
    rc = B.lib().dr_gather_dot_backward(
        user_table.data_ptr(), user_table.size(0), item_table.data_ptr(), item_table.size(0),
        user_table.size(1), user_id.contiguous().data_ptr(), item_id.contiguous().data_ptr(),
        user_id.numel(), grad_out.data_ptr(), B.ptr(grad_user), B.ptr(grad_item), B.ptr(err),
        B.stream(dev),
    )
    B.check(rc, "dr_gather_dot_backward")


# --------------------------------------------------------------------------- top-K
# Widths with a scan instantiation per table dtype (include/divrec_hip.h); any
# other width is served by zero-padding both tables (zero columns add exact
# zeros to every dot product).
SCORE_WIDTHS = {torch.bfloat16: (32, 64, 128, 256, 512), torch.float32: (32, 64, 128, 256)}


def score_width(dtype: torch.dtype, d: int) -> int:
    """The scan width an embedding of width ``d`` runs at (d itself or the
    next supported width, reached by zero-padding)."""
    _need(dtype in SCORE_WIDTHS, "score_topk tables must be bf16 or fp32")
    for w in SCORE_WIDTHS[dtype]:
        if d <= w:
            return w
    raise ValueError(f"embedding_dim {d} is wider than the widest {dtype} scan "
                     f"({SCORE_WIDTHS[dtype][-1]})")


def pad_columns(table: torch.Tensor, width: int) -> torch.Tensor:
    """``table`` [rows, d] widened to ``width`` columns with zeros (a copy);
    the table itself when it already has that width."""
    if table.size(1) == width:
        return table
    out = torch.zeros((table.size(0), width), dtype=table.dtype, device=table.device)
    out[:, :table.size(1)] = table
    return out


def score_topk(
    user_table: torch.Tensor,
    item_table: torch.Tensor,
    k: int,
    user_ids: Optional[torch.Tensor] = None,
    n_users: Optional[int] = None,
    item_base: int = 0,
    exclude: Optional[Tuple[torch.Tensor, torch.Tensor]] = None,
    init_thr: Optional[torch.Tensor] = None,
    stats: Optional[dict] = None,
) -> Tuple[torch.Tensor, torch.Tensor]:
    """Top-k items per user over the catalog slice ``item_table`` (global ids
    ``item_base + row``); order = score desc, item id asc.

    ``init_thr`` (fp32 [n], optional): only items scoring strictly above the
    user's threshold are ranked (dr_score_topk_seeded); slots past the last
    such item hold item -1 / score -inf. Used by the item-sharded multi-GPU
    top-k with thresholds from a sample of the whole catalog.

    The tables' dtype picks the arithmetic: bf16 tables run the bf16 MFMA scan
    (exact products, fp32 sums: the fast mode), fp32 tables the fp32 MFMA scan
    (an exact fp32 fmaf chain per score: the reference's arithmetic up to the
    summation order). Widths without a scan instance are zero-padded here: a
    copy of both tables on every call (O((U + I) d) bytes; pad once and pass
    the padded tables when calling repeatedly on a large catalog).

    ``user_ids`` (int64) selects user rows; if None the first ``n_users`` rows
    (default: all) are scored. ``exclude = (rowptr int64 [n+1], items int32)``
    is a CSR of GLOBAL item ids (sorted per row) never to recommend.
    Returns (scores fp32 [n, k], items int32 [n, k]).

    ``stats`` (a dict, optional): filled with ``guess_failures`` = [users the
    first-tier guessed threshold failed, users every guess failed] of this
    call (dr_score_topk_fail_counts; one synchronising read).
    """
    dev = B.require_device(user_table, item_table, user_ids)
    _need(user_table.dtype == item_table.dtype and user_table.dtype in SCORE_WIDTHS,
          "score_topk tables must both be bf16 or both fp32")
    _need(user_table.dim() == 2 and item_table.dim() == 2, "tables must be 2-D")
    d = user_table.size(1)
    _need(item_table.size(1) == d, "tables must share embedding_dim")
    _contig(user_table, "user_table"), _contig(item_table, "item_table")
    w = score_width(user_table.dtype, d)
    user_table, item_table = pad_columns(user_table, w), pad_columns(item_table, w)
    _need(1 <= k <= 1024, "k must be in [1, 1024]")
    if user_ids is not None:
        _need(user_ids.dtype == torch.int64 and user_ids.dim() == 1, "user_ids must be 1-D int64")
        user_ids = user_ids.contiguous()
        n = user_ids.numel()
        if n:
            lo, hi = int(user_ids.min()), int(user_ids.max())
            _need(0 <= lo and hi < user_table.size(0), "user_ids out of range")
    else:
        n = user_table.size(0) if n_users is None else int(n_users)
        _need(0 <= n <= user_table.size(0), "n_users out of range")
    n_items = item_table.size(0)
    _need(k <= n_items or exclude is not None or init_thr is not None or n_items == 0,
          "k must be <= number of items")
    rowptr = cols = None
    if exclude is not None:
        rowptr, cols = exclude
        B.require_device(rowptr, cols)
        _need(rowptr.dtype == torch.int64 and rowptr.numel() == n + 1, "rowptr must be int64 [n+1]")
        _need(cols.dtype == torch.int32, "excluded items must be int32")
        rowptr, cols = rowptr.contiguous(), cols.contiguous()
        if cols.numel() == 0:
            cols = torch.zeros(1, dtype=torch.int32, device=dev)
    scores = torch.empty((n, k), dtype=torch.float32, device=dev)
    items = torch.empty((n, k), dtype=torch.int32, device=dev)
    if n == 0:
        return scores, items
    L = B.lib()
    dt = B.dtype_code(user_table.dtype)
    if init_thr is not None:
        B.require_device(init_thr)
        _need(init_thr.dtype == torch.float32 and init_thr.numel() == n,
              "init_thr must be fp32 [n_users]")
        init_thr = init_thr.contiguous()
        ws_bytes = L.dr_score_topk_seeded_workspace(n, n_items, dt, w, k)
        ws = torch.empty(max(int(ws_bytes), 1), dtype=torch.uint8, device=dev)
        rc = L.dr_score_topk_seeded(
            user_table.data_ptr(), B.ptr(user_ids), n, item_table.data_ptr(), n_items,
            int(item_base), dt, w, int(k), init_thr.data_ptr(), B.ptr(rowptr), B.ptr(cols),
            scores.data_ptr(), items.data_ptr(), ws.data_ptr(), ws.numel(), B.stream(dev),
        )
        B.check(rc, "dr_score_topk_seeded")
        return scores, items
    ws_bytes = L.dr_score_topk_workspace(n, n_items, dt, w, k)
    ws = torch.empty(max(int(ws_bytes), 1), dtype=torch.uint8, device=dev)
    rc = L.dr_score_topk(
        user_table.data_ptr(), B.ptr(user_ids), n, item_table.data_ptr(), n_items, int(item_base),
        dt, w, int(k), B.ptr(rowptr), B.ptr(cols), scores.data_ptr(), items.data_ptr(),
        ws.data_ptr(), ws.numel(), B.stream(dev),
    )
    B.check(rc, "dr_score_topk")
    if stats is not None:
        import ctypes

        torch.cuda.synchronize(dev)
        fc = (ctypes.c_int32 * 2)()
        B.check(L.dr_score_topk_fail_counts(ws.data_ptr(), n, n_items, dt, w, int(k),
                                            ctypes.addressof(fc)), "dr_score_topk_fail_counts")
        stats["guess_failures"] = [int(fc[0]), int(fc[1])]
    return scores, items


PLAN_FIELDS = ("users_per_wg", "user_blocks", "head_blocks", "tail_chunks", "chunk_items", "grid",
               "cap", "sample_stride", "sample_rows", "sample_rank", "head_keys", "tail_keys",
               "first_tier_rank")


def score_topk_plan(n_users: int, n_items: int, dtype: torch.dtype, d: int, k: int) -> dict:
    """The launch plan dr_score_topk uses for this call shape on the current
    device (no device work): user blocks, head/tail split, guess stride, ...
    (PLAN_FIELDS). Tests use it to prove which plan they exercised.
    ``sample_rank`` is the guess's safe (second-tier) rank ks in the sample,
    ``first_tier_rank`` the rank ks1 <= ks the main scan starts from."""
    import ctypes

    w = score_width(dtype, d)
    n_f = len(PLAN_FIELDS)
    out = (ctypes.c_int64 * n_f)()
    rc = B.lib().dr_score_topk_plan(int(n_users), int(n_items), B.dtype_code(dtype), w, int(k),
                                    ctypes.addressof(out), n_f)
    B.check(rc, "dr_score_topk_plan")
    return dict(zip(PLAN_FIELDS, (int(x) for x in out)))


def sample_thresholds(user_table: torch.Tensor, sample_rows: torch.Tensor, ks1: int, ks: int,
                      user_ids: Optional[torch.Tensor] = None) -> torch.Tensor:
    """The guessed thresholds of the item-sharded top-k (dr_sample_thresholds):
    ``sample_rows`` are the whole catalog's rows at the guess stride; returns
    fp32 [2, n]: strictly below each user's ks1-th (row 0, first tier) and
    ks-th (row 1, safe tier) best tile-max score of the sample (the
    dr_score_topk guess's tile-max sample scan; -inf when there are fewer)."""
    dev = B.require_device(user_table, sample_rows, user_ids)
    _need(user_table.dtype == sample_rows.dtype and user_table.dtype in SCORE_WIDTHS,
          "user table and sample rows must both be bf16 or both fp32")
    _need(user_table.dim() == 2 and sample_rows.dim() == 2 and
          sample_rows.size(1) == user_table.size(1), "2-D tables of one width")
    _need(1 <= ks1 <= ks <= 256, "need 1 <= ks1 <= ks <= 256")
    _contig(user_table, "user_table")
    w = score_width(user_table.dtype, user_table.size(1))
    user_table = pad_columns(user_table, w)
    sample_rows = pad_columns(sample_rows.contiguous(), w)
    if user_ids is not None:
        _need(user_ids.dtype == torch.int64 and user_ids.dim() == 1, "user_ids must be 1-D int64")
        user_ids = user_ids.contiguous()
        n = user_ids.numel()
    else:
        n = user_table.size(0)
    out = torch.empty((2, n), dtype=torch.float32, device=dev)
    if n == 0:
        return out
    L = B.lib()
    dt = B.dtype_code(user_table.dtype)
    ws_bytes = L.dr_sample_thresholds_workspace(n, sample_rows.size(0), dt, w, int(ks))
    ws = torch.empty(max(int(ws_bytes), 1), dtype=torch.uint8, device=dev)
    rc = L.dr_sample_thresholds(user_table.data_ptr(), B.ptr(user_ids), n,
                                sample_rows.data_ptr(), sample_rows.size(0), dt, w, int(ks1),
                                int(ks), out[0].data_ptr(), out[1].data_ptr(), ws.data_ptr(),
                                ws.numel(), B.stream(dev))
    B.check(rc, "dr_sample_thresholds")
    return out


def topk_merge(
    scores: torch.Tensor, items: torch.Tensor, k_out: Optional[int] = None
) -> Tuple[torch.Tensor, torch.Tensor]:
    """Merge per-part sorted top-k lists [parts, n, k_in] -> [n, k_out]."""
    dev = B.require_device(scores, items)
    _need(scores.dim() == 3 and scores.shape == items.shape, "expected [parts, n, k] inputs")
    _need(scores.dtype == torch.float32 and items.dtype == torch.int32, "fp32 scores, int32 items")
    parts, n, k_in = scores.shape
    k_out = k_in if k_out is None else int(k_out)
    _need(1 <= k_out <= parts * k_in, "k_out must be in [1, parts * k_in]")
    _need(parts * k_in <= 2048 or k_out <= 1024, "k_out must be <= 1024 when parts * k_in > 2048")
    out_s = torch.empty((n, k_out), dtype=torch.float32, device=dev)
    out_i = torch.empty((n, k_out), dtype=torch.int32, device=dev)
    if n == 0:
        return out_s, out_i
    rc = B.lib().dr_topk_merge(
        scores.contiguous().data_ptr(), items.contiguous().data_ptr(), parts, n, k_in, k_out,
        out_s.data_ptr(), out_i.data_ptr(), B.stream(dev),
    )
    B.check(rc, "dr_topk_merge")
    return out_s, out_i


# --------------------------------------------------------------------------- ILD
def _recs(recs: torch.Tensor) -> Tuple[torch.Tensor, int]:
    _need(recs.dim() == 2, "recommendations must be [n_users, k]")
    _need(recs.dtype in (torch.int32, torch.int64), "recommendations must be int32 or int64")
    return recs.contiguous(), B.dtype_code(recs.dtype)


def ild_dense(recs: torch.Tensor, dist: torch.Tensor) -> torch.Tensor:
    """Per-user ILD against a dense [I, I] distance matrix (fp32/fp64/int32/int64)."""
    dev = B.require_device(recs, dist)
    recs, rc_dt = _recs(recs)
    _need(dist.dim() == 2 and dist.size(0) == dist.size(1), "distance matrix must be [I, I]")
    _need(dist.dtype in (torch.float32, torch.float64, torch.int32, torch.int64),
          "distance matrix dtype must be float32/float64/int32/int64")
    dist = dist.contiguous()
    n, k = recs.shape
    out = torch.empty(n, dtype=torch.float32, device=dev)
    if n == 0:
        return out
    err = B.error_counter(dev)
    rc = B.lib().dr_ild_dense(
        recs.data_ptr(), rc_dt, n, k, dist.data_ptr(), B.dtype_code(dist.dtype), dist.size(0),
        out.data_ptr(), err.data_ptr(), B.stream(dev),
    )
    B.check(rc, "dr_ild_dense")
    B.raise_if_out_of_range(err, "dr_ild_dense")
    return out


def ild_dense_pair_sum(recs: torch.Tensor, dist: torch.Tensor) -> torch.Tensor:
    """Per-user UN-normalised pair sum sum_{p<q} D[r_p, r_q] (the reference's
    user_ild), accumulated in D's precision; float64 [n] (exact for fp32 and
    integer D)."""
    dev = B.require_device(recs, dist)
    recs, rc_dt = _recs(recs)
    _need(dist.dim() == 2 and dist.size(0) == dist.size(1), "distance matrix must be [I, I]")
    _need(dist.dtype in (torch.float32, torch.float64, torch.int32, torch.int64),
          "distance matrix dtype must be float32/float64/int32/int64")
    dist = dist.contiguous()
    n, k = recs.shape
    out = torch.empty(n, dtype=torch.float64, device=dev)
    if n == 0:
        return out
    err = B.error_counter(dev)
    rc = B.lib().dr_ild_dense_pair_sum(
        recs.data_ptr(), rc_dt, n, k, dist.data_ptr(), B.dtype_code(dist.dtype), dist.size(0),
        out.data_ptr(), err.data_ptr(), B.stream(dev),
    )
    B.check(rc, "dr_ild_dense_pair_sum")
    B.raise_if_out_of_range(err, "dr_ild_dense_pair_sum")
    return out


def ild_labels(recs: torch.Tensor, labels: torch.Tensor) -> torch.Tensor:
    """Per-user ILD with D[i,j] = (labels[i] == labels[j]) computed on the fly."""
    dev = B.require_device(recs, labels)
    recs, rc_dt = _recs(recs)
    labels = labels.to(torch.int64).contiguous()
    n, k = recs.shape
    out = torch.empty(n, dtype=torch.float32, device=dev)
    if n == 0:
        return out
    err = B.error_counter(dev)
    rc = B.lib().dr_ild_labels(
        recs.data_ptr(), rc_dt, n, k, labels.data_ptr(), labels.numel(), out.data_ptr(),
        err.data_ptr(), B.stream(dev),
    )
    B.check(rc, "dr_ild_labels")
    B.raise_if_out_of_range(err, "dr_ild_labels")
    return out


_KINDS = {"cosine": B.DR_ILD_COSINE, "dot": B.DR_ILD_DOT, "euclidean": B.DR_ILD_EUCLIDEAN}
ILD_WIDTHS = (32, 64, 128, 256)  # dr_ild_embedding instances; others are zero-padded
MMR_WIDTHS = (64, 128)           # dr_mmr_rerank instances; others are zero-padded


def _width_of(widths, d: int, what: str) -> int:
    for w in widths:
        if d <= w:
            return w
    raise ValueError(f"{what} supports embedding_dim <= {widths[-1]}, got {d}")


def ild_embedding(recs: torch.Tensor, item_table: torch.Tensor, kind: str = "cosine",
                  check: bool = True) -> torch.Tensor:
    """Per-user ILD with D computed from bf16 item embeddings (cosine/dot/euclidean).
    A list with an id outside the table gives NaN; with ``check`` the call
    reads the count (one sync) and raises IndexError."""
    dev = B.require_device(recs, item_table)
    recs, rc_dt = _recs(recs)
    _need(item_table.dtype == torch.bfloat16 and item_table.dim() == 2, "item_table must be bf16 2-D")
    _contig(item_table, "item_table")
    _need(kind in _KINDS, f"kind must be one of {sorted(_KINDS)}")
    # a width without a kernel instance (e.g. d = 100) is zero-padded per call,
    # never cached: writes through .data or raw pointers bump no version a
    # cache could key on. Repeated callers pad once themselves
    # (EmbeddingDistance holds its padded table; pad_columns is public).
    item_table = pad_columns(item_table, _width_of(ILD_WIDTHS, item_table.size(1), "embedding ILD"))
    n, k = recs.shape
    _need(k <= 16384, "embedding ILD supports k <= 16384")
    out = torch.empty(n, dtype=torch.float32, device=dev)
    if n == 0:
        return out
    err = B.error_counter(dev) if check else None
    rc = B.lib().dr_ild_embedding(
        recs.data_ptr(), rc_dt, n, k, item_table.data_ptr(), item_table.size(0),
        item_table.size(1), _KINDS[kind], out.data_ptr(), B.ptr(err), B.stream(dev),
    )
    B.check(rc, "dr_ild_embedding")
    B.raise_if_out_of_range(err, "dr_ild_embedding")
    return out


# --------------------------------------------------------------------------- BPR
def bpr_fwd_bwd(
    user_table: torch.Tensor,
    item_table: torch.Tensor,
    user_id: torch.Tensor,
    pos_id: torch.Tensor,
    neg_id: torch.Tensor,
    grad_scale: float,
    grad_user: Optional[torch.Tensor],
    grad_item: Optional[torch.Tensor],
    err: Optional[torch.Tensor] = None,
    check: bool = True,
) -> Tuple[torch.Tensor, torch.Tensor]:
    """Fused BPR forward + backward; returns per-triple (loss fp32, hit int32)
    and accumulates dense gradients into grad_user / grad_item. Ids are
    range-checked on the device (an invalid triple adds nothing): with
    ``check`` and no ``err`` the call reads the count (one sync) and raises
    IndexError; otherwise the count goes to the caller's ``err`` (may be None),
    checked by the caller (pair_wise_train_loop: once per epoch)."""
    dev = B.require_device(user_table, item_table, user_id, pos_id, neg_id, grad_user, grad_item)
    _need(user_table.dtype == torch.float32 and item_table.dtype == torch.float32, "fp32 tables")
    for t in (user_id, pos_id, neg_id):
        _need(t.dtype == torch.int64 and t.dim() == 1 and t.numel() == user_id.numel(),
              "ids must be 1-D int64 of equal length")
    n = user_id.numel()
    loss = torch.empty(n, dtype=torch.float32, device=dev)
    hit = torch.empty(n, dtype=torch.int32, device=dev)
    own = err is None and check
    if own:
        err = B.error_counter(dev)
    rc = B.lib().dr_bpr_fwd_bwd(
        user_table.data_ptr(), user_table.size(0), item_table.data_ptr(), item_table.size(0),
        user_table.size(1), user_id.contiguous().data_ptr(), pos_id.contiguous().data_ptr(),
        neg_id.contiguous().data_ptr(), n, float(grad_scale), loss.data_ptr(), hit.data_ptr(),
        B.ptr(grad_user), B.ptr(grad_item), B.ptr(err), B.stream(dev),
    )
    B.check(rc, "dr_bpr_fwd_bwd")
    if own:
        B.raise_if_out_of_range(err, "dr_bpr_fwd_bwd")
    return loss, hit


def adam_dense(
    param: torch.Tensor, grad: torch.Tensor, exp_avg: torch.Tensor, exp_avg_sq: torch.Tensor,
    lr: float, beta1: float, beta2: float, eps: float, weight_decay: float, step: int,
) -> None:
    dev = B.require_device(param, grad, exp_avg, exp_avg_sq)
    for t in (param, grad, exp_avg, exp_avg_sq):
        _need(t.dtype == torch.float32 and t.is_contiguous() and t.numel() == param.numel(),
              "adam tensors must be contiguous fp32 of equal size")
    rc = B.lib().dr_adam_dense(
        param.data_ptr(), grad.data_ptr(), exp_avg.data_ptr(), exp_avg_sq.data_ptr(),
        param.numel(), float(lr), float(beta1), float(beta2), float(eps), float(weight_decay),
        int(step), B.stream(dev),
    )
    B.check(rc, "dr_adam_dense")


def adam_rows(
    param: torch.Tensor, grad: torch.Tensor, exp_avg: torch.Tensor, exp_avg_sq: torch.Tensor,
    rows: torch.Tensor, lr: float, beta1: float, beta2: float, eps: float, step: int,
    zero_grad: bool = True,
) -> None:
    """torch.optim.SparseAdam's update over the UNIQUE rows ``rows`` of 2-D
    fp32 tables (gradient values read from the dense ``grad``); with
    ``zero_grad`` the touched gradient rows are zeroed afterwards."""
    dev = B.require_device(param, grad, exp_avg, exp_avg_sq, rows)
    _need(param.dim() == 2, "adam_rows: param must be a 2-D table")
    for t in (param, grad, exp_avg, exp_avg_sq):
        _need(t.dtype == torch.float32 and t.is_contiguous() and t.shape == param.shape,
              "adam_rows tensors must be contiguous fp32 tables of equal shape")
    rows = rows.to(torch.int64).contiguous()
    _need(rows.dim() == 1, "adam_rows: rows must be 1-D")
    rc = B.lib().dr_adam_rows(
        param.data_ptr(), grad.data_ptr(), exp_avg.data_ptr(), exp_avg_sq.data_ptr(),
        param.size(1), rows.data_ptr(), rows.numel(), float(lr), float(beta1), float(beta2),
        float(eps), int(step), 1 if zero_grad else 0, B.stream(dev),
    )
    B.check(rc, "dr_adam_rows")


# --------------------------------------------------------------------------- pairwise sampler
def sample_pairwise(users: torch.Tensor, pos_rowptr: torch.Tensor, pos_items: torch.Tensor,
                    n_items: int, m: int, seed: int,
                    exclude: Optional[Tuple[torch.Tensor, torch.Tensor]] = None,
                    expand: bool = True):
    """PairWiseDataset's per-user sampling on the device (dr_sample_pairwise).
    Returns (pos [n, m] int32, neg [n, m] int32, triples) where triples is
    (uid, pid, nid) int64 [n*m*m] in the reference's pos-major order, or None
    without ``expand``. Raises IndexError, as the reference does, when a user
    has no positives or no allowed negative (this reads one device counter)."""
    dev = B.require_device(users, pos_rowptr, pos_items)
    _need(pos_items.dtype == torch.int32 and pos_rowptr.dtype == torch.int64,
          "positives CSR must be int64 rowptr / int32 items")
    users = users.to(torch.int64).contiguous()
    n = users.numel()
    pos = torch.empty((n, m), dtype=torch.int32, device=dev)
    neg = torch.empty((n, m), dtype=torch.int32, device=dev)
    err = torch.zeros(1, dtype=torch.int32, device=dev)
    trip = None
    if expand:
        trip = tuple(torch.empty(n * m * m, dtype=torch.int64, device=dev) for _ in range(3))
    er, ei = (None, None) if exclude is None else exclude
    rc = B.lib().dr_sample_pairwise(
        users.data_ptr(), n, pos_rowptr.contiguous().data_ptr(), pos_items.contiguous().data_ptr(),
        B.ptr(er), B.ptr(ei), int(n_items), int(m), int(seed) & ((1 << 64) - 1),
        pos.data_ptr(), neg.data_ptr(), *(B.ptr(t) for t in (trip or (None,) * 3)),
        err.data_ptr(), B.stream(dev),
    )
    B.check(rc, "dr_sample_pairwise")
    if int(err.item()) != 0:
        raise IndexError("Cannot choose from an empty sequence (a user without positives, "
                         "or without any allowed negative)")
    return pos, neg, trip


# --------------------------------------------------------------------------- catalog histogram
def catalog_histogram(recs: torch.Tensor, n_items: int) -> Tuple[torch.Tensor, torch.Tensor]:
    """(counts int32 [n_items], position sums int64 [n_items]) of the item ids
    in ``recs`` [n, k]; entries outside [0, n_items) are skipped."""
    dev = B.require_device(recs)
    recs, rc_dt = _recs(recs)
    n, k = recs.shape
    _need(n_items >= 1, "n_items must be >= 1")
    counts = torch.zeros(int(n_items), dtype=torch.int32, device=dev)
    pos_sum = torch.zeros(int(n_items), dtype=torch.int64, device=dev)
    if n == 0 or k == 0:
        return counts, pos_sum
    rc = B.lib().dr_catalog_histogram(recs.data_ptr(), rc_dt, n, k, int(n_items),
                                      counts.data_ptr(), pos_sum.data_ptr(), B.stream(dev))
    B.check(rc, "dr_catalog_histogram")
    return counts, pos_sum


# --------------------------------------------------------------------------- MMR
def mmr_rerank(
    cand_items: torch.Tensor, cand_scores: torch.Tensor, item_table: torch.Tensor, k_out: int,
    lam: float = 0.5, check: bool = True,
) -> torch.Tensor:
    """Greedy MMR over per-user candidates (int32 [n, C] + fp32 [n, C]) -> int32 [n, k_out].
    Candidate ids < 0 are empty slots; with ``check`` an id >= the table's row
    count raises IndexError after the call (one counter read), as indexing the
    table would (without it such candidates are silently never picked).
    Widths other than 64 / 128 are zero-padded per call (no cache, so every
    write to the table is seen; pass a pre-padded table to avoid the copy)."""
    dev = B.require_device(cand_items, cand_scores, item_table)
    _need(cand_items.dtype == torch.int32 and cand_scores.dtype == torch.float32,
          "int32 candidate ids, fp32 scores")
    _need(cand_items.dim() == 2 and cand_items.shape == cand_scores.shape, "[n, C] inputs")
    _need(item_table.dtype == torch.bfloat16 and item_table.dim() == 2, "item_table must be bf16 2-D")
    item_table = pad_columns(item_table.contiguous(),
                             _width_of(MMR_WIDTHS, item_table.size(1), "mmr_rerank"))
    n, C = cand_items.shape
    out = torch.empty((n, int(k_out)), dtype=torch.int32, device=dev)
    if n == 0:
        return out
    err = B.error_counter(dev) if check else None
    rc = B.lib().dr_mmr_rerank(
        cand_items.contiguous().data_ptr(), cand_scores.contiguous().data_ptr(), n, C,
        item_table.contiguous().data_ptr(), item_table.size(0), item_table.size(1), int(k_out),
        float(lam), out.data_ptr(), B.ptr(err), B.stream(dev),
    )
    B.check(rc, "dr_mmr_rerank")
    B.raise_if_out_of_range(err, "dr_mmr_rerank")
    return out


# --------------------------------------------------------------------------- rank metrics
def rank_metrics(
    recs: torch.Tensor, pos_rowptr: torch.Tensor, pos_items: torch.Tensor
) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor, torch.Tensor]:
    """(precision@k, recall@k, AP@k, NDCG@k) per user of ``recs`` [n, k] against
    positives given as CSR (rowptr int64 [n+1], items int32 sorted per row)."""
    dev = B.require_device(recs, pos_rowptr, pos_items)
    recs, rc_dt = _recs(recs)
    n, k = recs.shape
    _need(pos_rowptr.dtype == torch.int64 and pos_rowptr.numel() == n + 1, "rowptr int64 [n+1]")
    _need(pos_items.dtype == torch.int32, "positives must be int32")
    outs = [torch.empty(n, dtype=torch.float32, device=dev) for _ in range(4)]
    if n == 0:
        return tuple(outs)
    items = pos_items.contiguous() if pos_items.numel() else torch.zeros(1, dtype=torch.int32, device=dev)
    rc = B.lib().dr_rank_metrics(
        recs.data_ptr(), rc_dt, n, k, pos_rowptr.contiguous().data_ptr(), items.data_ptr(),
        *(o.data_ptr() for o in outs), B.stream(dev),
    )
    B.check(rc, "dr_rank_metrics")
    return tuple(outs)
