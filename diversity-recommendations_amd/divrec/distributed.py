"""Item-row-sharded top-K over several GPUs of one node.

The reference has no distributed code; this is the build's scale-out of
get_model_recommendations (reference divrec/train/utils.py:53-77). One process
per GPU (torchrun), ``torch.distributed`` with the "nccl" backend (= RCCL over
xGMI on ROCm):

  1. rank r owns the contiguous item rows [lo_r, hi_r) of the catalog and every
     user row; it computes the partial top-k of ALL users over its rows
     (dr_score_topk, global ids = lo_r + row);
  2. ONE exchange: all_to_all of the partials, so rank r receives, from every
     rank, the partial lists of its own user slice [u_lo_r, u_hi_r)
     (G-fold less traffic than an all_gather of everything);
  3. rank r merges the G partial lists of its users (dr_topk_merge).

Because the order (score desc, item id asc) is a total order and a score does
not depend on which shard computed it, the merged lists are bit-identical to
single-device dr_score_topk over the whole catalog.

Grid layout (``grid_layout``): the G ranks form a (G / S) x S grid. The S
ranks of a row share one user slice and row-shard the item table S ways; the
exchange above runs inside the row (a process group of S ranks). S = G is
pure item sharding (the north-star layout, bench.py's default); S = 1 is pure
user sharding (no exchange). The scan's survivor stream costs
~users * k * ln(items / k) per rank, so at fixed U x I fewer item shards mean
less of it.

User-sharded metrics (config 5: MMR re-rank + ILD):
every rank owns a user slice and the whole (replicated) item table; the only
collective is ``global_mean``, one all_reduce of (sum, count).
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import Any, Callable, Optional, Tuple

import torch
import torch.distributed as dist

Partial = Tuple[torch.Tensor, torch.Tensor]  # (scores fp32 [n, k], items int32 [n, k])
_SOLO = "solo"  # group sentinel: this rank alone holds the whole catalog (no exchange)


def shard_range(n: int, world: int, rank: int) -> Tuple[int, int]:
    """Contiguous balanced split of range(n) into `world` parts; part `rank`."""
    base, rem = divmod(n, world)
    lo = rank * base + min(rank, rem)
    return lo, lo + base + (1 if rank < rem else 0)


@dataclass
class GridLayout:
    """This rank's place in a (user_groups x item_shards) grid of ranks."""

    world: int
    rank: int
    item_shards: int   # S: ranks that row-shard the item table for one user slice
    user_groups: int   # G / S
    item_shard: int    # column of this rank: item rows shard_range(I, S, item_shard)
    user_group: int    # row of this rank: users shard_range(U, G / S, user_group)
    group: Any         # process group of this row (None = the default group)

    def item_range(self, n_items: int) -> Tuple[int, int]:
        return shard_range(n_items, self.item_shards, self.item_shard)

    def user_range(self, n_users: int) -> Tuple[int, int]:
        return shard_range(n_users, self.user_groups, self.user_group)


def grid_layout(item_shards: int) -> GridLayout:
    """Place every rank of the default group in the grid; ranks u*S .. u*S+S-1
    form row u. Collective: every rank must call it (dist.new_group)."""
    world, rank = dist.get_world_size(), dist.get_rank()
    if item_shards < 1 or world % item_shards:
        raise ValueError(f"item_shards={item_shards} must divide the world size {world}")
    groups = world // item_shards
    group = None
    if 1 < item_shards < world:
        for u in range(groups):  # every rank creates every row group, in the same order
            g = dist.new_group(list(range(u * item_shards, (u + 1) * item_shards)))
            if u == rank // item_shards:
                group = g
    if item_shards == 1:
        group = _SOLO
    return GridLayout(world, rank, item_shards, groups, rank % item_shards,
                      rank // item_shards, group)


def exchange_partials(scores: torch.Tensor, items: torch.Tensor, group=None) -> Partial:
    """all_to_all of per-user partial top-k lists.

    Input: this rank's partial lists for ALL n users ([n, k] each).
    Output: [world, n_r, k] scores / items — the partial lists of this rank's
    user slice from every rank (row p = rank p's shard)."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    n, k = scores.shape
    packed = torch.stack([scores.view(torch.int32), items], dim=2).reshape(n, 2 * k).contiguous()
    in_splits = [shard_range(n, world, p)[1] - shard_range(n, world, p)[0] for p in range(world)]
    lo, hi = shard_range(n, world, rank)
    n_r = hi - lo
    # gloo (CPU tests, the one-GPU multi-rank rehearsal) exchanges host
    # tensors; RCCL exchanges the device tensors in place over xGMI
    staged = packed.is_cuda and dist.get_backend(group) == "gloo"
    src = packed.cpu() if staged else packed
    out = torch.empty((world * n_r, 2 * k), dtype=torch.int32, device=src.device)
    dist.all_to_all_single(out, src, output_split_sizes=[n_r] * world,
                           input_split_sizes=in_splits, group=group)
    if staged:
        out = out.to(scores.device)
    out = out.view(world, n_r, k, 2)
    return out[..., 0].contiguous().view(torch.float32), out[..., 1].contiguous()


def global_mean(values: torch.Tensor, group=None) -> torch.Tensor:
    """Mean of per-user values (e.g. ILD) held by the ranks of ``group``, each
    for its own user slice: ONE all_reduce of the float64 (sum, count) pair.
    Equals ScoreWithReduction's 'mean' (sum / size, base_losses.py:22-27) over
    the concatenated values up to fp32 rounding of the final quotient."""
    t = torch.stack([values.detach().to(torch.float64).sum(),
                     torch.tensor(float(values.numel()), dtype=torch.float64,
                                  device=values.device)])
    staged = t.is_cuda and dist.get_backend(group) == "gloo"
    src = t.cpu() if staged else t
    dist.all_reduce(src, group=group)
    return (src[0] / src[1]).to(torch.float32).to(values.device)


# --------------------------------------------------------------------------- global thresholds
# Each shard of a pure item sharding would otherwise keep its LOCAL top-k: a
# survivor stream of ~k (1 + ln(I_shard / k)) keys per user on every one of
# the S shards, where only ~k / S of each shard's items can reach the global
# top-k. So the ranks first agree on a per-user threshold guessed from a
# strided sample of the WHOLE catalog (the same rule as dr_score_topk's own
# guess: stride by catalog length, rank ks = mean + 6 sigma + 3 of the user's
# top-k inside the sample), and each shard keeps only items above it
# (dr_score_topk_seeded). The guess is verified after the merge: a user left
# with fewer than k items is recomputed with plain per-shard top-k lists, so
# the result is the exact global top-k in every case.
GUESS_SIGMA = 6.0
# Users of the last thresholded_exchange call, summed over the ranks of its
# group, whose guess failed and who were recomputed by the exact fallback
# (observability for tests and the bench; not used by the path itself).
LAST_FALLBACK_USERS = 0


def sample_stride(n_items: int, k: int) -> int:
    """The sample stride of dr_score_topk's guess (csrc/score_topk.hip guess_for)."""
    st = 32
    while k < 256 and st < 128 and n_items // (2 * st) >= 65536:
        st *= 2
    return st


def guess_rank(k: int, frac: float) -> int:
    mu = k * frac
    return min(k, int(math.ceil(mu + GUESS_SIGMA * math.sqrt(mu) + 3.0)))


def threshold_below(kth: torch.Tensor) -> torch.Tensor:
    """A threshold strictly below each score (topk_threshold_kernel's rule);
    -inf where there is no finite score."""
    below = kth - torch.clamp(kth.abs() * 2.0 ** -20, min=2.0 ** -100)
    return torch.where(below < kth, below, torch.full_like(kth, -math.inf))


def _all_gather_rows(x: torch.Tensor, sizes, group) -> torch.Tensor:
    """Concatenate every rank's x (rank p holds sizes[p] rows) in rank order."""
    world = len(sizes)
    m = max(max(sizes), 1)
    staged = x.is_cuda and dist.get_backend(group) == "gloo"
    src = x.cpu() if staged else x
    pad = torch.zeros((m,) + tuple(src.shape[1:]), dtype=src.dtype, device=src.device)
    pad[: src.shape[0]] = src
    outs = [torch.empty_like(pad) for _ in range(world)]
    dist.all_gather(outs, pad, group=group)
    out = torch.cat([o[: sizes[p]] for p, o in enumerate(outs)])
    return out.to(x.device) if staged else out


def global_thresholds(user_table: torch.Tensor, item_shard: torch.Tensor, lo: int, hi: int,
                      n_items: int, k: int, group, user_ids: Optional[torch.Tensor] = None,
                      local_topk: Optional[Callable[..., Partial]] = None) -> torch.Tensor:
    """Per-user thresholds for all n users from a sample of the whole catalog:
    every rank contributes its shard's rows at global positions j * stride,
    the samples are all_gathered, each rank ranks ITS merge slice of users
    against them and the thresholds are all_gathered back. fp32 [n]."""
    if local_topk is None:
        from divrec import ops

        local_topk = ops.score_topk
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    st = sample_stride(n_items, k)
    j0 = -(-lo // st)  # first global sample position j * st inside [lo, hi)
    rows = item_shard[j0 * st - lo: hi - lo: st]
    # the shards may be any contiguous split: exchange the sample sizes first
    mine = torch.tensor([rows.size(0)], dtype=torch.int64, device=item_shard.device)
    sizes = [int(c) for c in _all_gather_rows(mine, [1] * world, group).cpu()]
    sample = _all_gather_rows(rows.contiguous(), sizes, group)
    n = user_table.size(0) if user_ids is None else user_ids.numel()
    u_lo, u_hi = shard_range(n, world, rank)
    ks = guess_rank(k, sample.size(0) / n_items) if sample.size(0) else 0
    thr = torch.full((u_hi - u_lo,), -math.inf, dtype=torch.float32, device=user_table.device)
    if ks and u_hi > u_lo and sample.size(0) >= ks:
        ids = (user_ids[u_lo:u_hi] if user_ids is not None
               else torch.arange(u_lo, u_hi, device=user_table.device))
        s, _ = local_topk(user_table, sample, ks, user_ids=ids, item_base=0)
        thr = threshold_below(s[:, ks - 1].contiguous())
    usizes = [shard_range(n, world, p)[1] - shard_range(n, world, p)[0] for p in range(world)]
    return _all_gather_rows(thr, usizes, group)


def thresholded_exchange(user_table: torch.Tensor, item_shard: torch.Tensor, lo: int, hi: int,
                         n_items: int, k: int, group, user_ids: Optional[torch.Tensor] = None,
                         local_topk: Optional[Callable[..., Partial]] = None,
                         merge: Optional[Callable[[torch.Tensor, torch.Tensor, int], Partial]] = None,
                         thr: Optional[torch.Tensor] = None,
                         local: Optional[Partial] = None) -> Partial:
    """Top-k of this rank's merge slice over the sharded catalog with global
    thresholds (computed here unless given): thresholded shard lists ->
    all_to_all -> merge -> verification, with an exact fallback for users the
    guess failed (a user with fewer than min(k, n_items) merged items)."""
    if local_topk is None or merge is None:
        from divrec import ops

        local_topk = local_topk or ops.score_topk
        merge = merge or ops.topk_merge
    if thr is None:
        thr = global_thresholds(user_table, item_shard, lo, hi, n_items, k, group, user_ids,
                                local_topk)
    if local is None:  # this shard's thresholded lists (the bench passes its timed call's)
        local = local_topk(user_table, item_shard, k, user_ids=user_ids, item_base=lo,
                           init_thr=thr)
    s, i = local
    ps, pi = exchange_partials(s, i, group)
    out_s, out_i = merge(ps, pi, k)
    # verification: the guess failed for a user left with fewer than k items
    need = min(k, n_items)
    bad = ((out_i[:, :need] < 0).any(dim=1)).nonzero().flatten()
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    n = user_table.size(0) if user_ids is None else user_ids.numel()
    u_lo, _ = shard_range(n, world, rank)
    mine = torch.tensor([bad.numel()], dtype=torch.int64, device=out_i.device)
    counts = _all_gather_rows(mine, [1] * world, group)
    cnt = [int(c) for c in counts.cpu()]
    global LAST_FALLBACK_USERS
    LAST_FALLBACK_USERS = sum(cnt)
    if sum(cnt) == 0:
        return out_s, out_i
    # exact fallback: plain per-shard top-k of every failed user, all_gathered
    pos = _all_gather_rows((bad + u_lo).to(torch.int64), cnt, group)
    fids = user_ids[pos] if user_ids is not None else pos
    fs, fi = local_topk(user_table, item_shard, k, user_ids=fids, item_base=lo,
                        init_thr=torch.full((len(pos),), -math.inf, dtype=torch.float32,
                                            device=out_s.device))
    gs = _all_gather_rows(fs.contiguous(), [len(pos)] * world, group).view(world, len(pos), k)
    gi = _all_gather_rows(fi.contiguous(), [len(pos)] * world, group).view(world, len(pos), k)
    off = sum(cnt[:rank])
    if bad.numel():
        ms, mi = merge(gs[:, off:off + bad.numel()].contiguous(),
                       gi[:, off:off + bad.numel()].contiguous(), k)
        out_s[bad], out_i[bad] = ms, mi
    return out_s, out_i


def sharded_score_topk(
    user_table: torch.Tensor,
    item_shard: torch.Tensor,
    item_base: int,
    k: int,
    user_ids: Optional[torch.Tensor] = None,
    group=None,
    local_topk: Optional[Callable[..., Partial]] = None,
    merge: Optional[Callable[[torch.Tensor, torch.Tensor, int], Partial]] = None,
    n_items: Optional[int] = None,
    global_thr: bool = False,
) -> Tuple[Partial, Tuple[int, int]]:
    """Top-k of this rank's user slice over the whole (sharded) catalog.
    ``global_thr`` (needs ``n_items``, the whole catalog's row count): shards
    keep only items above thresholds guessed from a sample of the whole
    catalog (thresholded_exchange); same result.

    Returns ((scores, items) for users [u_lo, u_hi), (u_lo, u_hi)); positions
    refer to ``user_ids`` if given, else to user rows 0..n-1. ``local_topk`` /
    ``merge`` default to the HIP kernels (divrec.ops.score_topk / topk_merge);
    they are injectable so the exchange logic is testable on CPU (gloo).
    """
    if local_topk is None or merge is None:
        from divrec import ops

        local_topk = local_topk or ops.score_topk
        merge = merge or ops.topk_merge
    if global_thr and (n_items is None or n_items < item_base + item_shard.size(0)):
        # checked before any collective: a failure on some ranks only, inside
        # the sequence of collectives, would leave the others waiting
        raise ValueError(f"global_thr needs n_items (the whole catalog's row count) >= "
                         f"item_base + shard rows = {item_base + item_shard.size(0)}, "
                         f"got {n_items}")
    world = 1 if group is _SOLO else dist.get_world_size(group)
    rank = 0 if group is _SOLO else dist.get_rank(group)
    n = user_table.size(0) if user_ids is None else user_ids.numel()
    if global_thr and world > 1:
        out = thresholded_exchange(user_table, item_shard, item_base,
                                   item_base + item_shard.size(0), n_items, k, group, user_ids,
                                   local_topk, merge)
        return out, shard_range(n, world, rank)
    s, i = local_topk(user_table, item_shard, k, user_ids=user_ids, item_base=item_base)
    if world == 1:
        return (s, i), (0, n)
    ps, pi = exchange_partials(s, i, group)
    out = merge(ps, pi, k)
    return out, shard_range(n, world, rank)
