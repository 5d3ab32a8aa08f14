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


class Comm:
    """The collectives of the exchange over one torch.distributed process group
    (RCCL over xGMI for device tensors; gloo exchanges host copies, for the CPU
    tests and the one-GPU multi-rank rehearsal). Every rank of the group must
    call each method in the same order. Any object with the same four members
    can stand in for it (tests run ranks as threads of one process)."""

    def __init__(self, group=None):
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)

    def _staged(self, x: torch.Tensor) -> bool:
        return x.is_cuda and dist.get_backend(self.group) == "gloo"

    def all_gather_rows(self, x: torch.Tensor, sizes) -> torch.Tensor:
        """Concatenate every rank's x (rank p holds sizes[p] rows) in rank order."""
        m = max(max(sizes), 1)
        staged = self._staged(x)
        src = x.cpu() if staged else x
        pad = torch.zeros((m,) + tuple(src.shape[1:]), dtype=src.dtype, device=src.device)
        pad[: src.shape[0]] = src
        outs = [torch.empty_like(pad) for _ in range(self.world)]
        dist.all_gather(outs, pad, group=self.group)
        out = torch.cat([o[: sizes[p]] for p, o in enumerate(outs)])
        return out.to(x.device) if staged else out

    def all_to_all_rows(self, x: torch.Tensor, in_splits, out_splits) -> torch.Tensor:
        """Rows [sum(in_splits[:p]), +in_splits[p]) of x go to rank p; the
        result holds out_splits[p] rows from every rank p, in rank order."""
        staged = self._staged(x)
        src = x.cpu() if staged else x
        out = torch.empty((sum(out_splits),) + tuple(src.shape[1:]), dtype=src.dtype,
                          device=src.device)
        dist.all_to_all_single(out, src, output_split_sizes=list(out_splits),
                               input_split_sizes=list(in_splits), group=self.group)
        return out.to(x.device) if staged else out

    def all_reduce_sum(self, t: torch.Tensor) -> torch.Tensor:
        staged = self._staged(t)
        src = t.cpu() if staged else t
        dist.all_reduce(src, group=self.group)
        return src.to(t.device) if staged else src


def as_comm(group) -> Any:
    """A Comm for a process group (None = the default group); a Comm-like
    object is returned as is."""
    return group if hasattr(group, "all_gather_rows") else Comm(group)


def exchange_partials(scores: torch.Tensor, items: torch.Tensor, group=None) -> Partial:
    """all_to_all of per-user partial top-k lists.

    Input: this rank's partial lists for ALL n users ([n, k] each).
    Output: [world, n_r, k] scores / items — the partial lists of this rank's
    user slice from every rank (row p = rank p's shard)."""
    comm = as_comm(group)
    world, rank = comm.world, comm.rank
    n, k = scores.shape
    packed = torch.stack([scores.view(torch.int32), items], dim=2).reshape(n, 2 * k).contiguous()
    in_splits = [shard_range(n, world, p)[1] - shard_range(n, world, p)[0] for p in range(world)]
    lo, hi = shard_range(n, world, rank)
    n_r = hi - lo
    out = comm.all_to_all_rows(packed, in_splits, [n_r] * world)
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
    t = as_comm(group).all_reduce_sum(t)
    return (t[0] / t[1]).to(torch.float32).to(values.device)


# --------------------------------------------------------------------------- global thresholds
# Each shard of a pure item sharding would otherwise keep its LOCAL top-k: a
# survivor stream of ~k (1 + ln(I_shard / k)) keys per user on every one of
# the S shards, where only ~k / S of each shard's items can reach the global
# top-k. So the ranks first agree on per-user thresholds guessed from a
# strided sample of the WHOLE catalog, with the single-device guess's rule
# (csrc/score_topk.hip guess_for): stride by catalog length, mu = k S / I of
# the user's true top k expected inside the sample, and two tiers:
#   1. the shards scan from the sample's ks1-th best score, ks1 = mu + 3 sigma
#      + 1 (about 0.1-0.4 % of users end with fewer than k merged items);
#   2. those users are rescanned on every shard from their safe threshold, the
#      sample's ks-th best, ks = mu + 6 sigma + 3 (the one-tier rule of round 2);
#   3. the users that fail the safe threshold too are rescanned from -inf.
# Every tier is verified after the merge (a user with fewer than k merged items
# failed it), so the result is the exact global top-k in every case.
GUESS_SIGMA = 6.0
GUESS_TAIL = 0.005  # first-tier rank: Poisson tail at most 0.5 % (csrc/score_topk.hip)
# Observability of the last thresholded_exchange call, summed over the ranks
# of its group (tests and the bench; not used by the path itself):
# LAST_FALLBACK_USERS = users whose first-tier guess failed (recomputed by a
# later tier); LAST_TIER_FAILURES = (first-tier, second-tier) failure counts.
LAST_FALLBACK_USERS = 0
LAST_TIER_FAILURES = (0, 0)


def sample_stride(n_items: int, k: int) -> int:
    """The sample stride of dr_score_topk's guess (csrc/score_topk.hip guess_for)."""
    st = 32
    while st < 128 and n_items // (2 * st) >= 65536:
        st *= 2
    return st


def guess_rank(k: int, frac: float) -> int:
    """Safe (second-tier) rank of the guess in the sample: mu + 6 sigma + 3."""
    mu = k * frac
    return min(k, int(math.ceil(mu + GUESS_SIGMA * math.sqrt(mu) + 3.0)))


def poisson_tail_rank(mu: float, tail: float = GUESS_TAIL) -> int:
    """Smallest j >= 1 with P(Poisson(mu) >= j) <= tail (score_topk.hip
    poisson_tail_rank: the same double-precision recurrence)."""
    pmf, cdf = math.exp(-mu), 0.0
    for j in range(1, 4096):
        cdf += pmf
        if 1.0 - cdf <= tail:
            return j
        pmf *= mu / j
    return 4096


def guess_ranks(k: int, frac: float) -> Tuple[int, int]:
    """(ks1, ks): the first-tier rank (the 0.5 % Poisson-tail rank of
    mu = k * frac, at most ks) and the safe rank, as guess_for computes them."""
    mu = k * frac
    ks = guess_rank(k, frac)
    return min(max(1, poisson_tail_rank(mu)), ks), ks


def threshold_below(kth: torch.Tensor) -> torch.Tensor:
    """A threshold strictly below each score (topk_threshold_kernel's rule);
    -inf where there is no finite score."""
    below = kth - torch.clamp(kth.abs() * 2.0 ** -20, min=2.0 ** -100)
    return torch.where(below < kth, below, torch.full_like(kth, -math.inf))


def _all_gather_rows(x: torch.Tensor, sizes, group) -> torch.Tensor:
    return as_comm(group).all_gather_rows(x, sizes)


def global_thresholds(user_table: torch.Tensor, item_shard: torch.Tensor, lo: int, hi: int,
                      n_items: int, k: int, group, user_ids: Optional[torch.Tensor] = None,
                      local_topk: Optional[Callable[..., Partial]] = None) -> torch.Tensor:
    """Per-user thresholds for all n users from a sample of the whole catalog:
    every rank contributes its shard's rows at global positions j * stride,
    the samples are all_gathered, each rank ranks ITS merge slice of users
    against them and the thresholds are all_gathered back. fp32 [2, n]: row 0
    the first tier (the shards' scan), row 1 the safe tier (the rescan of the
    users the first tier failed); -inf where the sample is too short.

    On the HIP kernels (no ``local_topk`` given) the ranking is
    dr_sample_thresholds: the single-GPU guess's tile-max sample scan, so the
    thresholds are lower bounds of the sample ranks. An injected
    ``local_topk`` (CPU tests) ranks the exact sample top-ks instead."""
    sample_thr = None
    if local_topk is None:
        from divrec import ops

        local_topk = ops.score_topk
        sample_thr = ops.sample_thresholds
    comm = as_comm(group)
    world, rank = comm.world, comm.rank
    st = sample_stride(n_items, k)
    j0 = -(-lo // st)  # first global sample position j * st inside [lo, hi)
    rows = item_shard[j0 * st - lo: hi - lo: st]
    # the shards may be any contiguous split: exchange the sample sizes first
    mine = torch.tensor([rows.size(0)], dtype=torch.int64, device=item_shard.device)
    sizes = [int(c) for c in comm.all_gather_rows(mine, [1] * world).cpu()]
    sample = comm.all_gather_rows(rows.contiguous(), sizes)
    n = user_table.size(0) if user_ids is None else user_ids.numel()
    u_lo, u_hi = shard_range(n, world, rank)
    # dr_sample_thresholds ranks the whole 32-row tiles of the sample only, and
    # guess_for takes mu from that rounded count: so does the HIP path here
    # (ADVICE r4), the two tiers then sit at the single-GPU guess's ranks
    n_s = sample.size(0) // 32 * 32 if sample_thr is not None else sample.size(0)
    ks1, ks = guess_ranks(k, n_s / n_items) if n_s else (0, 0)
    thr = torch.full((u_hi - u_lo, 2), -math.inf, dtype=torch.float32, device=user_table.device)
    if ks and u_hi > u_lo and n_s >= ks:
        ids = (user_ids[u_lo:u_hi] if user_ids is not None
               else torch.arange(u_lo, u_hi, device=user_table.device))
        if sample_thr is not None:
            thr = sample_thr(user_table, sample, ks1, ks, user_ids=ids).t().contiguous()
        else:
            s, _ = local_topk(user_table, sample, ks, user_ids=ids, item_base=0)
            thr[:, 0] = threshold_below(s[:, ks1 - 1].contiguous())
            thr[:, 1] = threshold_below(s[:, ks - 1].contiguous())
    usizes = [shard_range(n, world, p)[1] - shard_range(n, world, p)[0] for p in range(world)]
    return comm.all_gather_rows(thr, usizes).t().contiguous()


def _rescan(comm, user_table, item_shard, lo, k, user_ids, bad, u_lo, cnt, thr_all, merge,
            local_topk, out_s, out_i):
    """Recompute the users `bad` (this rank's merge-slice positions; cnt = every
    rank's count) on every shard from thresholds thr_all[position] (None:
    -inf), and merge their lists into out_s / out_i. Returns the positions
    (within bad) of users still left with fewer than k items."""
    world, rank = comm.world, comm.rank
    pos = comm.all_gather_rows((bad + u_lo).to(torch.int64), cnt)
    fids = user_ids[pos] if user_ids is not None else pos
    init = (torch.full((len(pos),), -math.inf, dtype=torch.float32, device=out_s.device)
            if thr_all is None else thr_all[pos].contiguous())
    fs, fi = local_topk(user_table, item_shard, k, user_ids=fids, item_base=lo, init_thr=init)
    gs = comm.all_gather_rows(fs.contiguous(), [len(pos)] * world).view(world, len(pos), k)
    gi = comm.all_gather_rows(fi.contiguous(), [len(pos)] * world).view(world, len(pos), k)
    off = sum(cnt[:rank])
    if bad.numel():
        ms, mi = merge(gs[:, off:off + bad.numel()].contiguous(),
                       gi[:, off:off + bad.numel()].contiguous(), k)
        out_s[bad], out_i[bad] = ms, mi


def _failed(out_i: torch.Tensor, rows: Optional[torch.Tensor], need: int) -> torch.Tensor:
    """Positions (of `rows`, or of every row) left with fewer than `need` items."""
    sel = out_i if rows is None else out_i[rows]
    f = (sel[:, :need] < 0).any(dim=1).nonzero().flatten()
    return f if rows is None else rows[f]


def thresholded_exchange(user_table: torch.Tensor, item_shard: torch.Tensor, lo: int, hi: int,
                         n_items: int, k: int, group, user_ids: Optional[torch.Tensor] = None,
                         local_topk: Optional[Callable[..., Partial]] = None,
                         merge: Optional[Callable[[torch.Tensor, torch.Tensor, int], Partial]] = None,
                         thr: Optional[torch.Tensor] = None,
                         local: Optional[Partial] = None) -> Partial:
    """Top-k of this rank's merge slice over the sharded catalog with global
    two-tier thresholds (computed here unless given, [2, n] as from
    global_thresholds; a [n] tensor is a one-tier guess): first-tier shard
    lists -> all_to_all -> merge -> verification; the users the first tier
    failed are rescanned on every shard from their safe thresholds and merged,
    and those that fail again from -inf, so the lists are exact (a user failed
    a tier when it is left with fewer than min(k, n_items) merged items)."""
    if local_topk is None or merge is None:
        from divrec import ops

        local_topk = local_topk or ops.score_topk
        merge = merge or ops.topk_merge
    comm = as_comm(group)
    if thr is None:
        thr = global_thresholds(user_table, item_shard, lo, hi, n_items, k, comm, user_ids,
                                local_topk)
    thr1, thr2 = (thr[0], thr[1]) if thr.dim() == 2 else (thr, None)
    if local is None:  # this shard's first-tier lists (the bench passes its timed call's)
        local = local_topk(user_table, item_shard, k, user_ids=user_ids, item_base=lo,
                           init_thr=thr1.contiguous())
    s, i = local
    ps, pi = exchange_partials(s, i, comm)
    out_s, out_i = merge(ps, pi, k)
    need = min(k, n_items)
    world, rank = comm.world, comm.rank
    n = user_table.size(0) if user_ids is None else user_ids.numel()
    u_lo, _ = shard_range(n, world, rank)
    dev = out_i.device

    def counts(x):
        c = comm.all_gather_rows(torch.tensor([x.numel()], dtype=torch.int64, device=dev),
                                 [1] * world)
        return [int(v) for v in c.cpu()]

    global LAST_FALLBACK_USERS, LAST_TIER_FAILURES
    bad = _failed(out_i, None, need)
    cnt = counts(bad)
    t1, t2 = sum(cnt), 0
    if t1 and thr2 is not None:  # second tier: the safe thresholds
        _rescan(comm, user_table, item_shard, lo, k, user_ids, bad, u_lo, cnt, thr2, merge,
                local_topk, out_s, out_i)
        bad = _failed(out_i, bad, need)
        cnt = counts(bad)
        t2 = sum(cnt)
    else:
        t2 = t1
    if t2:  # last tier: from -inf
        _rescan(comm, user_table, item_shard, lo, k, user_ids, bad, u_lo, cnt, None, merge,
                local_topk, out_s, out_i)
    LAST_FALLBACK_USERS = t1
    LAST_TIER_FAILURES = (t1, t2)
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
    comm = None if group is _SOLO else as_comm(group)
    world = 1 if comm is None else comm.world
    rank = 0 if comm is None else comm.rank
    n = user_table.size(0) if user_ids is None else user_ids.numel()
    if global_thr and world > 1:
        out = thresholded_exchange(user_table, item_shard, item_base,
                                   item_base + item_shard.size(0), n_items, k, comm, user_ids,
                                   local_topk, merge)
        return out, shard_range(n, world, rank)
    s, i = local_topk(user_table, item_shard, k, user_ids=user_ids, item_base=item_base)
    if world == 1:
        return (s, i), (0, n)
    ps, pi = exchange_partials(s, i, comm)
    out = merge(ps, pi, k)
    return out, shard_range(n, world, rank)
