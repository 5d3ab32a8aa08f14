"""The N>1 path (item-row shards + one all_to_all + merge) on CPU with gloo,
world_size 2 and 3: the per-rank merged lists must equal the single-process
top-k over the whole catalog. The local top-k / merge are injected from the
oracle (CPU checker); the exchange itself is the production code."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle
from divrec.distributed import exchange_partials, global_mean, shard_range, sharded_score_topk


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _local_topk(user_table, item_shard, k, user_ids=None, item_base=0):
    U = user_table.numpy() if user_ids is None else user_table.numpy()[user_ids.numpy()]
    items, scores = oracle.recommend_topk(U, item_shard.numpy(), k, return_scores=True)
    return torch.from_numpy(scores.astype(np.float32)), torch.from_numpy((items + item_base).astype(np.int32))


def _merge(ps, pi, k):
    s, i = oracle.topk_merge(ps.numpy(), pi.numpy(), k)
    return torch.from_numpy(s), torch.from_numpy(i.astype(np.int32))


def _worker(rank, world, port, U, I, k, user_ids, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        lo, hi = shard_range(I.shape[0], world, rank)
        (s, i), (ulo, uhi) = sharded_score_topk(torch.from_numpy(U), torch.from_numpy(I[lo:hi]), lo, k,
                                                user_ids=user_ids, local_topk=_local_topk, merge=_merge)
        q.put((rank, ulo, uhi, s.numpy(), i.numpy()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,n_users,user_ids", [(2, 37, False), (3, 20, True), (2, 1, False)])
def test_sharded_topk_equals_single_device(world, n_users, user_ids):
    rng = np.random.default_rng(world * 100 + n_users)
    U = rng.integers(-3, 4, size=(n_users + 5, 16)).astype(np.float32)   # integer scores: many ties
    I = rng.integers(-3, 4, size=(1001, 16)).astype(np.float32)
    k = 25
    uids = torch.from_numpy(rng.permutation(n_users + 5)[:n_users].astype(np.int64)) if user_ids else None
    Uq = U[uids.numpy()] if user_ids else U
    ref_i, ref_s = oracle.recommend_topk(Uq, I, k, return_scores=True)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, U, I, k, uids, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    seen = 0
    for rank, ulo, uhi, s, i in sorted(got):
        assert (ulo, uhi) == shard_range(Uq.shape[0], world, rank)
        assert np.array_equal(i, ref_i[ulo:uhi])
        assert np.array_equal(s, ref_s[ulo:uhi].astype(np.float32))
        seen += uhi - ulo
    assert seen == Uq.shape[0]


def _exchange_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        n, k = 7, 3
        s = torch.full((n, k), float(rank)) + torch.arange(n, dtype=torch.float32)[:, None] / 10
        i = torch.full((n, k), rank, dtype=torch.int32) * 1000 + torch.arange(n, dtype=torch.int32)[:, None]
        ps, pi = exchange_partials(s, i)
        q.put((rank, ps.numpy(), pi.numpy()))
    finally:
        dist.destroy_process_group()


def test_exchange_routes_user_slices():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_exchange_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict((r, (s, i)) for r, s, i in (q.get(timeout=120) for _ in range(world)))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(world):
        lo, hi = shard_range(7, world, r)
        s, i = got[r]
        assert s.shape == (world, hi - lo, 3)
        for src in range(world):   # row block `src` came from rank src, users lo..hi
            assert np.array_equal(i[src, :, 0], src * 1000 + np.arange(lo, hi))
            assert np.allclose(s[src, :, 0], src + np.arange(lo, hi) / 10)


def _grid_worker(rank, world, port, S, U, I, k, q):
    from divrec.distributed import grid_layout

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        lay = grid_layout(S)
        ulo, uhi = lay.user_range(U.shape[0])
        lo, hi = lay.item_range(I.shape[0])
        (s, i), (a, b) = sharded_score_topk(torch.from_numpy(U[ulo:uhi]), torch.from_numpy(I[lo:hi]),
                                            lo, k, group=lay.group, local_topk=_local_topk,
                                            merge=_merge)
        q.put((rank, lay.user_group, lay.item_shard, ulo + a, ulo + b, s.numpy(), i.numpy()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,S", [(4, 2), (4, 1), (4, 4), (2, 1)])
def test_grid_layout_equals_single_device(world, S):
    """(world/S) x S grid: users split over rows, item rows over the S ranks of a
    row, exchange inside the row only. Every user is owned by exactly one rank
    and its list equals the single-device top-k over the whole catalog."""
    rng = np.random.default_rng(world * 10 + S)
    U = rng.integers(-3, 4, size=(45, 16)).astype(np.float32)
    I = rng.integers(-3, 4, size=(803, 16)).astype(np.float32)
    k = 20
    ref_i, ref_s = oracle.recommend_topk(U, I, k, return_scores=True)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_grid_worker, args=(r, world, port, S, U, I, k, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = [q.get(timeout=180) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    owned = np.zeros(U.shape[0], dtype=int)
    for rank, ug, ish, a, b, s, i in got:
        assert (ug, ish) == (rank // S, rank % S)
        assert np.array_equal(i, ref_i[a:b])
        assert np.array_equal(s, ref_s[a:b].astype(np.float32))
        owned[a:b] += 1
    assert (owned == 1).all()


def _k1000_worker(rank, world, port, U, I, k, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from divrec.distributed import grid_layout
        lay = grid_layout(world)  # pure item sharding: S = world, the bench default
        lo, hi = lay.item_range(I.shape[0])
        (s, i), (ulo, uhi) = sharded_score_topk(torch.from_numpy(U), torch.from_numpy(I[lo:hi]), lo,
                                                k, group=lay.group, local_topk=_local_topk,
                                                merge=_merge)
        q.put((rank, ulo, uhi, s.numpy(), i.numpy()))
    finally:
        dist.destroy_process_group()


def test_item_sharded_8_ranks_k1000():
    """World size 8, pure 8-way item sharding (the north-star layout) at
    k = 1000 (config 5's candidate lists): the production exchange moves
    8 x 1000 partial entries per user; every user's merged list equals the
    single-device top-1000."""
    world, k = 8, 1000
    rng = np.random.default_rng(81000)
    U = rng.integers(-3, 4, size=(19, 8)).astype(np.float32)
    I = rng.integers(-3, 4, size=(8 * 1100 + 5, 8)).astype(np.float32)
    ref_i, ref_s = oracle.recommend_topk(U, I, k, return_scores=True)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_k1000_worker, args=(r, world, port, U, I, k, q))
             for r in range(world)]
    for p in procs:
        p.start()
    got = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    owned = np.zeros(U.shape[0], dtype=int)
    for rank, ulo, uhi, s, i in got:
        assert (ulo, uhi) == shard_range(U.shape[0], world, rank)
        assert np.array_equal(i, ref_i[ulo:uhi])
        assert np.array_equal(s, ref_s[ulo:uhi].astype(np.float32))
        owned[ulo:uhi] += 1
    assert (owned == 1).all()


def _mean_worker(rank, world, port, vals, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        lo, hi = shard_range(vals.size, world, rank)
        q.put((rank, float(global_mean(torch.from_numpy(vals[lo:hi])))))
    finally:
        dist.destroy_process_group()


def test_user_sharded_ild_mean():
    """Config 5's users sharded over ranks: the mean ILD from one all_reduce of
    (sum, count) equals the reference's 'mean' reduction (sum / size) over all
    users, uneven slices included."""
    world = 3
    vals = np.random.default_rng(5).random(1001).astype(np.float32)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_mean_worker, args=(r, world, port, vals, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want = float(oracle.reduce_values(vals, "mean"))
    for _, m in got:
        assert m == pytest.approx(want, rel=1e-6)


def _local_topk_thr(user_table, item_shard, k, user_ids=None, item_base=0, init_thr=None):
    """CPU checker of dr_score_topk_seeded: integer tables (exact scores); the
    top-k of the items scoring strictly above init_thr, padded with -1/-inf."""
    U = user_table.numpy() if user_ids is None else user_table.numpy()[user_ids.numpy()]
    S = U.astype(np.float64) @ item_shard.numpy().astype(np.float64).T
    if init_thr is not None:
        S = np.where(S > init_thr.numpy()[:, None].astype(np.float64), S, -np.inf)
    order = np.argsort(-S, axis=1, kind="stable")[:, :k]
    s = np.take_along_axis(S, order, axis=1)
    i = np.where(np.isfinite(s), order + item_base, -1)
    if s.shape[1] < k:  # shard shorter than k
        pad = k - s.shape[1]
        s = np.pad(s, ((0, 0), (0, pad)), constant_values=-np.inf)
        i = np.pad(i, ((0, 0), (0, pad)), constant_values=-1)
    return torch.from_numpy(s.astype(np.float32)), torch.from_numpy(i.astype(np.int32))


def _merge_pad(ps, pi, k):
    s, i = ps.numpy().astype(np.float64), pi.numpy().astype(np.int64)
    parts, n, kin = s.shape
    s = s.transpose(1, 0, 2).reshape(n, parts * kin)
    i = i.transpose(1, 0, 2).reshape(n, parts * kin)
    key_s = np.where(i >= 0, s, -np.inf)
    key_i = np.where(i >= 0, i, np.iinfo(np.int64).max)
    order = np.lexsort((key_i, -key_s), axis=1)[:, :k]
    so, io = np.take_along_axis(key_s, order, 1), np.take_along_axis(i, order, 1)
    io = np.where(np.isfinite(so), io, -1)
    return torch.from_numpy(so.astype(np.float32)), torch.from_numpy(io.astype(np.int32))


def _thr_worker(rank, world, port, U, I, k, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        lo, hi = shard_range(I.shape[0], world, rank)
        (s, i), (ulo, uhi) = sharded_score_topk(
            torch.from_numpy(U), torch.from_numpy(I[lo:hi]), lo, k, local_topk=_local_topk_thr,
            merge=_merge_pad, n_items=I.shape[0], global_thr=True)
        q.put((rank, ulo, uhi, s.numpy(), i.numpy()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,k,hot", [(2, 25, False), (3, 25, False), (4, 40, True)])
def test_sharded_topk_global_thresholds(world, k, hot):
    """Shards keep only items above per-user thresholds guessed from a sample
    of the whole catalog (every 32nd global row, all_gathered): the merged
    lists equal the single-process top-k. hot=True makes every sampled row
    every user's best item, so the guess fails for all users (32 hot items <
    k = 40 above the threshold) and the exact fallback recomputes them."""
    rng = np.random.default_rng(world * 7 + k)
    lo_v = 0 if hot else -3
    U = rng.integers(lo_v, 4, size=(45, 16)).astype(np.float32)
    I = rng.integers(-3, 4, size=(1001, 16)).astype(np.float32)
    if hot:
        I[::32] = 3.0
    ref_i, ref_s = oracle.recommend_topk(U, I, k, return_scores=True)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_thr_worker, args=(r, world, port, U, I, k, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    seen = 0
    for rank, ulo, uhi, s, i in sorted(got):
        assert np.array_equal(i, ref_i[ulo:uhi])
        assert np.array_equal(s, ref_s[ulo:uhi].astype(np.float32))
        seen += uhi - ulo
    assert seen == U.shape[0]


def _thr8_worker(rank, world, port, U, I, k, bounds, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from divrec import distributed
        from divrec.distributed import grid_layout

        lay = grid_layout(world)  # pure item sharding (S = world): bench.py's default at 8 GPUs
        lo, hi = bounds[rank], bounds[rank + 1]
        (s, i), (ulo, uhi) = sharded_score_topk(
            torch.from_numpy(U), torch.from_numpy(I[lo:hi]), lo, k, group=lay.group,
            local_topk=_local_topk_thr, merge=_merge_pad, n_items=I.shape[0], global_thr=True)
        q.put((rank, ulo, uhi, s.numpy(), i.numpy(), distributed.LAST_FALLBACK_USERS))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("hot", [False, True])
def test_item_sharded_8_ranks_global_thresholds_uneven(hot):
    """World size 8 with global thresholds (the default 8-GPU path), k = 100
    and an uneven contiguous item split (one shard shorter than k): merged
    lists equal the single-process top-k. hot=True puts 40 hot rows at the
    global sample positions (every 32nd row): the sample rank of the guess is
    17 < 40 < k, so every non-negative user fails the guess and is recomputed
    by the exact fallback."""
    world, k = 8, 100
    rng = np.random.default_rng(8100 + hot)
    U = np.concatenate([rng.integers(0, 4, size=(15, 16)),
                        rng.integers(-3, 4, size=(16, 16))]).astype(np.float32)
    I = rng.integers(-3, 4, size=(6007, 16)).astype(np.float32)
    if hot:
        I[np.arange(40) * 32] = 3.0
    bounds = [0, 40, 900, 1000, 2500, 2600, 4100, 5000, 6007]  # shard 0 has 40 < k rows
    ref_i, ref_s = oracle.recommend_topk(U, I, k, return_scores=True)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_thr8_worker, args=(r, world, port, U, I, k, bounds, q))
             for r in range(world)]
    for p in procs:
        p.start()
    got = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    owned = np.zeros(U.shape[0], dtype=int)
    fb = set()
    for rank, ulo, uhi, s, i, nfb in got:
        assert (ulo, uhi) == shard_range(U.shape[0], world, rank)
        assert np.array_equal(i, ref_i[ulo:uhi])
        assert np.array_equal(s, ref_s[ulo:uhi].astype(np.float32))
        owned[ulo:uhi] += 1
        fb.add(nfb)
    assert (owned == 1).all()
    assert len(fb) == 1 and ((fb.pop() >= 15) if hot else True)


def test_global_thresholds_need_n_items():
    """global_thr without the whole catalog's row count fails before any
    collective: a ValueError on every rank, not a hang."""
    with pytest.raises(ValueError, match="n_items"):
        sharded_score_topk(torch.zeros(3, 4), torch.zeros(10, 4), 0, 2, global_thr=True)
    with pytest.raises(ValueError, match="n_items"):
        sharded_score_topk(torch.zeros(3, 4), torch.zeros(10, 4), 5, 2, n_items=12, global_thr=True)


def test_two_tier_thresholds_8_thread_ranks():
    """The default 8-GPU path's two-tier guess (divrec.distributed.
    thresholded_exchange, the product function) with 8 ranks as threads of
    this process (tests/thread_comm.py) and the CPU checker top-k. k = 50 at
    sample stride 32: the first-tier rank in the sample is ks1 = 7, the safe
    rank ks = 13. Group A's best items are 8 hot rows at sample positions, so
    its first tier keeps only those 8 (fails) and its safe tier reaches past
    them (succeeds); group B's 20 hot rows defeat both tiers (the -inf
    rescan); group C passes the first tier. Lists equal the single-process
    top-k for every user; the tier counts show who took which tier."""
    from divrec import distributed as D
    from divrec.distributed import guess_ranks, sample_stride
    from thread_comm import ThreadHub

    world, k, d = 8, 50, 16
    rng = np.random.default_rng(2024)
    ni = 6007
    st = sample_stride(ni, k)
    assert st == 32 and guess_ranks(k, (ni // st + 1) / ni) == (7, 13)
    I = rng.integers(-3, 4, size=(ni, d)).astype(np.float32)
    I[:, 14:] = 0.0
    I[np.arange(8) * st, 15] = 100.0          # group A's hot rows
    I[np.arange(10, 30) * st, 14] = 100.0     # group B's hot rows
    U = rng.integers(-3, 4, size=(40, d)).astype(np.float32)
    U[:, 14:] = 0.0
    U[:12, 15] = 5.0   # group A
    U[12:20, 14] = 5.0  # group B
    bounds = [0, 40, 900, 1000, 2500, 2600, 4100, 5000, ni]  # shard 0 has 40 < k rows
    ref_i, ref_s = oracle.recommend_topk(U, I, k, return_scores=True)

    def rank_main(comm):
        lo, hi = bounds[comm.rank], bounds[comm.rank + 1]
        (s, i), (ulo, uhi) = sharded_score_topk(
            torch.from_numpy(U), torch.from_numpy(I[lo:hi]), lo, k, group=comm,
            local_topk=_local_topk_thr, merge=_merge_pad, n_items=ni, global_thr=True)
        return ulo, uhi, s.numpy(), i.numpy()

    got = ThreadHub(world).run(rank_main)
    owned = np.zeros(U.shape[0], dtype=int)
    for r, (ulo, uhi, s, i) in enumerate(got):
        assert (ulo, uhi) == shard_range(U.shape[0], world, r)
        assert np.array_equal(i, ref_i[ulo:uhi])
        assert np.array_equal(s, ref_s[ulo:uhi].astype(np.float32))
        owned[ulo:uhi] += 1
    assert (owned == 1).all()
    t1, t2 = D.LAST_TIER_FAILURES
    assert t1 >= 20 and 8 <= t2 < t1, D.LAST_TIER_FAILURES
    assert D.LAST_FALLBACK_USERS == t1


def test_thread_comm_matches_exchange_contract():
    """exchange_partials over the thread comm routes user slices as over gloo
    (test_exchange_routes_user_slices), so the thread harness is a faithful
    stand-in for the process group."""
    from thread_comm import ThreadHub

    world, n, k = 3, 7, 3

    def rank_main(comm):
        s = torch.full((n, k), float(comm.rank)) + torch.arange(n, dtype=torch.float32)[:, None] / 10
        i = torch.full((n, k), comm.rank, dtype=torch.int32) * 1000 + torch.arange(n, dtype=torch.int32)[:, None]
        return exchange_partials(s, i, comm)

    for r, (ps, pi) in enumerate(ThreadHub(world).run(rank_main)):
        lo, hi = shard_range(n, world, r)
        assert ps.shape == (world, hi - lo, k)
        for src in range(world):
            assert np.array_equal(pi[src, :, 0].numpy(), src * 1000 + np.arange(lo, hi))
