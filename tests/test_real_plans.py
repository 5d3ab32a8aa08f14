"""The scan plans the benchmark configurations actually run, pinned against an
exact reference.

dr_score_topk picks its plan from the call's shape (csrc/score_topk.hip
make_plan / guess_for): the sample stride of the guessed thresholds grows with
the catalog (32 below 4.2M rows, 64 from 4.2M, 128 from 8.4M), and a grid whose
last round would leave CUs idle splits its tail user blocks into catalog
chunks. The headline (BASELINE configs[3] at one GPU: 1M users x 10M items,
d = 128, k = 100) runs stride 128 with a 6-way split tail over 209 blocks;
config 2 (1M x 1M, d = 64) runs stride 32 unsplit over two rounds. These tests
run exactly those plans (asserted through dr_score_topk_plan) and compare the
lists with the exact top-k, the reference's get_model_recommendations
(/root/reference/divrec/train/utils.py:53-77) with its tie order fixed to
(score desc, item id asc).

Integer-valued tables make every score an exact integer in fp32 (|score| <=
9 d), so the lists AND scores must be bit-identical; the reference scores are
computed in float64 on the device (exact for these integers) and ranked by a
stable descending sort over ascending item ids, which is the key order.

* small shapes, planner knobs (dr_set_plan_knob): guess_stride 64 / 128 with
  scan_slots split plans, exclusions, duplicate user ids and "hot"
  sample rows that make the guess fail for a user group (device-counted
  rescan);
* full size: 1M x 10M d = 128 k = 100 and 1M x 1M d = 64 k = 100, the calls
  bench.py times, checked on ~1200 users drawn from head blocks, split-tail
  blocks and the last partial block, plus an exclusion run and a hot-row
  rescan group.
"""
import os

import numpy as np
import pytest
import torch

import oracle
from divrec import ops

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _Env(**kv):
    """Set planner knobs (dr_set_plan_knob, through divrec._backend.plan_knobs)
    for a block; None leaves a knob at its default."""
    from divrec import _backend
    return _backend.plan_knobs(**{k: v for k, v in kv.items() if v is not None})


def exact_topk_f64(U64: torch.Tensor, I64: torch.Tensor, k: int, frozen=None, block: int = 16):
    """Exact (score desc, id asc) top-k of the rows of U64 over I64 (float64
    device tensors holding integers: every score exact). frozen[r]: item ids
    excluded for row r (scored -inf). Returns (items int64 [n, k], scores
    float64 [n, k]) on the CPU."""
    outi, outs = [], []
    for b in range(0, U64.shape[0], block):
        S = U64[b:b + block] @ I64.T
        if frozen is not None:
            for r in range(S.shape[0]):
                f = frozen[b + r]
                if len(f):
                    S[r, torch.as_tensor(np.asarray(f, dtype=np.int64), device=S.device)] = -np.inf
        kth = torch.topk(S, k, dim=1).values[:, -1]
        for r in range(S.shape[0]):
            cand = torch.nonzero(S[r] >= kth[r]).flatten()  # ascending ids
            v, o = torch.sort(S[r, cand], descending=True, stable=True)
            outi.append(cand[o[:k]].cpu())
            outs.append(v[:k].cpu())
        del S
    return torch.stack(outi).numpy(), torch.stack(outs).numpy()


def _int_table_dev(n, d, seed, lo=-3, hi=3):
    g = torch.Generator(device=DEV).manual_seed(seed)
    return torch.randint(lo, hi + 1, (n, d), generator=g, device=DEV).to(torch.bfloat16)


def _check(users_tab, items_tab, it, s, rows, k, frozen=None, user_ids=None):
    """Compare output rows `rows` (positions) with the exact top-k."""
    sel = rows if user_ids is None else user_ids[rows]
    U64 = users_tab[torch.as_tensor(sel, device=DEV)].double()
    I64 = items_tab.double()
    fz = None if frozen is None else [frozen[r] for r in rows]
    ref_i, ref_s = exact_topk_f64(U64, I64, k, fz)
    del I64
    got_i = it[torch.as_tensor(rows, device=DEV)].cpu().numpy().astype(np.int64)
    got_s = s[torch.as_tensor(rows, device=DEV)].cpu().numpy()
    bad = np.nonzero((got_i != ref_i).any(axis=1))[0]
    assert bad.size == 0, f"{bad.size}/{len(rows)} users differ, first at position {rows[bad[0]]}"
    assert np.array_equal(got_s, ref_s.astype(np.float32))


# --------------------------------------------------------------------------- small shapes, forced plans
@pytest.mark.parametrize("d,stride,slots", [(128, 128, 3), (128, 64, 3), (64, 128, None),
                                            (64, 64, 2), (128, 128, None), (32, 64, 3)])
def test_forced_stride_split_rescan_exact(d, stride, slots):
    """Guess stride forced to 64 / 128 (the strides of >= 4.2M-row catalogs),
    with and without a split-tail plan: integer tables, exclusions of some
    users' best items, duplicate and permuted user ids, and 12 hot rows at
    sample positions j * stride that are the best items of every non-negative
    user (group A): the rank of the guess in the sample is < 12 for k = 50,
    so A's threshold is the hot score, only the 12 hot items pass it and every
    A user fails the guess and is rescanned. Lists and scores exact."""
    rng = np.random.default_rng(d * 1000 + stride + (slots or 0))
    upwg = 2048 if d <= 64 else 1024
    ni, k = (1 << 18) + 777, 50
    nu = (slots or 1) * upwg + 333  # slots + 1 user blocks: one full round + a split tail
    half = nu // 2
    U = np.concatenate([rng.integers(0, 4, size=(half, d)),
                        rng.integers(-3, 4, size=(nu - half, d))]).astype(np.float32)
    I = rng.integers(-3, 4, size=(ni, d)).astype(np.float32)
    I[np.arange(12) * stride] = 3.0  # hot sample rows
    users = np.concatenate([rng.permutation(nu), rng.integers(0, nu, 50)]).astype(np.int64)
    frozen = [rng.choice(ni, size=int(rng.integers(0, 25)), replace=False) for _ in users]
    for n in range(0, len(users), 53):  # exclude a hot row and some of the user's best items
        best = np.argsort(-(I @ U[users[n]]), kind="stable")[:8]
        frozen[n] = np.union1d(frozen[n], np.concatenate([best, [stride * 3]]))
    rowptr, cols = oracle.exclusion_csr(frozen)
    Ub, Ib = torch.from_numpy(U).to(DEV).to(torch.bfloat16), torch.from_numpy(I).to(DEV).to(torch.bfloat16)
    with _Env(guess_stride=stride, scan_slots=slots):
        plan = ops.score_topk_plan(len(users), ni, torch.bfloat16, d, k)
        s, it = ops.score_topk(Ub, Ib, k, user_ids=torch.from_numpy(users).to(DEV),
                               exclude=(torch.from_numpy(rowptr).to(DEV),
                                        torch.from_numpy(cols).to(DEV)))
    assert plan["sample_stride"] == stride and plan["sample_rank"] < 12
    if slots:
        assert plan["tail_chunks"] > 1 and plan["head_blocks"] > 0
    _check(Ub, Ib, it, s, np.arange(len(users)), k, frozen, users)


def test_forced_stride_k1000_split():
    """k = 1000 (config 5's candidate lists) at 2^18 rows samples at stride 32; forced
    to 64 with a split tail (long lists split in two): exact."""
    rng = np.random.default_rng(31337)
    d, ni, k = 128, (1 << 18) + 5, 1000
    nu = 3 * 1024 + 17
    U = rng.integers(-3, 4, size=(nu, d)).astype(np.float32)
    I = rng.integers(-3, 4, size=(ni, d)).astype(np.float32)
    Ub, Ib = torch.from_numpy(U).to(DEV).to(torch.bfloat16), torch.from_numpy(I).to(DEV).to(torch.bfloat16)
    with _Env(guess_stride=64, scan_slots=3):  # 4 blocks: 3 head + a split tail
        plan = ops.score_topk_plan(nu, ni, torch.bfloat16, d, k)
        s, it = ops.score_topk(Ub, Ib, k)
    assert plan["sample_stride"] == 64 and plan["tail_chunks"] == 2
    rows = np.concatenate([np.arange(0, nu, 29), [nu - 1]])
    _check(Ub, Ib, it, s, rows, k)


@pytest.mark.parametrize("d,k,nu", [(64, 100, 2 * 2048 + 700), (128, 1000, 3 * 1024 + 55),
                                    (128, 100, 5 * 1024 + 1)])
def test_second_tier_every_user_exact(d, k, nu):
    """The two-tier guess with the first tier forced almost useless
    (guess_z1 = -5: the main scan starts from the sample's best score or
    so): nearly every user fails the first tier and is recomputed by the
    second tier, whose device-side plan splits the many failing blocks over
    the grid and whose streaming finalize merges any number of keys per user
    (k = 1000: more than one 2048-key round). Exclusions of some users' best
    items; lists exact; the failure counts show who took which tier."""
    rng = np.random.default_rng(d + k + nu)
    ni = (1 << 18) + 5
    U = rng.integers(-3, 4, size=(nu, d)).astype(np.float32)
    I = rng.integers(-3, 4, size=(ni, d)).astype(np.float32)
    frozen = [rng.choice(ni, size=int(rng.integers(0, 20)), replace=False) for _ in range(nu)]
    for n in range(0, nu, 71):
        frozen[n] = np.union1d(frozen[n], np.argsort(-(I @ U[n]), kind="stable")[:12])
    rowptr, cols = oracle.exclusion_csr(frozen)
    Ub, Ib = torch.from_numpy(U).to(DEV).to(torch.bfloat16), torch.from_numpy(I).to(DEV).to(torch.bfloat16)
    st = {}
    with _Env(guess_z1=-5):
        s, it = ops.score_topk(Ub, Ib, k, exclude=(torch.from_numpy(rowptr).to(DEV),
                                                   torch.from_numpy(cols).to(DEV)), stats=st)
    t1, t2 = st["guess_failures"]
    assert t1 >= 0.9 * nu and t2 <= t1 // 10, st
    rows = np.unique(np.concatenate([np.arange(0, nu, 7), [nu - 1]]))
    _check(Ub, Ib, it, s, rows, k, frozen=frozen)


def test_second_tier_hot_rows_exact():
    """8 hot rows at stride-32 sample positions are the best items of a
    non-negative user group: the first-tier rank in the sample (ks1 = 7 for
    k = 50) is below 8, so the group fails the first tier; the safe rank
    (13) reaches 5 normal sample items past the hot rows, so the second tier
    succeeds for nearly all of them (a user with 5 of its top ~42 normal
    items in the sample, ~1 %, takes the -inf rescan). Lists exact."""
    rng = np.random.default_rng(1010)
    d, ni, k, nu = 64, (1 << 18) + 31, 50, 2 * 2048 + 99
    plan = ops.score_topk_plan(nu, ni, torch.bfloat16, d, k)
    assert plan["sample_stride"] == 32
    U = np.concatenate([rng.integers(0, 4, size=(nu // 2, d)),
                        rng.integers(-3, 4, size=(nu - nu // 2, d))]).astype(np.float32)
    I = rng.integers(-3, 4, size=(ni, d)).astype(np.float32)
    I[np.arange(8) * 32] = 3.0
    Ub, Ib = torch.from_numpy(U).to(DEV).to(torch.bfloat16), torch.from_numpy(I).to(DEV).to(torch.bfloat16)
    st = {}
    s, it = ops.score_topk(Ub, Ib, k, stats=st)
    t1, t2 = st["guess_failures"]
    assert t1 >= nu // 2 and t2 <= t1 // 10, st
    _check(Ub, Ib, it, s, np.arange(0, nu, 3), k)


# --------------------------------------------------------------------------- full size
def _sample_rows(rng, plan, n_users, n_head, n_tail, n_last):
    """Positions from head blocks, from split-tail blocks and from the last
    (partial) user block, plus every block boundary around the head/tail cut."""
    upwg = plan["users_per_wg"]
    head_end = min(plan["head_blocks"] * upwg, n_users)
    last0 = (plan["user_blocks"] - 1) * upwg
    rows = [rng.choice(head_end, n_head, replace=False)]
    if head_end < n_users:
        rows.append(head_end + rng.choice(last0 - head_end, n_tail, replace=False))
    rows.append(np.arange(max(last0, n_users - n_last), n_users))
    edge = [0, upwg - 1, upwg, head_end - 1, head_end, head_end + upwg - 1, last0 - 1, last0,
            n_users - 1]
    rows.append(np.asarray([e for e in edge if 0 <= e < n_users]))
    return np.unique(np.concatenate(rows))


def test_headline_plan_1m_x_10m_exact():
    """BASELINE configs[3] at one GPU, the call bench.py times: 1M users x 10M
    items, d = 128, k = 100 — stride-128 guess, 6-way split tail over the 209
    blocks of the 4th round. Integer tables generated on the device; 12 hot
    rows at sample positions are the best items of a non-negative user group
    spread over head and tail blocks (their guess fails: rescan). Checked: ~1200
    users from head blocks, tail blocks and the last partial block, and 200 of
    the hot group; then the same call with an exclusion CSR (the sampled users'
    best items excluded)."""
    U_n, I_n, d, k = 1_000_000, 10_000_000, 128, 100
    plan = ops.score_topk_plan(U_n, I_n, torch.bfloat16, d, k)
    assert (plan["sample_stride"], plan["tail_chunks"], plan["head_blocks"],
            plan["user_blocks"]) == (128, 6, 768, 977), plan
    rng = np.random.default_rng(2026)
    users = _int_table_dev(U_n, d, 11)
    items = _int_table_dev(I_n, d, 12)
    items[torch.arange(12, device=DEV) * 128] = 3.0
    hot = np.unique(rng.choice(U_n, 3000, replace=False))
    hot_t = torch.as_tensor(hot, device=DEV)
    users[hot_t] = users[hot_t].abs()  # non-negative rows: the hot items are their best
    s, it = ops.score_topk(users, items, k)
    rows = _sample_rows(rng, plan, U_n, 400, 500, 300)
    _check(users, items, it, s, rows, k)
    _check(users, items, it, s, rng.choice(hot, 200, replace=False), k)
    # exclusions: each sampled user loses its exact top-10 and 20 random items
    rows2 = rows[::3]
    ref_i, _ = exact_topk_f64(users[torch.as_tensor(rows2, device=DEV)].double(), items.double(), 10)
    frozen = [[] for _ in range(U_n)]
    for r, best in zip(rows2, ref_i):
        frozen[r] = np.union1d(best, rng.choice(I_n, 20, replace=False))
    rowptr, cols = oracle.exclusion_csr(frozen)
    s2, it2 = ops.score_topk(users, items, k, exclude=(torch.from_numpy(rowptr).to(DEV),
                                                       torch.from_numpy(cols).to(DEV)))
    _check(users, items, it2, s2, rows2, k, frozen=frozen)
    # users without exclusions get the same lists in the exclusion run
    rest = torch.as_tensor(np.setdiff1d(rows, rows2), device=DEV)
    assert torch.equal(it2[rest], it[rest]) and torch.equal(s2[rest], s[rest])


def test_config2_plan_1m_x_1m_d64_exact():
    """BASELINE configs[1], the call bench.py --workload score1m times: 1M x 1M,
    d = 64, k = 100 — stride-32 guess, 489 user blocks of 2048 (two rounds,
    unsplit). Integer tables; ~1200 users from both rounds and the last
    partial block, and a hot-row rescan group."""
    U_n, I_n, d, k = 1_000_000, 1_000_000, 64, 100
    plan = ops.score_topk_plan(U_n, I_n, torch.bfloat16, d, k)
    assert (plan["sample_stride"], plan["tail_chunks"], plan["user_blocks"]) == (32, 1, 489), plan
    rng = np.random.default_rng(64)
    users = _int_table_dev(U_n, d, 21)
    items = _int_table_dev(I_n, d, 22)
    # 20 hot rows at stride-32 sample positions; the guess's sample rank is 17
    items[torch.arange(20, device=DEV) * 32] = 3.0
    hot = np.unique(rng.choice(U_n, 3000, replace=False))
    hot_t = torch.as_tensor(hot, device=DEV)
    users[hot_t] = users[hot_t].abs()
    s, it = ops.score_topk(users, items, k)
    rows = np.unique(np.concatenate([_sample_rows(rng, plan, U_n, 500, 0, 300),
                                     256 * 2048 + rng.choice(U_n - 256 * 2048, 400, replace=False)]))
    _check(users, items, it, s, rows, k)
    _check(users, items, it, s, rng.choice(hot, 200, replace=False), k)


def test_configs3_eight_way_item_shards_full_size():
    """BASELINE configs[3] as bench.py --gpus 8 lays it out: the 10M-item
    catalog row-sharded 8 ways (1.25M rows per rank), run by the product
    function itself — divrec.distributed.sharded_score_topk(global_thr=True):
    global two-tier sample thresholds, dr_score_topk_seeded per shard, the
    all_to_all of partial lists, dr_topk_merge, verification and the tier-2 /
    -inf rescans — with the eight ranks as threads of this process on cuda:0
    (tests/thread_comm.py stands in for RCCL). Integer tables; 7 hot rows (+3)
    at global sample positions defeat group A's first tier (rank 5) but not
    its safe tier (rank 10); 12 hot rows (-3) defeat both tiers of the
    non-positive group B (the -inf rescan). Checked: the tier counts, and the
    merged lists of ~1000 users, both groups included, against the exact top-k
    of the whole catalog."""
    from divrec import distributed as D
    from thread_comm import ThreadHub

    U_n, I_n, d, k, S = 1_000_000, 10_000_000, 128, 100, 8
    rng = np.random.default_rng(8)
    users = _int_table_dev(U_n, d, 31)
    items = _int_table_dev(I_n, d, 32)
    st = D.sample_stride(I_n, k)
    assert st == ops.score_topk_plan(U_n, I_n, torch.bfloat16, d, k)["sample_stride"] == 128
    assert D.guess_ranks(k, (I_n // st) / I_n) == (5, 10)
    items[torch.arange(7, device=DEV) * st] = 3.0            # group A's hot rows (shard 0)
    items[torch.arange(20, 32, device=DEV) * st] = -3.0      # group B's hot rows
    grp = rng.choice(U_n, 2000, replace=False)
    ga, gb = np.sort(grp[:1000]), np.sort(grp[1000:])
    ga_t, gb_t = torch.as_tensor(ga, device=DEV), torch.as_tensor(gb, device=DEV)
    users[ga_t] = users[ga_t].abs()
    users[gb_t] = -users[gb_t].abs()
    torch.cuda.synchronize()

    def rank_main(comm):
        lo, hi = D.shard_range(I_n, S, comm.rank)
        (s, i), (ulo, uhi) = D.sharded_score_topk(users, items[lo:hi], lo, k, group=comm,
                                                  n_items=I_n, global_thr=True)
        return ulo, uhi, s, i

    got = ThreadHub(S).run(rank_main)
    torch.cuda.synchronize()
    t1, t2 = D.LAST_TIER_FAILURES
    assert t1 >= 2000 - 20 and 1000 - 10 <= t2 < t1 - 900, D.LAST_TIER_FAILURES
    assert [(a, b) for a, b, _, _ in got] == [D.shard_range(U_n, S, r) for r in range(S)]
    ms = torch.cat([g[2] for g in got])
    mi = torch.cat([g[3] for g in got])
    del got
    rows = np.unique(np.concatenate([rng.choice(U_n, 700, replace=False),
                                     rng.choice(ga, 150, replace=False),
                                     rng.choice(gb, 150, replace=False)]))
    _check(users, items, mi, ms, rows, k)


def test_config5_plan_1m_x_10m_k1000_then_mmr():
    """BASELINE configs[4] at one GPU, the calls bench.py --workload mmr times:
    the top-1000 scan of 1M users over the 10M-item catalog (d = 128; stride-128
    two-tier guess on the dense sample path, CAP 2048 with staged survivors,
    long-list flush) and the MMR re-rank of those 1000 candidates to 100 on
    the persistent grid. Integer tables; 60 hot rows at sample positions are
    the best items of a non-negative user group, whose first-tier (rank 17)
    and safe (rank 28) thresholds both fall inside the hot
    scores: the group goes through every tier down to the -inf rescan. Checked:
    ~600 users from head, split-tail and last blocks plus 100 of the hot group
    against the exact top-1000 (lists and scores); then MMR over all 1M lists:
    lambda = 1 equals each list's first 100 for every user, and at lambda = 0.5
    ~200 users spread over the grid (first users of their CU, prefetched users,
    the last round) replay as valid greedy steps in float64."""
    U_n, I_n, d, k = 1_000_000, 10_000_000, 128, 1000
    plan = ops.score_topk_plan(U_n, I_n, torch.bfloat16, d, k)
    assert (plan["sample_stride"], plan["cap"], plan["user_blocks"]) == (128, 2048, 977), plan
    assert (plan["first_tier_rank"], plan["sample_rank"]) == (17, 28), plan
    rng = np.random.default_rng(5005)
    users = _int_table_dev(U_n, d, 41)
    items = _int_table_dev(I_n, d, 42)
    items[torch.arange(60, device=DEV) * 128] = 3.0
    hot = np.unique(rng.choice(U_n, 1000, replace=False))
    hot_t = torch.as_tensor(hot, device=DEV)
    users[hot_t] = users[hot_t].abs()
    st = {}
    s, it = ops.score_topk(users, items, k, stats=st)
    t1, t2 = st["guess_failures"]
    assert t1 >= len(hot) and t2 >= len(hot) - 10, st
    rows = _sample_rows(rng, plan, U_n, 250, 200, 100)
    _check(users, items, it, s, rows, k)
    _check(users, items, it, s, rng.choice(hot, 100, replace=False), k)
    # MMR on the persistent grid over every user's real top-1000 list
    top = ops.mmr_rerank(it, s, items, 100, 1.0)
    assert torch.equal(top, it[:, :100])
    picks = ops.mmr_rerank(it, s, items, 100, 0.5).cpu().numpy()
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    sel = np.unique(np.concatenate([np.arange(0, 40), rng.choice(np.arange(cus, U_n - cus), 120,
                                                                  replace=False),
                                    np.arange(U_n - 40, U_n)]))
    sel_t = torch.as_tensor(sel, device=DEV)
    cand, sc = it[sel_t].cpu().numpy(), s[sel_t].cpu().numpy()
    # the replay needs only the selected users' candidate rows: ids remapped
    uniq = np.unique(cand)
    E = items[torch.as_tensor(uniq, device=DEV, dtype=torch.int64)].float().cpu().numpy()
    remap = lambda x: np.where(x >= 0, np.searchsorted(uniq, x), -1)  # noqa: E731
    from test_hip_kernels import _mmr_check_positions

    assert _mmr_check_positions(remap(picks[sel]), remap(cand), sc, E, 0.5, tol=1e-4) == 0


def test_bench_headline_own_tables_fp64():
    """The call bench.py times, on bench.py's own tables (N(0, 1/sqrt(d))
    bf16, seeded per 1M-row block; bench.gen_table), checked against float64
    with the gap-aware rule of test_score_topk_float_tolerance for ~1024
    users drawn from head, split-tail and last user blocks
    (bench.check_user_sample / bench.fp64_gap_check): every returned score
    within tol = 1e-5 sqrt(d/64) of its float64 value, the list sorted within
    tol, every item above the exact k-th score - 2 tol, and every item clearly
    inside the exact top-k (margin > 2 tol) returned. The integer-table plan
    tests above fix the same plan with exact scores; this one is the timed
    workload's own survivor and compaction dynamics."""
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench

    U_n, I_n, d, k = 1_000_000, 10_000_000, 128, 100
    U = bench.gen_table(U_n, d, 1, DEV)
    I = bench.gen_table(I_n, d, 2, DEV)
    plan = ops.score_topk_plan(U_n, I_n, torch.bfloat16, d, k)
    assert plan["tail_chunks"] > 1 and plan["sample_stride"] == 128  # the headline's plan
    s, i = ops.score_topk(U, I, k)
    sel = bench.check_user_sample(U_n, I_n, d, k, 1024)
    upw, head = plan["users_per_wg"], plan["head_blocks"]
    assert (sel < head * upw).sum() > 300 and (sel >= (plan["user_blocks"] - 1) * upw).sum() > 200
    res = bench.fp64_gap_check(U, I, s, i, sel, k)
    assert res["ok"], res
    assert res["users_checked"] >= 1000


def test_bpr_config3_full_size():
    """Config 3 at its BASELINE size: one
    pair_wise_train_loop-equivalent step (divrec/train/utils.py:144-152 with
    LogSigmoidDifferenceLoss, log_sigmoid_difference_loss.py:11-14) on two
    1M x 128 fp32 tables with 1,048,576 uniform triples, through the fused
    dr_bpr_fwd_bwd, against float64 on the device: the mean loss within rel
    1e-6; every AUC hit equal to (s_p >= s_n) except on float64 near-ties
    (|s_p - s_n| <= 1e-5), where fp32 summation order may flip it; both dense
    gradient tables (fp32 atomics, any order) within rel 1e-4 of float64
    index_add_ (the tolerance of test_bpr_fwd_bwd) everywhere; then one
    dr_adam_dense step equal to torch.optim.Adam on 4096 sampled rows of each
    table (atol 1e-6, the test_adam_dense_matches_torch bar)."""
    g = torch.Generator(device=DEV).manual_seed(33)
    n, d, B = 1_000_000, 128, 1 << 20
    U = torch.randn(n, d, generator=g, device=DEV) / d ** 0.5
    I = torch.randn(n, d, generator=g, device=DEV) / d ** 0.5
    uid = torch.randint(0, n, (B,), generator=g, device=DEV)
    pid = torch.randint(0, n, (B,), generator=g, device=DEV)
    nid = torch.randint(0, n, (B,), generator=g, device=DEV)
    gU = torch.zeros_like(U)
    gI = torch.zeros_like(I)
    loss, hit = ops.bpr_fwd_bwd(U, I, uid, pid, nid, 1.0 / B, gU, gI)

    Ud, Id = U.double(), I.double()
    u, p, q = Ud[uid], Id[pid], Id[nid]
    sp, sn = (u * p).sum(1), (u * q).sum(1)
    x = sp - sn
    ref_loss = torch.nn.functional.softplus(-x).mean()
    assert abs(loss.double().mean() - ref_loss) <= 1e-6 * abs(ref_loss)
    flip = (hit.bool() != (sp >= sn))
    assert not bool((flip & (x.abs() > 1e-5)).any())
    gcoef = (-torch.sigmoid(-x) / B).unsqueeze(1)
    # a user row's term g (p - n) may be formed as g p - g n in fp32: its
    # error scales with |g| (|p| + |n|), not with the (cancelling) difference
    tU, mU, tI = gcoef * (p - q), gcoef.abs() * (p.abs() + q.abs()), gcoef * u
    del p, q, u
    for got, idx, terms, mags in ((gU, (uid,), (tU,), (mU,)),
                                  (gI, (pid, nid), (tI, -tI), (tI.abs(), tI.abs()))):
        ref = torch.zeros_like(Ud)
        mag = torch.zeros_like(Ud)  # sum of |terms|: the scale of an fp32 sum's error
        for ix, t, a in zip(idx, terms, mags):
            ref.index_add_(0, ix, t)
            mag.index_add_(0, ix, a)
        err = (got.double() - ref).abs()
        # rel 1e-4 of the value, or 1e-5 of the terms' magnitude where the
        # terms cancel (a row's few fp32 adds in any order)
        assert bool((err <= torch.maximum(1e-4 * ref.abs(), 1e-5 * mag)).all()), float(err.max())
        del ref, mag, err
    del tU, mU, tI

    rows = torch.randperm(n, generator=g, device=DEV)[:4096]
    for P, G in ((U, gU), (I, gI)):
        ref = P[rows].clone().requires_grad_(True)
        ref.grad = G[rows].clone()
        opt = torch.optim.Adam([ref], lr=1e-3)
        opt.step()
        m, v = torch.zeros_like(P), torch.zeros_like(P)
        ops.adam_dense(P, G, m, v, 1e-3, 0.9, 0.999, 1e-8, 0.0, 1)
        assert torch.allclose(P[rows], ref.detach(), atol=1e-6, rtol=0)


def test_staged_scan_beyond_2_28_rows_exact():
    """A d = 32 bf16 (staged) scan of one unit longer than 2^28 rows: 64
    users over 2^28 + 4096 + 17 integer-valued item rows with the catalog
    split off (scan_split = 1), so a single workgroup's unit names tiles past
    2^23 (the old 23-bit staged-block field). A few planted hot rows sit
    past row 2^28 and near the end. Lists equal the exact top-k from a
    float64 scan of the same rows (integer tables: exact scores, ties broken
    by id)."""
    from divrec import _backend
    rng = np.random.default_rng(28)
    nu, ni, d, k = 64, (1 << 28) + 4096 + 17, 32, 10
    U = torch.from_numpy(rng.integers(-2, 3, size=(nu, d)).astype(np.float32)).to(DEV)
    g = torch.Generator(device=DEV).manual_seed(5)
    I = torch.randint(-1, 2, (ni, d), generator=g, device=DEV, dtype=torch.int8).to(torch.bfloat16)
    hot = torch.tensor([(1 << 28) + 5, (1 << 28) + 4000, ni - 1, 17], device=DEV)
    I[hot] = (U[:4] * 2).to(torch.bfloat16)  # user j's best possible row for j < 4
    Ub = U.to(torch.bfloat16)
    with _backend.plan_knobs(scan_split=1):
        s, i = ops.score_topk(Ub, I, k)
    best_s = torch.full((nu, k), -float("inf"), dtype=torch.float64, device=DEV)
    best_i = torch.zeros((nu, k), dtype=torch.int64, device=DEV)
    Ud = U.double()
    for c0 in range(0, ni, 1 << 24):
        S = Ud @ I[c0:c0 + (1 << 24)].double().T
        # ties by id ascending: the key (score, -id), scores integral
        key = S * (1 << 30) - torch.arange(c0, c0 + S.shape[1], device=DEV, dtype=torch.float64)
        kv, ki = torch.topk(key, k, dim=1)
        cand_i = torch.cat([best_i, ki + c0], 1)
        cand_k = torch.cat([best_s * (1 << 30) - best_i.double(), kv], 1)
        top = torch.topk(cand_k, k, dim=1).indices
        best_i = torch.gather(cand_i, 1, top)
        best_s = (Ud.unsqueeze(1) * I[best_i].double()).sum(-1)
    assert torch.equal(i.long(), best_i)
    assert torch.equal(s.double(), best_s)
    assert bool((i[:4, 0].long() == hot).all())
