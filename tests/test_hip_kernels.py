"""GPU parity tests: every C-ABI kernel against the CPU oracle on seeded inputs.

Integer and byte/index work is checked bit-exactly; floating point within the
tolerance stated next to each assertion. Inputs with
integer-valued embeddings make every score exact in fp32, so the top-K tests
on them are bit-exact including ties (tie-break: score desc, item id asc).
"""
import numpy as np
import pytest
import torch

import oracle
from divrec import _backend, ops
from topk_checks import fp32_row_tol, gap_check

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _int_table(rng, n, d, lo=-3, hi=3):
    return rng.integers(lo, hi + 1, size=(n, d)).astype(np.float32)


def _bf16(x):
    return torch.from_numpy(x).to(DEV).to(torch.bfloat16)


# --------------------------------------------------------------------------- gather_dot
@pytest.mark.parametrize("d", [32, 64, 96, 128, 256])
@pytest.mark.parametrize("dtype", ["f32", "bf16"])
def test_gather_dot(d, dtype):
    rng = np.random.default_rng(d)
    U = rng.standard_normal((300, d)).astype(np.float32)
    I = rng.standard_normal((500, d)).astype(np.float32)
    if dtype == "bf16":
        U, I = oracle.as_bf16_f32(U), oracle.as_bf16_f32(I)
    n = 5003
    uid = rng.integers(0, 300, n)
    iid = rng.integers(0, 500, n)
    tdt = torch.float32 if dtype == "f32" else torch.bfloat16
    got = ops.gather_dot(
        torch.from_numpy(U).to(DEV).to(tdt), torch.from_numpy(I).to(DEV).to(tdt),
        torch.from_numpy(uid).to(DEV), torch.from_numpy(iid).to(DEV),
    ).cpu().numpy()
    ref = oracle.mf_forward(U, I, uid, iid)
    # tolerance: fp32 sum-order difference, |err| <= 4e-7 * d * max|u*i|
    scale = np.abs(U[uid] * I[iid]).max(axis=1) * d
    assert np.all(np.abs(got - ref) <= 4e-7 * scale + 1e-6)


def test_gather_dot_integer_exact():
    rng = np.random.default_rng(7)
    U, I = _int_table(rng, 50, 128), _int_table(rng, 70, 128)
    uid, iid = rng.integers(0, 50, 999), rng.integers(0, 70, 999)
    got = ops.gather_dot(torch.from_numpy(U).to(DEV), torch.from_numpy(I).to(DEV),
                         torch.from_numpy(uid).to(DEV), torch.from_numpy(iid).to(DEV))
    assert np.array_equal(got.cpu().numpy(), oracle.mf_forward(U, I, uid, iid))


def _run_ids(rng, n, n_rows, max_run):
    """Ids in runs of random length 1..max_run (runs straddle every unroll
    and span boundary of the gather)."""
    out = []
    while len(out) < n:
        out += [int(rng.integers(0, n_rows))] * int(rng.integers(1, max_run + 1))
    return np.asarray(out[:n], dtype=np.int64)


@pytest.mark.parametrize("pattern", ["full", "mxm", "runs"])
@pytest.mark.parametrize("d,dtype", [(100, "f32"), (128, "f32"), (64, "bf16"), (100, "bf16"),
                                     (256, "bf16")])
def test_gather_dot_run_patterns(pattern, d, dtype):
    """The reference's own call patterns, whose repeated rows the gather reads
    once per run: RankingDataset's (torch.full((n,), u), candidates)
    (base_datasets.py:165-171), PairWiseDataset's m x m product, model(u, pos)
    and model(u, neg) (:94-107), and random run lengths. Same tolerance as
    test_gather_dot."""
    rng = np.random.default_rng(d + len(pattern))
    nu, ni = 300, 4000
    U = rng.standard_normal((nu, d)).astype(np.float32)
    I = rng.standard_normal((ni, d)).astype(np.float32)
    if dtype == "bf16":
        U, I = oracle.as_bf16_f32(U), oracle.as_bf16_f32(I)
    if pattern == "full":
        uid = np.full(ni - 37, 7, dtype=np.int64)
        iid = np.setdiff1d(np.arange(ni), rng.choice(ni, 37, replace=False)).astype(np.int64)
    elif pattern == "mxm":
        m, users = 20, rng.choice(nu, 97, replace=False)
        pos = rng.integers(0, ni, (97, m))
        neg = rng.integers(0, ni, (97, m))
        uid = np.repeat(users, m * m)
        iid = np.concatenate([np.repeat(pos, m, axis=1).ravel(),  # model(u, pos): p_a m times
                              np.tile(neg, (1, m)).ravel()])      # model(u, neg): cycling
        uid = np.concatenate([uid, uid])
    else:
        n = 50_003
        uid, iid = _run_ids(rng, n, nu, 9), _run_ids(rng, n, ni, 5)
    tdt = torch.float32 if dtype == "f32" else torch.bfloat16
    got = ops.gather_dot(torch.from_numpy(U).to(DEV).to(tdt), torch.from_numpy(I).to(DEV).to(tdt),
                         torch.from_numpy(uid).to(DEV), torch.from_numpy(iid).to(DEV)).cpu().numpy()
    ref = oracle.mf_forward(U, I, uid, iid)
    scale = np.abs(U[uid] * I[iid]).max(axis=1) * d
    assert np.all(np.abs(got - ref) <= 4e-7 * scale + 1e-6)


def test_ids_out_of_range_raise_index_error():
    """nn.Embedding / tensor indexing raise IndexError on an id outside the
    table (the reference's behaviour); the kernels never read such a row:
    gather_dot, the MF forward on host and device ids, the fused BPR step,
    the training loop and the three ILD modes."""
    from divrec import _backend, models
    rng = np.random.default_rng(0)
    U = torch.from_numpy(rng.standard_normal((10, 32)).astype(np.float32)).to(DEV)
    I = torch.from_numpy(rng.standard_normal((20, 32)).astype(np.float32)).to(DEV)
    ok = torch.arange(5, device=DEV)
    for bad_u, bad_i in (([0, 10, 2, 3, 4], ok), (ok, [0, 1, -1, 3, 4]), (ok, [0, 1, 2, 3, 20])):
        bu = torch.as_tensor(bad_u, device=DEV)
        bi = torch.as_tensor(bad_i, device=DEV)
        with pytest.raises(IndexError):
            ops.gather_dot(U, I, bu, bi)
        with pytest.raises(IndexError):
            ops.bpr_fwd_bwd(U, I, bu, bi, ok, 0.2, torch.zeros_like(U), torch.zeros_like(I))
    err = _backend.error_counter(torch.device(DEV))
    out = ops.gather_dot(U, I, torch.tensor([0, 10, 2], device=DEV),
                         torch.tensor([0, 1, 2], device=DEV), err=err, check=False)
    assert int(err.item()) == 1 and torch.isnan(out[1]) and not torch.isnan(out[[0, 2]]).any()
    gU, gI = torch.zeros_like(U), torch.zeros_like(I)
    ops.bpr_fwd_bwd(U, I, torch.tensor([0, 99], device=DEV), torch.tensor([1, 1], device=DEV),
                    torch.tensor([2, 2], device=DEV), 1.0, gU, gI, err=err, check=False)
    assert int(err.item()) == 2 and not gU[1:].any()  # the bad triple added nothing
    mf = models.MatrixFactorization(10, 20, 32).to(DEV)
    for uid, iid in (([0, 10], [0, 1]), ([0, 1], [0, 25])):
        with pytest.raises(IndexError):  # host ids: checked before the upload
            mf(torch.LongTensor(uid), torch.LongTensor(iid))
        with pytest.raises(IndexError):  # device ids: checked by the kernel
            mf(torch.tensor(uid, device=DEV), torch.tensor(iid, device=DEV))
    recs = torch.tensor([[0, 1, 2], [3, -1, 4]], device=DEV)
    with pytest.raises(IndexError):
        ops.ild_dense(recs, torch.rand(20, 20, device=DEV))
    with pytest.raises(IndexError):
        ops.ild_dense(recs, torch.randint(0, 5, (20, 20), device=DEV))
    with pytest.raises(IndexError):
        ops.ild_labels(recs, torch.randint(0, 3, (20,), device=DEV))
    with pytest.raises(IndexError):
        ops.ild_embedding(recs, I.to(torch.bfloat16))
    vals = ops.ild_embedding(recs, I.to(torch.bfloat16), check=False)
    assert not torch.isnan(vals[0]) and torch.isnan(vals[1])


@pytest.mark.parametrize("d", [32, 64, 100, 128, 300])
def test_gather_dot_backward(d):
    rng = np.random.default_rng(3 + d)
    U = rng.standard_normal((40, d)).astype(np.float32)
    I = rng.standard_normal((60, d)).astype(np.float32)
    uid, iid = rng.integers(0, 40, 2000), rng.integers(0, 60, 2000)
    go = rng.standard_normal(2000).astype(np.float32)
    gU = torch.zeros(40, d, device=DEV)
    gI = torch.zeros(60, d, device=DEV)
    ops.gather_dot_backward(torch.from_numpy(U).to(DEV), torch.from_numpy(I).to(DEV),
                            torch.from_numpy(uid).to(DEV), torch.from_numpy(iid).to(DEV),
                            torch.from_numpy(go).to(DEV), gU, gI)
    rU = np.zeros((40, d)); np.add.at(rU, uid, go[:, None].astype(np.float64) * I[iid])
    rI = np.zeros((60, d)); np.add.at(rI, iid, go[:, None].astype(np.float64) * U[uid])
    assert np.allclose(gU.cpu().numpy(), rU, rtol=1e-4, atol=1e-4)
    assert np.allclose(gI.cpu().numpy(), rI, rtol=1e-4, atol=1e-4)


# --------------------------------------------------------------------------- score_topk
@pytest.mark.parametrize("d", [32, 64, 128, 256, 512])  # 512: the compacting plan (no CAP-2048 instance)
@pytest.mark.parametrize("k", [1, 10, 100])
def test_score_topk_integer_exact(d, k):
    rng = np.random.default_rng(1000 * d + k)
    nu, ni = 37 + d, 2000 + 13  # partial user block, partial item tile
    U, I = _int_table(rng, nu, d), _int_table(rng, ni, d)
    s, it = ops.score_topk(_bf16(U), _bf16(I), k)
    ref_i, ref_s = oracle.recommend_topk(U, I, k, return_scores=True)
    assert np.array_equal(it.cpu().numpy().astype(np.int64), ref_i)
    assert np.array_equal(s.cpu().numpy(), ref_s)


def test_score_topk_ties_exact():
    # values in {-1, 0, 1} at d=32: massive ties; order must be score desc, id asc
    rng = np.random.default_rng(11)
    U, I = _int_table(rng, 70, 32, -1, 1), _int_table(rng, 3000, 32, -1, 1)
    s, it = ops.score_topk(_bf16(U), _bf16(I), 100)
    ref_i = oracle.recommend_topk(U, I, 100)
    assert np.array_equal(it.cpu().numpy().astype(np.int64), ref_i)


def test_score_topk_user_ids_and_item_base():
    rng = np.random.default_rng(5)
    U, I = _int_table(rng, 300, 64), _int_table(rng, 4000, 64)
    users = np.array([299, 0, 17, 17, 150], dtype=np.int64)
    s, it = ops.score_topk(_bf16(U), _bf16(I), 20, user_ids=torch.from_numpy(users).to(DEV),
                           item_base=1_000_000)
    ref_i = oracle.recommend_topk(U, I, 20, users=users)
    assert np.array_equal(it.cpu().numpy().astype(np.int64) - 1_000_000, ref_i)


def test_score_topk_exclusion_exact():
    rng = np.random.default_rng(9)
    nu, ni, d, k = 130, 3000, 64, 50
    U, I = _int_table(rng, nu, d), _int_table(rng, ni, d)
    frozen = [rng.choice(ni, size=rng.integers(0, 400), replace=False) for _ in range(nu)]
    # make some excluded items the best ones (worst case for the threshold)
    for u in range(0, nu, 3):
        best = np.argsort(-(I @ U[u]), kind="stable")[:30]
        frozen[u] = np.union1d(frozen[u], best)
    rowptr, cols = oracle.exclusion_csr(frozen)
    s, it = ops.score_topk(_bf16(U), _bf16(I), k,
                           exclude=(torch.from_numpy(rowptr).to(DEV), torch.from_numpy(cols).to(DEV)))
    ref_i = oracle.recommend_topk(U, I, k, frozen=frozen)
    assert np.array_equal(it.cpu().numpy().astype(np.int64), ref_i)


def test_score_topk_chunked_catalog_exact():
    # large catalog, few users: the planner splits items into chunks and merges
    rng = np.random.default_rng(21)
    U, I = _int_table(rng, 40, 32), _int_table(rng, 300_001, 32)
    s, it = ops.score_topk(_bf16(U), _bf16(I), 100)
    ref_i, ref_s = oracle.recommend_topk(U, I, 100, return_scores=True)
    assert np.array_equal(it.cpu().numpy().astype(np.int64), ref_i)
    assert np.array_equal(s.cpu().numpy(), ref_s)


def test_score_topk_guess_rescan_exact():
    """Catalogs >= 2^18 rows start from a threshold guessed on a strided sample
    (every 32nd row) and rescan users the guess failed. Here the sampled rows
    0, 32, ... 608 are "hot": the best items of every non-negative user (group
    A). The guess's rank in the sample is ks = 13 for k = 50, so A's guessed
    threshold is the hot score, it admits only those 20 items (< k) and all of A must be
    rescanned; non-positive users (group B) rank them last and are not. With
    duplicate / permuted user ids and exclusions (some hot items excluded)
    the lists must equal the oracle's exactly."""
    rng = np.random.default_rng(77)
    d, ni, k = 64, (1 << 18) + 123, 50
    U = np.concatenate([_int_table(rng, 48, d, 0, 3), _int_table(rng, 48, d, -3, 0)])
    I = _int_table(rng, ni, d)
    I[np.arange(20) * 32] = 3.0  # hot sample rows
    users = np.concatenate([rng.permutation(96), rng.integers(0, 96, 24)]).astype(np.int64)
    frozen = [rng.choice(ni, size=rng.integers(0, 50), replace=False) for _ in users]
    for n in range(0, len(users), 4):
        frozen[n] = np.union1d(frozen[n], [0, 64, 288])
    rowptr, cols = oracle.exclusion_csr(frozen)
    s, it = ops.score_topk(_bf16(U), _bf16(I), k, user_ids=torch.from_numpy(users).to(DEV),
                           exclude=(torch.from_numpy(rowptr).to(DEV), torch.from_numpy(cols).to(DEV)))
    ref_i, ref_s = oracle.recommend_topk(U, I, k, users=users, frozen=frozen, return_scores=True)
    assert np.array_equal(it.cpu().numpy().astype(np.int64), ref_i)
    assert np.array_equal(s.cpu().numpy(), ref_s)


@pytest.mark.parametrize("nu,ni,d,k,dtype", [(300, 300, 64, 600, "bf16"), (70, 2048, 128, 100, "f32"),
                                            (16384, 1000, 32, 20, "bf16"), (500, 1, 64, 5, "f32")])
def test_score_topk_small_catalog_keeps_every_key(nu, ni, d, k, dtype):
    """Small catalogs keep every key (round 6: CAP >= n_items, no compaction,
    the finalize sorts all of them): k above the catalog (the list's tail is
    item -1 / score -inf), exactly 2048 rows, the 16384-user bound, a
    one-row catalog; best items excluded for some users. Exact against the
    oracle (integer tables)."""
    rng = np.random.default_rng(nu + ni + k)
    U, I = _int_table(rng, nu, d), _int_table(rng, ni, d)
    t = _f32 if dtype == "f32" else _bf16
    plan = ops.score_topk_plan(nu, ni, torch.float32 if dtype == "f32" else torch.bfloat16, d, k)
    assert plan["cap"] >= ni and plan["head_keys"] >= max(ni, k)
    sel = np.unique(np.concatenate([np.arange(0, nu, max(1, nu // 97)), [nu - 1]]))
    frozen = [np.zeros(0, np.int64) for _ in range(nu)]
    for n in sel[::3]:
        frozen[n] = np.argsort(-(I @ U[n]), kind="stable")[:min(5, ni - 1)]
    rowptr, cols = oracle.exclusion_csr(frozen)
    s, it = ops.score_topk(t(U), t(I), k, exclude=(torch.from_numpy(rowptr).to(DEV),
                                                 torch.from_numpy(cols).to(DEV)))
    got_i, got_s = it.cpu().numpy()[sel], s.cpu().numpy()[sel]
    for r, n in enumerate(sel):  # one user at a time: list lengths differ when k > candidates
        ref_i, ref_s = oracle.recommend_topk(U, I, k, users=[n], frozen=[frozen[n]],
                                             return_scores=True)
        m = ref_i.shape[1]  # min(k, candidates)
        assert np.array_equal(got_i[r, :m].astype(np.int64), ref_i[0])
        assert np.array_equal(got_s[r, :m], ref_s[0])
        assert (got_i[r, m:] == -1).all() and np.isneginf(got_s[r, m:]).all()


@pytest.mark.parametrize("k,d,dtype,slots", [(1, 128, "bf16", None), (2, 64, "bf16", 2),
                                           (5, 32, "f32", None), (1, 64, "f32", 2)])
def test_score_topk_guess_small_k_exact(k, d, dtype, slots):
    """The guessed-threshold path at the smallest list lengths (k = 1, 2, 5:
    the sample's safe rank ks is clipped to k, the first-tier rank to ks),
    bf16 and fp32 tables, with and without a split plan (scan_slots), users
    whose single best item is excluded, and duplicate user ids: lists and
    scores equal the oracle's (integer tables: exact scores, ties by id)."""
    rng = np.random.default_rng(k * 100 + d)
    ni = (1 << 18) + 77
    nu = 2 * (2048 if d <= 64 else 1024) + 35 if slots else 150
    U, I = _int_table(rng, nu, d), _int_table(rng, ni, d)
    users = np.concatenate([rng.permutation(nu), rng.integers(0, nu, 20)]).astype(np.int64)
    sel = np.arange(0, len(users), max(1, len(users) // 120))  # the users checked
    frozen = [np.zeros(0, np.int64) for _ in users]
    for n in sel[::2]:
        frozen[n] = np.argsort(-(I @ U[users[n]]), kind="stable")[:3]  # the best 3 excluded
    rowptr, cols = oracle.exclusion_csr(frozen)
    t = _f32 if dtype == "f32" else _bf16
    knobs = {"scan_slots": slots} if slots else {}
    with _backend.plan_knobs(**knobs):
        plan = ops.score_topk_plan(len(users), ni, torch.float32 if dtype == "f32" else torch.bfloat16,
                                   d, k)
        s, it = ops.score_topk(t(U), t(I), k, user_ids=torch.from_numpy(users).to(DEV),
                               exclude=(torch.from_numpy(rowptr).to(DEV),
                                        torch.from_numpy(cols).to(DEV)))
    assert plan["sample_stride"] > 0 and plan["sample_rank"] == k
    if slots:
        assert plan["tail_chunks"] > 1
    ref_i, ref_s = oracle.recommend_topk(U, I, k, users=users[sel], frozen=[frozen[n] for n in sel],
                                         return_scores=True)
    assert np.array_equal(it.cpu().numpy()[sel].astype(np.int64), ref_i)
    assert np.array_equal(s.cpu().numpy()[sel], ref_s)


@pytest.mark.parametrize("d", [32, 64, 128])
def test_score_topk_many_workgroups_exact(d):
    """More users than one workgroup holds (2048 at d <= 64, 1024 at d = 128):
    several user blocks, the last one partial."""
    rng = np.random.default_rng(500 + d)
    nu, ni, k = 4100 + d, 1500 + 7, 10
    U, I = _int_table(rng, nu, d), _int_table(rng, ni, d)
    s, it = ops.score_topk(_bf16(U), _bf16(I), k)
    ref_i, ref_s = oracle.recommend_topk(U, I, k, return_scores=True)
    assert np.array_equal(it.cpu().numpy().astype(np.int64), ref_i)
    assert np.array_equal(s.cpu().numpy(), ref_s)


def _exact_topk_torch(U, I, k, block=256):
    """Integer-valued tables: fp32 scores are exact, so a stable descending
    sort over ascending item ids IS the (score desc, id asc) order. Used where
    the per-user oracle loop would take minutes; it is pinned to the oracle by
    test_score_topk_integer_exact's cases."""
    Ud = torch.from_numpy(U).to(DEV)
    Id = torch.from_numpy(I).to(DEV)
    outs, outi = [], []
    for b in range(0, Ud.shape[0], block):
        S = Ud[b:b + block] @ Id.T
        v, i = torch.sort(S, dim=1, descending=True, stable=True)
        outs.append(v[:, :k].cpu())
        outi.append(i[:, :k].cpu())
    return torch.cat(outi).numpy().astype(np.int64), torch.cat(outs).numpy()


@pytest.mark.parametrize("d", [32, 64, 128])
def test_score_topk_nan_rows_never_ranked(d):
    """Item rows holding NaN (a NaN score for every user): the hot test's
    maximum propagates NaN and counts it as a hit, the exact per-score tests
    behind it never admit a NaN score, so NaN items are never recommended and
    every other list is the exact top-k of the finite items (round 5; the
    round-4 maxNum test skipped NaN the same way). The reference would sort
    NaN scores with argsort (divrec/train/utils.py:73): a documented
    divergence. 300K rows: the guessed-threshold path,
    with NaN rows at sample positions too."""
    rng = np.random.default_rng(300 + d)
    nu, ni, k = 3000, 300_011, 50
    U = _int_table(rng, nu, d)
    I = _int_table(rng, ni, d)
    bad = np.unique(np.concatenate([np.arange(0, 40) * 32, rng.choice(ni, 200, replace=False)]))
    I[bad, d // 2] = np.nan
    s, it = ops.score_topk(_bf16(U), _bf16(I), k)
    it = it.cpu().numpy().astype(np.int64)
    assert not np.isin(it, bad).any()
    Ifin = I.copy()
    Ifin[bad] = 0.0
    ref_i, ref_s = _exact_topk_torch(U, Ifin, k + len(bad))
    # the finite items' order: drop the zeroed NaN rows from the exact lists
    keep = ~np.isin(ref_i, bad)
    exp_i = np.stack([r[m][:k] for r, m in zip(ref_i, keep)])
    exp_s = np.stack([r[m][:k] for r, m in zip(ref_s, keep)])
    assert np.array_equal(it, exp_i)
    assert np.array_equal(s.cpu().numpy(), exp_s)


@pytest.mark.parametrize("d", [64, 128])
def test_score_topk_guess_rescan_many_units_exact(d):
    """Every user fails the guess (hot sampled rows) and there are more of
    them than one workgroup holds: the device-counted rescan runs several
    user blocks, the last one partial, and writes each list to its position."""
    rng = np.random.default_rng(88 + d)
    ni, k = (1 << 18) + 77, 20
    nu = 2 * (2048 if d <= 64 else 1024) + 333
    U = _int_table(rng, nu, d, 0, 3)
    I = _int_table(rng, ni, d)
    # 12 hot sample rows: the best items of every (non-negative) user. The
    # guess's rank in the sample is ks = ceil(mu + 6 sqrt(mu) + 3) = 9 for
    # k = 20 (mu = k / 32), so the guessed threshold is the hot score and only
    # the 12 hot items (< k) pass it: every user fails and is rescanned.
    I[np.arange(12) * 32] = 3.0
    s, it = ops.score_topk(_bf16(U), _bf16(I), k)
    ref_i, ref_s = _exact_topk_torch(U, I, k)
    assert np.array_equal(it.cpu().numpy().astype(np.int64), ref_i)
    assert np.array_equal(s.cpu().numpy(), ref_s)


def _Slots(n):
    """Workgroup-slot count the scan planner plans for (the scan_slots knob,
    dr_set_plan_knob): small counts reach the split-tail plans with small inputs."""
    from divrec import _backend
    return _backend.plan_knobs(scan_slots=n)


def _exact_topk_torch_excl(U, I, k, frozen, block=256):
    """_exact_topk_torch with each user's frozen items scored -inf (integer
    tables: exact scores, stable sort = (score desc, id asc))."""
    Ud, Id = torch.from_numpy(U).to(DEV), torch.from_numpy(I).to(DEV)
    outi = []
    for b in range(0, Ud.shape[0], block):
        S = Ud[b:b + block] @ Id.T
        for r in range(S.shape[0]):
            f = frozen[b + r]
            if len(f):
                S[r, torch.from_numpy(np.asarray(f, dtype=np.int64)).to(DEV)] = -float("inf")
        outi.append(torch.sort(S, dim=1, descending=True, stable=True).indices[:, :k].cpu())
    return torch.cat(outi).numpy().astype(np.int64)


@pytest.mark.parametrize("d,slots,n_full", [(128, 4, 6), (64, 3, 6), (32, 3, 3), (32, 5, 1)])
def test_score_topk_split_tail_exact(d, slots, n_full):
    """Grid-tail plans: with `slots` workgroup slots, the user blocks past the
    last full round are each split into catalog chunks (DESIGN.md §3.1 grid
    tail), their chunk buffers end-compacted and merged by the finalize. The
    lists (with exclusions, duplicate user ids and a partial last block) must
    equal the exact top-k."""
    rng = np.random.default_rng(900 + d)
    upwg = 2048 if d <= 64 else 1024
    nu, ni, k = n_full * upwg + 333, 300_007, 50
    U, I = _int_table(rng, nu, d), _int_table(rng, ni, d)
    users = np.concatenate([np.arange(nu - 40), rng.integers(0, nu, 40)]).astype(np.int64)
    frozen = [rng.choice(ni, size=int(rng.integers(0, 30)), replace=False) for _ in users]
    for n in range(0, len(users), 97):  # exclude some of the user's best items
        best = np.argsort(-(I @ U[users[n]]), kind="stable")[:10]
        frozen[n] = np.union1d(frozen[n], best)
    rowptr, cols = oracle.exclusion_csr(frozen)
    with _Slots(slots):
        s, it = ops.score_topk(_bf16(U), _bf16(I), k, user_ids=torch.from_numpy(users).to(DEV),
                               exclude=(torch.from_numpy(rowptr).to(DEV),
                                        torch.from_numpy(cols).to(DEV)))
    ref_i = _exact_topk_torch_excl(U[users], I, k, frozen)
    assert np.array_equal(it.cpu().numpy().astype(np.int64), ref_i)


@pytest.mark.parametrize("d", [64, 128])
def test_score_topk_split_tail_rescan_exact(d):
    """A split tail whose every user fails the guessed threshold (hot sampled
    rows): the fail list comes from the chunked finalize, and the rescan
    (whole-catalog units) rewrites every list."""
    rng = np.random.default_rng(188 + d)
    ni, k = (1 << 18) + 77, 20
    nu = 2 * (2048 if d <= 64 else 1024) + 333
    U = _int_table(rng, nu, d, 0, 3)
    I = _int_table(rng, ni, d)
    I[np.arange(12) * 32] = 3.0  # see test_score_topk_guess_rescan_many_units_exact
    with _Slots(2):
        s, it = ops.score_topk(_bf16(U), _bf16(I), k)
    ref_i, ref_s = _exact_topk_torch(U, I, k)
    assert np.array_equal(it.cpu().numpy().astype(np.int64), ref_i)
    assert np.array_equal(s.cpu().numpy(), ref_s)


def test_score_topk_split_tail_fp32_exact():
    """The fp32 scan under a split-tail plan."""
    rng = np.random.default_rng(4242)
    nu, ni, k = 2 * 1024 + 100, 300_007, 30
    U, I = _int_table(rng, nu, 64), _int_table(rng, ni, 64)
    with _Slots(2):
        s, it = ops.score_topk(torch.from_numpy(U).to(DEV), torch.from_numpy(I).to(DEV), k)
    ref_i, ref_s = _exact_topk_torch(U, I, k)
    assert np.array_equal(it.cpu().numpy().astype(np.int64), ref_i)
    assert np.array_equal(s.cpu().numpy(), ref_s)


def test_score_topk_guess_large_exclusion_exact():
    """Guessed thresholds over a 2^19+-row catalog (a 16K-row sample): integer
    tables, several user blocks, exclusions of some users' best items,
    duplicate ids: lists equal the exact top-k."""
    rng = np.random.default_rng(4711)
    d, ni, k = 64, (1 << 19) + 321, 50
    nu = 2 * 2048 + 77
    U, I = _int_table(rng, nu, d), _int_table(rng, ni, d)
    users = np.concatenate([np.arange(nu - 30), rng.integers(0, nu, 30)]).astype(np.int64)
    frozen = [rng.choice(ni, size=int(rng.integers(0, 20)), replace=False) for _ in users]
    for n in range(0, len(users), 257):
        best = np.argsort(-(I @ U[users[n]]), kind="stable")[:15]
        frozen[n] = np.union1d(frozen[n], best)
    rowptr, cols = oracle.exclusion_csr(frozen)
    s, it = ops.score_topk(_bf16(U), _bf16(I), k, user_ids=torch.from_numpy(users).to(DEV),
                           exclude=(torch.from_numpy(rowptr).to(DEV), torch.from_numpy(cols).to(DEV)))
    ref_i = _exact_topk_torch_excl(U[users], I, k, frozen)
    assert np.array_equal(it.cpu().numpy().astype(np.int64), ref_i)


def test_score_topk_guess_hot_sample_rows_exact():
    """8 hot rows at catalog rows 0, 1024, ..., 7168 (all in the stride-32
    sample) are every user's best items: the guessed rank in the sample is 9
    (k = 20), so each threshold sits just below the user's best non-hot sample
    score; lists and scores equal the exact top-k."""
    rng = np.random.default_rng(99)
    d, ni, k = 64, (1 << 19) + 77, 20
    nu = 2048 + 100
    U = _int_table(rng, nu, d, 0, 3)
    I = _int_table(rng, ni, d)
    I[np.arange(8) * 1024] = 3.0
    s, it = ops.score_topk(_bf16(U), _bf16(I), k)
    ref_i, ref_s = _exact_topk_torch(U, I, k)
    assert np.array_equal(it.cpu().numpy().astype(np.int64), ref_i)
    assert np.array_equal(s.cpu().numpy(), ref_s)


@pytest.mark.parametrize("d,ni,slots", [(64, 5000, None), (128, 300_007, 2), (32, 300_007, None)])
def test_score_topk_seeded_thresholds_exact(d, ni, slots):
    """dr_score_topk_seeded: the top-k of the items scoring strictly above a
    caller threshold per user (-inf: plain top-k; +inf: an empty list; ties at
    the threshold excluded), lists padded with -1 / -inf; a split-tail plan
    too (slots = 2). Integer tables: exact against a masked stable sort."""
    rng = np.random.default_rng(d + ni)
    nu, k = 2 * (2048 if d <= 64 else 1024) + 55, 30
    U, I = _int_table(rng, nu, d), _int_table(rng, ni, d)
    Ud, Id = torch.from_numpy(U).to(DEV), torch.from_numpy(I).to(DEV)
    S = Ud @ Id.T
    top = torch.topk(S, 41, dim=1).values
    thr = top[:, 40].clone()  # ~40 items above most thresholds
    thr[::7] = -float("inf")
    thr[3::11] = float("inf")
    thr[5::13] = top[5::13, 10]  # ~10 above: padded lists
    ctx = _Slots(slots) if slots else None
    if ctx:
        ctx.__enter__()
    try:
        s, it = ops.score_topk(_bf16(U), _bf16(I), k, init_thr=thr.contiguous())
    finally:
        if ctx:
            ctx.__exit__(None, None, None)
    M = torch.where(S > thr[:, None], S, torch.full_like(S, -float("inf")))
    v, o = torch.sort(M, dim=1, descending=True, stable=True)
    v, o = v[:, :k], o[:, :k]
    ref_i = torch.where(torch.isfinite(v), o, torch.full_like(o, -1))
    assert torch.equal(it.to(torch.int64).cpu(), ref_i.cpu())
    assert torch.equal(s.cpu(), v.cpu())


def test_score_topk_guess_float_large():
    """Guessed-threshold path on a float catalog (2^19 rows, d=128): every user
    takes the guess (few or no rescans), lists within the float tolerance."""
    rng = np.random.default_rng(3)
    d, k = 128, 100
    U = oracle.as_bf16_f32(rng.standard_normal((64, d)).astype(np.float32) / np.sqrt(d))
    I = oracle.as_bf16_f32(rng.standard_normal((1 << 19, d)).astype(np.float32) / np.sqrt(d))
    s, it = ops.score_topk(_bf16(U), _bf16(I), k)
    s, it = s.cpu().numpy(), it.cpu().numpy().astype(np.int64)
    S = U.astype(np.float64) @ I.astype(np.float64).T
    tol = 1e-5 * np.sqrt(d / 64)
    kth = -np.sort(-S, axis=1)[:, k - 1]
    assert np.all(np.abs(s - np.take_along_axis(S, it, axis=1)) <= tol)
    for u in range(S.shape[0]):
        assert np.isin(np.nonzero(S[u] > kth[u] + 2 * tol)[0], it[u]).all()


def test_score_topk_float_tolerance():
    rng = np.random.default_rng(2)
    d, k = 128, 100
    U = oracle.as_bf16_f32(rng.standard_normal((200, d)).astype(np.float32) / np.sqrt(d))
    I = oracle.as_bf16_f32(rng.standard_normal((20000, d)).astype(np.float32) / np.sqrt(d))
    s, it = ops.score_topk(_bf16(U), _bf16(I), k)
    s, it = s.cpu().numpy(), it.cpu().numpy().astype(np.int64)
    S = U.astype(np.float64) @ I.astype(np.float64).T
    tol = 1e-5 * np.sqrt(d / 64)  # |score error| bound vs float64 (scores are O(1))
    got_true = np.take_along_axis(S, it, axis=1)
    assert np.all(np.abs(s - got_true) <= tol)
    assert np.all(np.diff(s, axis=1) <= 0)
    kth = -np.sort(-S, axis=1)[:, k - 1]
    # every returned item is within tol of the true top-k; every item clearly
    # inside the true top-k (margin > 2 tol) is returned
    assert np.all(got_true >= kth[:, None] - 2 * tol)
    for u in range(S.shape[0]):
        must = np.nonzero(S[u] > kth[u] + 2 * tol)[0]
        assert np.isin(must, it[u]).all()


# --------------------------------------------------------------------------- fp32-faithful scan
def _f32(x):
    return torch.from_numpy(np.ascontiguousarray(x, dtype=np.float32)).to(DEV)


@pytest.mark.parametrize("d", [32, 64, 100, 128, 256])
@pytest.mark.parametrize("k", [1, 10, 100])
def test_score_topk_fp32_integer_exact(d, k):
    """fp32 tables (v_mfma_f32_32x32x2_f32 scan): integer-valued scores are
    exact, so lists AND scores equal the oracle bit for bit, ties included;
    d=100 runs zero-padded to 128."""
    rng = np.random.default_rng(7000 + 1000 * d + k)
    nu, ni = 37 + d, 2000 + 13
    U, I = _int_table(rng, nu, d), _int_table(rng, ni, d)
    s, it = ops.score_topk(_f32(U), _f32(I), k)
    ref_i, ref_s = oracle.recommend_topk(U, I, k, return_scores=True)
    assert np.array_equal(it.cpu().numpy().astype(np.int64), ref_i)
    assert np.array_equal(s.cpu().numpy(), ref_s)


@pytest.mark.parametrize("d", [64, 100, 128])
def test_score_topk_fp32_float_faithful(d):
    """Raw N(0,1) fp32 tables (nn.Embedding's init, not bf16-representable).
    Scores: within 5e-7 * sum_j |u_j i_j| of the exact (float64) score — an
    fp32 fmaf chain's error (a numpy emulation of the scan's k order peaks at
    3.4e-7 over 600K N(0,1) pairs at d = 64..128). Lists: equal to the oracle's (the reference's fp32
    sum(u * i) loop) except where exact scores are within the fp32 tolerance
    (tests/topk_checks.py)."""
    rng = np.random.default_rng(90 + d)
    nu, ni, k = 150, 5000, 100
    U = rng.standard_normal((nu, d)).astype(np.float32)
    I = rng.standard_normal((ni, d)).astype(np.float32)
    s, it = ops.score_topk(_f32(U), _f32(I), k)
    s, it = s.cpu().numpy(), it.cpu().numpy().astype(np.int64)
    S = U.astype(np.float64) @ I.astype(np.float64).T
    A = np.abs(U.astype(np.float64)) @ np.abs(I.astype(np.float64)).T
    rows = np.arange(nu)[:, None]
    assert np.all(np.abs(s - S[rows, it]) <= 5e-7 * A[rows, it])
    assert np.all(np.diff(s, axis=1) <= 0)
    ref_i = oracle.recommend_topk(U, I, k)
    bad = gap_check(it, ref_i, U, I, None, fp32_row_tol(U, I))
    assert bad <= nu // 16


def test_score_topk_fp32_vs_bf16_mode():
    """bf16-representable fp32 tables: the fp32 scan and the bf16 scan see the
    same values; integer-valued ones give identical lists and scores."""
    rng = np.random.default_rng(44)
    U, I = _int_table(rng, 300, 128), _int_table(rng, 7000, 128)
    s32, i32 = ops.score_topk(_f32(U), _f32(I), 50)
    s16, i16 = ops.score_topk(_bf16(U), _bf16(I), 50)
    assert torch.equal(i32, i16) and torch.equal(s32, s16)


# --------------------------------------------------------------------------- k = 1000 (config 5's candidate lists)
def _excl(rng, U, I, nu, ni, n_max=300):
    frozen = [rng.choice(ni, size=rng.integers(0, n_max), replace=False) for _ in range(nu)]
    for u in range(0, nu, 3):  # the best items excluded: the worst case for the thresholds
        best = np.argsort(-(I @ U[u]), kind="stable")[:40]
        frozen[u] = np.union1d(frozen[u], best)
    return frozen


@pytest.mark.parametrize("d,k,dtype", [(64, 1000, "bf16"), (128, 1000, "bf16"), (128, 1024, "bf16"),
                                     (64, 1000, "f32")])
def test_score_topk_k1000_guess_exclusion_exact(d, k, dtype):
    """k = 1000 / 1024 (CAP 2048 candidate buffers, 32-key-per-lane finalize
    sort) over a 2^18+-row catalog, so the guessed-threshold path runs, with
    exclusions: lists and scores equal the oracle (integer tables, exact
    scores, massive ties). bf16 d = 128 and fp32 d = 64 (the same 256-B rows)
    run the staged long-list instance (56-KB stages, round 6)."""
    rng = np.random.default_rng(d + k)
    nu, ni = 24, (1 << 18) + 999
    U, I = _int_table(rng, nu, d), _int_table(rng, ni, d)
    frozen = _excl(rng, U, I, nu, ni)
    rowptr, cols = oracle.exclusion_csr(frozen)
    t = _f32 if dtype == "f32" else _bf16
    s, it = ops.score_topk(t(U), t(I), k,
                           exclude=(torch.from_numpy(rowptr).to(DEV), torch.from_numpy(cols).to(DEV)))
    ref_i, ref_s = oracle.recommend_topk(U, I, k, frozen=frozen, return_scores=True)
    assert np.array_equal(it.cpu().numpy().astype(np.int64), ref_i)
    assert np.array_equal(s.cpu().numpy(), ref_s)


@pytest.mark.parametrize("dtype", ["bf16", "f32"])
def test_score_topk_k1000_many_users_exact(dtype):
    """k = 1000 over more users than one workgroup holds, short catalog (no
    guess): fp32 and bf16 scans, exclusion of the best items."""
    rng = np.random.default_rng(1000)
    d, nu, ni, k = 64, 2100, 3000, 1000
    U, I = _int_table(rng, nu, d), _int_table(rng, ni, d)
    frozen = _excl(rng, U, I, nu, ni, n_max=100)
    rowptr, cols = oracle.exclusion_csr(frozen)
    t = _f32 if dtype == "f32" else _bf16
    s, it = ops.score_topk(t(U), t(I), k,
                           exclude=(torch.from_numpy(rowptr).to(DEV), torch.from_numpy(cols).to(DEV)))
    sel = np.arange(0, nu, 7)  # an oracle sample of the users (the per-user loop is slow)
    ref_i, ref_s = oracle.recommend_topk(U, I, k, users=sel, frozen=[frozen[u] for u in sel],
                                         return_scores=True)
    assert np.array_equal(it.cpu().numpy()[sel].astype(np.int64), ref_i)
    assert np.array_equal(s.cpu().numpy()[sel], ref_s)


def test_score_topk_sharded_k1000_equals_single_pass():
    """Config 5's candidate lists from an item-sharded catalog: 8 row shards
    (global ids through item_base), each a top-1000, merged by the streaming
    merge (8 x 1000 > 2048 entries) — bit-identical to one pass."""
    rng = np.random.default_rng(808)
    d, nu, ni, k = 128, 300, 40000, 1000
    U, I = _int_table(rng, nu, d), _int_table(rng, ni, d)
    Ub, Ib = _bf16(U), _bf16(I)
    full_s, full_i = ops.score_topk(Ub, Ib, k)
    bounds = np.linspace(0, ni, 9).astype(int)
    parts = [ops.score_topk(Ub, Ib[lo:hi], k, item_base=int(lo))
             for lo, hi in zip(bounds[:-1], bounds[1:])]
    ms, mi = ops.topk_merge(torch.stack([p[0] for p in parts]), torch.stack([p[1] for p in parts]), k)
    assert torch.equal(mi, full_i) and torch.equal(ms, full_s)


def test_topk_merge_streaming_matches_oracle():
    """parts * k_in > 2048 entries per user (8 x 1000): the streaming merge
    kernel, with empty slots, against the oracle."""
    rng = np.random.default_rng(14)
    P, n, k_in, k_out = 8, 37, 1000, 1000
    sc = rng.integers(-50, 50, size=(P, n, k_in)).astype(np.float32)
    items = np.stack([rng.permutation(200000)[: n * k_in].reshape(n, k_in)
                      for _ in range(P)]).astype(np.int32)
    for p in range(P):
        for u in range(n):
            o = np.lexsort((items[p, u], -sc[p, u]))
            sc[p, u], items[p, u] = sc[p, u][o], items[p, u][o]
    items[2, 5, 600:] = -1
    sc[2, 5, 600:] = -np.inf
    items[:, 7, 10:] = -1  # a user with only 80 entries: the tail must be empty
    sc[:, 7, 10:] = -np.inf
    ms, mi = ops.topk_merge(torch.from_numpy(sc).to(DEV), torch.from_numpy(items).to(DEV), k_out)
    rs, ri = oracle.topk_merge(sc, items, k_out)
    assert np.array_equal(mi.cpu().numpy().astype(np.int64), ri)
    assert np.array_equal(ms.cpu().numpy(), rs)


def test_topk_merge_matches_oracle():
    rng = np.random.default_rng(4)
    P, n, k = 4, 33, 25
    sc = rng.integers(-5, 5, size=(P, n, k)).astype(np.float32)
    sc = -np.sort(-sc, axis=2)
    items = np.stack([rng.permutation(10000)[: n * k].reshape(n, k) for _ in range(P)]).astype(np.int32)
    # sort each list by (score desc, item asc) so inputs are valid partials
    for p in range(P):
        for u in range(n):
            o = np.lexsort((items[p, u], -sc[p, u]))
            sc[p, u], items[p, u] = sc[p, u][o], items[p, u][o]
    items[1, 3, 20:] = -1  # empty slots
    ms, mi = ops.topk_merge(torch.from_numpy(sc).to(DEV), torch.from_numpy(items).to(DEV), 40)
    rs, ri = oracle.topk_merge(sc, items, 40)
    assert np.array_equal(mi.cpu().numpy().astype(np.int64), ri)
    assert np.array_equal(ms.cpu().numpy(), rs)


# --------------------------------------------------------------------------- ILD
@pytest.mark.parametrize("k", [1, 2, 10, 100])
def test_ild_dense_f32_bit_exact(k):
    rng = np.random.default_rng(k)
    ni = 500
    D = rng.random((ni, ni)).astype(np.float32)
    recs = rng.integers(0, ni, size=(64, k))
    recs[0, :] = recs[0, 0]  # duplicates (diagonal included)
    got = ops.ild_dense(torch.from_numpy(recs).to(DEV), torch.from_numpy(D).to(DEV)).cpu().numpy()
    ref = oracle.ild_sequential(recs, D)
    assert np.array_equal(got, ref, equal_nan=True)


@pytest.mark.parametrize("dt", [np.int32, np.int64])
def test_ild_dense_int_exact(dt):
    rng = np.random.default_rng(1)
    D = rng.integers(0, 3, size=(300, 300)).astype(dt)
    recs = rng.integers(0, 300, size=(50, 10)).astype(np.int32)
    got = ops.ild_dense(torch.from_numpy(recs).to(DEV), torch.from_numpy(D).to(DEV)).cpu().numpy()
    assert np.array_equal(got, oracle.ild_sequential(recs, D))


def test_ild_labels_exact():
    rng = np.random.default_rng(8)
    labels = rng.integers(0, 4, size=5000)
    recs = rng.integers(0, 5000, size=(300, 100))
    got = ops.ild_labels(torch.from_numpy(recs).to(DEV), torch.from_numpy(labels).to(DEV)).cpu().numpy()
    assert np.array_equal(got, oracle.ild_labels(recs, labels))
    # and the literal reference algorithm on the dense int matrix (20 users)
    D = (labels[:, None] == labels[None, :]).astype(np.int32)
    assert np.array_equal(got[:20], oracle.ild_sequential(recs[:20], D))


@pytest.mark.parametrize("d", [32, 64, 128, 256])
@pytest.mark.parametrize("k", [2, 10, 100, 128])
@pytest.mark.parametrize("kind", ["cosine", "dot", "euclidean"])
def test_ild_embedding(d, k, kind):
    rng = np.random.default_rng(d + k)
    E = oracle.as_bf16_f32(rng.standard_normal((3000, d)).astype(np.float32))
    recs = rng.integers(0, 3000, size=(40, k))
    got = ops.ild_embedding(torch.from_numpy(recs).to(DEV), _bf16(E), kind).cpu().numpy()
    ref = oracle.ild_embedding_f64(recs, E, kind)
    # fp32 Gram + fp32 pair sum vs float64: rel 2e-5 (k <= 128)
    assert np.allclose(got, ref, rtol=2e-5, atol=2e-5 * np.abs(ref).max())


@pytest.mark.parametrize("d", [32, 64, 128])
@pytest.mark.parametrize("k", [1, 2, 10, 31, 33, 64, 100, 128])
@pytest.mark.parametrize("rec_dtype", [torch.int64, torch.int32])
def test_ild_embedding_stream_matches_wave_per_user(d, k, rec_dtype):
    """The streamed persistent-grid ILD (k <= 128, d <= 128; the default for
    k > 40, forced here by ild_stream = 1 for every k):
    int64 and int32 lists, more users than the grid's waves (each wave's
    pipeline runs many users, its last ones re-issued as padding), a ring of
    one list's pieces, of 1.5 and 3 lists (ild_bufs) and the LDS-sized
    default, which must agree bit for bit (the same arithmetic, only the
    pipeline depth differs). Bad ids give NaN and count once per user. Against float64 and
    against the one-wave-per-user kernel (ild_stream = 0, per-pair
    epilogue; the streamed one sums each Gram column weighted, so the fp32
    rounding differs) the bar is the usual rel 2e-5."""
    rng = np.random.default_rng(d * 1000 + k)
    E = oracle.as_bf16_f32(rng.standard_normal((5000, d)).astype(np.float32))
    Et = _bf16(E)
    nu = 3 * 1024 + 77  # > the 1024 waves of a 256-CU grid: several users per wave
    recs = rng.integers(0, 5000, size=(nu, k))
    recs[5, k // 2] = 5000  # out of range
    recs[nu - 1, 0] = -1
    rt = torch.from_numpy(recs).to(DEV, rec_dtype)
    for kind in ("cosine", "dot", "euclidean"):
        with _backend.plan_knobs(ild_stream=0):
            base = ops.ild_embedding(rt, Et, kind, check=False).cpu().numpy()
        first = None
        ni = -(-k // (64 // (d // 8)))  # 1-KB pieces per list
        for bufs in (None, ni, max(ni * 3 // 2, ni + 1), min(3 * ni, 64)):
            err = torch.zeros(1, dtype=torch.int32, device=DEV)
            with _backend.plan_knobs(ild_stream=1, **({} if bufs is None else {"ild_bufs": bufs})):
                out = torch.empty(nu, dtype=torch.float32, device=DEV)
                rc = _backend.lib().dr_ild_embedding(
                    rt.data_ptr(), _backend.dtype_code(rec_dtype), nu, k, Et.data_ptr(), 5000, d,
                    {"cosine": 0, "dot": 1, "euclidean": 2}[kind], out.data_ptr(), err.data_ptr(),
                    _backend.stream(torch.device(DEV)))
                assert rc == 0
            got = out.cpu().numpy()
            assert int(err.item()) == 2
            assert np.isnan(got[5]) and np.isnan(got[nu - 1])
            if first is None:
                first = got
            assert np.array_equal(got, first, equal_nan=True), (kind, bufs)
            sc = np.nanmax(np.abs(base)) if k > 1 else 1.0
            assert np.allclose(got, base, rtol=2e-5, atol=2e-5 * sc, equal_nan=True), (kind, bufs)
        ok = np.ones(nu, bool)
        ok[[5, nu - 1]] = False
        ref = oracle.ild_embedding_f64(recs[ok][:300], E, kind)
        if k == 1:
            assert np.isnan(got[ok][:300]).all()  # 0 / 0, as the reference
        else:
            assert np.allclose(got[ok][:300], ref, rtol=2e-5, atol=2e-5 * np.abs(ref).max())


def test_ild_embedding_routes_short_lists_to_the_per_user_kernel():
    """Default plan: d = 128 cosine / dot lists of k > 40 take the streamed
    kernel; short lists, d = 64 / 32 and euclidean the one-wave-per-user
    kernel (faster there). The default output equals the forced kernel's
    bit for bit in each case."""
    rng = np.random.default_rng(40)
    for d, kind, k, forced in ((128, "cosine", 10, 0), (128, "cosine", 40, 0),
                               (128, "cosine", 41, 1), (128, "dot", 64, 1),
                               (128, "euclidean", 100, 0), (64, "cosine", 100, 0),
                               (32, "dot", 100, 0)):
        E = _bf16(oracle.as_bf16_f32(rng.standard_normal((3000, d)).astype(np.float32)))
        rt = torch.from_numpy(rng.integers(0, 3000, size=(2000, k))).to(DEV)
        got = ops.ild_embedding(rt, E, kind)
        with _backend.plan_knobs(ild_stream=forced):
            ref = ops.ild_embedding(rt, E, kind)
        assert torch.equal(got, ref), (d, kind, k)


def test_ild_embedding_stream_small_grids():
    """Fewer users than waves (idle waves return at once), one user, and a
    wave with exactly one user: the pipeline's padding re-issues that user."""
    rng = np.random.default_rng(3)
    E = oracle.as_bf16_f32(rng.standard_normal((700, 128)).astype(np.float32))
    for nu in (1, 3, 1023, 1025):
        recs = rng.integers(0, 700, size=(nu, 100))
        rt = torch.from_numpy(recs).to(DEV)
        got = ops.ild_embedding(rt, _bf16(E), "cosine").cpu().numpy()  # k = 100: streamed
        with _backend.plan_knobs(ild_stream=0):
            base = ops.ild_embedding(rt, _bf16(E), "cosine").cpu().numpy()
        assert np.allclose(got, base, rtol=2e-5, atol=1e-6)
        ref = oracle.ild_embedding_f64(recs[:50], E, "cosine")
        assert np.allclose(got[:50], ref, rtol=2e-5, atol=1e-6)


# --------------------------------------------------------------------------- BPR + Adam
@pytest.mark.parametrize("d", [100, 128, 256])  # 100: the reference experiments' embedding_dim
def test_bpr_fwd_bwd(d):
    rng = np.random.default_rng(6)
    nu, ni, B = 200, 300, 4096
    U = rng.standard_normal((nu, d)).astype(np.float32) * 0.3
    I = rng.standard_normal((ni, d)).astype(np.float32) * 0.3
    uid, pid, nid = rng.integers(0, nu, B), rng.integers(0, ni, B), rng.integers(0, ni, B)
    gU = torch.zeros(nu, d, device=DEV)
    gI = torch.zeros(ni, d, device=DEV)
    loss, hit = ops.bpr_fwd_bwd(torch.from_numpy(U).to(DEV), torch.from_numpy(I).to(DEV),
                                torch.from_numpy(uid).to(DEV), torch.from_numpy(pid).to(DEV),
                                torch.from_numpy(nid).to(DEV), 1.0 / B, gU, gI)
    rl, ra, rU, rI = oracle.bpr_forward_backward(U, I, uid, pid, nid)
    assert abs(loss.double().mean().item() - rl) <= 1e-5 * abs(rl)
    assert abs(hit.double().mean().item() - ra) <= 1.0 / B
    assert np.allclose(gU.cpu().numpy(), rU, rtol=1e-4, atol=1e-7)
    assert np.allclose(gI.cpu().numpy(), rI, rtol=1e-4, atol=1e-7)


def test_adam_dense_matches_torch():
    rng = np.random.default_rng(12)
    p0 = rng.standard_normal(10007).astype(np.float32)
    grads = [rng.standard_normal(10007).astype(np.float32) for _ in range(3)]
    # torch reference on the same device
    pt = torch.nn.Parameter(torch.from_numpy(p0.copy()).to(DEV))
    opt = torch.optim.Adam([pt], lr=1e-3, foreach=False)
    p = torch.from_numpy(p0.copy()).to(DEV)
    m = torch.zeros_like(p)
    v = torch.zeros_like(p)
    for step, g in enumerate(grads, 1):
        pt.grad = torch.from_numpy(g).to(DEV)
        opt.step()
        ops.adam_dense(p, torch.from_numpy(g).to(DEV), m, v, 1e-3, 0.9, 0.999, 1e-8, 0.0, step)
    assert torch.allclose(p, pt.detach(), rtol=0, atol=1e-6)


# --------------------------------------------------------------------------- MMR
@pytest.mark.parametrize("lam", [1.0, 0.7, 0.3])
def test_mmr_rerank(lam):
    rng = np.random.default_rng(int(lam * 10))
    d, ni, n, C, kout = 128, 5000, 8, 300, 40
    E = oracle.as_bf16_f32(rng.standard_normal((ni, d)).astype(np.float32))
    cand = np.stack([rng.choice(ni, C, replace=False) for _ in range(n)]).astype(np.int32)
    sc = rng.standard_normal((n, C)).astype(np.float32)
    got = ops.mmr_rerank(torch.from_numpy(cand).to(DEV), torch.from_numpy(sc).to(DEV), _bf16(E),
                         kout, lam).cpu().numpy()
    assert oracle.mmr_check(got, cand, sc, E, lam, tol=1e-4) == 0
    if lam == 1.0:  # pure relevance: equals top-k by score (ties: lowest position)
        ref = np.take_along_axis(cand, np.argsort(-sc, axis=1, kind="stable")[:, :kout], axis=1)
        assert np.array_equal(got, ref)


def _mmr_check_positions(picks, cand, sc, E, lam, tol):
    """float64 replay that also handles invalid (-1) candidates: each pick must
    be a live candidate whose MMR value is within tol of the step maximum, and
    -1 must appear exactly when no live candidate is left."""
    bad = 0
    for u in range(cand.shape[0]):
        valid = cand[u] >= 0
        X = E[np.where(valid, cand[u], 0)].astype(np.float64)
        Xn = X / np.linalg.norm(X, axis=1, keepdims=True)
        sims = Xn @ Xn.T
        s = sc[u].astype(np.float64)
        alive = valid.copy()
        pen = None
        for it in picks[u]:
            if not alive.any():
                bad += int(it != -1)
                continue
            val = lam * s - (1 - lam) * (pen if pen is not None else 0.0)
            val[~alive] = -np.inf
            hits = np.nonzero(alive & (cand[u] == it))[0]
            if len(hits) == 0 or val[hits].max() < val.max() - tol:
                bad += 1
                continue
            j = hits[np.argmax(val[hits])]
            alive[j] = False
            pen = sims[:, j] if pen is None else np.maximum(pen, sims[:, j])
    return bad


@pytest.mark.parametrize("d,C,kout,lam", [(128, 1000, 100, 0.5), (128, 1024, 100, 0.9),
                                          (64, 1024, 64, 0.3), (64, 777, 100, 0.0),
                                          (128, 1000, 100, 1.0)])
def test_mmr_rerank_config5_shape(d, C, kout, lam):
    """Config-5 shapes (1000 -> 100, scores sorted descending as a top-k list
    gives them); every pick a valid greedy step within 1e-4 (float64 replay)."""
    rng = np.random.default_rng(d + C + kout)
    ni, n = 20000, 12
    E = oracle.as_bf16_f32((rng.standard_normal((ni, d)) / np.sqrt(d)).astype(np.float32))
    cand = np.stack([rng.choice(ni, C, replace=False) for _ in range(n)]).astype(np.int32)
    sc = -np.sort(-rng.random((n, C)), axis=1).astype(np.float32)
    got = ops.mmr_rerank(torch.from_numpy(cand).to(DEV), torch.from_numpy(sc).to(DEV), _bf16(E),
                         kout, lam).cpu().numpy()
    assert _mmr_check_positions(got, cand, sc, E, lam, tol=1e-4) == 0
    if lam == 1.0:
        assert np.array_equal(got, cand[:, :kout])


@pytest.mark.parametrize("lam", [1.0, 0.5])
def test_mmr_rerank_ties(lam):
    """Tie-saturated lists: equal scores everywhere (user 0, 1) and 100 items
    repeated 10 times with equal scores per item (users 2, 3). More than a
    wave's probe count of equal values sit at the top of every wave, so a batch
    can have no probe that beats its bound: the bound's candidate (the best key
    outside the probes) is then picked on its own. lam = 1 with equal scores
    must return the candidates in position order (ties: lowest position)."""
    rng = np.random.default_rng(21)
    d, ni, C, kout = 128, 5000, 1000, 100
    E = oracle.as_bf16_f32((rng.standard_normal((ni, d)) / np.sqrt(d)).astype(np.float32))
    cand = np.stack([rng.choice(ni, C, replace=False) for _ in range(2)]
                    + [np.repeat(rng.choice(ni, C // 10, replace=False), 10) for _ in range(2)]
                    ).astype(np.int32)
    sc = np.full(cand.shape, 0.25, np.float32)
    sc[2:] = np.repeat(-np.sort(-rng.random((2, C // 10))), 10, axis=1)
    got = ops.mmr_rerank(torch.from_numpy(cand).to(DEV), torch.from_numpy(sc).to(DEV), _bf16(E),
                         kout, lam).cpu().numpy()
    assert _mmr_check_positions(got, cand, sc, E, lam, tol=1e-4) == 0
    if lam == 1.0:
        assert np.array_equal(got[:2], cand[:2, :kout])
        assert np.array_equal(got[2:], cand[2:, :kout])


def test_mmr_rerank_invalid_candidates():
    """-1 candidates are never picked; once the live ones run out the tail is -1."""
    rng = np.random.default_rng(5)
    d, ni, n, C, kout = 64, 3000, 6, 200, 150
    E = oracle.as_bf16_f32(rng.standard_normal((ni, d)).astype(np.float32))
    cand = np.stack([rng.choice(ni, C, replace=False) for _ in range(n)]).astype(np.int32)
    for u in range(n):  # 0, 35, 70, ... invalid entries: fewer live than kout for most users
        cand[u, rng.choice(C, 35 * u, replace=False)] = -1
    sc = rng.standard_normal((n, C)).astype(np.float32)
    got = ops.mmr_rerank(torch.from_numpy(cand).to(DEV), torch.from_numpy(sc).to(DEV), _bf16(E),
                         kout, 0.6).cpu().numpy()
    assert _mmr_check_positions(got, cand, sc, E, 0.6, tol=1e-4) == 0
    for u in range(n):
        n_live = int((cand[u] >= 0).sum())
        assert (got[u, :min(n_live, kout)] >= 0).all()
        assert (got[u, n_live:] == -1).all()


@pytest.mark.parametrize("d,C,lam", [(128, 1000, 0.5), (64, 777, 0.3), (128, 1000, 1.0)])
def test_mmr_rerank_persistent_prefetch(d, C, lam):
    """More users than CUs: each workgroup of the persistent grid runs several
    users, all but its first with ids, scores and tile-0 rows prefetched by
    LDS-DMA during the previous user. Empty (-1) candidates and an
    out-of-range id on prefetched users; lam = 1 must equal the top-k by score
    (ties: lowest position) for every user, lam < 1 every pick a valid greedy
    step (float64 replay) for users of the prefetched range."""
    rng = np.random.default_rng(d + C)
    ni, n, kout = 30000, 700, 100
    E = oracle.as_bf16_f32((rng.standard_normal((ni, d)) / np.sqrt(d)).astype(np.float32))
    cand = np.stack([rng.choice(ni, C, replace=False) for _ in range(n)]).astype(np.int32)
    sc = -np.sort(-rng.random((n, C)), axis=1).astype(np.float32)
    for u in range(300, n, 37):  # empty slots on prefetched users, some in tile 0
        cand[u, rng.choice(C, 50, replace=False)] = -1
    got = ops.mmr_rerank(torch.from_numpy(cand).to(DEV), torch.from_numpy(sc).to(DEV), _bf16(E),
                         kout, lam).cpu().numpy()
    if lam == 1.0:
        for u in range(n):
            live = cand[u][cand[u] >= 0]
            assert np.array_equal(got[u], live[:kout]), u
    else:
        users = np.concatenate([np.arange(0, 8), rng.choice(np.arange(256, n), 24, replace=False)])
        assert _mmr_check_positions(got[users], cand[users], sc[users], E, lam, tol=1e-4) == 0
    bad = cand.copy()
    bad[500, 3] = ni + 7  # an out-of-range id on a prefetched user: IndexError, as indexing would
    with pytest.raises(IndexError):
        ops.mmr_rerank(torch.from_numpy(bad).to(DEV), torch.from_numpy(sc).to(DEV), _bf16(E), kout, lam)


# --------------------------------------------------------------------------- catalog histogram
@pytest.mark.parametrize("dt", [torch.int32, torch.int64])
def test_catalog_histogram_exact(dt):
    """Counts and 0-based position sums per item (Entropy's torch.unique counts,
    PRI's avg_rank sums), exact; -1 and out-of-range entries are skipped."""
    rng = np.random.default_rng(8)
    n, k, ni = 5000, 37, 3000
    recs = rng.integers(-1, ni + 2, size=(n, k))
    counts, pos = ops.catalog_histogram(torch.from_numpy(recs).to(DEV, dt), ni)
    ok = (recs >= 0) & (recs < ni)
    ref_c = np.bincount(recs[ok], minlength=ni)
    ref_p = np.bincount(recs[ok], weights=np.broadcast_to(np.arange(k), recs.shape)[ok], minlength=ni)
    assert np.array_equal(counts.cpu().numpy(), ref_c)
    assert np.array_equal(pos.cpu().numpy(), ref_p.astype(np.int64))


def test_pri_avg_rank_matches_reference_formula():
    """avg_rank = the reference's per-item sum(positions) / len(positions) as float32."""
    from divrec.metrics.popularity_rank_correlation_for_items import avg_rank

    rng = np.random.default_rng(13)
    recs = rng.integers(0, 500, size=(300, 20))
    items, avg = avg_rank(torch.from_numpy(recs).to(DEV))
    ranks = {}
    for row in recs:
        for p, it in enumerate(row):
            ranks.setdefault(int(it), []).append(p)
    ref_items = np.array(sorted(ranks))
    ref_avg = np.array([sum(ranks[i]) / len(ranks[i]) for i in ref_items], dtype=np.float32)
    assert np.array_equal(items.cpu().numpy(), ref_items)
    assert np.array_equal(avg.cpu().numpy(), ref_avg)


def test_mmr_rerank_out_of_range_raises():
    """A candidate id past the table raises IndexError (as indexing it
    would); with check=False it is skipped like an empty slot."""
    rng = np.random.default_rng(9)
    d, ni, n, C, kout = 128, 2000, 4, 64, 10
    E = oracle.as_bf16_f32(rng.standard_normal((ni, d)).astype(np.float32))
    cand = np.stack([rng.choice(ni, C, replace=False) for _ in range(n)]).astype(np.int32)
    sc = rng.standard_normal((n, C)).astype(np.float32)
    bad = cand.copy()
    bad[2, 7] = ni + 5
    args = (torch.from_numpy(bad).to(DEV), torch.from_numpy(sc).to(DEV), _bf16(E), kout, 0.5)
    with pytest.raises(IndexError):
        ops.mmr_rerank(*args)
    got = ops.mmr_rerank(*args, check=False).cpu().numpy()
    skip = bad.copy()
    skip[2, 7] = -1
    assert _mmr_check_positions(got, skip, sc, E, 0.5, tol=1e-4) == 0
    assert not (got == ni + 5).any()


@pytest.mark.parametrize("d", [100, 128])
def test_bpr_fwd_bwd_mxm_runs(d):
    """The reference's triple layout (PairWiseDataset: users in order, m*m
    triples each, each positive repeated m times in a row, the negatives
    cycled): runs of equal ids are summed in registers before the atomics.
    Gradients against the oracle, with an out-of-range id inside a run."""
    rng = np.random.default_rng(16)
    nu, ni, m, n_users = 50, 400, 20, 45
    U = rng.standard_normal((nu, d)).astype(np.float32) * 0.3
    I = rng.standard_normal((ni, d)).astype(np.float32) * 0.3
    users = rng.choice(nu, n_users)
    pos = rng.integers(0, ni, (n_users, m))
    neg = rng.integers(0, ni, (n_users, m))
    uid = np.repeat(users, m * m)
    pid = np.repeat(pos, m, axis=1).reshape(-1)
    nid = np.tile(neg, (1, m)).reshape(-1)
    B = uid.size
    gU = torch.zeros(nu, d, device=DEV)
    gI = torch.zeros(ni, d, device=DEV)
    loss, hit = ops.bpr_fwd_bwd(torch.from_numpy(U).to(DEV), torch.from_numpy(I).to(DEV),
                                torch.from_numpy(uid).to(DEV), torch.from_numpy(pid).to(DEV),
                                torch.from_numpy(nid).to(DEV), 1.0 / B, gU, gI)
    rl, ra, rU, rI = oracle.bpr_forward_backward(U, I, uid, pid, nid)
    assert abs(loss.double().mean().item() - rl) <= 1e-5 * abs(rl)
    assert abs(hit.double().mean().item() - ra) <= 1.0 / B
    assert np.allclose(gU.cpu().numpy(), rU, rtol=1e-4, atol=1e-7)
    assert np.allclose(gI.cpu().numpy(), rI, rtol=1e-4, atol=1e-7)
    # an invalid positive in the middle of a run: that triple adds nothing, raises
    bad = pid.copy()
    bad[5 * m * m + 7] = ni + 3
    gU.zero_()
    gI.zero_()
    with pytest.raises(IndexError):
        ops.bpr_fwd_bwd(torch.from_numpy(U).to(DEV), torch.from_numpy(I).to(DEV),
                        torch.from_numpy(uid).to(DEV), torch.from_numpy(bad).to(DEV),
                        torch.from_numpy(nid).to(DEV), 1.0 / B, gU, gI)
    keep = np.ones(B, dtype=bool)
    keep[5 * m * m + 7] = False
    _, _, rU2, rI2 = oracle.bpr_forward_backward(U, I, uid[keep], pid[keep], nid[keep])
    # the oracle averages over its own batch size: rescale to 1/B
    sc = keep.sum() / B
    assert np.allclose(gU.cpu().numpy(), rU2 * sc, rtol=1e-4, atol=1e-7)
    assert np.allclose(gI.cpu().numpy(), rI2 * sc, rtol=1e-4, atol=1e-7)


@pytest.mark.parametrize("d,C", [(128, 1), (64, 40), (128, 200)])
def test_mmr_rerank_persistent_prefetch_short_lists(d, C):
    """Short candidate lists (C < 256: the prefetch pads s_nitem with entry C - 1
    and tile 0 is only partly live) with k_out == C and more users than CUs:
    lambda = 1 returns each list in score order, lambda = 0.5 replays as valid
    greedy steps on prefetched users."""
    rng = np.random.default_rng(d * 7 + C)
    ni, n = 5000, 700
    E = oracle.as_bf16_f32((rng.standard_normal((ni, d)) / np.sqrt(d)).astype(np.float32))
    cand = np.stack([rng.choice(ni, C, replace=False) for _ in range(n)]).astype(np.int32)
    sc = -np.sort(-rng.random((n, C)), axis=1).astype(np.float32)
    ct, st = torch.from_numpy(cand).to(DEV), torch.from_numpy(sc).to(DEV)
    top = ops.mmr_rerank(ct, st, _bf16(E), C, 1.0).cpu().numpy()
    assert np.array_equal(top, cand)
    got = ops.mmr_rerank(ct, st, _bf16(E), C, 0.5).cpu().numpy()
    users = np.concatenate([np.arange(0, 4), rng.choice(np.arange(256, n), 20, replace=False)])
    assert _mmr_check_positions(got[users], cand[users], sc[users], E, 0.5, tol=1e-4) == 0
    assert all(sorted(got[u].tolist()) == sorted(cand[u].tolist()) for u in users)


def test_padded_item_table_sees_data_writes():
    """ILD / MMR on a width without a kernel instance (d = 100) pad the item
    table per call, with no cache: writes through ``.data`` (which
    bump no autograd version) and in-place updates are always seen, like
    score_topk's (test_score_topk_sees_data_writes)."""
    rng = np.random.default_rng(100)
    ni, d, n, k = 3000, 100, 50, 10
    E = torch.from_numpy(rng.standard_normal((ni, d)).astype(np.float32)).to(DEV).to(torch.bfloat16)
    recs = torch.from_numpy(rng.integers(0, ni, (n, k))).to(DEV)
    a = ops.ild_embedding(recs, E, "dot")
    assert torch.equal(a, ops.ild_embedding(recs, ops.pad_columns(E, 128), "dot"))
    ver = E._version
    E.data.mul_(2.0)  # no version bump
    assert E._version == ver
    assert torch.allclose(ops.ild_embedding(recs, E, "dot"), 4 * a, rtol=1e-5)
    # MMR at lambda = 0 (pure diversity) on the padded table: the picks follow
    # the rows, so a .data write that swaps two candidates' rows changes them
    C = 64
    torch.manual_seed(7)
    cand = torch.stack([torch.randperm(ni, device=DEV)[:C] for _ in range(n)]).to(torch.int32)
    sc = torch.sort(torch.rand(n, C, device=DEV), dim=1, descending=True).values
    p1 = ops.mmr_rerank(cand, sc, E, 8, 0.0)
    assert torch.equal(p1, ops.mmr_rerank(cand, sc, ops.pad_columns(E, 128), 8, 0.0))
    E.data[cand[:, 1].long()] = E.data[cand[:, 0].long()]  # candidate 1 duplicates candidate 0
    p2 = ops.mmr_rerank(cand, sc, E, 8, 0.0)
    assert torch.equal(p2, ops.mmr_rerank(cand, sc, ops.pad_columns(E, 128), 8, 0.0))
    assert not torch.equal(p1, p2)


@pytest.mark.parametrize("dense", [1, 0])
@pytest.mark.parametrize("d,n_sample,ks1,ks,ids", [(128, 78125, 5, 10, False), (64, 31250, 10, 17, True),
                                                   (128, 70, 1, 3, False), (64, 5000, 50, 68, True),
                                                   (32, 31, 1, 2, False), (64, 40000, 29, 32, False)])
def test_sample_thresholds_group_max(d, n_sample, ks1, ks, ids, dense):
    """dr_sample_thresholds (the item-sharded path's guess): the whole 32-row
    tiles of the sample, tile-transposed (sample q T + r -> row q of tile r),
    one max per user and tile (its 32 rows), thresholds strictly below each
    user's ks1-th / ks-th best tile max (-inf with fewer tiles). Integer tables:
    every score exact, so the thresholds must equal a torch restatement bit for
    bit, and never exceed the exact sample ranks. Both forms of the sample
    scan: dense tile maxima ranked per user by topk_threshold_dense_kernel
    (ks <= 32, the default) and the compaction path (sample_dense = 0, and
    ks = 68 with the default)."""
    from divrec.distributed import threshold_below

    rng = np.random.default_rng(d + n_sample + ks)
    nu = 2500
    U = _int_table(rng, nu, d)
    Sm = _int_table(rng, n_sample, d)
    uids = rng.permutation(nu)[:1800].astype(np.int64) if ids else None
    Ub, Sb = _bf16(U), _bf16(Sm)
    with _backend.plan_knobs(sample_dense=dense):
        out = ops.sample_thresholds(Ub, Sb, ks1, ks,
                                    user_ids=None if uids is None else torch.from_numpy(uids).to(DEV))
    Uq = U if uids is None else U[uids]
    Sp = n_sample // 32 * 32
    ref = torch.full((2, Uq.shape[0]), -float("inf"))
    if Sp:
        T = Sp // 32
        idx = np.array([(p % 32) * T + p // 32 for p in range(Sp)])
        sc = torch.from_numpy(Uq.astype(np.float64) @ Sm[idx].astype(np.float64).T)
        gm = sc.view(-1, T, 32).amax(dim=2)  # one max per user and tile
        top = torch.sort(gm, dim=1, descending=True).values
        for row, kk in ((0, ks1), (1, ks)):
            if T >= kk:
                ref[row] = threshold_below(top[:, kk - 1].float())
        exact = torch.sort(torch.from_numpy(Uq.astype(np.float64) @ Sm.astype(np.float64).T), dim=1,
                           descending=True).values
        assert (ref[1].double() <= exact[:, ks - 1]).all()  # a lower bound of the exact rank
    assert torch.equal(out.cpu(), ref)


@pytest.mark.parametrize("d,k,dtype", [(64, 100, torch.bfloat16), (128, 100, torch.bfloat16),
                                       (32, 20, torch.bfloat16), (64, 100, torch.float32),
                                       (128, 1000, torch.bfloat16)])
def test_score_topk_dense_sample_matches_compaction(d, k, dtype):
    """The guessed-threshold path with the sample scan's dense tile maxima
    (round 5, the default for ks <= 72; k = 1000: ks = 68) against its compaction path
    (sample_dense = 0): the thresholds are the same order statistic of the same
    tile maxima, so the first-tier / second-tier failure counts must be equal
    and the lists identical, and identical to the unseeded scan's.
    Random-normal tables (realistic, tie-free thresholds); 4100 users: several
    user blocks, the last one partial; 300K rows: seeded at stride 32."""
    rng = np.random.default_rng(d * 3 + k)
    nu, ni = 4100, 300_011
    U = (rng.standard_normal((nu, d)) / np.sqrt(d)).astype(np.float32)
    I = (rng.standard_normal((ni, d)) / np.sqrt(d)).astype(np.float32)
    Ut, It = torch.from_numpy(U).to(DEV).to(dtype), torch.from_numpy(I).to(DEV).to(dtype)
    plan = ops.score_topk_plan(nu, ni, dtype, d, k)
    assert plan["sample_stride"] == 32 and plan["sample_rank"] <= 72
    out = {}
    for dense in (1, 0):
        st = {}
        with _backend.plan_knobs(sample_dense=dense):
            s, i = ops.score_topk(Ut, It, k, stats=st)
        out[dense] = (s.cpu(), i.cpu(), st["guess_failures"])
    assert out[1][2] == out[0][2]
    assert torch.equal(out[1][1], out[0][1]) and torch.equal(out[1][0], out[0][0])
    with _backend.plan_knobs(scan_seed=0):  # the plain scan from -inf: same scores, same order
        s0, i0 = ops.score_topk(Ut, It, k)
    assert torch.equal(out[1][1], i0.cpu()) and torch.equal(out[1][0], s0.cpu())


@pytest.mark.parametrize("slots", [0, 7])
def test_score_topk_dense_sample_chunked_units(slots):
    """Few users over a long catalog: one user block, so the sample plan splits
    its 131072 sample rows into catalog chunks (two on 256 slots; more with 7
    planned slots), each unit writing its tiles' maxima at the global tile
    index. Dense and compaction sample scans and the unseeded scan give
    identical lists, and the lists are exact (integer tables)."""
    rng = np.random.default_rng(4242 + slots)
    nu, ni, d, k = 70, 32 * 131072 + 45, 32, 300
    U, I = _int_table(rng, nu, d), _int_table(rng, ni, d)
    Ut, It = _bf16(U), _bf16(I)
    # stride 32 forced: k = 300 samples this 4.2M-row catalog at 64 by default
    knobs = {"guess_stride": 32, **({"scan_slots": slots} if slots else {})}
    with _backend.plan_knobs(**knobs):
        plan = ops.score_topk_plan(nu, ni, torch.bfloat16, d, k)
    assert plan["sample_stride"] == 32 and plan["sample_rows"] == 131072
    out = []
    for extra in ({}, {"sample_dense": 0}, {"scan_seed": 0}):
        with _backend.plan_knobs(**knobs, **extra):
            s, i = ops.score_topk(Ut, It, k)
        out.append((s.cpu(), i.cpu()))
    for s, i in out[1:]:
        assert torch.equal(i, out[0][1]) and torch.equal(s, out[0][0])
    ref_i, ref_s = _exact_topk_torch(U, I, k)
    assert np.array_equal(out[0][1].numpy().astype(np.int64), ref_i)


@pytest.mark.parametrize("d,k", [(128, 129), (64, 300), (256, 200), (32, 1000), (128, 1000)])
@pytest.mark.parametrize("kind", ["cosine", "dot", "euclidean"])
def test_ild_embedding_long_lists(d, k, kind):
    """Lists longer than the register-resident kernel's 128 rows (VERDICT r3,
    missing 5: the reference's user_ild takes any length): the streaming
    kernel, tile sums in double, against the float64 oracle; duplicates in a
    list (diagonal pairs) and a list with an out-of-range id (NaN, IndexError)."""
    rng = np.random.default_rng(d * 7 + k)
    ni = 5000
    E = oracle.as_bf16_f32(rng.standard_normal((ni, d)).astype(np.float32))
    recs = rng.integers(0, ni, size=(12, k))
    recs[1, : k // 2] = recs[1, 0]  # repeated items
    got = ops.ild_embedding(torch.from_numpy(recs).to(DEV), _bf16(E), kind).cpu().numpy()
    ref = oracle.ild_embedding_f64(recs, E, kind)
    assert np.allclose(got, ref, rtol=2e-5, atol=2e-5 * np.abs(ref).max())
    bad = recs.copy()
    bad[3, k - 1] = ni + 1
    out = ops.ild_embedding(torch.from_numpy(bad).to(DEV), _bf16(E), kind, check=False).cpu().numpy()
    assert np.isnan(out[3]) and np.allclose(np.delete(out, 3), np.delete(got, 3))
    with pytest.raises(IndexError):
        ops.ild_embedding(torch.from_numpy(bad).to(DEV), _bf16(E), kind)


@pytest.mark.parametrize("kind", ["cosine", "dot", "euclidean"])
def test_ild_embedding_longest_lists(kind):
    """The advertised upper bound, k = 16384 (64 KB of per-row terms in the
    dynamically sized LDS array), and k = 16383 (a partial last tile), at
    d = 32 against a float64 restatement of the reference's pair sum
    (divrec/losses/intra_list_diversity_score.py:36-42) on the device."""
    rng = np.random.default_rng(16384)
    ni, d = 20000, 32
    E = oracle.as_bf16_f32(rng.standard_normal((ni, d)).astype(np.float32))
    Et = torch.from_numpy(E).to(DEV).double()
    for k in (16384, 16383):
        recs = rng.integers(0, ni, size=(2, k))
        got = ops.ild_embedding(torch.from_numpy(recs).to(DEV), _bf16(E), kind).cpu().numpy()
        for u in range(2):
            x = Et[torch.from_numpy(recs[u]).to(DEV)]
            g = x @ x.t()
            if kind == "cosine":
                n = g.diagonal().sqrt()
                dist = 1.0 - g / (n[:, None] * n[None, :])
            elif kind == "dot":
                dist = g
            else:
                sq = g.diagonal()
                dist = (sq[:, None] + sq[None, :] - 2.0 * g).clamp_min(0.0).sqrt()
            ref = (dist.triu(1).sum() / (k * (k - 1))).item()
            scale = dist.abs().mean().item()
            assert abs(got[u] - ref) <= 2e-5 * max(abs(ref), scale), (k, u, got[u], ref)
            del g, dist


@pytest.mark.parametrize("k", [1025, 3000])
def test_ild_labels_long_lists_exact(k):
    """Label ILD beyond the 1024-entry LDS staging: exact counts, the same
    fp32 quotient as the short kernel (count / (k (k - 1)) in fp32)."""
    rng = np.random.default_rng(k)
    labels = rng.integers(0, 5, size=20000)
    recs = rng.integers(0, 20000, size=(20, k))
    got = ops.ild_labels(torch.from_numpy(recs).to(DEV), torch.from_numpy(labels).to(DEV)).cpu().numpy()
    assert np.array_equal(got, oracle.ild_labels(recs, labels))


def test_ild_drop_in_long_lists():
    """IntraListDiversityScore with a lazy EmbeddingDistance and 300-item lists
    (the reference's recommendations_loss at that length) equals the float64
    oracle within the embedding tolerance."""
    from divrec import losses
    from divrec.losses import EmbeddingDistance

    rng = np.random.default_rng(300)
    ni, d, k = 4000, 64, 300
    E = oracle.as_bf16_f32(rng.standard_normal((ni, d)).astype(np.float32))
    recs = torch.from_numpy(rng.integers(0, ni, size=(6, k)))
    ild = losses.IntraListDiversityScore(distance_matrix=EmbeddingDistance(torch.from_numpy(E), "cosine"),
                                         reduction="none")
    got = ild.recommendations_loss(None, recs).cpu().numpy()
    ref = oracle.ild_embedding_f64(recs.numpy(), E, "cosine")
    assert np.allclose(got, ref, rtol=2e-5, atol=2e-5)
