"""Drop-in API on the GPU against the golden vectors the REFERENCE produced
(tests/golden/make_golden.py). Every call goes through the divrec package ->
ctypes -> libdivrec_hip.so. Tolerances:
  * indices: exact on integer-valued tables; on float tables exact wherever
    the reference's neighbouring scores are separated by more than the score
    tolerance (bf16 products are exact in fp32, only the summation order
    differs: |ds| <= 1e-5 * sqrt(d/64) for O(1) scores);
  * ILD from a dense D: bit-exact (same fp32 accumulation order);
  * accuracy metrics on identical lists: rel 1e-6;
  * BPR loss rel 1e-6, grads rel 1e-5 (fp32 atomics reorder the sums).
"""
import os
import random

import numpy as np
import pytest
import torch

import oracle
from divrec import datasets, losses, metrics, models, ops, train
from topk_checks import fp32_row_tol, gap_check
from divrec.losses import EmbeddingDistance, LabelEquality

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")
DEV = torch.device("cuda", 0)


def load(name):
    return np.load(os.path.join(GOLD, f"{name}.npz"), allow_pickle=False)


def mf_from(U, I, device=DEV):
    mf = models.MatrixFactorization(U.shape[0], I.shape[0], U.shape[1])
    with torch.no_grad():
        mf.user_embeddings.weight.copy_(torch.from_numpy(U))
        mf.item_embeddings.weight.copy_(torch.from_numpy(I))
    return mf.to(device)


def ranking_dataset(g, n_users, n_items):
    train_ds = datasets.UserItemInteractionsDataset(torch.from_numpy(g["train"]),
                                                    number_of_users=n_users, number_of_items=n_items)
    test_ds = datasets.UserItemInteractionsDataset(torch.from_numpy(g["test"]),
                                                   number_of_users=n_users, number_of_items=n_items)
    return datasets.RankingDataset(test_ds, frozen=train_ds)


def assert_topk_gap_exact(got, ref, U, I, frozen_csr, tol):
    """got == ref except where the reference's own ordering is within tol."""
    S = U.astype(np.float64) @ I.astype(np.float64).T
    rowptr, cols = frozen_csr
    bad = 0
    for u in range(ref.shape[0]):
        if np.array_equal(got[u], ref[u]):
            continue
        s = S[u].copy()
        s[cols[rowptr[u]:rowptr[u + 1]]] = -np.inf
        # the returned list must be a valid top-k under a tol-perturbation:
        # sorted by score within tol, and no omitted item clearly better
        gs = s[got[u]]
        assert np.all(np.diff(gs) <= 2 * tol), u
        kth = np.sort(s)[::-1][len(ref[u]) - 1]
        assert np.all(gs >= kth - 2 * tol), u
        must = np.nonzero(s > kth + 2 * tol)[0]
        assert set(must.tolist()) <= set(got[u].tolist()), u
        bad += 1
    return bad


@pytest.mark.parametrize("d", [32, 64, 128])
def test_mf_forward_golden(d):
    g = load(f"mf_forward_d{d}")
    mf = mf_from(g["U"], g["I"])
    with torch.no_grad():
        out = mf(torch.from_numpy(g["uid"]), torch.from_numpy(g["iid"])).cpu().numpy()
    scale = np.abs(g["U"][g["uid"]] * g["I"][g["iid"]]).sum(axis=1)
    assert np.all(np.abs(out - g["out"]) <= 5e-7 * scale)


def test_mf_backward_matches_torch():
    g = load("mf_forward_d64")
    mf = mf_from(g["U"], g["I"])
    uid, iid = torch.from_numpy(g["uid"]), torch.from_numpy(g["iid"])
    w = torch.linspace(-1, 1, uid.numel())
    (mf(uid, iid) * w.to(DEV)).sum().backward()
    U = torch.from_numpy(g["U"]).requires_grad_()
    I = torch.from_numpy(g["I"]).requires_grad_()
    ((U[uid] * I[iid]).sum(1) * w).sum().backward()
    assert torch.allclose(mf.user_embeddings.weight.grad.cpu(), U.grad, rtol=1e-5, atol=1e-6)
    assert torch.allclose(mf.item_embeddings.weight.grad.cpu(), I.grad, rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("name", ["recs_int_k10", "recs_int_k100"])
def test_recommendations_integer_exact(name):
    g = load(name)
    U, I, k = g["U"], g["I"], int(g["k"])
    rds = ranking_dataset(g, U.shape[0], I.shape[0])
    recs = train.get_model_recommendations(rds, mf_from(U, I), k)
    assert recs.dtype == torch.int64 and recs.device.type == "cpu"
    assert np.array_equal(recs.numpy(), g["recs"])


@pytest.mark.parametrize("name", ["recs_float_k10", "recs_float_k100"])
def test_recommendations_float_gap_exact(name):
    g = load(name)
    U, I, k = g["U"], g["I"], int(g["k"])
    rds = ranking_dataset(g, U.shape[0], I.shape[0])
    recs = train.get_model_recommendations(rds, mf_from(U, I), k).numpy()
    rowptr, cols = rds.exclusion_csr()
    tol = 1e-5 * max(1.0, float(np.abs(U).max() * np.abs(I).max() * U.shape[1] / 8))
    bad = assert_topk_gap_exact(recs, g["recs"], U, I, (rowptr.numpy(), cols.numpy()), tol)
    assert bad <= U.shape[0] // 16


@pytest.mark.parametrize("name", ["recs_fp32_d100_k10", "recs_fp32_d100_k100",
                                  "recs_fp32_d100_k1000"])
def test_recommendations_raw_fp32_d100(name):
    """The reference's own model configuration: embedding_dim 100 (the
    experiments' config.yaml:7) and raw N(0,1) fp32 weights. The default
    (fp32-faithful) scoring equals the reference's lists except at near-ties
    of the exact scores (fp32 tolerance, tests/topk_checks.py)."""
    g = load(name)
    U, I, k = g["U"], g["I"], int(g["k"])
    rds = ranking_dataset(g, U.shape[0], I.shape[0])
    recs = train.get_model_recommendations(rds, mf_from(U, I), k)
    assert recs.dtype == torch.int64 and recs.shape == (U.shape[0], k)
    rowptr, cols = rds.exclusion_csr()
    bad = gap_check(recs.numpy(), g["recs"], U, I, (rowptr.numpy(), cols.numpy()),
                    fp32_row_tol(U, I))
    assert bad <= max(1, U.shape[0] // 32)


def test_recommendations_bf16_mode_is_explicit():
    """precision='bf16' ranks the tables' bf16 rounding (the fast mode): on
    raw fp32 weights it is NOT the reference's ranking, which is why fp32 is
    the default. Its lists equal the fp32 scan of the bf16-rounded tables."""
    g = load("recs_fp32_d100_k100")
    U, I = g["U"], g["I"]
    mf = mf_from(U, I)
    rds = ranking_dataset(g, U.shape[0], I.shape[0])
    excl = rds.exclusion_csr()
    items16, _ = mf.score_topk(100, exclude=excl, precision="bf16")
    rounded = mf_from(oracle.as_bf16_f32(U), oracle.as_bf16_f32(I))
    items32, _ = rounded.score_topk(100, exclude=excl, precision="fp32")
    assert torch.equal(items16, items32)
    assert (items16.cpu().numpy() != g["recs"]).any(axis=1).sum() > 0


def test_ml100k_d100_end_to_end():
    """configs[0] at the reference experiments' width: d=100, raw fp32 weights,
    top-10 + dense cosine ILD + accuracy / diversity metrics through
    recommendations_score_loop."""
    g = load("ml100k_d100")
    U, I = g["U"], g["I"]
    nu, ni = U.shape[0], I.shape[0]
    rds = ranking_dataset(g, nu, ni)
    mf = mf_from(U, I)
    It = torch.from_numpy(I)
    En = It / It.norm(dim=1, keepdim=True)
    ild = losses.IntraListDiversityScore(distance_matrix=1.0 - En @ En.T, reduction="none")
    te = torch.from_numpy(g["test"])
    res = train.recommendations_score_loop(rds, mf, [ild], 10)
    recs = train.get_model_recommendations(rds, mf, 10).numpy()
    rowptr, cols = rds.exclusion_csr()
    bad = gap_check(recs, g["recs"], U, I, (rowptr.numpy(), cols.numpy()), fp32_row_tol(U, I))
    assert bad <= nu // 100
    same = (recs == g["recs"]).all(axis=1)
    assert np.array_equal(res[0].cpu().numpy()[same], g["ild"][same])
    lazy = losses.IntraListDiversityScore(distance_matrix=EmbeddingDistance(It, "cosine"),
                                          reduction="none")  # d=100 zero-padded, bf16 Gram
    ref_recs = torch.from_numpy(g["recs"])
    assert np.allclose(lazy(None, ref_recs).cpu().numpy(), g["ild"], rtol=2e-3, atol=2e-3)
    for fn, key in ((metrics.precision_at_k, "precision"), (metrics.recall_at_k, "recall"),
                    (metrics.average_precision_at_k, "ap"),
                    (metrics.normalized_discounted_cumulative_gain, "ndcg")):
        assert np.allclose(fn(te, ref_recs).cpu().numpy(), g[key], rtol=1e-6, atol=1e-7), key


def test_scoring_tables_follow_fused_training():
    """train -> recommend -> train -> recommend: the fused Adam steps write the
    parameters through raw pointers; the scoring tables (cached padded fp32 at
    d=100, cached bf16) must follow them (the version bump in fused_adam_step)."""
    rng = np.random.default_rng(61)
    nu, ni, d = 30, 200, 100
    inter = np.stack([rng.integers(0, nu, 600), rng.integers(0, ni, 600)], axis=1)
    data = datasets.UserItemInteractionsDataset(
        torch.from_numpy(inter).long(), number_of_users=nu, number_of_items=ni,
        user_features=datasets.Features(torch.zeros(nu, 1), ["x"]),
        item_features=datasets.Features(torch.zeros(ni, 1), ["x"]))
    rds = datasets.RankingDataset(data, frozen=data)
    torch.manual_seed(2)
    mf = models.MatrixFactorization(nu, ni, d).to(DEV)
    opt = torch.optim.Adam(mf.parameters(), lr=5e-2)
    for precision in ("fp32", "bf16", "fp32"):
        random.seed(3)
        train.pair_wise_train_loop(datasets.PairWiseDataset(data, max_sampled=4), mf,
                                   losses.LogSigmoidDifferenceLoss(), opt, batch_size=64)
        got, _ = mf.score_topk(10, exclude=rds.exclusion_csr(), precision=precision)
        fresh = mf_from(mf.user_embeddings.weight.detach().cpu().numpy(),
                        mf.item_embeddings.weight.detach().cpu().numpy())
        want, _ = fresh.score_topk(10, exclude=rds.exclusion_csr(), precision=precision)
        assert torch.equal(got, want), precision


def test_get_model_recommendations_longer_than_scan_k():
    """k > 1024 (beyond dr_score_topk): the reference returns lists of any
    length (utils.py:53-77), so the MF path falls back to the per-user loop on
    the model's HIP forward. Integer tables: exact against the oracle."""
    rng = np.random.default_rng(1100)
    nu, ni, d, k = 6, 1500, 16, 1100
    U = rng.integers(-3, 4, size=(nu, d)).astype(np.float32)
    I = rng.integers(-3, 4, size=(ni, d)).astype(np.float32)
    tr = np.stack([np.repeat(np.arange(nu), 5), rng.integers(0, ni, nu * 5)], axis=1)
    te = np.stack([np.arange(nu), rng.integers(0, ni, nu)], axis=1)
    g = {"train": tr.astype(np.int64), "test": te.astype(np.int64)}
    rds = ranking_dataset(g, nu, ni)
    got = train.get_model_recommendations(rds, mf_from(U, I), k).numpy()
    frozen = [np.unique(tr[tr[:, 0] == u, 1]) for u in range(nu)]
    ref = oracle.recommend_topk(U, I, k, frozen=frozen)
    assert got.shape == (nu, k) and np.array_equal(got, ref)


@pytest.mark.parametrize("precision", ["fp32", "bf16"])
def test_score_topk_sees_data_writes(precision):
    """Writes through ``weight.data`` bump no autograd version:
    ranking after such a write must use the new weights (d = 100: the padded
    fp32 copy; bf16: the converted copy)."""
    torch.manual_seed(5)
    mf = models.MatrixFactorization(40, 300, 100).to(DEV)
    before, _ = mf.score_topk(10, precision=precision)
    mf.item_embeddings.weight.data.normal_()
    mf.user_embeddings.weight.data.mul_(-1.0)
    got, _ = mf.score_topk(10, precision=precision)
    fresh = mf_from(mf.user_embeddings.weight.detach().cpu().numpy(),
                    mf.item_embeddings.weight.detach().cpu().numpy())
    want, _ = fresh.score_topk(10, precision=precision)
    assert torch.equal(got, want) and not torch.equal(got, before)


def test_pair_wise_train_loop_out_of_range_raises():
    """A batch with an item id outside the model's table: the reference's
    nn.Embedding raises IndexError; so does the fused loop (host batches are
    checked before the upload)."""
    data = datasets.UserItemInteractionsDataset(
        torch.LongTensor([[0, 1], [1, 2], [1, 30]]), number_of_users=2, number_of_items=31,
        user_features=datasets.Features(torch.zeros(2, 1), ["x"]),
        item_features=datasets.Features(torch.zeros(31, 1), ["x"]))
    mf = models.MatrixFactorization(2, 20, 16).to(DEV)  # fewer items than the data
    opt = torch.optim.Adam(mf.parameters(), lr=1e-2)
    random.seed(1)
    with pytest.raises(IndexError):
        train.pair_wise_train_loop(datasets.PairWiseDataset(data, max_sampled=3), mf,
                                   losses.LogSigmoidDifferenceLoss(), opt, batch_size=4)


def test_recommendations_ragged_lists_raise_like_reference():
    """A user with fewer candidates than k: the reference's
    torch.LongTensor(recommendations) raises on ragged lists (utils.py:77);
    equal short lists come back short."""
    train_ds = datasets.UserItemInteractionsDataset(torch.LongTensor([[0, 1], [0, 2], [1, 3]]),
                                                    number_of_users=2, number_of_items=5)
    test_ds = datasets.UserItemInteractionsDataset(torch.LongTensor([[0, 0], [1, 0]]),
                                                   number_of_users=2, number_of_items=5)
    mf = models.MatrixFactorization(2, 5, 32).to(DEV)
    with pytest.raises(ValueError):
        train.get_model_recommendations(datasets.RankingDataset(test_ds, frozen=train_ds), mf, 4)
    recs = train.get_model_recommendations(datasets.RankingDataset(test_ds, frozen=train_ds), mf, 3)
    assert recs.shape == (2, 3)
    assert not set(recs[0].tolist()) & {1, 2} and 3 not in recs[1].tolist()


def test_ml100k_config1_end_to_end():
    """configs[0]: ML-100K-shaped MF d=32, top-10, cosine ILD + accuracy and
    diversity metrics, all through the drop-in API."""
    g = load("ml100k_cfg1")
    U, I = g["U"], g["I"]
    nu, ni = U.shape[0], I.shape[0]
    rds = ranking_dataset(g, nu, ni)
    mf = mf_from(U, I)
    recs = train.get_model_recommendations(rds, mf, 10)
    rowptr, cols = rds.exclusion_csr()
    bad = assert_topk_gap_exact(recs.numpy(), g["recs"], U, I, (rowptr.numpy(), cols.numpy()), 2e-5)
    assert bad <= nu // 50
    # ILD with the reference's dense cosine D (torch fp32, built like the reference)
    It = torch.from_numpy(I)
    En = It / It.norm(dim=1, keepdim=True)
    Dc = 1.0 - En @ En.T
    ild = losses.IntraListDiversityScore(distance_matrix=Dc, reduction="none")
    ref_recs = torch.from_numpy(g["recs"])
    assert np.array_equal(ild(None, ref_recs).cpu().numpy(), g["ild"])
    (res,) = train.recommendations_score_loop(rds, mf, [ild], 10)
    same = (recs.numpy() == g["recs"]).all(axis=1)
    assert np.array_equal(res.cpu().numpy()[same], g["ild"][same])
    # ILD with D computed on the fly from the embeddings (bf16 Gram tiles)
    lazy = losses.IntraListDiversityScore(distance_matrix=EmbeddingDistance(It, "cosine"),
                                          reduction="none")
    assert np.allclose(lazy(None, ref_recs).cpu().numpy(), g["ild"], rtol=1e-5, atol=2e-6)
    # accuracy metrics on the reference's lists
    te = torch.from_numpy(g["test"])
    for fn, key in ((metrics.precision_at_k, "precision"), (metrics.recall_at_k, "recall"),
                    (metrics.average_precision_at_k, "ap"),
                    (metrics.normalized_discounted_cumulative_gain, "ndcg")):
        assert np.allclose(fn(te, ref_recs).cpu().numpy(), g[key], rtol=1e-6, atol=1e-7), key
    full = datasets.UserItemInteractionsDataset(torch.cat([torch.from_numpy(g["train"]), te]),
                                                number_of_users=nu, number_of_items=ni)
    assert float(metrics.EntropyDiversityScore(dataset=full)(te, ref_recs)) == pytest.approx(
        float(g["entropy"]), rel=1e-6)
    assert float(metrics.PRI(dataset=full)(te, ref_recs)) == pytest.approx(float(g["pri"]), rel=1e-5)
    assert float(metrics.MeanAveragePrecisionAtKScore()(te, ref_recs)) == pytest.approx(
        float(g["map"]), rel=1e-6)


@pytest.mark.parametrize("k", [1, 2, 10, 100])
def test_ild_dense_golden_bit_exact(k):
    g = load(f"ild_dense_k{k}")
    D = torch.from_numpy(g["D"])
    recs = torch.from_numpy(g["recs"]).to(DEV)
    got = losses.IntraListDiversityScore(distance_matrix=D, reduction="none")(None, recs)
    assert np.array_equal(got.cpu().numpy(), g["out"], equal_nan=True)
    if k > 1:
        s = losses.IntraListDiversityScore(distance_matrix=D, reduction="sum")(None, recs)
        assert float(s) == pytest.approx(float(g["sum"]), rel=1e-6)
    # user_ild: the reference's raw combinations sum per list, bit-exact (0 for k = 1)
    raw = [losses.IntraListDiversityScore.user_ild(row, D) for row in recs.cpu()]
    if k == 1:
        assert all(v == 0 for v in raw)
    else:
        assert all(v.dtype == D.dtype and v.dim() == 0 for v in raw)
    assert np.array_equal(np.asarray([float(v) for v in raw], dtype=np.float32), g["user_ild"])


def test_ild_labels_golden():
    g = load("ild_labels")
    recs = torch.from_numpy(g["recs"])
    lab = torch.from_numpy(g["labels"])
    got = losses.IntraListDiversityScore(distance_matrix=LabelEquality(lab), reduction="none")
    assert np.array_equal(got(None, recs).cpu().numpy(), g["out"])
    ds = datasets.UserItemInteractionsDataset(
        torch.LongTensor([[0, 0]]), number_of_items=lab.numel(),
        item_features=datasets.Features(lab[:, None].float(), ["partition"]))
    unf = losses.IntraListBinaryUnfairnessScore(dataset=ds, reduction="none")
    assert np.array_equal(unf(None, recs).cpu().numpy(), g["out"])


def test_ild_cosine_golden():
    g = load("ild_cosine")
    recs = torch.from_numpy(g["recs"])
    dense = losses.IntraListDiversityScore(distance_matrix=torch.from_numpy(g["D"]), reduction="none")
    assert np.array_equal(dense(None, recs).cpu().numpy(), g["out"])
    lazy = losses.IntraListDiversityScore(
        distance_matrix=EmbeddingDistance(torch.from_numpy(g["E"]), "cosine"), reduction="none")
    assert np.allclose(lazy(None, recs).cpu().numpy(), g["out"], rtol=1e-5, atol=2e-6)


def test_bpr_step_golden():
    g = load("bpr_step")
    mf = mf_from(g["U0"], g["I0"])
    opt = torch.optim.Adam(mf.parameters(), lr=1e-3)
    U, I = mf.user_embeddings.weight, mf.item_embeddings.weight
    U.grad, I.grad = torch.zeros_like(U), torch.zeros_like(I)
    B = g["uid"].size
    lv, hit = ops.bpr_fwd_bwd(U.data, I.data, *(torch.from_numpy(g[n]).to(DEV)
                                                 for n in ("uid", "pid", "nid")), 1.0 / B, U.grad, I.grad)
    assert float(lv.sum() / B) == pytest.approx(float(g["loss"]), rel=1e-6)
    assert float(hit.float().mean()) == pytest.approx(float(g["auc"]), abs=1e-7)
    assert np.allclose(U.grad.cpu().numpy(), g["gU"], rtol=1e-5, atol=1e-8)
    assert np.allclose(I.grad.cpu().numpy(), g["gI"], rtol=1e-5, atol=1e-8)
    train.fused_adam_step(opt)
    assert np.allclose(U.detach().cpu().numpy(), g["U1"], rtol=0, atol=1e-6)
    assert np.allclose(I.detach().cpu().numpy(), g["I1"], rtol=0, atol=1e-6)


def test_pair_wise_train_loop_golden():
    g = load("bpr_loop")
    tr = torch.from_numpy(g["train"])
    data = datasets.UserItemInteractionsDataset(
        tr, user_features=datasets.Features(torch.zeros(12, 1), ["x"]),
        item_features=datasets.Features(torch.zeros(40, 1), ["x"]))
    mf = mf_from(g["U0"], g["I0"])
    random.seed(int(g["seed"]))
    pw = datasets.PairWiseDataset(data, max_sampled=int(g["max_sampled"]))
    opt = torch.optim.Adam(mf.parameters(), lr=float(g["lr"]))
    mean_loss, (mean_auc,) = train.pair_wise_train_loop(
        pw, mf, losses.LogSigmoidDifferenceLoss(), opt, scores=[metrics.AUCScore()],
        batch_size=int(g["batch_size"]))
    assert mean_loss == pytest.approx(float(g["mean_loss"]), rel=1e-5)
    assert mean_auc == pytest.approx(float(g["mean_auc"]), abs=1e-6)
    assert np.allclose(mf.user_embeddings.weight.detach().cpu().numpy(), g["U1"], atol=1e-5)
    assert np.allclose(mf.item_embeddings.weight.detach().cpu().numpy(), g["I1"], atol=1e-5)


def test_rank_metrics_against_oracle_formulas():
    rng = np.random.default_rng(3)
    nu, ni, k = 200, 500, 37
    recs = torch.from_numpy(np.stack([rng.choice(ni, k, replace=False) for _ in range(nu)]))
    inter = torch.from_numpy(np.stack([np.repeat(np.arange(nu), 12),
                                       rng.integers(0, ni, nu * 12)], 1))
    inter[inter[:, 0] == 5, 0] = 6  # user 5 has no positives: recall NaN
    p, r, ap, nd = (f(inter, recs).cpu().numpy() for f in (
        metrics.precision_at_k, metrics.recall_at_k, metrics.average_precision_at_k,
        metrics.normalized_discounted_cumulative_gain))
    for u in range(nu):
        pos = inter[inter[:, 0] == u, 1].numpy()
        rel = np.isin(recs[u].numpy(), pos).astype(np.float64)
        assert p[u] == pytest.approx(rel.sum() / k, rel=1e-6)
        if len(pos):
            assert r[u] == pytest.approx(rel.sum() / len(pos), rel=1e-6)
        else:
            assert np.isnan(r[u])
        cum = np.cumsum(rel) / np.arange(1, k + 1)
        assert ap[u] == pytest.approx(cum.sum() / k, rel=1e-5, abs=1e-7)
        disc = 1 / np.log2(np.arange(2, k + 2))
        assert nd[u] == pytest.approx((rel * disc).sum() / disc.sum(), rel=1e-5, abs=1e-7)


def test_score_topk_api_exclusion_and_user_subset():
    rng = np.random.default_rng(11)
    U = rng.integers(-3, 4, size=(50, 64)).astype(np.float32)
    I = rng.integers(-3, 4, size=(3000, 64)).astype(np.float32)
    mf = mf_from(U, I)
    frozen = [sorted(set(rng.integers(0, 3000, 40).tolist())) for _ in range(20)]
    rowptr, cols = oracle.exclusion_csr(frozen)
    uids = torch.arange(10, 30)
    items, scores = mf.score_topk(25, user_ids=uids, exclude=(torch.from_numpy(rowptr),
                                                             torch.from_numpy(cols)))
    ref = oracle.recommend_topk(U[10:30], I, 25, frozen=frozen)
    assert np.array_equal(items.cpu().numpy(), ref)


# --------------------------------------------------------------------------- lazy (row-sparse) Adam
def _sparse_adam_reference(P0, steps, lr, betas, eps):
    """torch.optim.SparseAdam on the CPU, fp32: steps = [(rows, grad_values)]."""
    p = torch.nn.Parameter(torch.from_numpy(P0.copy()))
    opt = torch.optim.SparseAdam([p], lr=lr, betas=betas, eps=eps)
    for rows, vals in steps:
        p.grad = torch.sparse_coo_tensor(torch.from_numpy(rows)[None, :], torch.from_numpy(vals),
                                         P0.shape).coalesce()
        opt.step()
    st = opt.state[p]
    return p.detach().numpy(), st["exp_avg"].numpy(), st["exp_avg_sq"].numpy()


def test_adam_rows_vs_torch_sparse_adam():
    """dr_adam_rows over three steps with different row sets, against
    (1) the oracle's restatement of SparseAdam's fp32 op sequence with IEEE
    sqrt / division: bit-exact for param, exp_avg, exp_avg_sq;
    (2) torch.optim.SparseAdam on the CPU: exp_avg / exp_avg_sq bit-exact,
    param within 1e-6 (torch's CPU vector sqrt is not correctly rounded: the
    last bit differs for ~0.7 % of inputs). Untouched rows keep their values
    and the touched gradient rows are zeroed."""
    rng = np.random.default_rng(31)
    n, d, lr, betas, eps = 500, 100, 3e-3, (0.85, 0.995), 1e-7
    P0 = rng.standard_normal((n, d)).astype(np.float32)
    steps = []
    for _ in range(3):
        rows = np.sort(rng.choice(n, size=137, replace=False)).astype(np.int64)
        vals = (rng.standard_normal((rows.size, d)) * 0.1).astype(np.float32)
        steps.append((rows, vals))
    refP, refM, refV = _sparse_adam_reference(P0, steps, lr, betas, eps)
    oP, oM, oV = P0.copy(), np.zeros_like(P0), np.zeros_like(P0)
    for t, (rows, vals) in enumerate(steps, start=1):
        oracle.sparse_adam_rows(oP, oM, oV, rows, vals, t, lr, *betas, eps)
    P = torch.from_numpy(P0).to(DEV)
    M, V = torch.zeros_like(P), torch.zeros_like(P)
    G = torch.zeros_like(P)
    for t, (rows, vals) in enumerate(steps, start=1):
        r = torch.from_numpy(rows).to(DEV)
        G[r] = torch.from_numpy(vals).to(DEV)
        ops.adam_rows(P, G, M, V, r[torch.randperm(r.numel(), device=DEV)], lr, *betas, eps, t)
        assert int(torch.count_nonzero(G)) == 0  # touched rows zeroed, the rest stayed zero
    assert np.array_equal(P.cpu().numpy(), oP)
    assert np.array_equal(M.cpu().numpy(), oM)
    assert np.array_equal(V.cpu().numpy(), oV)
    assert np.array_equal(M.cpu().numpy(), refM)
    assert np.array_equal(V.cpu().numpy(), refV)
    assert np.allclose(P.cpu().numpy(), refP, rtol=0, atol=1e-6)


def test_pair_wise_train_loop_sparse_adam():
    """pair_wise_train_loop with torch.optim.SparseAdam takes the fused BPR
    kernel + dr_adam_rows path. Reference: the same batches through an
    nn.Embedding(sparse=True) copy of the model and torch's SparseAdam on the
    CPU. Gradients differ only by the fp32 atomic summation order (rel 1e-5),
    so the parameters after the epoch agree within 1e-5."""
    rng = np.random.default_rng(8)
    nu, ni, d, lr = 12, 40, 32, 1e-2
    U0 = rng.standard_normal((nu, d)).astype(np.float32)
    I0 = rng.standard_normal((ni, d)).astype(np.float32)
    inter = np.stack([rng.integers(0, nu, 150), rng.integers(0, ni, 150)], axis=1)
    data = datasets.UserItemInteractionsDataset(
        torch.from_numpy(inter).long(), number_of_users=nu, number_of_items=ni,
        user_features=datasets.Features(torch.zeros(nu, 1), ["x"]),
        item_features=datasets.Features(torch.zeros(ni, 1), ["x"]))
    random.seed(5)
    pw = datasets.PairWiseDataset(data, max_sampled=4)
    batches = [(u.clone(), p.clone(), n.clone()) for u, p, n, *_ in pw.loader(batch_size=64)]

    mf = mf_from(U0, I0)
    opt = torch.optim.SparseAdam(list(mf.parameters()), lr=lr)
    random.seed(5)
    pw = datasets.PairWiseDataset(data, max_sampled=4)
    mean_loss, (mean_auc,) = train.pair_wise_train_loop(
        pw, mf, losses.LogSigmoidDifferenceLoss(), opt, scores=[metrics.AUCScore()],
        batch_size=64)

    Ue = torch.nn.Embedding(nu, d, sparse=True)
    Ie = torch.nn.Embedding(ni, d, sparse=True)
    with torch.no_grad():
        Ue.weight.copy_(torch.from_numpy(U0))
        Ie.weight.copy_(torch.from_numpy(I0))
    ref_opt = torch.optim.SparseAdam(list(Ue.parameters()) + list(Ie.parameters()), lr=lr)
    ref_losses = []
    for u, p, n in batches:
        sp = torch.sum(Ue(u) * Ie(p), dim=1)
        sn = torch.sum(Ue(u) * Ie(n), dim=1)
        loss = -torch.nn.functional.logsigmoid(sp - sn).mean()
        loss.backward()
        ref_opt.step()
        ref_opt.zero_grad()
        ref_losses.append(float(loss.detach()))
    assert mean_loss == pytest.approx(sum(ref_losses) / len(ref_losses), rel=1e-5)
    assert np.allclose(mf.user_embeddings.weight.detach().cpu().numpy(),
                       Ue.weight.detach().numpy(), rtol=0, atol=1e-5)
    assert np.allclose(mf.item_embeddings.weight.detach().cpu().numpy(),
                       Ie.weight.detach().numpy(), rtol=0, atol=1e-5)


# --------------------------------------------------------------------------- device pairwise sampler
def _sampler_fixture(rng, nu=60, ni=500):
    inter = np.stack([np.repeat(np.arange(nu), 6), rng.integers(0, ni, nu * 6)], axis=1)
    inter = np.concatenate([inter, inter[:40]])  # duplicate pairs: frozenset semantics
    frozen = np.stack([rng.integers(0, nu, 900), rng.integers(0, ni, 900)], axis=1)
    data = datasets.UserItemInteractionsDataset(torch.from_numpy(inter).long(),
                                                number_of_users=nu, number_of_items=ni)
    fz = datasets.UserItemInteractionsDataset(torch.from_numpy(frozen).long(),
                                              number_of_users=nu, number_of_items=ni)
    pos = [set(inter[inter[:, 0] == u, 1].tolist()) for u in range(nu)]
    frz = [set(frozen[frozen[:, 0] == u, 1].tolist()) for u in range(nu)]
    return data, fz, pos, frz


def test_sample_pairwise_layout_membership_determinism():
    """dr_sample_pairwise vs the reference's PairWiseDataset contract
    (base_datasets.py:70-107): every positive is one of the user's positives,
    every negative is outside positives and frozen, triples are the m x m
    product in positive-major order for users in order; same seed -> same
    draws, another seed -> other draws."""
    rng = np.random.default_rng(40)
    data, fz, pos, frz = _sampler_fixture(rng)
    m = 16
    ds = datasets.DevicePairWiseDataset(data, frozen=fz, max_sampled=m, device=DEV, seed=3)
    users = torch.arange(60, device=DEV)
    p, n, (uid, pid, nid) = ops.sample_pairwise(users, *ds.pos_csr, 500, m, 77, exclude=ds.excl_csr)
    p, n = p.cpu().numpy(), n.cpu().numpy()
    uid, pid, nid = (t.cpu().numpy().reshape(60, m, m) for t in (uid, pid, nid))
    for u in range(60):
        assert set(p[u].tolist()) <= pos[u]
        assert not (set(n[u].tolist()) & (pos[u] | frz[u]))
        assert n[u].min() >= 0 and n[u].max() < 500
        assert np.all(uid[u] == u)
        assert np.array_equal(pid[u], np.repeat(p[u][:, None], m, axis=1))  # positive-major
        assert np.array_equal(nid[u], np.repeat(n[u][None, :], m, axis=0))
    p2, n2, _ = ops.sample_pairwise(users, *ds.pos_csr, 500, m, 77, exclude=ds.excl_csr,
                                    expand=False)
    assert np.array_equal(p2.cpu().numpy(), p) and np.array_equal(n2.cpu().numpy(), n)
    p3, n3, _ = ops.sample_pairwise(users, *ds.pos_csr, 500, m, 78, exclude=ds.excl_csr,
                                    expand=False)
    assert not np.array_equal(n3.cpu().numpy(), n)


def test_sample_pairwise_uniform():
    """Draws are uniform over the populations random.choices samples: the
    user's unique positives and items - positives - frozen (chi-square,
    p > 1e-4 for each)."""
    from scipy.stats import chisquare
    ni, m = 400, 40000
    inter = np.array([[0, i] for i in (3, 9, 9, 27, 100, 250, 399)], dtype=np.int64)
    frozen = np.array([[0, i] for i in range(150, 200)], dtype=np.int64)
    data = datasets.UserItemInteractionsDataset(torch.from_numpy(inter), number_of_users=1,
                                                number_of_items=ni)
    fz = datasets.UserItemInteractionsDataset(torch.from_numpy(frozen), number_of_users=1,
                                              number_of_items=ni)
    ds = datasets.DevicePairWiseDataset(data, frozen=fz, max_sampled=1, device=DEV)
    p, n, _ = ops.sample_pairwise(torch.zeros(1, dtype=torch.int64, device=DEV), *ds.pos_csr, ni,
                                  m, 5, exclude=ds.excl_csr, expand=False)
    p, n = p.cpu().numpy().ravel(), n.cpu().numpy().ravel()
    P = [3, 9, 27, 100, 250, 399]
    allowed = sorted(set(range(ni)) - set(P) - set(range(150, 200)))
    assert set(p.tolist()) == set(P) and set(n.tolist()) <= set(allowed)
    assert chisquare([np.sum(p == i) for i in P]).pvalue > 1e-4
    assert chisquare([np.sum(n == i) for i in allowed]).pvalue > 1e-4


def test_sample_pairwise_user_without_positives_raises():
    data = datasets.UserItemInteractionsDataset(torch.tensor([[0, 1], [2, 3]]),
                                                number_of_users=3, number_of_items=10)
    ds = datasets.DevicePairWiseDataset(data, max_sampled=2, device=DEV)
    with pytest.raises(IndexError):  # the reference: random.choices([]) -> IndexError
        list(ds.loader(batch_size=4))


def test_device_pairwise_dataset_trains():
    """pair_wise_train_loop over DevicePairWiseDataset (fused BPR + fused Adam):
    every batch but the last has batch_size triples, the loss falls over
    epochs and AUC rises above chance."""
    rng = np.random.default_rng(41)
    data, fz, _, _ = _sampler_fixture(rng)
    ds = datasets.DevicePairWiseDataset(data, frozen=fz, max_sampled=10, device=DEV, seed=1)
    sizes = [b[0].numel() for b in ds.loader(batch_size=512)]
    assert sum(sizes) == 60 * 100 and all(s == 512 for s in sizes[:-1])
    torch.manual_seed(0)
    mf = models.MatrixFactorization(60, 500, 32).to(DEV)
    opt = torch.optim.Adam(mf.parameters(), lr=5e-2)
    hist = [train.pair_wise_train_loop(ds, mf, losses.LogSigmoidDifferenceLoss(), opt,
                                       scores=[metrics.AUCScore()], batch_size=512)
            for _ in range(5)]
    assert all(np.isfinite(h[0]) for h in hist)
    assert hist[-1][0] < hist[0][0]
    assert hist[-1][1][0] > 0.6


class _DeviceBatches:
    """A PairWiseDataset stand-in whose loader yields device batches (as
    DevicePairWiseDataset does): (user, pos, neg, None, None, None)."""

    def __init__(self, batches):
        self.batches = batches

    def loader(self, **_):
        for u, p, n in self.batches:
            yield u, p, n, None, None, None


@pytest.mark.parametrize("sparse", [False, True])
def test_pair_wise_train_loop_bad_device_batch_leaves_no_trace(sparse):
    """A device batch with an out-of-range item id raises IndexError before
    the fused kernel runs: the gradient tables stay as they were,
    so a caller that catches the error and trains on gets exactly the clean
    run's weights (dense Adam and the lazy SparseAdam path)."""
    torch.manual_seed(3)
    nu, ni, d = 50, 80, 32
    a = models.MatrixFactorization(nu, ni, d).to(DEV)
    b = models.MatrixFactorization(nu, ni, d).to(DEV)
    b.load_state_dict(a.state_dict())
    mk = (lambda m: torch.optim.SparseAdam(m.parameters(), lr=1e-2)) if sparse else \
        (lambda m: torch.optim.Adam(m.parameters(), lr=1e-2))
    oa, ob = mk(a), mk(b)
    g = torch.Generator(device=DEV).manual_seed(5)
    good = [tuple(torch.randint(0, n, (64,), generator=g, device=DEV) for n in (nu, ni, ni))
            for _ in range(2)]
    bad_n = good[0][2].clone()
    bad_n[17] = ni + 3
    loss = losses.LogSigmoidDifferenceLoss()
    with pytest.raises(IndexError):
        train.pair_wise_train_loop(_DeviceBatches([(good[0][0], good[0][1], bad_n)]), a, loss, oa)
    for m in (a,):
        for p_ in m.parameters():
            assert p_.grad is None or not p_.grad.any()  # nothing was accumulated
    train.pair_wise_train_loop(_DeviceBatches(good), a, loss, oa)
    train.pair_wise_train_loop(_DeviceBatches(good), b, loss, ob)
    for pa, pb in zip(a.parameters(), b.parameters()):
        assert torch.equal(pa, pb)
