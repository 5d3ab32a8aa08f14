"""Pin the CPU oracle to the golden vectors produced by the REFERENCE itself
(tests/golden/make_golden.py). CPU only; bit-exact where the reference is
deterministic."""
import os

import numpy as np
import pytest

import oracle
from topk_checks import fp32_row_tol, gap_check

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def load(name):
    return np.load(os.path.join(GOLD, f"{name}.npz"), allow_pickle=False)


@pytest.mark.parametrize("d", [32, 64, 128])
def test_mf_forward(d):
    g = load(f"mf_forward_d{d}")
    got = oracle.mf_forward(g["U"], g["I"], g["uid"], g["iid"])
    # torch.sum(dim=1) and numpy's sum differ only in summation order:
    # |delta| <= 8 eps_fp32 * sum_d |u_d i_d|
    scale = np.abs(g["U"][g["uid"]] * g["I"][g["iid"]]).sum(axis=1)
    assert np.all(np.abs(got - g["out"]) <= 5e-7 * scale)


def _frozen(train, n_users):
    fz = [[] for _ in range(n_users)]
    for u, i in train:
        fz[int(u)].append(int(i))
    return fz


@pytest.mark.parametrize("name", ["recs_float_k10", "recs_float_k100", "recs_int_k10", "recs_int_k100"])
def test_recommendations(name):
    g = load(name)
    U, I, k = g["U"], g["I"], int(g["k"])
    recs = oracle.recommend_topk(U, I, k, frozen=_frozen(g["train"], U.shape[0]))
    assert np.array_equal(recs, g["recs"])


@pytest.mark.parametrize("name", ["recs_fp32_d100_k10", "recs_fp32_d100_k100",
                                  "recs_fp32_d100_k1000", "ml100k_d100"])
def test_recommendations_raw_fp32(name):
    """Raw N(0,1) fp32 tables at d=100: the oracle's fp32 sums (numpy order)
    against the reference's (torch order) — equal except at near-ties."""
    g = load(name)
    U, I = g["U"], g["I"]
    k = int(g["k"]) if "k" in g.files else 10
    frozen = _frozen(g["train"], U.shape[0])
    recs = oracle.recommend_topk(U, I, k, frozen=frozen)
    bad = gap_check(recs, g["recs"], U, I, oracle.exclusion_csr(frozen), fp32_row_tol(U, I))
    assert bad <= max(1, U.shape[0] // 64)
    if name == "ml100k_d100":
        ild = oracle.ild_embedding_f64(g["recs"], I, "cosine")
        assert np.allclose(ild, g["ild"], rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("k", [1, 2, 10, 100])
def test_ild_dense_bit_exact(k):
    g = load(f"ild_dense_k{k}")
    got = oracle.ild_sequential(g["recs"], g["D"])
    assert np.array_equal(got, g["out"], equal_nan=True)
    if k > 1:
        assert np.float32(np.sum(got.astype(np.float64))) == pytest.approx(float(g["sum"]), rel=1e-6)
    assert bool(g["mean_raises"])  # the reference's 'mean' forward raises IndexError
    # user_ild: the raw pair sums, exactly the reference's values
    assert np.array_equal(oracle.ild_pair_sums(g["recs"], g["D"]).astype(np.float32),
                          g["user_ild"])


def test_ild_labels_exact():
    g = load("ild_labels")
    assert np.array_equal(oracle.ild_labels(g["recs"], g["labels"]), g["out"])
    D = (g["labels"][:, None] == g["labels"][None, :]).astype(np.int32)
    assert np.array_equal(oracle.ild_sequential(g["recs"], D), g["out"])


def test_ild_cosine_from_dense():
    g = load("ild_cosine")
    assert np.array_equal(oracle.ild_sequential(g["recs"], g["D"]), g["out"])
    f64 = oracle.ild_embedding_f64(g["recs"], g["E"], "cosine")
    assert np.allclose(f64, g["out"], rtol=2e-6, atol=1e-6)


def test_bpr_step():
    g = load("bpr_step")
    loss, auc, gU, gI = oracle.bpr_forward_backward(g["U0"], g["I0"], g["uid"], g["pid"], g["nid"])
    assert loss == pytest.approx(float(g["loss"]), rel=1e-6)
    assert auc == pytest.approx(float(g["auc"]), abs=1e-7)
    assert np.allclose(gU, g["gU"], rtol=1e-5, atol=1e-8)
    assert np.allclose(gI, g["gI"], rtol=1e-5, atol=1e-8)
    # one Adam(lr=1e-3) step from zero moments
    U1, _, _ = oracle.adam_step(g["U0"], g["gU"], 0.0, 0.0, step=1)
    I1, _, _ = oracle.adam_step(g["I0"], g["gI"], 0.0, 0.0, step=1)
    assert np.allclose(U1, g["U1"], rtol=0, atol=2e-7)
    assert np.allclose(I1, g["I1"], rtol=0, atol=2e-7)


def test_reference_torch_restatements():
    """The torch restatements bench.py times as CPU baselines reproduce the
    reference: MatrixFactorization.forward and one pair_wise_train_loop batch
    (loss, Adam step) bit for bit against the reference-generated fixtures."""
    import torch

    for d in (32, 64, 128):
        g = load(f"mf_forward_d{d}")
        out = oracle.reference_mf_forward(torch.from_numpy(g["U"]), torch.from_numpy(g["I"]),
                                          torch.from_numpy(g["uid"]), torch.from_numpy(g["iid"]))
        assert np.array_equal(out.numpy(), g["out"])
    g = load("bpr_step")
    losses, U1, I1 = oracle.reference_bpr_steps(
        torch.from_numpy(g["U0"]), torch.from_numpy(g["I0"]),
        [(torch.from_numpy(g["uid"]), torch.from_numpy(g["pid"]), torch.from_numpy(g["nid"]))])
    assert np.float32(losses[0]) == g["loss"]
    assert np.array_equal(U1.numpy(), g["U1"]) and np.array_equal(I1.numpy(), g["I1"])


def test_ml100k_cfg1_recs_and_ild():
    g = load("ml100k_cfg1")
    U, I = g["U"], g["I"]
    recs = oracle.recommend_topk(U, I, 10, frozen=_frozen(g["train"], U.shape[0]))
    assert np.array_equal(recs, g["recs"])
    En = I / np.linalg.norm(I.astype(np.float64), axis=1, keepdims=True)
    ild = oracle.ild_embedding_f64(g["recs"], I, "cosine")
    assert np.allclose(ild, g["ild"], rtol=1e-5, atol=1e-6)
    del En


def test_topk_merge_equals_single_pass_k1000():
    rng = np.random.default_rng(3)
    U = rng.integers(-2, 3, size=(6, 16)).astype(np.float32)
    I = rng.integers(-2, 3, size=(5000, 16)).astype(np.float32)
    full_i, full_s = oracle.recommend_topk(U, I, 1000, return_scores=True)
    bounds = np.linspace(0, 5000, 9).astype(int)
    parts = [oracle.recommend_topk(U, I[lo:hi], 1000, return_scores=True)
             for lo, hi in zip(bounds[:-1], bounds[1:])]
    ms, mi = oracle.topk_merge(np.stack([p[1] for p in parts]),
                               np.stack([p[0] + lo for p, lo in zip(parts, bounds)]), 1000)
    assert np.array_equal(mi, full_i)
    assert np.array_equal(ms, full_s)


def test_topk_merge_equals_single_pass():
    rng = np.random.default_rng(0)
    U = rng.integers(-2, 3, size=(20, 16)).astype(np.float32)
    I = rng.integers(-2, 3, size=(1000, 16)).astype(np.float32)
    full_i, full_s = oracle.recommend_topk(U, I, 30, return_scores=True)
    parts_s, parts_i = [], []
    for lo, hi in ((0, 333), (333, 700), (700, 1000)):
        i, s = oracle.recommend_topk(U, I[lo:hi], 30, return_scores=True)
        parts_s.append(s)
        parts_i.append(i + lo)
    ms, mi = oracle.topk_merge(np.stack(parts_s), np.stack(parts_i), 30)
    assert np.array_equal(mi, full_i)
    assert np.array_equal(ms, full_s)


def test_mmr_lambda_one_is_topk():
    rng = np.random.default_rng(1)
    E = rng.standard_normal((200, 8))
    cand = np.stack([rng.choice(200, 50, replace=False) for _ in range(4)])
    sc = rng.standard_normal((4, 50))
    got = oracle.mmr_greedy(cand, sc, E, 10, 1.0)
    ref = np.take_along_axis(cand, np.argsort(-sc, axis=1, kind="stable")[:, :10], axis=1)
    assert np.array_equal(got, ref)
    assert oracle.mmr_check(got, cand, sc, E, 1.0) == 0
    got5 = oracle.mmr_greedy(cand, sc, E, 10, 0.5)
    assert oracle.mmr_check(got5, cand, sc, E, 0.5) == 0


def test_oracle_sparse_adam_rows_vs_torch():
    """The oracle's SparseAdam restatement (the bit-exact target of
    dr_adam_rows) against torch.optim.SparseAdam on the CPU: moments bit-exact;
    the parameter within 1e-6 (torch's CPU vector sqrt is not correctly
    rounded, the oracle's is)."""
    import torch
    rng = np.random.default_rng(12)
    n, d, lr, betas, eps = 200, 48, 1e-2, (0.9, 0.999), 1e-8
    P0 = rng.standard_normal((n, d)).astype(np.float32)
    p = torch.nn.Parameter(torch.from_numpy(P0.copy()))
    opt = torch.optim.SparseAdam([p], lr=lr, betas=betas, eps=eps)
    oP, oM, oV = P0.copy(), np.zeros_like(P0), np.zeros_like(P0)
    for t in range(1, 4):
        rows = np.sort(rng.choice(n, size=60, replace=False)).astype(np.int64)
        vals = rng.standard_normal((rows.size, d)).astype(np.float32)
        p.grad = torch.sparse_coo_tensor(torch.from_numpy(rows)[None, :], torch.from_numpy(vals),
                                         P0.shape).coalesce()
        opt.step()
        oracle.sparse_adam_rows(oP, oM, oV, rows, vals, t, lr, *betas, eps)
    st = opt.state[p]
    assert np.array_equal(oM, st["exp_avg"].numpy())
    assert np.array_equal(oV, st["exp_avg_sq"].numpy())
    assert np.allclose(oP, p.detach().numpy(), rtol=0, atol=1e-6)
