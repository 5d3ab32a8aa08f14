"""Host-side logic on CPU: datasets, CSR builders, naming, planner-independent
API behaviour. No GPU calls."""
import os

import numpy as np
import pytest
import torch

import oracle
from divrec.datasets import Features, PairWiseDataset, RankingDataset, UserItemInteractionsDataset
from divrec.distributed import shard_range
from divrec.losses import IntraListDiversityScore, LogSigmoidDifferenceLoss
from divrec.metrics import AUCScore, PrecisionAtKScore
from divrec.models import MatrixFactorization, RandomModel
from divrec.utils import to_camel_case

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def test_metric_names():
    assert to_camel_case("IntraListDiversityScore") == "intra_list_diversity_score"
    assert to_camel_case("AUCScore") == "auc_score"
    assert to_camel_case("PRI") == "pri"
    assert IntraListDiversityScore(distance_matrix=None).name == "intra_list_diversity_score"
    assert PrecisionAtKScore().name == "precision_atk_score"  # the reference rule, verbatim


def test_interactions_dataset_derivations():
    inter = torch.LongTensor([[0, 3], [2, 1], [2, 5]])
    ds = UserItemInteractionsDataset(inter)
    assert (ds.number_of_users, ds.number_of_items, ds.number_of_interactions) == (3, 6, 3)
    assert torch.equal(ds.interaction_scores, torch.ones(3))
    ds2 = UserItemInteractionsDataset(inter, number_of_users=10, number_of_items=4)
    assert (ds2.number_of_users, ds2.number_of_items) == (10, 6)
    with pytest.raises(AssertionError):
        UserItemInteractionsDataset(torch.LongTensor([[0, 1, 2]]))
    f = Features(torch.zeros(6, 2), ["a", "partition"])
    assert "partition" in f and len(f) == 6 and f["partition"].shape == (6,)


def test_ranking_dataset_candidates_and_csr():
    rng = np.random.default_rng(0)
    tr = torch.LongTensor([(u, int(i)) for u in range(5) for i in rng.choice(30, 7, replace=False)])
    te = torch.LongTensor([(u, int(i)) for u in range(5) for i in rng.choice(30, 2, replace=False)])
    train = UserItemInteractionsDataset(tr, number_of_users=5, number_of_items=30)
    test = UserItemInteractionsDataset(te, number_of_users=5, number_of_items=30)
    rds = RankingDataset(test, frozen=train)
    rowptr, cols = rds.exclusion_csr()
    for u, (rep, pos, cands, uf, itf) in enumerate(rds):
        frozen = tr[tr[:, 0] == u, 1].tolist()
        assert torch.equal(cands, torch.from_numpy(oracle.candidates_for_user(30, frozen)))
        assert rep.tolist() == [u] * len(cands)
        assert sorted(cols[rowptr[u]:rowptr[u + 1]].tolist()) == sorted(set(frozen))
    # no frozen: every item is a candidate (the reference crashes here)
    _, _, cands, _, _ = next(iter(RankingDataset(test)))
    assert torch.equal(cands, torch.arange(30))
    assert RankingDataset(test).exclusion_csr() is None


def test_pairwise_sampling_matches_reference_stream():
    import random

    g = np.load(os.path.join(GOLD, "pairwise_triples.npz"), allow_pickle=False)
    tr = torch.from_numpy(g["train"])
    n_items = int(g["n_items"])
    data = UserItemInteractionsDataset(tr, user_features=Features(torch.zeros(12, 1), ["x"]),
                                       item_features=Features(torch.zeros(n_items, 1), ["x"]))
    random.seed(int(g["seed"]))
    got = [row[:3] for row in PairWiseDataset(data, max_sampled=int(g["max_sampled"]))]
    assert np.array_equal(np.asarray(got, dtype=np.int64), g["triples"])


def test_shard_range_partitions():
    for n in (0, 1, 7, 10_000_001):
        for w in (1, 2, 3, 8):
            parts = [shard_range(n, w, r) for r in range(w)]
            assert parts[0][0] == 0 and parts[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(parts, parts[1:]))
            assert max(h - l for l, h in parts) - min(h - l for l, h in parts) <= 1


def test_models_state_dict_and_cpu_guard():
    mf = MatrixFactorization(7, 9, 16)
    assert set(mf.state_dict()) == {"user_embeddings.weight", "item_embeddings.weight"}
    with pytest.raises(RuntimeError, match="ROCm device"):
        mf(torch.LongTensor([0]), torch.LongTensor([1]))
    assert RandomModel(3, 4)(torch.LongTensor([0, 1]), torch.LongTensor([2, 3])).shape == (2,)


def test_pairwise_losses_are_elementwise():
    pos, neg = torch.tensor([1.0, 0.0, -2.0]), torch.tensor([0.0, 0.0, 1.0])
    loss = LogSigmoidDifferenceLoss(reduction="none")  # ignored, as the reference
    assert loss.reduction == "mean"
    assert torch.allclose(loss.pair_wise(pos, neg), -torch.nn.functional.logsigmoid(pos - neg))
    assert AUCScore(reduction="none")(pos, neg).tolist() == [1, 1, 0]


def test_device_pairwise_dataset_csr_and_no_cpu_fallback():
    """DevicePairWiseDataset's CSRs hold each user's UNIQUE items, sorted
    (frozenset semantics of base_datasets.py:74-85); sampling itself is HIP
    only, so a CPU-resident dataset fails loudly instead of falling back."""
    from divrec.datasets import DevicePairWiseDataset
    inter = torch.tensor([[0, 5], [0, 2], [0, 5], [2, 7], [2, 1], [2, 9]])
    fz = torch.tensor([[1, 3], [2, 0]])
    data = UserItemInteractionsDataset(inter, number_of_users=3, number_of_items=10)
    frozen = UserItemInteractionsDataset(fz, number_of_users=3, number_of_items=10)
    ds = DevicePairWiseDataset(data, frozen=frozen, max_sampled=4, device="cpu")
    rowptr, items = ds.pos_csr
    assert rowptr.tolist() == [0, 2, 2, 5] and items.tolist() == [2, 5, 1, 7, 9]
    assert items.dtype == torch.int32 and rowptr.dtype == torch.int64
    erow, eitems = ds.excl_csr
    assert erow.tolist() == [0, 0, 1, 2] and eitems.tolist() == [3, 0]
    assert len(ds) == 3 * 16
    with pytest.raises(RuntimeError):
        next(iter(ds.loader(batch_size=8)))
    with pytest.raises(ValueError):
        DevicePairWiseDataset(data, max_sampled=0, device="cpu")


def test_user_item_csr_matches_unique_rows():
    """user_item_csr (1-D key unique) == torch.unique(dim=0) order, with
    duplicates, users past n_users and an empty user."""
    rng = np.random.default_rng(3)
    inter = torch.from_numpy(np.stack([rng.integers(0, 60, 3000), rng.integers(0, 500, 3000)], 1))
    inter = torch.cat([inter, inter[:200], torch.LongTensor([[70, 1], [5, 499]])])
    ds = UserItemInteractionsDataset(inter, number_of_users=80, number_of_items=500)
    rowptr, items = ds.user_item_csr(65)
    ref = torch.unique(inter, dim=0)
    ref = ref[ref[:, 0] < 65]
    assert rowptr.numel() == 66 and int(rowptr[-1]) == ref.shape[0]
    assert torch.equal(items.to(torch.int64), ref[:, 1])
    counts = torch.bincount(ref[:, 0], minlength=65)
    assert torch.equal(rowptr[1:] - rowptr[:-1], counts)


def test_pmc_summaries_feed_bench_traffic(tmp_path):
    """tools/pmc_kernels.py reduces per-dispatch FETCH/WRITE rows of our
    kernels only (x2 on FETCH, KB -> B); bench.pmc_traffic groups them by
    workload phase and sums instantiations of one kernel."""
    import csv
    import importlib.util
    import json

    root = os.path.dirname(os.path.dirname(__file__))
    spec = importlib.util.spec_from_file_location("pmc_kernels",
                                                  os.path.join(root, "tools", "pmc_kernels.py"))
    pk = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(pk)
    assert pk.short_name("void dr_topk::score_scan_kernel<128, 512, false, false>(dr_topk::TopkArgs)") \
        == "score_scan_kernel<128,512,false,false>"
    assert pk.short_name("void (anonymous namespace)::adam_kernel(float*, float const*)") == "adam_kernel"
    fields = ["Dispatch_Id", "Kernel_Name", "Counter_Name", "Counter_Value"]
    rows = [(1, "void (anonymous namespace)::bpr_kernel<4>(float const*)", 10.0),
            (2, "void at::native::(anonymous namespace)::foo<float>(int)", 99.0),
            (3, "void (anonymous namespace)::bpr_kernel<4>(float const*)", 20.0),
            (4, "void (anonymous namespace)::bpr_kernel<4>(float const*)", 30.0),
            (5, "void (anonymous namespace)::bpr_kernel<4>(float const*)", 40.0)]
    for name, counter, scale in (("f.csv", "FETCH_SIZE", 1.0), ("w.csv", "WRITE_SIZE", 0.5)):
        with open(tmp_path / name, "w", newline="") as f:
            w = csv.DictWriter(f, fieldnames=fields)
            w.writeheader()
            for d, k, v in rows:
                w.writerow({"Dispatch_Id": d, "Kernel_Name": k, "Counter_Name": counter,
                            "Counter_Value": v * scale})
    out = tmp_path / "pmc_bpr.json"
    import sys

    from divrec import _backend

    bid = _backend.build_id()
    # the profiled runs' own bench lines carry the build id that gets stamped
    (tmp_path / "f.log").write_text("note\n" + json.dumps({"metric": "x", "build_id": bid}) + "\n")
    (tmp_path / "w.log").write_text(json.dumps({"metric": "x", "build_id": bid}) + "\n")
    (tmp_path / "old.log").write_text(json.dumps({"metric": "x", "build_id": "0123456789abcdef"}))
    argv = sys.argv

    def run(logs):
        sys.argv = ["pmc_kernels.py", str(tmp_path / "f.csv"), str(tmp_path / "w.csv"),
                    "--workload", "bpr", "--reps", "2", "--config", "bpr", "--out", str(out),
                    "--logs"] + [str(tmp_path / x) for x in logs]
        try:
            pk.main()
        finally:
            sys.argv = argv

    with pytest.raises(SystemExit):  # runs of two builds: refused
        run(["f.log", "old.log"])
    run(["f.log", "w.log"])
    rec = json.load(open(out))
    assert rec["build_id"] == bid
    assert list(rec["kernels"]) == ["bpr_kernel<4>"]  # the torch kernel is dropped
    hb = rec["kernels"]["bpr_kernel<4>"]["hbm_bytes"]
    assert hb == [1024.0 * (2 * v + 0.5 * v) for v in (10.0, 20.0, 30.0, 40.0)]
    # bench.py: phase groups of `reps` dispatches, averaged per call
    import shutil

    bench_spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(root, "bench.py"))
    bench = importlib.util.module_from_spec(bench_spec)
    bench_spec.loader.exec_module(bench)
    (tmp_path / "profiles").mkdir()
    shutil.copy(out, tmp_path / "profiles" / "pmc_bpr.json")
    bench.ROOT = str(tmp_path)
    assert bench.pmc_traffic("bpr", "bpr", "bpr_kernel", group=0) == (hb[0] + hb[1]) / 2
    assert bench.pmc_traffic("bpr", "bpr", "bpr_kernel", group=1) == (hb[2] + hb[3]) / 2
    assert bench.pmc_traffic("bpr", "bpr", "bpr_kernel", per_step=2) == sum(hb) / 2
    assert bench.pmc_traffic("bpr", "other-config", "bpr_kernel") is None
    assert bench.pmc_traffic("bpr", "bpr", "bpr_kernel", group=2) is None
    # a record of another build (or without an id) is never used
    rec["build_id"] = "0123456789abcdef"
    json.dump(rec, open(tmp_path / "profiles" / "pmc_bpr.json", "w"))
    assert bench.pmc_traffic("bpr", "bpr", "bpr_kernel", group=0) is None
    del rec["build_id"]
    json.dump(rec, open(tmp_path / "profiles" / "pmc_bpr.json", "w"))
    assert bench.pmc_traffic("bpr", "bpr", "bpr_kernel", group=0) is None


def test_global_threshold_helpers():
    """The host side of the item-sharded global thresholds mirrors the scan's
    own guess (csrc/score_topk.hip guess_for / topk_threshold_kernel): stride
    32 / 64 / 128 by catalog length (32 for long lists), rank = mean + 6 sigma
    + 3, thresholds strictly below the k-th sample score and -inf without one."""
    from divrec.distributed import guess_rank, sample_stride, threshold_below

    assert sample_stride(1_000_000, 100) == 32
    assert sample_stride(5_000_000, 100) == 64
    assert sample_stride(10_000_000, 100) == 128
    assert sample_stride(10_000_000, 1000) == 128  # long lists too (round 6)
    assert guess_rank(100, 1 / 32) == 17  # the config-2 guess (ks = 17)
    assert guess_rank(100, 78125 / 10_000_000) == 10
    assert guess_rank(5, 0.9) == 5  # never above k
    from divrec.distributed import guess_ranks

    # first tier: the smallest rank whose Poisson(mu) tail is <= 0.5 %
    assert guess_ranks(100, 1 / 32) == (9, 17)  # config 2: first tier 9, safe 17
    assert guess_ranks(100, 78125 / 10_000_000) == (5, 10)
    assert guess_ranks(1000, 1 / 32) == (48, 68)  # config 5's top-1000 scan
    assert guess_ranks(3, 0.01) == (2, 3)
    from scipy.stats import poisson

    from divrec.distributed import poisson_tail_rank
    for mu in (0.03, 0.78, 1.5623, 3.125, 31.25, 200.0):
        j = poisson_tail_rank(mu)
        assert poisson.sf(j - 1, mu) <= 0.005 < (poisson.sf(j - 2, mu) if j > 1 else 1.0), mu
    s = torch.tensor([1.0, -2.5, 0.0, float("-inf"), float("nan"), 3e-39])
    t = threshold_below(s)
    assert bool((t[:3] < s[:3]).all()) and bool((t[5:] < s[5:]).all())
    assert torch.isinf(t[3]) and t[3] < 0 and torch.isinf(t[4]) and t[4] < 0


def test_fp64_gap_check_rule_on_cpu():
    """bench.fp64_gap_check (the bench line's "check" field) on the CPU: exact
    float64 top-k lists pass; a list missing a clearly-inside item, a score
    off by more than tol, or an item far below the k-th fail."""
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench

    g = torch.Generator().manual_seed(5)
    nu, ni, d, k = 64, 5000, 32, 10
    U = (torch.randn(nu, d, generator=g) / d ** 0.5).to(torch.bfloat16)
    I = (torch.randn(ni, d, generator=g) / d ** 0.5).to(torch.bfloat16)
    S = U.double() @ I.double().T
    s, i = torch.topk(S, k, dim=1)
    sel = torch.arange(nu)
    ok = bench.fp64_gap_check(U, I, s.float(), i.int(), sel, k, chunk=1000, extra=8)
    assert ok["ok"] and ok["users_not_in_exact_float64_order"] == 0
    bad = i.clone()
    bad[3, 0] = torch.argsort(S[3])[0]  # the user's worst item instead of its best
    assert not bench.fp64_gap_check(U, I, s.float(), bad.int(), sel, k, chunk=1000, extra=8)["ok"]
    off = s.float().clone()
    off[7, 4] += 1e-3
    assert not bench.fp64_gap_check(U, I, off, i.int(), sel, k, chunk=1000, extra=8)["ok"]


def test_embedding_distance_device_copy_follows_its_table():
    """EmbeddingDistance keeps its bf16, zero-padded copy between calls and
    rebuilds it when the source changes in a way torch records (in-place
    update, new tensor, new shape) or on refresh() (no stale
    padded copy). Host logic only: the copy is built on the CPU here."""
    import torch
    from divrec.losses import EmbeddingDistance

    cpu = torch.device("cpu")
    E = torch.randn(10, 100)
    D = EmbeddingDistance(E, "cosine")
    t0 = D.table(cpu)
    assert t0.shape == (10, 128) and t0.dtype == torch.bfloat16 and not t0[:, 100:].any()
    assert D.table(cpu) is t0  # cached
    E.add_(1.0)  # an optimizer-style in-place step bumps the version
    t1 = D.table(cpu)
    assert t1 is not t0 and torch.equal(t1[:, :100], E.to(torch.bfloat16))
    D.item_table = torch.randn(12, 100)
    assert D.table(cpu).shape == (12, 128)
    t2 = D.table(cpu)
    D.item_table.data[0, 0] = 5.0  # a .data write: no version torch records
    assert D.table(cpu) is t2  # documented: such writes need refresh()
    D.refresh()
    t3 = D.table(cpu)
    assert t3 is not t2 and float(t3[0, 0]) == 5.0


def test_user_item_csr_cache_follows_the_interactions():
    """UserItemInteractionsDataset.user_item_csr keeps its CSR between calls
    and rebuilds it when the interactions change, including writes torch does
    not record (.data, a numpy view): the key holds value checksums."""
    import torch
    from divrec.datasets import UserItemInteractionsDataset

    inter = torch.tensor([[0, 3], [0, 1], [2, 2], [1, 0], [0, 1]], dtype=torch.int64)
    ds = UserItemInteractionsDataset(inter.clone(), number_of_users=3, number_of_items=4)
    a = ds.user_item_csr()
    assert a[0].tolist() == [0, 2, 3, 4] and a[1].tolist() == [1, 3, 0, 2]
    assert ds.user_item_csr() is a  # cached
    ds.interactions.data[4, 1] = 2  # unrecorded write: (0, 1) duplicate -> (0, 2)
    b = ds.user_item_csr()
    assert b is not a and b[0].tolist() == [0, 3, 4, 5] and b[1].tolist() == [1, 2, 3, 0, 2]
    ds.interactions.numpy()[3, 0] = 2  # numpy view: user 1's item moves to user 2
    c = ds.user_item_csr()
    assert c[0].tolist() == [0, 3, 3, 5] and c[1].tolist() == [1, 2, 3, 0, 2]
    assert ds.user_item_csr(2)[0].tolist() == [0, 3, 3]  # another n_users: another key


def test_rank_metrics_shared_inside_an_evaluation_loop(monkeypatch):
    """Inside shared_rank_metrics() the four accuracy metrics of one
    (interactions, recommendations) pair come from ONE dr_rank_metrics call
    (train.recommendations_score_loop opens the block); outside it every call
    computes. Host logic: the kernel call is replaced by a counter."""
    import torch
    from divrec import _backend
    from divrec.metrics import _rank

    calls = []

    def fake(recs, rowptr, items):
        calls.append(1)
        n = recs.size(0)
        return tuple(torch.full((n,), float(i)) for i in range(4))

    monkeypatch.setattr(_backend, "default_device", lambda: torch.device("cpu"))
    monkeypatch.setattr(_rank.ops, "rank_metrics", fake)
    inter = torch.tensor([[0, 1], [1, 2]])
    recs = torch.tensor([[1, 2], [2, 0]])
    with _rank.shared_rank_metrics():
        r1 = _rank.rank_metrics(inter, recs)
        r2 = _rank.rank_metrics(inter, recs)
        _rank.rank_metrics(inter, recs.clone())  # another tensor: computed
    assert r1 is r2 and len(calls) == 2
    _rank.rank_metrics(inter, recs)
    assert len(calls) == 3
