"""Generate golden vectors by running the REFERENCE divrec implementation.

Run in the build container only (the reference tree is not on the GPU box):

    PYTHONDONTWRITEBYTECODE=1 PYTHONPATH=/root/reference python tests/golden/make_golden.py

It imports the reference package ``divrec`` from /root/reference, calls the
reference entry points of the hot path on small seeded inputs and writes the
inputs and outputs as .npz fixtures next to this script. Nothing from the
reference is copied: only data (inputs and the values its code returned).

Fixtures (one .npz each):
  mf_forward_*    MatrixFactorization.forward (matrix_factorization.py:26-28)
  recs_*          get_model_recommendations over RankingDataset(test, frozen=train)
                  (train/utils.py:53-77, datasets/base_datasets.py:136-171)
  ild_*           IntraListDiversityScore / IntraListBinaryUnfairnessScore
                  recommendations_loss (losses/intra_list_diversity_score.py:20-63)
  bpr_step        one pair_wise_train_loop batch: loss, AUC, grads, Adam step
                  (train/utils.py:130-164, losses/log_sigmoid_difference_loss.py:11-14)
  bpr_loop        pair_wise_train_loop over a seeded PairWiseDataset (random.choices)
  ml100k_cfg1     config 1: ML-100K-shaped synthetic MF d=32 top-10 + ILD
  recs_fp32_d100_* get_model_recommendations with raw N(0,1) fp32 weights (the
                  nn.Embedding init, no bf16 rounding) at the reference
                  experiments' embedding_dim 100, k = 10 / 100 / 1000
  ml100k_d100     config 1 at d=100 with raw fp32 weights: top-10 + ILD + metrics
"""
from __future__ import annotations

import os
import random
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))


def _import_reference():
    import divrec  # noqa: F401  (must resolve to /root/reference/divrec)

    path = os.path.dirname(divrec.__file__)
    assert path.startswith("/root/reference"), f"not the reference package: {path}"
    from divrec import datasets, losses, metrics, models, train

    return datasets, losses, metrics, models, train


def bf16_round(t: torch.Tensor) -> torch.Tensor:
    return t.to(torch.bfloat16).to(torch.float32)


def save(name: str, **arrays):
    out = {}
    for k, v in arrays.items():
        if isinstance(v, torch.Tensor):
            v = v.detach().cpu().numpy()
        out[k] = np.asarray(v)
    np.savez_compressed(os.path.join(HERE, f"{name}.npz"), **out)
    print(f"wrote {name}.npz: " + ", ".join(f"{k}{list(np.shape(v))}" for k, v in out.items()))


def synthetic_split(rng, n_users, n_items, n_train, n_test):
    """Per user: n_train train and n_test test items, disjoint."""
    tr, te = [], []
    for u in range(n_users):
        items = rng.choice(n_items, size=n_train + n_test, replace=False)
        tr += [(u, int(i)) for i in items[:n_train]]
        te += [(u, int(i)) for i in items[n_train:]]
    return torch.LongTensor(tr), torch.LongTensor(te)


def main():
    datasets, losses, metrics, models, train = _import_reference()
    torch.manual_seed(0)

    # ---------------------------------------------------------------- MF forward
    for d in (32, 64, 128):
        g = torch.Generator().manual_seed(d)
        mf = models.MatrixFactorization(50, 80, d)
        with torch.no_grad():
            mf.user_embeddings.weight.copy_(torch.randn(50, d, generator=g))
            mf.item_embeddings.weight.copy_(torch.randn(80, d, generator=g))
        uid = torch.randint(0, 50, (500,), generator=g)
        iid = torch.randint(0, 80, (500,), generator=g)
        with torch.no_grad():
            out = mf(uid, iid)
            save(f"mf_forward_d{d}", U=mf.user_embeddings.weight, I=mf.item_embeddings.weight,
                 uid=uid, iid=iid, out=out)

    # ---------------------------------------------------------------- recommendations
    def run_recs(name, U, I, k, stable_ties):
        rng = np.random.default_rng(len(name))
        nu, ni = U.shape[0], I.shape[0]
        tr, te = synthetic_split(rng, nu, ni, 30, 10)
        train_ds = datasets.UserItemInteractionsDataset(tr, number_of_users=nu, number_of_items=ni)
        test_ds = datasets.UserItemInteractionsDataset(te, number_of_users=nu, number_of_items=ni)
        mf = models.MatrixFactorization(nu, ni, U.shape[1])
        with torch.no_grad():
            mf.user_embeddings.weight.copy_(U)
            mf.item_embeddings.weight.copy_(I)
        rds = datasets.RankingDataset(test_ds, frozen=train_ds)
        orig = torch.argsort
        if stable_ties:
            # the build's defined tie-break (score desc, item id asc) is
            # argsort(stable=True); the reference's own call is unstable
            # (train/utils.py:73), which only matters when scores tie.
            train.utils.torch.argsort = lambda x, descending=False: orig(
                x, descending=descending, stable=True)
        try:
            with torch.no_grad():
                recs = train.get_model_recommendations(rds, mf, k)
        finally:
            train.utils.torch.argsort = orig
        save(name, U=U, I=I, train=tr, test=te, k=np.int64(k), recs=recs)

    g = torch.Generator().manual_seed(1234)
    for k in (10, 100):
        U = bf16_round(torch.randn(64, 64, generator=g) / 8.0)
        I = bf16_round(torch.randn(2000, 64, generator=g) / 8.0)
        run_recs(f"recs_float_k{k}", U, I, k, stable_ties=False)
        U = torch.randint(-3, 4, (64, 64), generator=g).float()
        I = torch.randint(-3, 4, (2000, 64), generator=g).float()
        run_recs(f"recs_int_k{k}", U, I, k, stable_ties=True)

    # ---------------------------------------------------------------- ILD
    g = torch.Generator().manual_seed(77)
    ni = 400
    D = torch.rand(ni, ni, generator=g)
    inter = torch.zeros((0, 2), dtype=torch.long)
    for k in (1, 2, 10, 100):
        recs = torch.randint(0, ni, (40, k), generator=g)
        recs[0] = recs[0, 0]  # a row with duplicates (diagonal entries included)
        ild = losses.IntraListDiversityScore(distance_matrix=D, reduction="none")
        vals = ild.recommendations_loss(inter, recs)
        ild_sum = losses.IntraListDiversityScore(distance_matrix=D, reduction="sum")
        total = ild_sum(inter, recs)
        mean_raises = False
        try:
            losses.IntraListDiversityScore(distance_matrix=D)(inter, recs)
        except IndexError:
            mean_raises = True
        # user_ild (:36-42): the raw combinations sum per list (a 0-d fp32
        # tensor; the int 0 of an empty sum for k = 1)
        raw = np.asarray([float(ild.user_ild(row, D)) for row in recs], dtype=np.float32)
        save(f"ild_dense_k{k}", D=D, recs=recs, out=vals, sum=total,
             mean_raises=np.bool_(mean_raises), user_ild=raw)

    # label equality (IntraListBinaryUnfairnessScore with a 'partition' feature)
    labels = torch.randint(0, 3, (ni,), generator=g)
    feats = datasets.Features(labels.unsqueeze(1).float(), ["partition"])
    ds = datasets.UserItemInteractionsDataset(
        torch.LongTensor([[0, 0]]), number_of_items=ni, item_features=feats)
    unf = losses.IntraListBinaryUnfairnessScore(dataset=ds, reduction="none")
    recs = torch.randint(0, ni, (50, 10), generator=g)
    save("ild_labels", labels=labels, recs=recs, out=unf.recommendations_loss(inter, recs))

    # cosine distance from a bf16-quantised item table (D built in fp32 torch)
    E = bf16_round(torch.randn(ni, 64, generator=g))
    En = E / E.norm(dim=1, keepdim=True)
    Dc = 1.0 - En @ En.T
    recs = torch.randint(0, ni, (50, 10), generator=g)
    cos = losses.IntraListDiversityScore(distance_matrix=Dc, reduction="none")
    save("ild_cosine", E=E, D=Dc, recs=recs, out=cos.recommendations_loss(inter, recs))

    # ---------------------------------------------------------------- BPR step
    g = torch.Generator().manual_seed(5)
    nu, ni, d, B = 30, 60, 16, 100
    mf = models.MatrixFactorization(nu, ni, d)
    with torch.no_grad():
        mf.user_embeddings.weight.copy_(torch.randn(nu, d, generator=g) * 0.5)
        mf.item_embeddings.weight.copy_(torch.randn(ni, d, generator=g) * 0.5)
    U0 = mf.user_embeddings.weight.detach().clone()
    I0 = mf.item_embeddings.weight.detach().clone()
    uid = torch.randint(0, nu, (B,), generator=g)
    pid = torch.randint(0, ni, (B,), generator=g)
    nid = torch.randint(0, ni, (B,), generator=g)
    loss_fn = losses.LogSigmoidDifferenceLoss()
    opt = torch.optim.Adam(mf.parameters(), lr=1e-3)
    pos = mf(uid, pid)
    neg = mf(uid, nid)
    loss = loss_fn(pos, neg)
    loss.backward()
    gU = mf.user_embeddings.weight.grad.detach().clone()
    gI = mf.item_embeddings.weight.grad.detach().clone()
    opt.step()
    auc = metrics.AUCScore()(pos.detach(), neg.detach())
    save("bpr_step", U0=U0, I0=I0, uid=uid, pid=pid, nid=nid, loss=loss.detach(), auc=auc,
         gU=gU, gI=gI, U1=mf.user_embeddings.weight, I1=mf.item_embeddings.weight)

    # pair_wise_train_loop end to end over a seeded PairWiseDataset
    rng = np.random.default_rng(9)
    tr, _ = synthetic_split(rng, 12, 40, 6, 0)
    ufe = datasets.Features(torch.zeros(12, 1), ["x"])
    ife = datasets.Features(torch.zeros(40, 1), ["x"])
    data = datasets.UserItemInteractionsDataset(tr, user_features=ufe, item_features=ife)
    torch.manual_seed(3)
    mf = models.MatrixFactorization(12, 40, 16)
    U0 = mf.user_embeddings.weight.detach().clone()
    I0 = mf.item_embeddings.weight.detach().clone()
    random.seed(42)
    pw = datasets.PairWiseDataset(data, max_sampled=5)
    opt = torch.optim.Adam(mf.parameters(), lr=1e-2)
    mean_loss, (mean_auc,) = train.pair_wise_train_loop(
        pw, mf, losses.LogSigmoidDifferenceLoss(), opt, scores=[metrics.AUCScore()],
        batch_size=64)
    random.seed(42)
    triples = []
    for row in datasets.PairWiseDataset(data, max_sampled=5):
        triples.append(row[:3])
    save("pairwise_triples", train=tr, triples=np.asarray(triples, dtype=np.int64),
         seed=np.int64(42), max_sampled=np.int64(5), n_items=np.int64(40))
    save("bpr_loop", train=tr, U0=U0, I0=I0, U1=mf.user_embeddings.weight,
         I1=mf.item_embeddings.weight, mean_loss=np.float64(mean_loss),
         mean_auc=np.float64(mean_auc), seed=np.int64(42), max_sampled=np.int64(5),
         batch_size=np.int64(64), lr=np.float64(1e-2))

    # ---------------------------------------------------------------- config 1
    g = torch.Generator().manual_seed(100)
    nu, ni, d = 943, 1682, 32
    U = bf16_round(torch.randn(nu, d, generator=g) / 4)
    I = bf16_round(torch.randn(ni, d, generator=g) / 4)
    rng = np.random.default_rng(100)
    tr, te = synthetic_split(rng, nu, ni, 96, 10)
    train_ds = datasets.UserItemInteractionsDataset(tr, number_of_users=nu, number_of_items=ni)
    test_ds = datasets.UserItemInteractionsDataset(te, number_of_users=nu, number_of_items=ni)
    mf = models.MatrixFactorization(nu, ni, d)
    with torch.no_grad():
        mf.user_embeddings.weight.copy_(U)
        mf.item_embeddings.weight.copy_(I)
    rds = datasets.RankingDataset(test_ds, frozen=train_ds)
    En = I / I.norm(dim=1, keepdim=True)
    Dc = 1.0 - En @ En.T
    ild = losses.IntraListDiversityScore(distance_matrix=Dc, reduction="none")
    with torch.no_grad():
        res = train.recommendations_score_loop(rds, mf, [ild], 10)
        recs = train.get_model_recommendations(rds, mf, 10)
    test_inter = te
    full_ds = datasets.UserItemInteractionsDataset(torch.cat([tr, te]), number_of_users=nu,
                                                   number_of_items=ni)
    with torch.no_grad():
        prec = metrics.precision_at_k(test_inter, recs)
        rec = metrics.recall_at_k(test_inter, recs)
        ap = metrics.average_precision_at_k(test_inter, recs)
        ndcg = metrics.normalized_discounted_cumulative_gain(test_inter, recs)
        ent = metrics.EntropyDiversityScore(dataset=full_ds)(test_inter, recs)
        pri = metrics.PRI(dataset=full_ds)(test_inter, recs)
        mapk = metrics.MeanAveragePrecisionAtKScore()(test_inter, recs)
    save("ml100k_cfg1", U=U, I=I, train=tr, test=te, recs=recs, ild=res[0], precision=prec,
         recall=rec, ap=ap, ndcg=ndcg, entropy=ent, pri=pri, map=mapk)

    # ---------------------------------------------------------------- raw fp32 weights, d=100
    # The reference experiments train MatrixFactorization at embedding_dim 100
    # (experiments/experiments/movie_lens_100k_mf_bpr/config.yaml:7) from
    # nn.Embedding's N(0,1) init: fp32 values that bf16 does not represent.
    g = torch.Generator().manual_seed(4321)
    U = torch.randn(64, 100, generator=g)
    I = torch.randn(2000, 100, generator=g)
    for k in (10, 100, 1000):
        run_recs(f"recs_fp32_d100_k{k}", U, I, k, stable_ties=False)

    g = torch.Generator().manual_seed(943)
    nu, ni, d = 943, 1682, 100
    U = torch.randn(nu, d, generator=g)
    I = torch.randn(ni, d, generator=g)
    rng = np.random.default_rng(943)
    tr, te = synthetic_split(rng, nu, ni, 96, 10)
    train_ds = datasets.UserItemInteractionsDataset(tr, number_of_users=nu, number_of_items=ni)
    test_ds = datasets.UserItemInteractionsDataset(te, number_of_users=nu, number_of_items=ni)
    mf = models.MatrixFactorization(nu, ni, d)
    with torch.no_grad():
        mf.user_embeddings.weight.copy_(U)
        mf.item_embeddings.weight.copy_(I)
    rds = datasets.RankingDataset(test_ds, frozen=train_ds)
    En = I / I.norm(dim=1, keepdim=True)
    Dc = 1.0 - En @ En.T
    ild = losses.IntraListDiversityScore(distance_matrix=Dc, reduction="none")
    with torch.no_grad():
        res = train.recommendations_score_loop(rds, mf, [ild], 10)
        recs = train.get_model_recommendations(rds, mf, 10)
    full_ds = datasets.UserItemInteractionsDataset(torch.cat([tr, te]), number_of_users=nu,
                                                   number_of_items=ni)
    with torch.no_grad():
        prec = metrics.precision_at_k(te, recs)
        rec = metrics.recall_at_k(te, recs)
        ap = metrics.average_precision_at_k(te, recs)
        ndcg = metrics.normalized_discounted_cumulative_gain(te, recs)
        ent = metrics.EntropyDiversityScore(dataset=full_ds)(te, recs)
        pri = metrics.PRI(dataset=full_ds)(te, recs)
        mapk = metrics.MeanAveragePrecisionAtKScore()(te, recs)
    save("ml100k_d100", U=U, I=I, train=tr, test=te, recs=recs, ild=res[0], precision=prec,
         recall=rec, ap=ap, ndcg=ndcg, entropy=ent, pri=pri, map=mapk)


if __name__ == "__main__":
    sys.exit(main())
