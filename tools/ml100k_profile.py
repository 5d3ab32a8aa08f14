"""Where config 1's evaluation step (bench.py --workload ml100k) spends its
wall time: get_model_recommendations and each of the seven scores timed apart
(device synchronised around each), median of 20 steps, plus a cProfile of one
step's host functions. Prints one JSON line, then the cProfile top 25.

    python tools/ml100k_profile.py
"""
import cProfile
import io
import json
import os
import pstats
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "diversity-recommendations_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from divrec import datasets, losses, metrics, models, train  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    nu, ni, d, k = 943, 1682, 32, 10
    rng = np.random.default_rng(100)
    tr, te = [], []
    for u in range(nu):
        its = rng.choice(ni, 106, replace=False)
        tr += [(u, int(i)) for i in its[10:]]
        te += [(u, int(i)) for i in its[:10]]
    tr_t, te_t = torch.tensor(tr, dtype=torch.int64), torch.tensor(te, dtype=torch.int64)
    train_ds = datasets.UserItemInteractionsDataset(tr_t, number_of_users=nu, number_of_items=ni)
    test_ds = datasets.UserItemInteractionsDataset(te_t, number_of_users=nu, number_of_items=ni)
    full = datasets.UserItemInteractionsDataset(torch.cat([tr_t, te_t]), number_of_users=nu,
                                                number_of_items=ni)
    rds = datasets.RankingDataset(test_ds, frozen=train_ds)
    mf = models.MatrixFactorization(nu, ni, d)
    It = mf.item_embeddings.weight.detach().clone()
    En = It / It.norm(dim=1, keepdim=True)
    Dc = 1.0 - En @ En.T
    mf = mf.to(dev)
    names = ["ild", "precision", "recall", "map", "ndcg", "entropy", "pri"]
    scores = [losses.IntraListDiversityScore(distance_matrix=Dc, reduction="none"),
              metrics.PrecisionAtKScore(), metrics.RecallAtKScore(),
              metrics.MeanAveragePrecisionAtKScore(), metrics.NDCGScore(),
              metrics.EntropyDiversityScore(dataset=full), metrics.PRI(dataset=full)]
    times = {n: [] for n in ["recommend"] + names + ["step"]}
    for rep in range(25):
        torch.cuda.synchronize()
        t_step = time.perf_counter()
        mf.eval()
        t0 = time.perf_counter()
        recs = train.get_model_recommendations(rds, mf, k)
        torch.cuda.synchronize()
        times["recommend"].append(time.perf_counter() - t0)
        inter = rds.data.interactions
        for n, sc in zip(names, scores):
            t0 = time.perf_counter()
            sc(inter, recs)
            torch.cuda.synchronize()
            times[n].append(time.perf_counter() - t0)
        times["step"].append(time.perf_counter() - t_step)
    med = {n: round(statistics.median(v[5:]) * 1e3, 3) for n, v in times.items()}
    print(json.dumps({"ms_median": med}), flush=True)
    pr = cProfile.Profile()
    pr.enable()
    train.recommendations_score_loop(rds, mf, scores, k)
    torch.cuda.synchronize()
    pr.disable()
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats("cumulative").print_stats(25)
    print(s.getvalue())


if __name__ == "__main__":
    main()
