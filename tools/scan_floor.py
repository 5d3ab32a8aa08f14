"""How much of a score scan is the survivor path? Times, on one shape, the
product dr_score_topk, the caller-seeded scan (dr_score_topk_seeded) started
just below each user's TRUE k-th score (the best any guess can do: ~k
survivors per user, no sample scan), and the seeded scan with +inf thresholds
(no survivor at all: MFMA + hot test + stage pipeline only, lists empty).

    python tools/scan_floor.py --users 1000000 --items 1000000 --dim 64
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "diversity-recommendations_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from bench import gen_table  # noqa: E402
from divrec import ops  # noqa: E402
from divrec.distributed import threshold_below  # noqa: E402


def timed(fn, reps=3):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--users", type=int, default=1_000_000)
    ap.add_argument("--items", type=int, default=1_000_000)
    ap.add_argument("--dim", type=int, default=64)
    ap.add_argument("--k", type=int, default=100)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    U, I = gen_table(a.users, a.dim, 1, dev), gen_table(a.items, a.dim, 2, dev)
    t_prod = timed(lambda: ops.score_topk(U, I, a.k))
    s, _ = ops.score_topk(U, I, a.k)
    exact = threshold_below(s[:, a.k - 1].contiguous())
    inf = torch.full((a.users,), float("inf"), device=dev)
    t_exact = timed(lambda: ops.score_topk(U, I, a.k, init_thr=exact))
    t_none = timed(lambda: ops.score_topk(U, I, a.k, init_thr=inf))
    flop = 2.0 * a.users * a.items * a.dim
    print(json.dumps({"users": a.users, "items": a.items, "dim": a.dim, "k": a.k,
                      "product_ms": t_prod, "exact_threshold_ms": t_exact, "no_survivor_ms": t_none,
                      "tflops": {"product": flop / t_prod / 1e9, "exact_threshold": flop / t_exact / 1e9,
                                 "no_survivor": flop / t_none / 1e9}}), flush=True)


if __name__ == "__main__":
    sys.exit(main())
