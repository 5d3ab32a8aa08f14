"""Attribute a score scan's HBM traffic to its survivor path (VERDICT r4
item 3): one product dr_score_topk call, then the seeded scan from each user's
exact k-th score (~k survivors per user) and from +inf (no survivors), one
dispatch each, and the seeded scan from the product's own first-tier guess,
under a rocprofv3 FETCH_SIZE or WRITE_SIZE pass (tools/gpu_r05_pmcfloor.sh).
The seeded dispatches differ only in their survivor streams, so their byte
counts split the product's traffic into item streaming, survivor-induced
traffic and the product plan's own.

    rocprofv3 --pmc FETCH_SIZE -d DIR -o fetch -- python3 tools/pmc_floor.py --k 1000
    python3 tools/pmc_floor.py --reduce DIR/fetch_counter_collection.csv FETCH_SIZE
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "diversity-recommendations_amd"))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))


def run(a):
    import torch

    from bench import gen_table
    from divrec import ops
    from divrec.distributed import threshold_below

    dev = torch.device("cuda", 0)
    U, I = gen_table(a.users, a.dim, 1, dev), gen_table(a.items, a.dim, 2, dev)
    s, _ = ops.score_topk(U, I, a.k)
    exact = threshold_below(s[:, a.k - 1].contiguous())
    inf = torch.full((a.users,), float("inf"), device=dev)
    ops.score_topk(U, I, a.k, init_thr=exact)
    ops.score_topk(U, I, a.k, init_thr=inf)
    # the product's own first-tier thresholds (the same sample guess through
    # dr_sample_thresholds), on the seeded call's plan: separates the
    # survivors' traffic from the plan's
    plan = ops.score_topk_plan(a.users, a.items, U.dtype, a.dim, a.k)
    st, S = plan["sample_stride"], plan["sample_rows"]
    if st:
        thr = ops.sample_thresholds(U, I[::st][:S].contiguous(), plan["first_tier_rank"],
                                    plan["sample_rank"])[0]
        ops.score_topk(U, I, a.k, init_thr=thr.contiguous())
    torch.cuda.synchronize()
    print(json.dumps({"users": a.users, "items": a.items, "dim": a.dim, "k": a.k}), flush=True)


def reduce(path, counter):
    from pmc_kernels import per_dispatch

    per = per_dispatch(path, counter)  # kernel -> bytes per dispatch, in launch order
    scale = 2 if counter == "FETCH_SIZE" else 1  # gfx950 wide reads (pmc_kernels.py)
    print(json.dumps({"counter": counter,
                      "gb": {n: [round(v * scale / 1e9, 3) for v in vs] for n, vs in per.items()}}))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--users", type=int, default=1_000_000)
    ap.add_argument("--items", type=int, default=10_000_000)
    ap.add_argument("--dim", type=int, default=128)
    ap.add_argument("--k", type=int, default=1000)
    ap.add_argument("--reduce", nargs=2, metavar=("CSV", "COUNTER"))
    a = ap.parse_args()
    if a.reduce:
        reduce(*a.reduce)
    else:
        run(a)


if __name__ == "__main__":
    main()
