"""Headline benchmark: scored pairs/s + ILD-eval users/s, 1M users x 10M items,
d=128, top-100 (BASELINE.json metric; configs[3], the 10M-item catalog).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    torchrun --nproc-per-node N --master-addr 127.0.0.1 ... bench.py --gpus N

One step = one pass of the hot path over the whole synthetic workload:
  score_topk (bf16 MFMA scores of every user x every item of this rank's item
  shard, fused top-k) -> [N>1: all_to_all of the partial top-k lists over RCCL
  + merge] -> cosine ILD of the final top-k lists (users sharded over ranks).
Inputs are resident in HBM before timing. Item rows are sharded contiguously
over ranks (the item table is also replicated for the ILD gathers); the total
work is fixed, so scaling is "strong". value = U*I / step time (max over ranks).

Rank 0 prints ONE JSON line. The `roofline` object is for the dominant kernel
(score_topk: bound = MFMA, achieved = 2*U*I_shard*d flop / average HIP-event
time of the call on its stream); `traffic` comes from a committed rocprofv3 PMC
summary (profiles/pmc_traffic.json) when one exists for this exact config.
`cpu_baseline` (N=1 only) times the CPU oracle — the reference algorithm,
restated — on a bounded user sample on this host.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "diversity-recommendations_amd"))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from divrec import ops  # noqa: E402
from divrec.distributed import exchange_partials, shard_range  # noqa: E402

MFMA_BF16_PEAK_TFLOPS = 2500.0  # MI355X dense bf16 (MI355X_MICROARCH.md)
HBM_PEAK_GBS = 8000.0


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--users", type=int, default=1_000_000)
    ap.add_argument("--items", type=int, default=10_000_000)
    ap.add_argument("--dim", type=int, default=128)
    ap.add_argument("--k", type=int, default=100)
    ap.add_argument("--ild-kind", default="cosine")
    ap.add_argument("--cpu-budget-s", type=float, default=15.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    return ap.parse_args()


def gen_table(rows: int, d: int, seed: int, device, block: int = 1 << 20) -> torch.Tensor:
    """N(0, 1/sqrt(d)) rows in bf16, generated per 1M-row block with its own
    seed so any contiguous shard is identical whatever the world size."""
    out = torch.empty((rows, d), dtype=torch.bfloat16, device=device)
    scale = 1.0 / d ** 0.5
    for b0 in range(0, rows, block):
        g = torch.Generator(device=device).manual_seed(seed * 100_003 + b0 // block)
        n = min(block, rows - b0)
        out[b0 : b0 + n] = (torch.randn((n, d), generator=g, device=device) * scale).to(torch.bfloat16)
    return out


def cpu_baseline(U: torch.Tensor, I: torch.Tensor, recs: torch.Tensor, k: int, budget_s: float):
    """Time the CPU oracle (reference algorithm restated) on a bounded sample."""
    sys.path.insert(0, ROOT)
    import numpy as np

    import oracle

    Uh = U[:64].float().cpu().numpy()
    Ih = I.float().cpu().numpy()
    n_items = Ih.shape[0]
    # scoring + top-k: per-user loop of the reference (fp32 products, sum, full sort)
    t0 = time.perf_counter()
    oracle.recommend_topk(Uh, Ih, k, users=[0])
    per_user = time.perf_counter() - t0
    n_users = int(max(1, min(16, budget_s * 0.8 // max(per_user, 1e-3))))
    t0 = time.perf_counter()
    oracle.recommend_topk(Uh, Ih, k, users=list(range(1, 1 + n_users)))
    dt = time.perf_counter() - t0
    pairs_per_s = n_users * n_items / dt
    # ILD (cosine, from embeddings): per-user pairwise sum of the reference formula
    rh = recs[:2000].long().cpu().numpy()
    t0 = time.perf_counter()
    oracle.ild_embedding_f64(rh, Ih, "cosine")
    ild_dt = time.perf_counter() - t0
    return {
        "value": pairs_per_s,
        "unit": "scored pairs/s",
        "cores": 1,
        "kind": "port",
        "sample": f"oracle.recommend_topk (reference get_model_recommendations loop: fp32 "
                  f"sum(u*i) + full stable argsort) for {n_users} users x {n_items} items in "
                  f"{dt:.1f}s; ILD: oracle.ild_embedding_f64 on {len(rh)} users "
                  f"-> {len(rh) / ild_dt:.0f} users/s",
        "ild_users_per_s": len(rh) / ild_dt,
    }


def load_traffic(cfg_key: str):
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if not os.path.exists(path):
        return None
    try:
        with open(path) as f:
            rec = json.load(f)
        if rec.get("config") == cfg_key:
            return rec.get("hbm_bytes_per_launch")
    except (OSError, ValueError):
        pass
    return None


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and rank == 0:
        print(f"note: --gpus {args.gpus} but WORLD_SIZE={world}; using WORLD_SIZE", file=sys.stderr)
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)

    U_n, I_n, d, k = args.users, args.items, args.dim, args.k
    users = gen_table(U_n, d, 1, dev)
    items = gen_table(I_n, d, 2, dev)  # replicated: ILD gathers arbitrary rows
    lo, hi = shard_range(I_n, world, rank)
    shard = items[lo:hi]
    u_lo, u_hi = shard_range(U_n, world, rank)
    torch.cuda.synchronize()

    ev = {n: [] for n in ("topk0", "topk1", "ild0", "ild1")}

    def step(record: bool):
        e = [torch.cuda.Event(enable_timing=True) for _ in range(4)] if record else None
        if e:
            e[0].record()
        s, i = ops.score_topk(users, shard, k, item_base=lo)
        if e:
            e[1].record()
        if world > 1:
            ps, pi = exchange_partials(s, i)
            s, i = ops.topk_merge(ps, pi, k)
        if e:
            e[2].record()
        ild = ops.ild_embedding(i, items, args.ild_kind)
        if e:
            e[3].record()
            ev["topk0"].append(e[0]); ev["topk1"].append(e[1])
            ev["ild0"].append(e[2]); ev["ild1"].append(e[3])
        return i, ild

    for _ in range(args.warmup):
        step(False)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        recs, ild = step(True)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    topk_s = sum(a.elapsed_time(b) for a, b in zip(ev["topk0"], ev["topk1"])) / 1e3 / args.steps
    ild_s = sum(a.elapsed_time(b) for a, b in zip(ev["ild0"], ev["ild1"])) / 1e3 / args.steps
    t = torch.tensor([dt, ild_s], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dt, ild_max = float(t[0]), float(t[1])
    step_s = dt / args.steps

    cfg_key = f"U{U_n}_I{I_n}_d{d}_k{k}_G{world}"
    flops = 2.0 * U_n * (hi - lo) * d
    achieved = flops / topk_s / 1e12
    traffic = load_traffic(cfg_key)
    result = {
        "metric": "scored pairs/sec + ILD-eval users/sec, 1M x 10M d=128 at 1/2/4/8 GPU",
        "value": U_n * I_n / step_s,
        "unit": "scored pairs/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": step_s * 1e3,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "bf16",
        "data": "synthetic (N(0,1/sqrt(d)) bf16 tables, seeded per 1M-row block)",
        "config": {
            "workload": f"score_topk + cosine ILD: {U_n} users x {I_n} items, d={d}, k={k} "
                        f"(BASELINE configs[3], item rows sharded over ranks)",
            "users": U_n, "items": I_n, "dim": d, "k": k,
            "parallelism": f"item-shard{world}" + ("+all_to_all" if world > 1 else ""),
        },
        "ild_users_per_s": U_n / ild_max,
        "score_topk_ms": topk_s * 1e3,
        "ild_ms": ild_max * 1e3,
        "roofline": {
            "bound": "mfma",
            "achieved": achieved,
            "peak": MFMA_BF16_PEAK_TFLOPS,
            "unit": "TFLOP/s",
            "frac": achieved / MFMA_BF16_PEAK_TFLOPS,
            "traffic": traffic,
            "kernel": "dr_score_topk = score_scan_kernel (MFMA scan + fused threshold top-k) + topk_finalize_kernel; timed together",
            "flop_per_launch": flops,
        },
        "cpu_baseline": None,
    }
    if world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline(users, items, recs, k, args.cpu_budget_s)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
