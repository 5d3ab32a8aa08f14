"""A/B timing of dr_mmr_rerank builds in one process (interleaved rounds), as
tools/variant_bench.py does for the score scan; outputs must be identical.

    python tools/mmr_ab.py --libs product,TAG,... [--users N]
"""
import argparse
import json
import statistics
import sys
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
sys.path.insert(0, os.path.join(ROOT, "diversity-recommendations_amd"))
import torch  # noqa: E402

from variant_bench import lib_for  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--libs", required=True)
    ap.add_argument("--users", type=int, default=262144)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--lam", type=float, default=0.5)
    ap.add_argument("--real", action="store_true",
                    help="candidates = the real top-C lists of random users (dr_score_topk)")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(1)
    n_items, d, C, kout = 10_000_000, 128, 1000, 100
    items = (torch.randn(n_items, d, generator=g, device=dev) / d ** 0.5).to(torch.bfloat16)
    if args.real:
        from divrec import ops

        users = (torch.randn(args.users, d, generator=g, device=dev) / d ** 0.5).to(torch.bfloat16)
        sc, cand = ops.score_topk(users, items, C)
        del users
    else:
        cand = torch.randint(0, n_items, (args.users, C), generator=g, device=dev, dtype=torch.int32)
        sc = torch.sort(torch.rand(args.users, C, generator=g, device=dev), dim=1,
                        descending=True).values
    tags = args.libs.split(",")
    libs = {t: lib_for(t) for t in tags}
    stream = torch.cuda.current_stream(dev).cuda_stream
    outs, times = {}, {t: [] for t in tags}

    def run(t):
        out = torch.empty(args.users, kout, dtype=torch.int32, device=dev)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        rc = libs[t].dr_mmr_rerank(cand.data_ptr(), sc.data_ptr(), args.users, C, items.data_ptr(),
                                   n_items, d, kout, args.lam, out.data_ptr(), None, stream)
        e1.record()
        assert rc == 0, libs[t].dr_last_error()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1), out

    for t in tags:
        outs[t] = run(t)[1].cpu()
    for r in range(args.rounds):
        for t in tags:
            times[t].append(run(t)[0])
        print(f"round {r}: " + " ".join(f"{t}={times[t][-1]:.1f}ms" for t in tags), file=sys.stderr, flush=True)
    res = {"users": args.users, "lam": args.lam, "candidates": "real top-C" if args.real else "random",
           "variants": {}}
    for t in tags:
        med = statistics.median(times[t])
        res["variants"][t] = {"median_ms": med, "users_per_s": args.users / med * 1e3,
                              "identical": bool(torch.equal(outs[t], outs[tags[0]])),
                              "users_differ": int((outs[t] != outs[tags[0]]).any(dim=1).sum())}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
