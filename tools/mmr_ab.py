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
    ap.add_argument("--check", type=int, default=64,
                    help="users per variant whose lists differ from the first tag to replay in float64")
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
        if t != tags[0] and args.check:
            res["variants"][t]["divergence"] = divergence(outs[tags[0]], outs[t], cand.cpu(), sc.cpu(),
                                                          items, args.lam, args.check)
    print(json.dumps(res), flush=True)


def divergence(a, b, cand, sc, items, lam, limit):
    """Where two variants' lists differ: the float64 MMR values of both choices
    at the first differing step (the common prefix is the selected set). A gap
    of a few fp32 ulps means an fp32 near-tie that the two cosine roundings
    order differently; both lists are then the exact greedy on their values."""
    rows = torch.nonzero((a != b).any(dim=1)).flatten()[:limit].tolist()
    worst_gap, worst_rel = 0.0, 0.0
    for u in rows:
        p = int(torch.nonzero(a[u] != b[u])[0])
        pos = {int(x): j for j, x in enumerate(cand[u].tolist())}
        S = [pos[int(x)] for x in a[u, :p].tolist()]
        E = items[cand[u].long().clamp(min=0)].double().cpu()
        E = E / E.norm(dim=1, keepdim=True)
        pen = (E @ E[S].T).max(dim=1).values if S else torch.zeros(len(E), dtype=torch.float64)
        val = lam * sc[u].double() - (1 - lam) * (pen if S else 0 * pen)
        va, vb = float(val[pos[int(a[u, p])]]), float(val[pos[int(b[u, p])]])
        worst_gap = max(worst_gap, abs(va - vb))
        worst_rel = max(worst_rel, abs(va - vb) / max(abs(va), 1e-30))
    return {"checked": len(rows), "max_abs_gap": worst_gap, "max_rel_gap": worst_rel}


if __name__ == "__main__":
    main()
