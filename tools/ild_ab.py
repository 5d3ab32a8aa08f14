"""A/B timing of dr_ild_embedding builds in one process (config-4 shape: 1M
users x top-100 lists over a 10M x 128 bf16 table, cosine); outputs must match.

    python tools/ild_ab.py --libs product,TAG,...
"""
import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
sys.path.insert(0, os.path.join(ROOT, "diversity-recommendations_amd"))
import torch  # noqa: E402

from variant_bench import lib_for  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--libs", required=True)
    ap.add_argument("--users", type=int, default=1_000_000)
    ap.add_argument("--k", type=int, default=100)
    ap.add_argument("--rounds", type=int, default=5)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(1)
    n_items, d = 10_000_000, 128
    items = (torch.randn(n_items, d, generator=g, device=dev) / d ** 0.5).to(torch.bfloat16)
    recs = torch.randint(0, n_items, (args.users, args.k), generator=g, device=dev, dtype=torch.int32)
    tags = args.libs.split(",")
    libs = {t: lib_for(t) for t in tags}
    stream = torch.cuda.current_stream(dev).cuda_stream
    outs, times = {}, {t: [] for t in tags}

    def run(t):
        out = torch.empty(args.users, device=dev)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        rc = libs[t].dr_ild_embedding(recs.data_ptr(), 2, args.users, args.k, items.data_ptr(),
                                      n_items, d, 0, out.data_ptr(), stream)
        e1.record()
        assert rc == 0, libs[t].dr_last_error()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1), out

    for t in tags:
        outs[t] = run(t)[1].cpu()
    for _ in range(args.rounds):
        for t in tags:
            times[t].append(run(t)[0])
    per_user = args.k * 8 + args.k * d * 2 + 4
    res = {"users": args.users, "k": args.k, "variants": {}}
    for t in tags:
        med = statistics.median(times[t])
        res["variants"][t] = {"median_ms": med, "users_per_s": args.users / med * 1e3,
                              "gbs": per_user * args.users / med / 1e6,
                              "max_abs_diff": float((outs[t] - outs[tags[0]]).abs().max())}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
