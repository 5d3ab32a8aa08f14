"""A/B timing of dr_ild_embedding plans in ONE process (config-4 shape by
default: 1M users x top-100 lists over a 10M x 128 bf16 table, cosine).

    python tools/ild_ab.py --variants stream,ild_stream=0,ild_bufs=1 [--users U --k K --dim D]

Each variant is "stream" (the default plan) or knobs of divrec._backend.PLAN_KNOBS
joined by "+" (e.g. "ild_stream=0": the one-wave-per-user kernel), optionally
prefixed by a library tag "TAG@" (libdivrec_hip_TAG.so, a --variant build of
build_native.py; default the product library). Variants run
round-robin on the same device inputs, timed with HIP events on the current
stream; every variant's output must equal the first one's bit for bit (the
streamed and per-user kernels sum the same pairs in the same order). Prints
one JSON line; exit status 1 on a mismatch.
"""
import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "diversity-recommendations_amd"))
import torch  # noqa: E402

from divrec import _backend as B  # noqa: E402

_KINDS = {"cosine": 0, "dot": 1, "euclidean": 2}


def lib_of(tag):
    if "@" not in tag:
        return B.lib()
    import ctypes
    name = tag.split("@")[0]
    lib = ctypes.CDLL(os.path.join(ROOT, "diversity-recommendations_amd", "divrec", "_lib",
                                   f"libdivrec_hip_{name}.so"))
    for fn in ("dr_ild_embedding", "dr_set_plan_knob", "dr_get_plan_knob", "dr_last_error"):
        res, argt = B.SIGNATURES[fn]
        getattr(lib, fn).restype, getattr(lib, fn).argtypes = res, argt
    return lib


def knobs_of(tag):
    tag = tag.split("@")[-1]
    if tag == "stream":
        return {}
    out = {}
    for kv in tag.split("+"):
        k, v = kv.split("=")
        out[k] = float(v)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="stream,ild_stream=0")
    ap.add_argument("--users", type=int, default=1_000_000)
    ap.add_argument("--items", type=int, default=10_000_000)
    ap.add_argument("--dim", type=int, default=128)
    ap.add_argument("--k", type=int, default=100)
    ap.add_argument("--kind", default="cosine")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--lists", choices=["uniform", "topk"], default="uniform",
                    help="topk: the top-k lists of bench.py's own tables (dr_score_topk)")
    ap.add_argument("--after-scan", action="store_true",
                    help="run the dr_score_topk call before every timed ILD launch "
                         "(bench.py's step order)")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(1)
    n_items, d = args.items, args.dim
    if args.lists == "topk" or args.after_scan:
        sys.path.insert(0, ROOT)
        from bench import gen_table
        from divrec import ops
        users = gen_table(args.users, d, 1, dev)
        items = gen_table(n_items, d, 2, dev)
    else:
        items = (torch.randn(n_items, d, generator=g, device=dev) / d ** 0.5).to(torch.bfloat16)
    if args.lists == "topk":
        recs = ops.score_topk(users, items, args.k)[1]
        torch.cuda.synchronize()
    else:
        recs = torch.randint(0, n_items, (args.users, args.k), generator=g, device=dev,
                             dtype=torch.int32)
    tags = args.variants.split(",")
    libs = {t: lib_of(t) for t in tags}
    stream = torch.cuda.current_stream(dev).cuda_stream
    outs, times = {}, {t: [] for t in tags}

    def run(t):
        out = torch.empty(args.users, device=dev)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        L = libs[t]
        kn = knobs_of(t)
        old = {n: L.dr_get_plan_knob(B.PLAN_KNOBS[n]) for n in kn}
        for n, v in kn.items():
            L.dr_set_plan_knob(B.PLAN_KNOBS[n], v)
        if args.after_scan:
            ops.score_topk(users, items, args.k)
        if True:
            e0.record()
            rc = L.dr_ild_embedding(recs.data_ptr(), B.DR_I32, args.users, args.k,
                                    items.data_ptr(), n_items, d, _KINDS[args.kind],
                                    out.data_ptr(), None, stream)
            e1.record()
        for n, v in old.items():
            L.dr_set_plan_knob(B.PLAN_KNOBS[n], v)
        assert rc == 0, L.dr_last_error()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1), out

    for t in tags:
        outs[t] = run(t)[1].cpu()
    for _ in range(args.rounds):
        for t in tags:
            times[t].append(run(t)[0])
    per_user = args.k * 4 + args.k * d * 2 + 4  # int32 lists
    res = {"users": args.users, "k": args.k, "d": d, "items": n_items, "kind": args.kind,
           "lists": args.lists, "after_scan": args.after_scan,
           "build_id": B.build_id(), "variants": {}}
    bad = False
    for t in tags:
        med = statistics.median(times[t])
        same = bool(torch.equal(outs[t], outs[tags[0]]))
        bad |= not same
        res["variants"][t] = {"median_ms": med, "min_ms": min(times[t]),
                              "users_per_s": args.users / med * 1e3,
                              "gbs": per_user * args.users / med / 1e6,
                              "frac_of_8tbs": per_user * args.users / med / 1e6 / 8000,
                              "identical": same}
    # diag libraries (built with -D DR_ILD_DIAG): per-wave phase cycles of the
    # last launch, averaged per user
    import ctypes
    import numpy as np
    for t in tags:
        L = libs[t]
        if not hasattr(L, "dr_ild_diag_read"):
            continue
        run(t)
        buf = np.zeros((8192, 8), dtype=np.uint64)
        L.dr_ild_diag_read.argtypes = [ctypes.c_void_p]
        if L.dr_ild_diag_read(buf.ctypes.data) == 0:
            act = buf[buf[:, 6] > 0]
            users = act[:, 6].sum()
            res["variants"][t]["diag_cycles_per_user"] = {
                n: float(act[:, i].sum() / users)
                for i, n in ((0, "wait"), (1, "lds_reads"), (2, "compute_and_issue"), (3, "tail"),
                             (5, "total"))}
    print(json.dumps(res), flush=True)
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
