"""A/B timing of dr_score_topk builds in ONE process (interleaved rounds).

    python diversity-recommendations_amd/build_native.py --variant NAME -D KEY=VAL ...
    python tools/variant_bench.py --libs product,NAME,... [--users U --items I --dim D --k K]

Each entry of --libs is a library tag: "product" is divrec/_lib/libdivrec_hip.so,
any other tag T is divrec/_lib/libdivrec_hip_T.so. A tag may carry planner
knobs, "product@scan_split=1" (several joined by "+"; names of
divrec._backend.PLAN_KNOBS, set through dr_set_plan_knob before each call;
round-4 libraries, which read DIVREC_<NAME> environment variables instead, get
those too): the same library timed under another plan. Every library is loaded into
this one process (separate code objects), fed the same device inputs, and timed
with HIP events on the current stream, round-robin, `--rounds` times. The
outputs of every build must equal the first build's bit for bit (the ranking
order is a total order, so any geometry gives the same lists); a mismatch is
reported and the exit status is 1. Prints one JSON line.
"""
import argparse
import ctypes
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "diversity-recommendations_amd")
sys.path.insert(0, PKG)

import torch  # noqa: E402

from divrec import _backend as B  # noqa: E402

LIBDIR = os.path.join(PKG, "divrec", "_lib")


# Tags starting with "abi1" are builds from before dr_score_topk took a table
# dtype (round 1 ABI: no dtype argument), kept to A/B the current build
# against the round-start kernels in one process.
_ABI1 = {"dr_score_topk_workspace": (ctypes.c_size_t, [ctypes.c_int64, ctypes.c_int64, ctypes.c_int,
                                                      ctypes.c_int]),
         "dr_score_topk": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64,
                                          ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64,
                                          ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                                          ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                          ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p])}


def lib_for(tag):
    tag = tag.split("@")[0]
    name = "libdivrec_hip.so" if tag == "product" else f"libdivrec_hip_{tag}.so"
    lib = ctypes.CDLL(os.path.join(LIBDIR, name))
    sigs = dict(B.SIGNATURES)
    if tag.startswith("abi1"):
        sigs.update(_ABI1)
    for fn in ("dr_score_topk_workspace", "dr_score_topk", "dr_last_error", "dr_mmr_rerank",
               "dr_set_plan_knob"):
        if not hasattr(lib, fn):
            continue  # libraries from before the knob ABI
        res, args = sigs[fn]
        f = getattr(lib, fn)
        f.restype, f.argtypes = res, args
    return lib


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--libs", required=True)
    ap.add_argument("--users", type=int, default=131072)
    ap.add_argument("--items", type=int, default=10_000_000)
    ap.add_argument("--dim", type=int, default=128)
    ap.add_argument("--k", type=int, default=100)
    ap.add_argument("--rounds", type=int, default=3)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(1234)
    d = args.dim
    U = (torch.randn(args.users, d, generator=g, device=dev) / d ** 0.5).to(torch.bfloat16)
    I = (torch.randn(args.items, d, generator=g, device=dev) / d ** 0.5).to(torch.bfloat16)
    tags = args.libs.split(",")
    libs = {t: lib_for(t) for t in tags}
    envs = {t: dict(kv.split("=", 1) for kv in t.split("@")[1].split("+")) if "@" in t else {}
            for t in tags}
    stream = torch.cuda.current_stream(dev).cuda_stream
    outs, times, fails = {}, {t: [] for t in tags}, {}

    def run(t):
        L = libs[t]
        knobs = {k.lower().replace("divrec_", ""): v for k, v in envs[t].items()}
        for name, i in B.PLAN_KNOBS.items():
            os.environ.pop("DIVREC_" + name.upper(), None)
            if hasattr(L, "dr_set_plan_knob"):
                L.dr_set_plan_knob(i, float(knobs[name]) if name in knobs else float("nan"))
        os.environ.update({"DIVREC_" + k.upper(): v for k, v in knobs.items()})
        dt = () if t.startswith("abi1") else (B.DR_BF16,)
        ws_bytes = L.dr_score_topk_workspace(args.users, args.items, *dt, d, args.k)
        ws = torch.empty(ws_bytes, dtype=torch.uint8, device=dev)
        s = torch.empty(args.users, args.k, device=dev)
        i = torch.empty(args.users, args.k, dtype=torch.int32, device=dev)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        rc = L.dr_score_topk(U.data_ptr(), None, args.users, I.data_ptr(), args.items, 0,
                             *dt, d,
                             args.k, None, None, s.data_ptr(), i.data_ptr(), ws.data_ptr(),
                             ws_bytes, stream)
        e1.record()
        if rc != 0:
            raise RuntimeError(f"{t}: {L.dr_last_error().decode()}")
        torch.cuda.synchronize()
        if hasattr(L, "dr_score_topk_fail_counts") and not t.startswith("abi1"):
            fc = (ctypes.c_int32 * 2)()
            L.dr_score_topk_fail_counts.argtypes = B.SIGNATURES["dr_score_topk_fail_counts"][1]
            if L.dr_score_topk_fail_counts(ws.data_ptr(), args.users, args.items, *dt, d, args.k,
                                           ctypes.addressof(fc)) == 0:
                fails[t] = [int(fc[0]), int(fc[1])]
        return e0.elapsed_time(e1), s, i

    for t in tags:  # warm-up + output capture
        _, s, i = run(t)
        outs[t] = (s.cpu(), i.cpu())
        print(f"warm {t}", file=sys.stderr, flush=True)
    for r in range(args.rounds):
        for t in tags:
            ms, _, _ = run(t)
            times[t].append(ms)
        print(f"round {r}: " + " ".join(f"{t}={times[t][-1]:.1f}ms" for t in tags),
              file=sys.stderr, flush=True)
    ref_s, ref_i = outs[tags[0]]
    flop = 2.0 * args.users * args.items * d
    res = {"users": args.users, "items": args.items, "dim": d, "k": args.k, "variants": {}}
    ok = True
    for t in tags:
        same = bool(torch.equal(outs[t][1], ref_i) and torch.equal(outs[t][0], ref_s))
        ok &= same
        med = statistics.median(times[t])
        res["variants"][t] = {"median_ms": med, "min_ms": min(times[t]),
                              "tflops": flop / (med * 1e-3) / 1e12, "identical": same,
                              "guess_failures": fails.get(t)}
    print(json.dumps(res), flush=True)
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
