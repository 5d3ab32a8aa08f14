"""Phase breakdown of dr_mmr_rerank from the instrumented variant library.

    python diversity-recommendations_amd/build_native.py --variant mmrdiag -D DR_MMR_DIAG
    python tools/mmr_diag.py [--users 65536] [--real]

Per wave: s_memtime cycles of each phase summed over users (kernel-side
atomics), printed per user and as shares of the wave's total.
"""
import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
sys.path.insert(0, os.path.join(ROOT, "diversity-recommendations_amd"))
import torch  # noqa: E402

from variant_bench import lib_for  # noqa: E402

PHASES = ["load", "select", "stage", "mma", "sync1", "rounds", "sync2", "fold", "batches", "total",
          "stage_barrier", "gt_writes"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--users", type=int, default=65536)
    ap.add_argument("--real", action="store_true")
    ap.add_argument("--lam", type=float, default=0.5)
    ap.add_argument("--lib", default="mmrdiag")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(1)
    n_items, d, C, kout = 10_000_000, 128, 1000, 100
    items = (torch.randn(n_items, d, generator=g, device=dev) / d ** 0.5).to(torch.bfloat16)
    if args.real:
        from divrec import ops

        users = (torch.randn(args.users, d, generator=g, device=dev) / d ** 0.5).to(torch.bfloat16)
        sc, cand = ops.score_topk(users, items, C)
    else:
        cand = torch.randint(0, n_items, (args.users, C), generator=g, device=dev, dtype=torch.int32)
        sc = torch.sort(torch.rand(args.users, C, generator=g, device=dev), dim=1,
                        descending=True).values
    lib = lib_for(args.lib)
    lib.dr_mmr_diag_read.argtypes = [ctypes.c_void_p, ctypes.c_int]
    buf = (ctypes.c_ulonglong * (8 * 16))()
    stream = torch.cuda.current_stream(dev).cuda_stream
    out = torch.empty(args.users, kout, dtype=torch.int32, device=dev)

    def run():
        rc = lib.dr_mmr_rerank(cand.data_ptr(), sc.data_ptr(), args.users, C, items.data_ptr(),
                               n_items, d, kout, args.lam, out.data_ptr(), None, stream)
        assert rc == 0, lib.dr_last_error()
        torch.cuda.synchronize()

    run()
    lib.dr_mmr_diag_read(buf, 1)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    run()
    e1.record()
    torch.cuda.synchronize()
    lib.dr_mmr_diag_read(buf, 1)
    rec = {"users": args.users, "candidates": "real" if args.real else "random", "lam": args.lam,
           "ms": e0.elapsed_time(e1), "per_user_cycles": {}}
    for w in range(8):
        v = [buf[w * 16 + i] / args.users for i in range(len(PHASES))]
        rec["per_user_cycles"][f"wave{w}"] = dict(zip(PHASES, v))
    w0 = rec["per_user_cycles"]["wave0"]
    w1 = rec["per_user_cycles"]["wave1"]
    rec["share_wave0"] = {p: w0[p] / w0["total"] for p in PHASES if p not in ("batches", "total", "stage_barrier", "gt_writes")}
    rec["share_wave1"] = {p: w1[p] / w1["total"] for p in PHASES if p not in ("batches", "total", "stage_barrier", "gt_writes")}
    print(json.dumps(rec))


if __name__ == "__main__":
    main()
