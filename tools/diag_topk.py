"""Phase breakdown of score_topk_kernel from the instrumented diag library.

    python diversity-recommendations_amd/build_native.py --diag   (build container)
    python tools/diag_topk.py --users 65536 --items 10000000 --dim 128 --k 100

Loads divrec/_lib/libdivrec_hip_diag.so (built with -DDR_TOPK_DIAG: s_memtime
stamps around each phase of the scan) and prints per-wave cycle shares. The
stamps fence the pipeline, so read the SHARES, not the absolute time.
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "diversity-recommendations_amd")
_tag = next((a.split("=", 1)[1] for a in sys.argv if a.startswith("--lib=")), "diag")
os.environ["DIVREC_HIP_LIB"] = os.path.join(PKG, "divrec", "_lib", f"libdivrec_hip_{_tag}.so")
sys.path.insert(0, PKG)
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from divrec import _backend as B  # noqa: E402

SLOTS = ["total", "prologue", "boundary", "mma_issue", "hits", "enqueue", "drain", "flush",
         "n_tiles", "n_enqueue", "n_drain", "n_flush", "n_stages", "realtime_100mhz"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--users", type=int, default=65536)
    ap.add_argument("--items", type=int, default=10_000_000)
    ap.add_argument("--dim", type=int, default=128)
    ap.add_argument("--k", type=int, default=100)
    ap.add_argument("--lib", default="diag", help="diag library tag (libdivrec_hip_<tag>.so)")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(1)
    U = (torch.randn(args.users, args.dim, generator=g, device=dev) / args.dim ** 0.5).to(torch.bfloat16)
    I = (torch.randn(args.items, args.dim, generator=g, device=dev) / args.dim ** 0.5).to(torch.bfloat16)
    L = B.lib()
    ws_bytes = L.dr_score_topk_workspace(args.users, args.items, B.DR_BF16, args.dim, args.k)
    out_s = torch.empty(args.users, args.k, device=dev)
    out_i = torch.empty(args.users, args.k, dtype=torch.int32, device=dev)
    res = {}
    for rep in range(2):
        ws = torch.zeros(ws_bytes, dtype=torch.uint8, device=dev)
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ev0.record()
        rc = L.dr_score_topk(U.data_ptr(), None, args.users, I.data_ptr(), args.items, 0,
                             B.DR_BF16, args.dim,
                             args.k, None, None, out_s.data_ptr(), out_i.data_ptr(), ws.data_ptr(),
                             ws_bytes, B.stream(dev))
        ev1.record()
        B.check(rc, "dr_score_topk")
        torch.cuda.synchronize()
        ms = ev0.elapsed_time(ev1)
    import ctypes
    fn = L.dr_score_topk_diag_offset
    fn.restype = ctypes.c_size_t
    fn.argtypes = [ctypes.c_int64, ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                   ctypes.c_void_p]
    grid = ctypes.c_int(0)
    off = fn(args.users, args.items, B.DR_BF16, args.dim, args.k, ctypes.byref(grid))
    # the kernel aligns the workspace base up to 256 B
    base = (-ws.data_ptr()) % 256
    blk = ws[base + off: base + off + grid.value * 8 * 16 * 8].view(torch.int64).cpu()
    recs = blk.view(grid.value * 8, 16).tolist()
    tot = [sum(r[i] for r in recs) for i in range(len(SLOTS))]
    res = {"kernel_ms": ms, "waves": len(recs)}
    for i, nm in enumerate(SLOTS):
        res[nm] = tot[i] / max(1, len(recs))
    cyc = res["total"]
    res["shares"] = {nm: round(res[nm] / cyc, 4) for nm in SLOTS[1:8]}
    res["tflops"] = 2.0 * args.users * args.items * args.dim / (ms * 1e-3) / 1e12
    res["cycles_per_tile"] = cyc / max(1, res["n_tiles"])
    # in-kernel shader clock: s_memtime cycles / s_memrealtime ticks (100 MHz)
    res["clock_ghz"] = cyc / max(1.0, res["realtime_100mhz"]) * 0.1
    # per SIMD-pair half: waves 0-3 (older, favoured by the arbiter's age
    # order) against their partners 4-7 on the same SIMDs
    for half, name in ((range(0, 4), "waves0_3"), (range(4, 8), "waves4_7")):
        sel = [r for i, r in enumerate(recs) if i % 8 in half]
        t = [sum(r[i] for r in sel) / max(1, len(sel)) for i in range(len(SLOTS))]
        res[name] = {nm: round(t[i] / max(1.0, t[0]), 4) for i, nm in enumerate(SLOTS[1:8], 1)}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
