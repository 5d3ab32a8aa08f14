"""MFMA utilisation per kernel from one rocprofv3 counter pass
(tools/gpu_pmc_mfma.sh): SQ_VALU_MFMA_BUSY_CYCLES, SQ_BUSY_CYCLES and
GRBM_GUI_ACTIVE per dispatch.

    python tools/pmc_mfma.py COUNTERS.csv --workload catalog --reps 1 \
        --config U1000000_I10000000_d128_k100_G1 --flops 2.56e15 \
        --kernel-ms 1775.0 [--out profiles/pmc_mfma_catalog.json]

Units (MI355X_MICROARCH.md, per-instruction constants): SQ_VALU_MFMA_BUSY_CYCLES
counts cycles, 32 per v_mfma_f32_32x32x16_bf16 on its SIMD, summed over the
chip; GRBM_GUI_ACTIVE counts the dispatch's GPU-busy cycles summed over the 8
XCDs. So a kernel's MFMA utilisation is

    mfma_busy_frac = MFMA_BUSY / (GRBM_GUI_ACTIVE / 8 x 1024 SIMDs)

at the clock the chip held, and its effective clock is GRBM_GUI_ACTIVE / 8 /
kernel time (--kernel-ms: the kernel-trace average of the same command, from a
separate unprofiled-counter pass). `expected_busy_from_flops` = flops / 1024
(2 x 32 x 32 x 16 flop per 32-cycle MFMA) cross-checks the counter against the
algorithmic flops of the launch (--flops, for the kernel named by --flops-kernel).
"""
import argparse
import csv
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_kernels import OURS, build_id_of, short_name  # noqa: E402

N_SIMDS = 1024
COUNTERS = ("SQ_VALU_MFMA_BUSY_CYCLES", "SQ_BUSY_CYCLES", "GRBM_GUI_ACTIVE")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--workload", required=True)
    ap.add_argument("--reps", type=int, required=True)
    ap.add_argument("--config", default="")
    ap.add_argument("--flops", type=float, default=0.0)
    ap.add_argument("--flops-kernel", default="score_scan_kernel")
    ap.add_argument("--kernel-ms", type=float, default=0.0)
    ap.add_argument("--out", default="")
    ap.add_argument("--logs", nargs="+", required=True,
                    help="bench output of the profiled runs (their build id is stamped)")
    args = ap.parse_args()
    bid = build_id_of(args.logs)
    per = {}  # (dispatch, name) -> {counter: value}
    with open(args.csv) as f:
        for r in csv.DictReader(f):
            if r["Counter_Name"] not in COUNTERS or not any(o in r["Kernel_Name"] for o in OURS):
                continue
            name = short_name(r["Kernel_Name"])
            if "::" in name:
                continue
            key = (int(r["Dispatch_Id"]), name)
            per.setdefault(key, {})[r["Counter_Name"]] = float(r["Counter_Value"])
    by_kernel = {}
    for (_, name), c in sorted(per.items()):
        by_kernel.setdefault(name, []).append(c)
    out = {}
    # group instantiations by base name (score_scan_kernel<...> -> score_scan_kernel)
    groups = {}
    for name, rows in by_kernel.items():
        groups.setdefault(name.split("<")[0], []).extend(rows)
        groups.setdefault(name, []).extend(rows)
    for name, rows in sorted(groups.items()):
        busy = sum(r.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) for r in rows) / args.reps
        sq = sum(r.get("SQ_BUSY_CYCLES", 0.0) for r in rows) / args.reps
        grbm = sum(r.get("GRBM_GUI_ACTIVE", 0.0) for r in rows) / args.reps
        simd_cycles = grbm / 8.0 * N_SIMDS
        rec = {"dispatches_per_call": len(rows) / args.reps, "mfma_busy_cycles": busy,
               "sq_busy_cycles": sq, "grbm_gui_active": grbm, "simd_cycles": simd_cycles,
               "mfma_busy_frac": busy / simd_cycles if simd_cycles else None,
               "counters": ", ".join(COUNTERS)}
        if name == args.flops_kernel and args.flops:
            rec["expected_busy_from_flops"] = args.flops / 1024.0
            rec["busy_over_expected"] = busy / (args.flops / 1024.0)
        if name == args.flops_kernel and args.kernel_ms:
            rec["clock_ghz"] = grbm / 8.0 / (args.kernel_ms * 1e-3) / 1e9
        out[name] = rec
    res = {"workload": args.workload, "config": args.config, "reps": args.reps, "build_id": bid,
           "method": "rocprofv3 --pmc " + " ".join(COUNTERS) + " (one pass); "
                     "mfma_busy_frac = MFMA_BUSY / (GRBM_GUI_ACTIVE / 8 x 1024 SIMDs)",
           "kernels": out}
    txt = json.dumps(res, indent=1)
    if args.out:
        with open(args.out, "w") as f:
            f.write(txt + "\n")
    print(txt)


if __name__ == "__main__":
    main()
