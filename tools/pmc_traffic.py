"""HBM traffic per dr_score_topk call from rocprofv3 PMC passes (tools/gpu_pmc.sh).

    python tools/pmc_traffic.py gpurun_out/pmc_fetch/fetch_counter_collection.csv \
        gpurun_out/pmc_write/write_counter_collection.csv --config U1000000_I10000000_d128_k100_G1

Sums FETCH_SIZE and WRITE_SIZE (KB) over the kernels of one dr_score_topk call
(score_scan_kernel, topk_threshold_kernel, topk_finalize_kernel; the passes
ran one bench step). Per MI355X_MICROARCH.md (HBM): FETCH_SIZE reads 1/2 of the
bytes of wide 16-B-per-lane streaming reads on gfx950 (LDS-DMA included), so
it is doubled; WRITE_SIZE is exact for 16-B streaming stores and uncalibrated
for the 8-B candidate stores (an upper bound there). Writes
profiles/pmc_traffic.json, which bench.py reads as roofline.traffic.
"""
import argparse
import csv
import json
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KERNELS = ("score_scan_kernel", "sample_rows_kernel", "topk_threshold_kernel",
           "topk_finalize_kernel")


def per_kernel(path, counter):
    out = {}
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        name = r["Kernel_Name"]
        short = next((k for k in KERNELS if k in name), None)
        if short:
            out[short] = out.get(short, 0.0) + float(r["Counter_Value"])
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_csv")
    ap.add_argument("write_csv")
    ap.add_argument("--config", required=True)
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "pmc_traffic.json"))
    args = ap.parse_args()
    f = per_kernel(args.fetch_csv, "FETCH_SIZE")
    w = per_kernel(args.write_csv, "WRITE_SIZE")
    fetch_b = 2.0 * sum(f.values()) * 1024.0
    write_b = sum(w.values()) * 1024.0
    rec = {
        "config": args.config,
        "hbm_bytes_per_launch": fetch_b + write_b,
        "fetch_bytes_corrected": fetch_b,
        "write_bytes": write_b,
        "fetch_size_kb": f,
        "write_size_kb": w,
        "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE, separate passes, one "
                  "bench step each; FETCH_SIZE x2 (gfx950), KB x 1024",
    }
    with open(args.out, "w") as fh:
        json.dump(rec, fh, indent=1)
    print(json.dumps(rec))


if __name__ == "__main__":
    main()
