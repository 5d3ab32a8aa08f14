"""HBM traffic of the headline scan per d = 128 stage size:
reduces the FETCH_SIZE / WRITE_SIZE passes of one `tools/variant_bench.py`
run per library (tools/runs/gpu_r06_stagefetch.sh) and the in-process A/B
timing of the same libraries into one record.

    python tools/stage_fetch.py --dir gpurun_out/r06sf --tags product,stage64 \
        --ab gpurun_out/r06sf/ab.json --out profiles/r06/stage_fetch/stage_fetch.json

Counter corrections as tools/pmc_kernels.py (MI355X_MICROARCH.md, HBM):
FETCH_SIZE x 2 for gfx950's 16-B-per-lane streaming reads, KB x 1024.
Each PMC run makes 2 dr_score_topk calls (warm-up + one round); every
kernel's per-dispatch values are averaged over them.
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_kernels import per_dispatch  # noqa: E402

STAGE_BYTES = {"product": 73728, "stage64": 65536}


def kernels(fetch_csv, write_csv):
    """Per kernel: dispatch count and the mean FETCH / WRITE of its dispatches.
    The seeded scan kernel runs twice per call (the main scan, then the small
    second-tier rescan): its main-scan dispatches are reported apart (the
    larger half by FETCH, in launch order every other dispatch)."""
    f = per_dispatch(fetch_csv, "FETCH_SIZE")
    w = per_dispatch(write_csv, "WRITE_SIZE")
    out = {}
    for name in sorted(set(f) | set(w)):
        fv, wv = f.get(name, []), w.get(name, [])
        rec = {"dispatches": max(len(fv), len(wv)),
               "fetch_gb": 2.0 * sum(fv) / max(len(fv), 1) / 1e9 if fv else None,
               "write_gb": sum(wv) / max(len(wv), 1) / 1e9 if wv else None}
        if len(fv) >= 2 and len(fv) % 2 == 0 and len(wv) == len(fv):
            big = [i for i in range(len(fv)) if fv[i] >= max(fv) / 4]
            rec["main_dispatches"] = len(big)
            rec["main_fetch_gb"] = 2.0 * sum(fv[i] for i in big) / len(big) / 1e9
            rec["main_write_gb"] = sum(wv[i] for i in big) / len(big) / 1e9
        out[name] = rec
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dir", required=True)
    ap.add_argument("--tags", default="product,stage64")
    ap.add_argument("--ab", required=True)
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    ab = json.load(open(a.ab))
    rec = {"workload": f"dr_score_topk {ab['users']} x {ab['items']}, d = {ab['dim']}, k = {ab['k']}",
           "columns": {}}
    for t in a.tags.split(","):
        ks = kernels(os.path.join(a.dir, t, "fetch", "fetch_counter_collection.csv"),
                     os.path.join(a.dir, t, "write", "write_counter_collection.csv"))
        main_scan = {n: v for n, v in ks.items() if n.startswith("score_scan_kernel<128,512,true")}
        v = ab["variants"][t]
        rec["columns"][t] = {"stage_bytes": STAGE_BYTES.get(t), "median_ms": v["median_ms"],
                             "min_ms": v["min_ms"], "identical": v["identical"],
                             "main_scan": main_scan, "kernels": ks}
    json.dump(rec, open(a.out, "w"), indent=1)
    for t, c in rec["columns"].items():
        ms = next(iter(c["main_scan"].values()), {})
        print(f"{t}: {c['median_ms']:.1f} ms, main-scan dispatch FETCH {ms.get('main_fetch_gb')} GB, "
              f"WRITE {ms.get('main_write_gb')} GB (mean over all {ms.get('dispatches')} dispatches "
              f"of the kernel incl. the second-tier rescans: {ms.get('fetch_gb')} / {ms.get('write_gb')})")


if __name__ == "__main__":
    main()
