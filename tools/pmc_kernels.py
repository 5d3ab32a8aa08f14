"""Per-dispatch HBM traffic of every divrec kernel in one bench workload, from
two rocprofv3 PMC passes (tools/gpu_pmc_kernels.sh).

    python tools/pmc_kernels.py FETCH.csv WRITE.csv --workload gather \
        --reps 2 --config "..." [--out profiles/r02_pmc_gather.json]

For every kernel of libdivrec_hip (names without namespaces / template
arguments) it records, per dispatch in launch order, FETCH_SIZE and WRITE_SIZE
converted to bytes. Corrections (MI355X_MICROARCH.md, HBM): FETCH_SIZE counts
1/2 of the bytes of wide 16-B-per-lane streaming reads on gfx950, so
`fetch_bytes` doubles it (`fetch_bytes_raw` keeps the counter's own value);
WRITE_SIZE is exact for 16-B streaming stores and for fp32 atomics; other
access widths are uncalibrated (the adam_kernel line, whose traffic is known
exactly, is the in-run calibration). `reps` = warmup + steps of the pass: the
dispatches of a kernel come in groups of `reps` (one group per workload
phase), which bench.py averages into `roofline.traffic`.

Provenance: --logs names the profiled runs' own bench output; the build id
(libdivrec_hip's source hash) their JSON lines print is stamped into the
record, and bench.py uses a record only when that id equals the id of the
library it has loaded. Runs of different builds are refused.
"""
import argparse
import csv
import json
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OURS = ("dr_topk::", "(anonymous namespace)::")


def short_name(full: str) -> str:
    """'void dr_topk::score_scan_kernel<128, 512, false, false>(...)' ->
    'score_scan_kernel<128,512,false,false>'."""
    name = re.sub(r"^void\s+", "", full)
    name = re.sub(r"\(anonymous namespace\)::", "", name)
    name = re.sub(r"^dr_topk::", "", name)
    depth, out = 0, []
    for ch in name:  # cut the parameter list (the first '(' at template depth 0)
        if ch == "<":
            depth += 1
        elif ch == ">":
            depth -= 1
        elif ch == "(" and depth == 0:
            break
        out.append(ch)
    return "".join(out).replace(" ", "")


def per_dispatch(path, counter):
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            if r["Counter_Name"] != counter or not any(o in r["Kernel_Name"] for o in OURS):
                continue
            name = short_name(r["Kernel_Name"])
            if "::" in name:  # torch / rocprim kernels in anonymous namespaces
                continue
            rows.append((int(r["Dispatch_Id"]), name,
                         float(r["Counter_Value"]) * 1024.0))
    rows.sort()
    out = {}
    for _, name, v in rows:
        out.setdefault(name, []).append(v)
    return out


def build_id_of(logs):
    """The one build id printed by the bench lines of these logs (error if
    none, or if the runs loaded different builds)."""
    ids = set()
    for path in logs:
        with open(path) as f:
            for line in f:
                line = line.strip()
                if line.startswith("{") and '"build_id"' in line:
                    try:
                        ids.add(json.loads(line)["build_id"])
                    except (ValueError, KeyError):
                        pass
    if len(ids) != 1:
        raise SystemExit(f"expected one build id in {logs}, found {sorted(ids)}")
    return ids.pop()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_csv")
    ap.add_argument("write_csv")
    ap.add_argument("--workload", required=True)
    ap.add_argument("--reps", type=int, required=True, help="warmup + steps of the PMC passes")
    ap.add_argument("--config", default="")
    ap.add_argument("--out", default="")
    ap.add_argument("--logs", nargs="+", required=True,
                    help="bench output of the profiled runs (their build id is stamped)")
    args = ap.parse_args()
    bid = build_id_of(args.logs)
    f = per_dispatch(args.fetch_csv, "FETCH_SIZE")
    w = per_dispatch(args.write_csv, "WRITE_SIZE")
    kernels = {}
    for name in sorted(set(f) | set(w)):
        fr, wr = f.get(name, []), w.get(name, [])
        kernels[name] = {"dispatches": max(len(fr), len(wr)),
                         "fetch_bytes_raw": fr, "fetch_bytes": [2.0 * x for x in fr],
                         "write_bytes": wr,
                         "hbm_bytes": [2.0 * a + b for a, b in zip(fr, wr)]}
    rec = {"workload": args.workload, "config": args.config, "reps": args.reps,
           "build_id": bid, "kernels": kernels,
           "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes of the "
                     "same command; per dispatch; FETCH_SIZE x2 (gfx950 wide-read correction), "
                     "KB x 1024"}
    out = args.out or os.path.join(ROOT, "profiles", f"pmc_{args.workload}.json")
    with open(out, "w") as fh:
        json.dump(rec, fh, indent=1)
    for name, k in kernels.items():
        hb = k["hbm_bytes"]
        print(f"{name:60s} n={k['dispatches']:3d} hbm/dispatch (first, last) = "
              f"{hb[0] / 1e9 if hb else 0:.3f} / {hb[-1] / 1e9 if hb else 0:.3f} GB")


if __name__ == "__main__":
    main()
