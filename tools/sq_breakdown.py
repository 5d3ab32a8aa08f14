"""Wave-cycle breakdown of the score scans from one rocprofv3 SQ counter pass
(tools/gpu_r04_sqpass.sh): per scan kernel instance, the counters summed over
its dispatches and the shares of SQ_WAVE_CYCLES spent parked (SQ_WAIT_ANY:
s_waitcnt / barrier), issue-stalled (SQ_WAIT_INST_ANY, of it LDS issue
SQ_WAIT_INST_LDS) and issuing (SQ_ACTIVE_INST_ANY), plus LDS bank-conflict
cycles against all LDS-array cycles.

    python tools/sq_breakdown.py <counter_collection.csv> [--out FILE]
"""
import argparse
import collections
import csv
import json
import re


def short(name):
    m = re.search(r"score_scan_kernel<([^>]*)>", name)
    return f"score_scan_kernel<{m.group(1)}>" if m else name.split("(")[0][-60:]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--out")
    a = ap.parse_args()
    tot = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for r in csv.DictReader(open(a.csv)):
        if "score_scan_kernel" not in r["Kernel_Name"]:
            continue
        k = short(r["Kernel_Name"])
        tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k].add(r["Dispatch_Id"])
    out = {}
    for k, c in tot.items():
        wc = c.get("SQ_WAVE_CYCLES", 0.0) or 1.0
        rec = {"dispatches": len(disp[k]), "counters": dict(c)}
        rec["share"] = {
            "parked_wait_any": c.get("SQ_WAIT_ANY", 0.0) / wc,
            "issue_stall_wait_inst_any": c.get("SQ_WAIT_INST_ANY", 0.0) / wc,
            "of_it_lds_issue": c.get("SQ_WAIT_INST_LDS", 0.0) / wc,
            "issuing_active_inst_any": c.get("SQ_ACTIVE_INST_ANY", 0.0) / wc,
        }
        lds = c.get("SQ_LDS_IDX_ACTIVE", 0.0)
        rec["lds_bank_conflict_over_idx_active"] = c.get("SQ_LDS_BANK_CONFLICT", 0.0) / lds if lds else None
        out[k] = rec
    s = json.dumps(out, indent=1)
    if a.out:
        open(a.out, "w").write(s)
    print(s)


if __name__ == "__main__":
    main()
