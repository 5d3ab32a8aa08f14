"""Per-kernel summary (calls, total/avg/min/max ns, share) from a rocprofv3
rocpd SQLite database — the same table `--stats` writes as CSV.

    python tools/rocpd_stats.py gpurun_out/prof/bench_results.db > profiles/<round>_stats.csv
"""
import csv
import sqlite3
import sys


def main(path):
    c = sqlite3.connect(path)
    rows = c.execute(
        "select name, count(*), sum(end - start), avg(end - start), min(end - start), "
        "max(end - start) from kernels group by name order by sum(end - start) desc").fetchall()
    total = sum(r[2] for r in rows) or 1
    w = csv.writer(sys.stdout)
    w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "MinNs", "MaxNs", "Percentage"])
    for name, n, tot, avg, mn, mx in rows:
        short = name if len(name) < 200 else name[:197] + "..."
        w.writerow([short, n, tot, f"{avg:.1f}", mn, mx, f"{100.0 * tot / total:.3f}"])


if __name__ == "__main__":
    main(sys.argv[1])
