"""Summarise a rocprofv3 --kernel-trace run (rocpd sqlite .db or *_kernel_stats.csv) into a
kernel-stats CSV (Name,Calls,TotalDurationNs,AverageNs,Percentage) and a top-N text table.

    python tools/prof_summary.py gpurun_out/prof1/run_results.db profiles/r01_v1_kernel_stats.csv
"""
import csv
import sqlite3
import sys


def load(path):
    if path.endswith(".csv"):
        rows = list(csv.DictReader(open(path)))
        return [(r["Name"], int(r["Calls"]), float(r["TotalDurationNs"])) for r in rows]
    db = sqlite3.connect(path)
    q = "select name, count(*), sum(duration) from kernels group by name order by sum(duration) desc"
    return [(n, int(c), float(d)) for n, c, d in db.execute(q)]


def main():
    rows = load(sys.argv[1])
    tot = sum(r[2] for r in rows)
    if len(sys.argv) > 2:
        with open(sys.argv[2], "w", newline="") as f:
            w = csv.writer(f)
            w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage"])
            for n, c, d in rows:
                w.writerow([n, c, int(d), d / c, round(100 * d / tot, 3)])
    print(f"total kernel time {tot / 1e6:.2f} ms over {sum(r[1] for r in rows)} launches")
    for n, c, d in rows[:40]:
        print(f"{d / 1e6:9.2f} ms {c:6d} x {d / c / 1e3:9.1f} us  {n[:120]}")


if __name__ == "__main__":
    main()
