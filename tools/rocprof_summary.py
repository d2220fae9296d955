"""Summarise a rocprofv3 --kernel-trace --stats output (rocpd SQLite .db or *_kernel_stats.csv)
into a per-kernel table (calls, total ms, avg us, share) for profiles/."""
import csv
import glob
import os
import sqlite3
import sys


def from_db(path):
    con = sqlite3.connect(path)
    rows = con.execute("select name, count(*), sum(end-start), avg(end-start), min(end-start), max(end-start) "
                       "from kernels group by name order by sum(end-start) desc").fetchall()
    return [(r[0], r[1], r[2] / 1e6, r[3] / 1e3, r[4] / 1e3, r[5] / 1e3) for r in rows]


def from_csv(path):
    out = []
    with open(path) as f:
        for r in csv.DictReader(f):
            out.append((r["Name"], int(r["Calls"]), float(r["TotalDurationNs"]) / 1e6, float(r["AverageNs"]) / 1e3,
                        float(r["MinNs"]) / 1e3, float(r["MaxNs"]) / 1e3))
    return out


def main(src, dst=None):
    if os.path.isdir(src):
        cands = glob.glob(os.path.join(src, "**", "*kernel_stats.csv"), recursive=True) or \
            glob.glob(os.path.join(src, "**", "*.db"), recursive=True)
        src = cands[0]
    rows = from_csv(src) if src.endswith(".csv") else from_db(src)
    tot = sum(r[2] for r in rows)
    lines = [f"# source: {os.path.basename(src)}   total kernel time {tot:.2f} ms",
             f"{'total_ms':>10} {'share':>6} {'calls':>6} {'avg_us':>10} {'min_us':>10} {'max_us':>10}  kernel"]
    for name, n, ms, avg, mn, mx in rows:
        lines.append(f"{ms:10.2f} {100 * ms / tot:5.1f}% {n:6d} {avg:10.1f} {mn:10.1f} {mx:10.1f}  {name[:140]}")
    text = "\n".join(lines) + "\n"
    if dst:
        with open(dst, "w") as f:
            f.write(text)
    print(text)


if __name__ == "__main__":
    main(*sys.argv[1:])
