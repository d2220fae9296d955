"""Idle gaps between consecutive kernels of a rocprofv3 --kernel-trace run (rocpd SQLite): total span, busy time and
the largest gaps with the kernels on either side (where a forward's wall time goes when it is not in kernels).

  python tools/gap_table.py DIR_OR_DB [N_TOP] [SKIP_FRACTION]

SKIP_FRACTION (default 0.5) drops that leading fraction of the trace (the warm-up step of a bench run)."""
import glob
import os
import sqlite3
import sys


def kernels(path):
    dbs = [path] if path.endswith(".db") else glob.glob(os.path.join(path, "**", "*.db"), recursive=True)
    rows = []
    for db in dbs:
        rows += sqlite3.connect(db).execute("select start, end, name from kernels order by start").fetchall()
    rows.sort()
    return rows


def short(name):
    name = name.replace("(anonymous namespace)::", "").replace("void ", "").replace("sesa::", "")
    return name.split("(")[0][:70]


def main():
    rows = kernels(sys.argv[1])
    top = int(sys.argv[2]) if len(sys.argv) > 2 else 15
    skip = float(sys.argv[3]) if len(sys.argv) > 3 else 0.5
    rows = rows[int(len(rows) * skip):]
    span = (rows[-1][1] - rows[0][0]) / 1e6
    busy = sum(e - s for s, e, _ in rows) / 1e6
    gaps = []
    end = rows[0][1]
    for i in range(1, len(rows)):
        s, e, n = rows[i]
        if s > end:
            gaps.append(((s - end) / 1e6, short(rows[i - 1][2]), short(n)))
        end = max(end, e)
    print(f"kernels {len(rows)}  span {span:.2f} ms  busy {busy:.2f} ms  idle {span - busy:.2f} ms "
          f"({sum(g[0] for g in gaps):.2f} ms in {len(gaps)} gaps)")
    for g in sorted(gaps, reverse=True)[:top]:
        print(f"  {g[0]:8.3f} ms  after {g[1]}  before {g[2]}")


if __name__ == "__main__":
    main()
