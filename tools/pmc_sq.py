"""Average SQ/GRBM counters per kernel name from rocprofv3 --pmc CSV passes (diagnostic)."""
import csv
import glob
import os
import sys
from collections import defaultdict


def main(*dirs):
    acc = defaultdict(lambda: defaultdict(list))
    import sqlite3
    for d in dirs:
        for db in glob.glob(os.path.join(d, "**", "*.db"), recursive=True):   # rocpd SQLite output
            per, names = defaultdict(dict), {}
            for did, name, cn, v in sqlite3.connect(db).execute(
                    "select dispatch_id, kernel_name, counter_name, value from counters_collection"):
                per[did][cn] = per[did].get(cn, 0.0) + float(v)
                names[did] = name[:90]
            for did, cs in per.items():
                for c, v in cs.items():
                    acc[names[did]][c].append(v)
        for fn in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            per = defaultdict(dict)
            names = {}
            with open(fn) as f:
                for r in csv.DictReader(f):
                    did = r.get("Dispatch_Id") or r.get("Correlation_Id")
                    per[did][r["Counter_Name"]] = per[did].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
                    names[did] = r.get("Kernel_Name", "")[:90]
            for did, cs in per.items():
                for c, v in cs.items():
                    acc[names[did]][c].append(v)
    for name, cs in acc.items():
        print(name)
        for c, vs in sorted(cs.items()):
            print(f"   {c:32s} {sum(vs) / len(vs):16.1f}  (n={len(vs)})")


if __name__ == "__main__":
    main(*sys.argv[1:])
