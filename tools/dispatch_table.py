"""Per-dispatch kernel table (in launch order) from a rocprofv3 --kernel-trace output, for mapping
kernel time onto MDX23C layers (diagnostic)."""
import csv
import glob
import os
import sys


def main(d, skip=0, limit=400):
    fns = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    rows = []
    for fn in fns:
        with open(fn) as f:
            for r in csv.DictReader(f):
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"],
                             r.get("Grid_Size_X", r.get("Grid_Size", "")), r.get("Workgroup_Size_X", "")))
    rows.sort()
    rows = rows[int(skip):int(skip) + int(limit)]
    for i, (s, e, n, g, w) in enumerate(rows):
        short = n.split("(")[0].replace("sesa::(anonymous namespace)::", "").replace("void ", "")
        print(f"{i:4d} {(e - s) / 1e3:9.1f} us  grid={g:>9s}  {short[:90]}")


if __name__ == "__main__":
    main(*sys.argv[1:])
