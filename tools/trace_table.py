"""Per-dispatch table (launch order) from a rocprofv3 --kernel-trace --output-format csv directory, with
short kernel names and per-kernel totals (diagnostic: mapping kernel time onto model layers)."""
import collections
import csv
import glob
import os
import re
import sys


def short(n):
    n = n.replace("sesa::(anonymous namespace)::", "").replace("void ", "")
    return re.sub(r"\((sesa::|float|long|int|HIP_|unsigned|DcArgs).*$", "", n)


def main(d, first=0, last=10 ** 9, match=""):
    fn = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r["Grid_Size_X"],
                   r["Grid_Size_Y"]) for r in csv.DictReader(open(fn)))
    agg = collections.defaultdict(float)
    for i, (s, e, n, gx, gy) in enumerate(rows[int(first):int(last)]):
        sn = short(n)
        agg[sn] += (e - s) / 1e3
        if match in sn:
            print(f"{i + int(first):5d} {(e - s) / 1e3:9.1f} us gx={gx:>10s} gy={gy:>6s} {sn[:100]}")
    print()
    for k, v in sorted(agg.items(), key=lambda x: -x[1]):
        print(f"{v:10.1f} us {k[:110]}")


if __name__ == "__main__":
    main(*sys.argv[1:])
