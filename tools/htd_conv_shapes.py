"""HTDemucs implicit-GEMM conv time per shape (diagnostic): joins the `[htd conv]` stderr lines of a
SESA_HTD_TRACE=1 run with the conv-mode `tok_gemm_kernel` dispatches of the same run's rocprofv3
--kernel-trace CSV (both in launch order; conv mode = the kernel's 8th template argument `true`).

Usage: python tools/htd_conv_shapes.py TRACE_STDERR_FILE ROCPROF_CSV_DIR [steps]
"""
import collections
import csv
import glob
import os
import re
import sys


def conv_dispatch(name):
    m = re.search(r"tok_gemm_kernel<([^>]*)>", name)
    if not m:
        return False
    args = [a.strip() for a in m.group(1).split(",")]
    return len(args) > 7 and args[7] == "true"


def main(trace_file, csv_dir, steps=1):
    shapes = [ln.split("] ", 1)[1].strip() for ln in open(trace_file) if ln.startswith("[htd conv]")]
    fn = glob.glob(os.path.join(csv_dir, "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"])
                  for r in csv.DictReader(open(fn)))
    convs = [(e - s) / 1e6 for s, e, n in rows if conv_dispatch(n)]
    if len(convs) != len(shapes):
        print(f"warning: {len(shapes)} traced launches, {len(convs)} conv dispatches; joining the first "
              f"{min(len(shapes), len(convs))}")
    agg = collections.defaultdict(lambda: [0.0, 0])
    for sh, ms in zip(shapes, convs):
        agg[sh][0] += ms
        agg[sh][1] += 1
    total = sum(v[0] for v in agg.values())
    print(f"# {len(convs)} conv launches, {total / steps:.1f} ms per step")
    print(" ms/step     n  avg_us  TF/s(alg)  shape")
    for sh, (ms, n) in sorted(agg.items(), key=lambda x: -x[1][0]):
        d = dict(zip(sh.split()[0::2], sh.split()[1::2]))
        fl = 2.0 * int(d["M"]) * int(d["N"]) * int(d["K"])
        print(f"{ms / steps:8.1f} {n:5d} {ms / n * 1e3:7.0f} {fl * n / (ms * 1e-3) / 1e12:9.1f}  {sh}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], int(sys.argv[3]) if len(sys.argv) > 3 else 1)
