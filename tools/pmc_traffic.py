"""HBM traffic per launch of the dominant kernel class from two rocprofv3 PMC passes.

Per MI355X_MICROARCH.md §HBM / cdna_hip_programming.md §7: FETCH_SIZE and WRITE_SIZE are collected
in SEPARATE passes (TCC slots), both in KiB; on gfx950 FETCH_SIZE reports exactly half of the bytes
of a wide coalesced streaming read, so it is doubled before comparing with byte counts.

usage: python tools/pmc_traffic.py <fetch_pass_dir> <write_pass_dir> <kernel-substring[|substring...]> [out.json]
                                    [kernel-class]
(a dispatch matches if its name contains any of the '|'-separated substrings: one kernel CLASS, as
bench.py's roofline times it).  With a kernel class (bench.py KSRC key) the summary is stamped with
``src_sha16`` of that class's sources in this tree and ``git_sha`` from $GIT_SHA, so bench.py reports
the figure only for the sources it was measured on.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def read_counter_db(path, counter):
    import sqlite3
    con = sqlite3.connect(path)
    per, names = defaultdict(float), {}
    for did, name, val in con.execute("select dispatch_id, kernel_name, value from counters_collection "
                                      "where counter_name = ?", (counter,)):
        per[did] += float(val)
        names[did] = name
    return per, names


def read_counter(d, counter):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        dbs = glob.glob(os.path.join(d, "**", "*.db"), recursive=True)
        if dbs:   # rocprofv3 >= 7: rocpd SQLite output
            return read_counter_db(dbs[0], counter)
        raise SystemExit(f"no counter_collection.csv / .db under {d}")
    per = defaultdict(float)   # dispatch id -> value
    names = {}
    for fn in files:
        with open(fn) as f:
            for r in csv.DictReader(f):
                if r.get("Counter_Name") != counter:
                    continue
                did = r.get("Dispatch_Id") or r.get("Correlation_Id")
                per[did] += float(r["Counter_Value"])
                names[did] = r.get("Kernel_Name", "")
    return per, names


def main(fetch_dir, write_dir, substr, out=None, kclass=None):
    f, fn = read_counter(fetch_dir, "FETCH_SIZE")
    w, wn = read_counter(write_dir, "WRITE_SIZE")
    subs = substr.split("|")
    fk = [v for k, v in f.items() if any(s in fn[k] for s in subs)]
    wk = [v for k, v in w.items() if any(s in wn[k] for s in subs)]
    if not fk or not wk:
        raise SystemExit(f"no dispatches matching {substr!r}")
    fetch_kib = sum(fk) / len(fk)
    write_kib = sum(wk) / len(wk)
    res = {"kernel_match": substr, "launches_fetch_pass": len(fk), "launches_write_pass": len(wk),
           "fetch_size_kib_avg": round(fetch_kib, 1), "write_size_kib_avg": round(write_kib, 1),
           "hbm_bytes_per_launch": round((2 * fetch_kib + write_kib) * 1024),
           # the profiled command runs SESA_PMC_STEPS bench steps (tools/pmc_refresh.sh: 1): bench.py divides the
           # per-step bytes by its own profile records per step (a record may cover several dispatches)
           "dispatches_per_step": round(len(fk) / float(os.environ.get("SESA_PMC_STEPS", "1")), 2),
           "hbm_bytes_per_step": round((2 * sum(fk) + sum(wk)) * 1024 / float(os.environ.get("SESA_PMC_STEPS", "1"))),
           "correction": "bytes = (2*FETCH_SIZE + WRITE_SIZE) * 1024 (gfx950 FETCH_SIZE counts half of "
                         "wide coalesced reads; MI355X_MICROARCH.md §HBM)"}
    if kclass:
        import importlib.util
        here = os.path.dirname(os.path.abspath(__file__))
        spec = importlib.util.spec_from_file_location("bench", os.path.join(here, "..", "bench.py"))
        bench = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(bench)
        res["kernel_class"] = kclass
        model = os.environ.get("SESA_PMC_MODEL") or None
        res["model"] = model
        res["src_sha16"] = bench.kernel_sources_sha16(kclass, model)
        res["git_sha"] = os.environ.get("GIT_SHA", "unknown")
        res["precision"] = os.environ.get("SESA_PMC_PRECISION", "bf16x3")
    print(json.dumps(res, indent=1))
    if out:
        with open(out, "w") as fo:
            json.dump(res, fo, indent=1)


if __name__ == "__main__":
    main(*sys.argv[1:])
