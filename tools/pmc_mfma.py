"""MFMA-pipe utilisation per kernel name from one rocprofv3 --pmc pass (rocpd SQLite output; diagnostic):
busy = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 x 1024 SIMDs), averaged over the kernel's dispatches
(weighted by GRBM_GUI_ACTIVE, i.e. by duration)."""
import glob
import os
import sqlite3
import sys
from collections import defaultdict


def main(d):
    per = defaultdict(lambda: defaultdict(float))
    names = {}
    for db in glob.glob(os.path.join(d, "**", "*.db"), recursive=True):
        for did, name, cn, v in sqlite3.connect(db).execute(
                "select dispatch_id, kernel_name, counter_name, value from counters_collection"):
            per[(db, did)][cn] += float(v)
            names[(db, did)] = name
    agg = defaultdict(lambda: defaultdict(float))
    cnt = defaultdict(int)
    for k, cs in per.items():
        nm = names[k][:110]
        cnt[nm] += 1
        for c, v in cs.items():
            agg[nm][c] += v
    rows = sorted(agg.items(), key=lambda kv: -kv[1].get("GRBM_GUI_ACTIVE", 0.0))
    print(f"{'mfma_busy':>9s} {'valu/mfma':>9s} {'lds/mfma':>8s} {'bank_cf/lds':>11s} {'n':>5s}  kernel")
    for nm, cs in rows:
        gui = cs.get("GRBM_GUI_ACTIVE", 0.0)
        if gui <= 0:
            continue
        busy = cs.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / (gui / 8 * 1024)
        mf = max(cs.get("SQ_INSTS_MFMA", 0.0), 1.0)
        lds = max(cs.get("SQ_INSTS_LDS", 0.0), 1.0)
        print(f"{busy:9.3f} {cs.get('SQ_INSTS_VALU', 0.0) / mf:9.2f} {cs.get('SQ_INSTS_LDS', 0.0) / mf:8.2f} "
              f"{cs.get('SQ_LDS_BANK_CONFLICT', 0.0) / lds:11.2f} {cnt[nm]:5d}  {nm}")


if __name__ == "__main__":
    main(sys.argv[1])
