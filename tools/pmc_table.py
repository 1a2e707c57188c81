"""Merge rocprofv3 --pmc counter_collection CSVs (one dir per pass) into a
per-kernel-launch table: python tools/pmc_table.py gpurun_out/pmce [filter]."""
import collections
import csv
import glob
import os
import sys

root = sys.argv[1]
filt = sys.argv[2] if len(sys.argv) > 2 else ""
table = collections.defaultdict(dict)   # (kernel, grid, ordinal) -> counters
for path in sorted(glob.glob(os.path.join(root, "p*", "*counter_collection.csv"))):
    seen = collections.Counter()
    rows = list(csv.DictReader(open(path)))
    by_dispatch = collections.defaultdict(dict)
    meta = {}
    for r in rows:
        d = r["Dispatch_Id"]
        by_dispatch[d][r["Counter_Name"]] = by_dispatch[d].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        meta[d] = (r["Kernel_Name"].replace("(anonymous namespace)::", "")[:40], r["Grid_Size"],
                   (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    for d in sorted(by_dispatch, key=int):
        name, grid, dur = meta[d]
        key = (name, grid, seen[(name, grid)])
        seen[(name, grid)] += 1
        table[key].update(by_dispatch[d])
        table[key].setdefault("dur_us", dur)
cols = sorted({c for v in table.values() for c in v if c != "dur_us"})
print("kernel|grid|#|dur_us|" + "|".join(cols))
for key, v in table.items():
    if filt and filt not in key[0]:
        continue
    if key[2] != 0:
        continue
    print("%s|%s|%d|%.1f|" % (key[0], key[1], key[2], v.get("dur_us", 0)) + "|".join("%.3g" % v.get(c, float("nan")) for c in cols))
