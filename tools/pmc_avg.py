"""Per-kernel average of every PMC counter per dispatch over the passes of
tools/pmc_cmd.sh: python tools/pmc_avg.py <outdir> [kernel-substring]"""
import collections
import csv
import glob
import os
import sys

out = sys.argv[1]
pat = sys.argv[2] if len(sys.argv) > 2 else ""
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(os.path.join(out, "p*", "**", "*counter_collection.csv"), recursive=True):
    with open(f) as fh:
        for row in csv.DictReader(fh):
            name = row["Kernel_Name"].replace("(anonymous namespace)::", "")
            name = name[5:] if name.startswith("void ") else name
            name = name.split("(")[0]
            if pat in name:
                acc[name][row["Counter_Name"]].append(float(row["Counter_Value"]))
for name, ctr in sorted(acc.items()):
    print(name)
    for c, v in sorted(ctr.items()):
        print(f"    {c:32s} {sum(v) / len(v):14.1f}  (n={len(v)})")
