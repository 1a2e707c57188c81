"""Per (kernel, grid) average durations from a rocprofv3 kernel_trace.csv."""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
filt = sys.argv[2] if len(sys.argv) > 2 else ""
d = collections.defaultdict(list)
for r in rows:
    n = r["Kernel_Name"].replace("(anonymous namespace)::", "")
    if filt and filt not in n:
        continue
    d[(n.split("(")[0][:60], r["Grid_Size_X"], r["Grid_Size_Y"])].append(
        (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for k, v in sorted(d.items()):
    print("%-60s %8s %4s  n=%3d  avg %8.1f us" % (k[0], k[1], k[2], len(v), sum(v) / len(v)))
