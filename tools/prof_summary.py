"""Summarise a rocprofv3 --stats kernel_stats.csv: per-kernel share, calls, avg."""
import csv
import sys

path = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof/run_kernel_stats.csv"
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 0
rows = list(csv.DictReader(open(path)))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"{'share':>7} {'total_us':>10} {'calls':>6} {'avg_us':>9}  kernel")
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:30]:
    name = r["Name"].replace("(anonymous namespace)::", "")
    print("%6.2f%% %10.1f %6s %9.1f  %s" % (100 * float(r["TotalDurationNs"]) / tot, float(r["TotalDurationNs"]) / 1e3,
                                          r["Calls"], float(r["AverageNs"]) / 1e3, name[:100]))
print("total GPU kernel time %.2f ms" % (tot / 1e6) + (f", {tot / 1e6 / steps:.3f} ms/step" if steps else ""))
