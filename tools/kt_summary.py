"""Per-kernel summary of a rocprofv3 --kernel-trace --stats run (run_kernel_stats.csv):
share, total, calls, average, short name; and the per-step total.
  python tools/kt_summary.py <dir with run_kernel_stats.csv> [steps]"""
import csv
import os
import re
import sys


def short(name):
    name = re.sub(r"\(anonymous namespace\)::", "", name)
    name = re.sub(r"^void ", "", name)
    depth, out = 0, []
    for ch in name:  # drop the argument list, keep template arguments
        if ch == "(" and depth == 0:
            break
        depth += ch == "<"
        depth -= ch == ">"
        out.append(ch)
    return "".join(out)[:100]


def main():
    d = sys.argv[1]
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else None
    rows = list(csv.DictReader(open(os.path.join(d, "run_kernel_stats.csv"))))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    print("  share   total_us  calls    avg_us  kernel")
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"])):
        t = float(r["TotalDurationNs"])
        print(f"{t / tot * 100:6.2f}% {t / 1e3:10.1f} {int(r['Calls']):6d} {float(r['AverageNs']) / 1e3:9.2f}  "
              f"{short(r['Name'])}")
    print(f"total GPU kernel time {tot / 1e6:.2f} ms" + (f", {tot / 1e3 / steps:.1f} us/step" if steps else ""))


if __name__ == "__main__":
    main()
