"""Per-kernel summary of a rocprofv3 kernel-trace SQLite database (rocpd
format, the rocprofv3 default output): share, total, calls, average, name.
  python tools/db_summary.py <run_results.db> [steps]"""
import sqlite3
import sys

from kt_summary import short


def main():
    c = sqlite3.connect(sys.argv[1])
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else None
    rows = c.execute("select name, count(*), sum(end-start), avg(end-start) from kernels "
                     "group by name order by sum(end-start) desc").fetchall()
    tot = sum(r[2] for r in rows)
    print("  share   total_us  calls    avg_us  kernel")
    for name, n, t, a in rows:
        print(f"{t / tot * 100:6.2f}% {t / 1e3:10.1f} {n:6d} {a / 1e3:9.2f}  {short(name)}")
    print(f"total GPU kernel time {tot / 1e6:.2f} ms")
    if steps:
        print(f"({steps} steps: {tot / 1e6 / steps:.3f} ms/step)")


if __name__ == "__main__":
    main()
