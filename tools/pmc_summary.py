"""Summarise a tools/profile.sh run (gpurun_out/prof_<tag>/) into profiles/:

  <round>_<tag>_kernel_stats.txt   per-kernel share / calls / avg (kernel trace)
  <round>_pmc_<config>.json        per-kernel averages of every PMC counter per
                                   dispatch + HBM bytes per dispatch
                                   (2*FETCH_SIZE + WRITE_SIZE, KiB -> B: the gfx950
                                   correction of MI355X_MICROARCH.md §HBM),
                                   keyed by the kernel name as rocprofv3 prints it
                                   with template arguments (what bench.py matches)

usage: python tools/pmc_summary.py gpurun_out/prof_<tag> <round> <config> [steps]
"""
import collections
import csv
import glob
import json
import os
import re
import sys


def short(name):
    name = name.replace("(anonymous namespace)::", "")
    name = re.sub(r"^void ", "", name)
    name = re.sub(r"^(\w+::)+", "", name)   # e.g. dgx_knn::knn_kernel<...>
    depth, out = 0, []
    for ch in name:  # drop the argument list, keep template arguments
        if ch == "(" and depth == 0:
            break
        depth += ch == "<"
        depth -= ch == ">"
        out.append(ch)
    return "".join(out).strip()


def kernel_stats(root):
    path = glob.glob(os.path.join(root, "kt", "**", "*kernel_stats.csv"), recursive=True)
    rows = list(csv.DictReader(open(path[0])))
    return sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))


def main():
    root, rnd, cfg = sys.argv[1], sys.argv[2], sys.argv[3]
    steps = int(sys.argv[4]) if len(sys.argv) > 4 else 0
    rows = kernel_stats(root)
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    lines = [f"rocprofv3 --kernel-trace --stats over bench.py ({cfg}); {root}",
             f"{'share':>7} {'total_us':>10} {'calls':>6} {'avg_us':>9}  kernel"]
    for r in rows[:40]:
        lines.append("%6.2f%% %10.1f %6s %9.2f  %s" % (100 * float(r["TotalDurationNs"]) / tot,
                                                    float(r["TotalDurationNs"]) / 1e3, r["Calls"],
                                                    float(r["AverageNs"]) / 1e3, short(r["Name"])))
    lines.append("total GPU kernel time %.2f ms" % (tot / 1e6) + (f", {tot / 1e6 / steps:.3f} ms/step" if steps else ""))
    os.makedirs("profiles", exist_ok=True)
    with open(f"profiles/{rnd}_{cfg}_kernel_stats.txt", "w") as f:
        f.write("\n".join(lines) + "\n")
    print("\n".join(lines[:25]))

    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    durs = collections.defaultdict(list)
    for path in sorted(glob.glob(os.path.join(root, "p*", "**", "*counter_collection.csv"), recursive=True)):
        per = collections.defaultdict(dict)
        meta = {}
        for r in csv.DictReader(open(path)):
            d = r["Dispatch_Id"]
            per[d][r["Counter_Name"]] = per[d].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
            meta[d] = short(r["Kernel_Name"])
        for d, cs in per.items():
            for c, v in cs.items():
                acc[meta[d]][c].append(v)
    avg_dur = {short(r["Name"]): float(r["AverageNs"]) for r in rows}
    kernels = {}
    for name, cs in acc.items():
        k = {c: sum(v) / len(v) for c, v in cs.items()}
        k["dispatches_sampled"] = max(len(v) for v in cs.values())
        if "FETCH_SIZE" in k and "WRITE_SIZE" in k:
            k["hbm_bytes"] = (2 * k["FETCH_SIZE"] + k["WRITE_SIZE"]) * 1024
        if name in avg_dur:
            k["avg_duration_ns"] = avg_dur[name]
            if "hbm_bytes" in k:
                k["hbm_GBps"] = k["hbm_bytes"] / avg_dur[name]
        if k.get("GRBM_GUI_ACTIVE", 0) > 0 and "SQ_VALU_MFMA_BUSY_CYCLES" in k:
            # MFMA-pipe busy cycles summed over the 1024 SIMDs / (kernel cycles x 1024);
            # kernel cycles = GRBM_GUI_ACTIVE / 8 (rocprofv3 sums the 8 XCDs)
            k["mfma_util"] = k["SQ_VALU_MFMA_BUSY_CYCLES"] / (k["GRBM_GUI_ACTIVE"] / 8 * 1024)
        kernels[name] = k
    out = {"config": cfg, "source": root,
           "method": "rocprofv3 --pmc passes (FETCH_SIZE | WRITE_SIZE | SQ_* | SQ_*) over bench.py, each its own "
                     "run; per-dispatch counter values averaged per kernel name; hbm_bytes = (2*FETCH_SIZE + "
                     "WRITE_SIZE) KiB -> bytes (gfx950 FETCH_SIZE counts half of a wide coalesced read); "
                     "avg_duration_ns from the kernel-trace pass",
           "kernels": kernels}
    with open(f"profiles/{rnd}_pmc_{cfg}.json", "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
    for name in sorted(kernels, key=lambda n: -kernels[n].get("avg_duration_ns", 0))[:12]:
        k = kernels[name]
        print("%-45s dur %7.1f us  hbm %8.2f MB  %6.0f GB/s  valu %9.0f  mfma_util %.3f" % (
            name[:45], k.get("avg_duration_ns", 0) / 1e3, k.get("hbm_bytes", 0) / 1e6, k.get("hbm_GBps", 0),
            k.get("SQ_INSTS_VALU", 0), k.get("mfma_util", 0)))


if __name__ == "__main__":
    main()
