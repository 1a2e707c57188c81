"""Turn a rocprofv3 PMC run over bench.py (tools/gpu_pmc_bench.sh -> gpurun_out/pmcb)
into profiles/<round>_knn_pmc.json: HBM bytes per kNN selection launch, averaged
over the launches of one training step the way bench.py averages its roofline
(FETCH_SIZE x 2 + WRITE_SIZE, the gfx950 correction of MI355X_MICROARCH.md:
FETCH_SIZE tallies 128-B requests at 64 B)."""
import collections
import csv
import glob
import json
import os
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmcb"
out = sys.argv[2] if len(sys.argv) > 2 else "profiles/r01_knn_pmc.json"
vals = collections.defaultdict(dict)
for path in glob.glob(os.path.join(root, "p*", "*counter_collection.csv")):
    order = collections.defaultdict(int)
    for r in csv.DictReader(open(path)):
        if "knn_kernel<" not in r["Kernel_Name"] or r["Counter_Name"] not in ("FETCH_SIZE", "WRITE_SIZE"):
            continue
        nm = r["Kernel_Name"]
        nm = nm[nm.index("knn_kernel<"):]
        key = (nm[:nm.index(">") + 1], r["Dispatch_Id"])
        vals[r["Counter_Name"]].setdefault(key, 0.0)
        vals[r["Counter_Name"]][key] += float(r["Counter_Value"])
per_kernel = collections.defaultdict(lambda: {"fetch_kb": [], "write_kb": []})
for (name, _), v in vals["FETCH_SIZE"].items():
    per_kernel[name]["fetch_kb"].append(v)
for (name, _), v in vals["WRITE_SIZE"].items():
    per_kernel[name]["write_kb"].append(v)
summary = {}
for name, d in per_kernel.items():
    f = sum(d["fetch_kb"]) / max(1, len(d["fetch_kb"]))
    w = sum(d["write_kb"]) / max(1, len(d["write_kb"]))
    summary[name] = {"fetch_bytes_x2": f * 1024 * 2, "write_bytes": w * 1024, "hbm_bytes": (2 * f + w) * 1024}
# one step: layer 1 (C=3, NSTEP 1), layers 2-3 (C=64, NSTEP 16), layer 4 (C=128, NSTEP 32)
weights = {"knn_kernel<1, 20, false>": 1, "knn_kernel<16, 20, false>": 2, "knn_kernel<32, 20, false>": 1}
tot = sum(summary[n]["hbm_bytes"] * c for n, c in weights.items() if n in summary)
cnt = sum(c for n, c in weights.items() if n in summary)
res = {"hbm_bytes_per_launch": tot / cnt if cnt else None,
       "per_kernel": summary,
       "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes over bench.py "
                 "(tools/gpu_pmc_bench.sh); bytes = 2*FETCH_SIZE + WRITE_SIZE (gfx950 correction), "
                 "averaged over one step's kNN launches (C=3, 64, 64, 128) like bench.py's roofline"}
os.makedirs(os.path.dirname(out), exist_ok=True)
json.dump(res, open(out, "w"), indent=1)
print(json.dumps(res, indent=1))
