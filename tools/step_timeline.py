"""Print one training step's kernel sequence (durations, grid) from a
rocprofv3 kernel-trace CSV: python tools/step_timeline.py <kernel_trace.csv> [step]"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
which = int(sys.argv[2]) if len(sys.argv) > 2 else 15
marks = [i for i, r in enumerate(rows) if "knn_image_kernel<1>" in r["Kernel_Name"]]
st, en = marks[which], marks[which + 1]
tot = 0.0
for r in rows[st:en]:
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    tot += d
    name = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "")
    name = name[:name.index("(")] if "(" in name else name
    print(f"{d:8.1f} us  grid {int(r['Grid_Size_X']):>7}x{r['Grid_Size_Y']:<3} lds {r['LDS_Block_Size']:>6} "
          f"vgpr {r['VGPR_Count']:>3}  {name[:70]}")
span = (int(rows[en]["Start_Timestamp"]) - int(rows[st]["Start_Timestamp"])) / 1e3
print(f"kernel time {tot:.1f} us, span {span:.1f} us")
