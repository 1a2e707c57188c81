"""Per-launch PMC summary (counters per wave; FETCH/WRITE in MB with the gfx950
FETCH_SIZE x2 correction of MI355X_MICROARCH.md) from tools/pmc_table.py output.
usage: python tools/pmc_table.py DIR FILTER > t; python tools/pmc_per_wave.py t"""
import sys

rows = [ln.rstrip("\n").split("|") for ln in open(sys.argv[1])]
hdr = rows[0]
keys = ["SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_SALU", "SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY",
        "SQ_ACTIVE_INST_ANY", "SQ_LDS_BANK_CONFLICT", "SQ_LDS_IDX_ACTIVE", "SQ_INSTS_VMEM_RD", "SQ_WAIT_INST_LDS"]
for r in rows[1:]:
    d = dict(zip(hdr, r))
    w = float(d.get("SQ_WAVES", "nan"))
    f = float(d.get("FETCH_SIZE", "nan")) * 2 / 1024
    wr = float(d.get("WRITE_SIZE", "nan")) / 1024
    dur = float(d["dur_us"])
    print(f"{d['kernel'][:34]:34s} grid={d['grid']:>8s} dur={dur:7.1f}us waves={w:6.0f} fetchx2={f:7.1f}MB "
          f"write={wr:6.1f}MB  ({(f + wr) / dur * 1e-3 if dur else 0:5.2f} TB/s)")
    print("    " + " ".join(f"{k.replace('SQ_', '')}={float(d.get(k, 'nan')) / w:.0f}" for k in keys))
