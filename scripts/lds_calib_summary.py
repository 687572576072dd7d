"""Summary of scripts/lds_calib.sh: per pattern, the LDS counters per wave-instruction (the
micro-kernel's 4096 explicit ds_read_b32 / ds_write_b32 per thread dominate its LDS instructions)
next to what the bank rule predicts (MI355X_MICROARCH.md §LDS)."""
import csv
import glob
import os
import sys

EXPECT = {  # kernel (demangled template arguments): (LDS-array cycles, extra conflict cycles) per wave-instruction
    "<1, false>": ("stride1 ds_read_b32", 2, 0), "<2, false>": ("stride2 ds_read_b32", 4, 2),
    "<32, false>": ("stride32 ds_read_b32", 64, 62), "<-1, false>": ("broadcast ds_read_b32", 2, 0),
    "<33, false>": ("stride33 ds_read_b32", 2, 0), "<32, true>": ("stride32 ds_write_b32", 64, 62),
}
READS, THREADS = 4096, 256

rows = []
for f in glob.glob(os.path.join(sys.argv[1], "**", "*counter_collection.csv"), recursive=True):
    with open(f) as fh:
        rows += list(csv.DictReader(fh))
per = {}
for r in rows:
    k = next((key for key in EXPECT if key in r["Kernel_Name"]), None)
    if k is None:
        continue
    d = per.setdefault(k, {"grid": int(r.get("Grid_Size", r.get("Grid_Size_X", 0)) or 0), "seen": set()})
    key = (r["Dispatch_Id"], r["Counter_Name"])  # (rocprofv3 may repeat a counter row)
    if key in d["seen"]:
        continue
    d["seen"].add(key)
    d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
print("pattern | waves | SQ_INSTS_LDS per wave | IDX_ACTIVE / LDS inst (expect) | BANK_CONFLICT / LDS inst (expect) | "
      "ADDR_CONFLICT / LDS inst | BANK/IDX")
for k, (name, e_idx, e_bank) in EXPECT.items():
    d = per.get(k)
    if not d:
        print(f"{name}: no data")
        continue
    waves = d["grid"] / 64 if d["grid"] else float("nan")  # Grid_Size counts work-items
    insts = d.get("SQ_INSTS_LDS", 0.0)
    idx, bank, addr = d.get("SQ_LDS_IDX_ACTIVE", 0.0), d.get("SQ_LDS_BANK_CONFLICT", 0.0), d.get("SQ_LDS_ADDR_CONFLICT", 0.0)
    print(f"{name} | {waves:.0f} | {insts / waves:.0f} | {idx / insts:.2f} ({e_idx}) | {bank / insts:.2f} ({e_bank}) | "
          f"{addr / insts:.2f} | {bank / idx if idx else 0:.3f}")
