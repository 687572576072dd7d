"""C5 wave counters per dispatch (scripts/r05_prof.sh's rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES
SQ_BUSY_CYCLES GRBM_GUI_ACTIVE pass) -> profiles/r05_c5_waves.txt.
Usage: python scripts/c5_waves.py gpurun_out/<tag>_c5_waves > profiles/r05_c5_waves.txt"""
import collections
import csv
import sys

base = sys.argv[1].rstrip("/") + "/"
agg, name = collections.defaultdict(dict), {}
for r in csv.DictReader(open(base + "run_counter_collection.csv")):
    d = int(r["Dispatch_Id"])
    agg[d][r["Counter_Name"]] = agg[d].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    name[d] = r["Kernel_Name"]
dur = {int(r["Dispatch_Id"]): int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
       for r in csv.DictReader(open(base + "run_kernel_trace.csv"))}
print("""# r05 C5 (10M x 64, light / heavy split) wave counters per dispatch: rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES
# SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace, bench.py --config c5_mixed --steps 3 --warmup 1 (scripts/r05_prof.sh, final build;
# this file: scripts/c5_waves.py). Each pass = two launches: the light region (68 % of rows, 64-row tiles,
# evaluate_tiles_kernel<true,false,6>) then the heavy one (12-row tiles, the container wave-scan instantiation
# <true,false,38> = labels | containers | kFeatRng). Resident waves per CU = 4 x SQ_WAVE_CYCLES (quad-cycles)
# / (GRBM_GUI_ACTIVE / 8 XCDs) / 256 CUs; the maximum at 4 workgroups of 4 waves is 16 (the unsplit layout of
# r04, 81 KB tiles, held 2 workgroups = 8 waves per CU).
""")
for d in sorted(agg):
    if "evaluate_tiles" not in name[d]:
        continue
    a = agg[d]
    res = 4 * a["SQ_WAVE_CYCLES"] / (a["GRBM_GUI_ACTIVE"] / 8) / 256
    kind = "light" if "6u>" in name[d] else "heavy"
    print(f"dispatch {d} ({kind}): SQ_WAVES {int(a['SQ_WAVES'])}  dur {dur[d] / 1e6:.3f} ms  "
          f"SQ_WAVE_CYCLES {a['SQ_WAVE_CYCLES']:.4g}  GRBM_GUI_ACTIVE {a['GRBM_GUI_ACTIVE']:.4g}  resident waves/CU {res:.2f}")
