"""Summarise rocprofv3 --pmc CSVs: mean counter value per dispatch of the tiled kernel.
usage: python scripts/pmc_summary.py gpurun_out/<tag>_<variant>_<pass> ...  (FETCH_SIZE is in KB)"""
import csv
import sys
from collections import defaultdict


def summarise(d, match="evaluate_tiled"):
    vals = defaultdict(list)
    dur = {}
    for r in csv.DictReader(open(f"{d}/run_counter_collection.csv")):
        if match not in r["Kernel_Name"]:
            continue
        vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
        dur[r["Dispatch_Id"]] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    out = {k: sum(v) / len(v) for k, v in vals.items()}
    out["dispatches"] = len(dur)
    return out


if __name__ == "__main__":
    for d in sys.argv[1:]:
        s = summarise(d)
        print(d, "  ".join(f"{k}={v:.4g}" for k, v in sorted(s.items())))
