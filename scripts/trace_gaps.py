"""Kernel-trace summary (rocprofv3 --kernel-trace csv): per kernel name, count and mean duration, and
for the tiled kernel the gap from one launch's end to the next one's start (the per-pass fixed cost
of back-to-back passes). usage: python scripts/trace_gaps.py <rocprof dir>..."""
import csv
import glob
import sys

for d in sys.argv[1:]:
    f = glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)[0]
    rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
    by = {}
    for r in rows:
        by.setdefault(r["Kernel_Name"][:60], []).append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    print(d)
    for k, v in sorted(by.items(), key=lambda kv: -sum(kv[1])):
        print(f"  {len(v):5d} x {sum(v) / len(v) / 1e3:9.2f} us  {k}")
    tiles = [r for r in rows if "evaluate_tiles" in r["Kernel_Name"]]
    gaps = [int(b["Start_Timestamp"]) - int(a["End_Timestamp"]) for a, b in zip(tiles, tiles[1:])]
    gaps = sorted(gaps[20:]) if len(gaps) > 40 else sorted(gaps)
    if gaps:
        print(f"  tile-kernel gaps: median {gaps[len(gaps) // 2] / 1e3:.2f} us, p10 {gaps[len(gaps) // 10] / 1e3:.2f}, "
              f"p90 {gaps[9 * len(gaps) // 10] / 1e3:.2f} (n={len(gaps)})")
