"""Summarise rocprofv3 --pmc CSVs: mean counter value per dispatch of the tiled kernel.
usage: python scripts/pmc_summary.py gpurun_out/<tag>_<variant>_<pass> ...  (FETCH_SIZE is in KB)"""
import csv
import sys
from collections import defaultdict


def summarise(d, match="evaluate_tiles"):
    vals = defaultdict(list)
    dur = {}
    for r in csv.DictReader(open(f"{d}/run_counter_collection.csv")):
        if match not in r["Kernel_Name"]:
            continue
        vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
        dur[r["Dispatch_Id"]] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    out = {k: sum(v) / len(v) for k, v in vals.items()}
    out["dispatches"] = len(dur)
    out["dur_ns"] = sum(dur.values()) / max(1, len(dur))
    return out


def write_traffic(fetch_dir, write_dir, out, config="c4_64", rows=1_000_000, tag="r01"):
    """profiles/traffic.json for bench.py: HBM bytes per tiled-kernel launch. FETCH_SIZE and
    WRITE_SIZE are in KB; FETCH_SIZE counts half of the bytes of wide coalesced reads on gfx950
    (MI355X_MICROARCH.md, HBM section), so it is doubled."""
    import json

    f, w = summarise(fetch_dir), summarise(write_dir)
    fetch = 2.0 * f["FETCH_SIZE"] * 1024.0
    write = w["WRITE_SIZE"] * 1024.0
    import hashlib
    import os
    lib = os.environ.get("KWGPU_LIB") or os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                                     "policy-server_amd", "libkwgpu.so")
    with open(lib, "rb") as fh:
        sha = hashlib.sha256(fh.read()).hexdigest()
    doc = {"round": tag, "config": config, "rows": rows, "kernel": "evaluate_tiles_kernel", "lib_sha256": sha,
           "fetch_bytes": fetch, "write_bytes": write, "bytes_per_launch": fetch + write,
           "source": f"rocprofv3 --pmc FETCH_SIZE ({fetch_dir}) and WRITE_SIZE ({write_dir}), separate passes; "
                     "FETCH_SIZE x2 (gfx950 calibration)"}
    with open(out, "w") as fh:
        json.dump(doc, fh, indent=1)
    return doc


if __name__ == "__main__":
    if sys.argv[1] == "--traffic":
        # --traffic fetch_dir write_dir out tag [config rows]
        a = sys.argv
        print(write_traffic(a[2], a[3], a[4], tag=a[5] if len(a) > 5 else "r02", config=a[6] if len(a) > 6 else "c4_64",
                            rows=int(a[7]) if len(a) > 7 else 1_000_000))
        sys.exit(0)
    if sys.argv[1] == "--derived":
        # --derived rows dir... : the ratios the DESIGN tables quote, from the merged passes
        rows = float(sys.argv[2])
        m = {}
        for d in sys.argv[3:]:
            m.update(summarise(d))
        g = lambda k: m.get(k, float("nan"))
        print(f"rows={rows:.0f} dur_ns={g('dur_ns'):.4g}")
        print(f"SQ_WAIT_ANY/SQ_WAVE_CYCLES={g('SQ_WAIT_ANY') / g('SQ_WAVE_CYCLES'):.3f}  "
              f"SQ_ACTIVE_INST_ANY/SQ_WAVE_CYCLES={g('SQ_ACTIVE_INST_ANY') / g('SQ_WAVE_CYCLES'):.3f}  "
              f"SQ_WAIT_INST_ANY/SQ_WAVE_CYCLES={g('SQ_WAIT_INST_ANY') / g('SQ_WAVE_CYCLES'):.3f}")
        print(f"LDS bank conflict / LDS active={g('SQ_LDS_BANK_CONFLICT') / g('SQ_LDS_IDX_ACTIVE'):.3f}")
        print(f"per request: VALU={g('SQ_INSTS_VALU') / rows:.1f} SALU={g('SQ_INSTS_SALU') / rows:.1f} "
              f"LDS={g('SQ_INSTS_LDS') / rows:.1f} SMEM={g('SQ_INSTS_SMEM') / rows:.2f} VMEM_RD={g('SQ_INSTS_VMEM_RD') / rows:.2f} "
              f"VMEM_WR={g('SQ_INSTS_VMEM_WR') / rows:.2f}")
        print(f"HBM bytes per request: fetch(x2)={2 * g('FETCH_SIZE') * 1024 / rows:.1f} write={g('WRITE_SIZE') * 1024 / rows:.1f}")
        sys.exit(0)
    for d in sys.argv[1:]:
        s = summarise(d)
        print(d, "  ".join(f"{k}={v:.4g}" for k, v in sorted(s.items())))
