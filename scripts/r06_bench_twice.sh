#!/bin/bash
# r06: the default bench line (C4, host modes and CPU baseline included) twice on one box, to put
# the end-to-end (bulk path) figures next to the pcie rates the same line measures.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
for k in 1 2; do
  timeout -k 10 400 python bench.py > gpurun_out/r06bt_$k.json 2> gpurun_out/r06bt_$k.err || exit $?
  python3 - gpurun_out/r06bt_$k.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
t = d["timing_modes"]
print("[bench] value=%.4g G req/s ms=%.4f" % (d["value"] / 1e9, d["ms_per_step"]))
for k in ("end_to_end", "end_to_end_pinned_columns", "end_to_end_pageable", "end_to_end_serial"):
    if k in t: print("   %-28s %.1f M req/s  %.2f ms" % (k, t[k]["value"] / 1e6, t[k]["ms"]))
p = t.get("pcie", {})
print("   pcie", {k: (round(v, 1) if isinstance(v, float) else v) for k, v in p.items() if k != "what"})
print("   cpu_baseline %.2f M req/s on %s cores" % (d["cpu_baseline"]["value"] / 1e6, d["cpu_baseline"]["cores"]))
PY
done
