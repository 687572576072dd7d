#!/bin/bash
# r06 closing record, part B: rocprofv3 kernel stats of every BASELINE config's bench run, then the
# PMC passes of scripts/pmc.sh on C4 (HBM traffic -> gpurun_out/<tag>_c4_traffic.json).
set -u
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$ROOT"; mkdir -p gpurun_out
TAG=${1:-r06p}
cd /tmp && export TMPDIR=/tmp
for cfg in c4_64 c1_namespace c2_trusted c3_group c5_mixed c6_256; do
  steps=20; [ $cfg = c5_mixed ] && steps=10
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/${TAG}_${cfg}_stats" -o run --output-format csv -- python3 "$ROOT/bench.py" --config $cfg --steps $steps --warmup 3 --no-cpu-baseline --no-host-modes > "$ROOT/gpurun_out/${TAG}_${cfg}_stats.json" 2> "$ROOT/gpurun_out/${TAG}_${cfg}_stats.err" || exit $?
  echo "[prof] $cfg stats ok"
done
cd "$ROOT" && bash scripts/pmc.sh ${TAG}_c4 || exit $?
