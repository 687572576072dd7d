#!/bin/bash
# One bench line + one rocprofv3 kernel-trace summary per BASELINE config:
#   gpurun_out/${TAG}_<config>.json and gpurun_out/${TAG}_<config>_prof/run_kernel_stats.csv
# Every GPU step has its own time limit; a fault / abort / timeout stops the script.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
TAG=${1:-cfg}
CFGS=${CFGS:-"c2_trusted c3_group c5_mixed c6_256"}
stop() { local rc=$1 what=$2; echo "[configs] $what exit $rc"; if [ "$rc" -ne 0 ]; then exit "$rc"; fi; }
for c in $CFGS; do
  timeout -k 10 400 python bench.py --config $c --no-host-modes > gpurun_out/${TAG}_$c.json 2> gpurun_out/${TAG}_$c.err
  stop $? "bench $c"
  tail -c 600 gpurun_out/${TAG}_$c.json
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/${TAG}_${c}_prof" \
     -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --config $c --steps 10 --no-cpu-baseline --no-host-modes \
     > "$GRAFT_REPO_ROOT/gpurun_out/${TAG}_${c}_prof.log" 2>&1)
  stop $? "prof $c"
done
echo "[configs] done"
