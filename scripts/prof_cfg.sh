#!/bin/bash
# rocprofv3 kernel-trace stats of bench.py per config (CFGS), extra env passed through (e.g.
# KW_PRECLASSIFY=1): gpurun_out/<tag>_<cfg>_prof/ and the bench line gpurun_out/<tag>_<cfg>.json.
set -u
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-prof}
cd /tmp && export TMPDIR=/tmp
for CFG in ${CFGS:-c4_64}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/${TAG}_${CFG}_prof" -o run --output-format csv -- python3 "$ROOT/bench.py" --config $CFG --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline --no-host-modes > "$ROOT/gpurun_out/${TAG}_${CFG}.json" 2> "$ROOT/gpurun_out/${TAG}_${CFG}.err"
  rc=$?; echo "[prof] $CFG exit $rc"
  if [ $rc -ne 0 ]; then tail -5 "$ROOT/gpurun_out/${TAG}_${CFG}.err"; exit $rc; fi
  grep -h "kernel" "$ROOT/gpurun_out/${TAG}_${CFG}_prof/run_kernel_stats.csv" | awk -F'",' '{print $1"\"", $2}' | cut -c1-160
done
