#!/bin/bash
# r06: the 125k-row C4 shard (1M over 8 GPUs) under a kernel trace: per-pass kernel
# durations and the gaps between consecutive passes, then the 1M pass for comparison.
set -u
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$ROOT"; mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
for r in 125000 1000000; do
  timeout -k 10 300 rocprofv3 --kernel-trace -d "$ROOT/gpurun_out/r06tr_$r" -o run --output-format csv -- python3 "$ROOT/bench.py" --rows $r --steps 200 --warmup 20 --no-cpu-baseline --no-host-modes > "$ROOT/gpurun_out/r06tr_$r.json" 2> "$ROOT/gpurun_out/r06tr_$r.err" || exit $?
  echo "[trace] rows=$r ok"
done
cd "$ROOT" && python3 scripts/trace_gaps.py gpurun_out/r06tr_125000 gpurun_out/r06tr_1000000
