#!/bin/bash
# PC sampling (host trap) of the bench's tile kernel: where waves sit (diagnostics).
set -u
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-pcs}
CFG=${CFG:-c4_64}
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method host_trap --pc-sampling-unit time \
  --pc-sampling-interval ${INTERVAL:-1} --kernel-include-regex evaluate_tiles -d "$ROOT/gpurun_out/${TAG}" -o run --output-format csv \
  -- python3 "$ROOT/bench.py" --config $CFG --steps 10 --warmup 2 --no-cpu-baseline --no-host-modes > "$ROOT/gpurun_out/${TAG}.log" 2>&1
rc=$?
echo "[pcs] exit $rc"; ls -la "$ROOT/gpurun_out/${TAG}" 2>/dev/null | head; tail -5 "$ROOT/gpurun_out/${TAG}.log"
exit $rc
