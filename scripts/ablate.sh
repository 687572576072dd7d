#!/bin/bash
# Phase ablation of the slot kernel (diagnostic): kernel time with classification / walk / output
# skipped (KW_TILE_DEBUG bits 1 / 2 / 4), then a kernel-trace profile of the default run.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
TAG=${1:-abl}
for d in ${DEBUGS:-0 1 2 4 6 7}; do
  KW_TILE_DEBUG=$d timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-host-modes > gpurun_out/${TAG}_d$d.json 2>gpurun_out/${TAG}_d$d.err
  rc=$?; echo "debug=$d rc=$rc $(python -c "import json;d=json.load(open('gpurun_out/${TAG}_d$d.json'));print(d['kernel_ms'], d['value']/1e6)" 2>/dev/null)"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
[ -n "${NOPROF:-}" ] && exit 0
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/${TAG}_prof" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 10 --warmup 2 --no-cpu-baseline > "$GRAFT_REPO_ROOT/gpurun_out/${TAG}_prof.log" 2>&1 || exit $?
cat "$GRAFT_REPO_ROOT/gpurun_out/${TAG}_prof/run_kernel_stats.csv"
echo done
