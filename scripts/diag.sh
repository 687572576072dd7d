#!/bin/bash
# Diagnostics of the tile kernel on one box: phase clocks (KW_TILE_DEBUG 512), then the kernel time
# with phases / sub-phases ablated (KW_TILE_DEBUG bits, capi.cpp), all at C4 unless CFG is set.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
TAG=${1:-diag}
CFG=${CFG:-c4_64}
KW_TILE_DEBUG=768 timeout -k 10 300 python bench.py --config $CFG --steps 2 --warmup 1 --no-cpu-baseline --no-host-modes > /dev/null 2> gpurun_out/${TAG}_phase.err || exit $?
grep -E "kw phase|kw tile\] launch" gpurun_out/${TAG}_phase.err | head -8
for d in ${DEBUGS:-0 1 2 4 6 7 1024 2048 4096}; do
  KW_TILE_DEBUG=$d timeout -k 10 300 python bench.py --config $CFG --steps 10 --warmup 2 --no-cpu-baseline --no-host-modes > gpurun_out/${TAG}_d$d.json 2>gpurun_out/${TAG}_d$d.err
  rc=$?; echo "debug=$d rc=$rc $(python -c "import json;d=json.load(open('gpurun_out/${TAG}_d$d.json'));print('%.4f' % d['kernel_ms']['evaluate'])" 2>/dev/null)"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
