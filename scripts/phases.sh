#!/bin/bash
# Phase clocks of the tile kernel's diagnostics instantiation under KW_TILE_DEBUG ablation bits
# (DEBUGS: values added to 512), then kernel time of the product instantiation per bit (KDEBUGS).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
CFG=${CFG:-c4_64}
for d in ${DEBUGS:-0 1 2 7}; do
  KW_TILE_DEBUG=$((512 + d)) timeout -k 10 300 python bench.py --config $CFG --steps 2 --warmup 1 --no-cpu-baseline --no-host-modes > /dev/null 2> gpurun_out/ph_$d.err || exit $?
  echo "debug=$d $(grep -E 'kw phase' gpurun_out/ph_$d.err | tail -1 | sed 's/.*cycles.tile//')"
done
for d in ${KDEBUGS:-}; do
  KW_TILE_DEBUG=$d timeout -k 10 300 python bench.py --config $CFG --steps 10 --warmup 2 --no-cpu-baseline --no-host-modes > gpurun_out/kd_$d.json 2>/dev/null || exit $?
  echo "kernel debug=$d $(python -c "import json;d=json.load(open('gpurun_out/kd_$d.json'));print('%.4f' % d['kernel_ms']['evaluate'])")"
done
