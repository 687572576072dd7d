#!/bin/bash
# C5 (10M) ablations of the current build (KW_TILE_DEBUG bits, diagnostics only: verdicts wrong): kernel ms.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
for rep in 1; do
  for dbg in 0 1 2 4 2048 4096 8192 16384; do
    KW_TILE_DEBUG=$dbg timeout -k 10 300 python bench.py --config c5_mixed --steps 10 --no-cpu-baseline --no-host-modes > gpurun_out/c5ab_$dbg.json 2> /dev/null || exit $?
    echo "[c5] debug=$dbg kernel_ms=$(python -c "import json;print('%.4f' % json.load(open('gpurun_out/c5ab_$dbg.json'))['kernel_ms']['evaluate'])")"
  done
done
