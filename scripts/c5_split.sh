#!/bin/bash
# C5 tile-capacity sweep: the share of tiles the planner may split (KW_TILE_SPLIT) vs occupancy.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
for sp in ${SPLITS:-0.02 0.05 0.1 0.2}; do
  KW_TILE_DEBUG=256 KW_TILE_SPLIT=$sp timeout -k 10 300 python bench.py --config c5_mixed --no-cpu-baseline --no-host-modes > gpurun_out/c5s_$sp.json 2> gpurun_out/c5s_$sp.err || exit $?
  echo "split=$sp $(python -c "import json;d=json.load(open('gpurun_out/c5s_$sp.json'));print('evaluate_ms=%.4f' % d['kernel_ms']['evaluate'])") $(grep -m1 'launch grid' gpurun_out/c5s_$sp.err)"
done
