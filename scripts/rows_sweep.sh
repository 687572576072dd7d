#!/bin/bash
# Tile-height sweep (KW_SLOT_ROWS) per config: kernel ms (HIP events) and the plan line (LDS, grid).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
TAG=${1:-rows}
for spec in ${SPECS:-c3_group:96,104,112,120,128 c2_trusted:96,104,112,120,128 c4_64:52,56,60,64}; do
  cfg=${spec%%:*}; rows=${spec#*:}
  for r in ${rows//,/ }; do
    KW_SLOT_ROWS=$r KW_TILE_DEBUG=256 timeout -k 10 300 python bench.py --config $cfg --steps 10 --no-cpu-baseline --no-host-modes > gpurun_out/${TAG}_${cfg}_$r.json 2> gpurun_out/${TAG}_${cfg}_$r.err || exit $?
    echo "[rows] $cfg $r kernel_ms=$(python -c "import json;print('%.4f' % json.load(open('gpurun_out/${TAG}_${cfg}_$r.json'))['kernel_ms']['evaluate'])") $(grep -o 'lds=[0-9]* area' gpurun_out/${TAG}_${cfg}_$r.err | tail -1) $(grep -o 'grid=[0-9]* occupancy=[0-9]*' gpurun_out/${TAG}_${cfg}_$r.err | tail -1)"
  done
done
