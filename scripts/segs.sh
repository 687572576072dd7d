#!/bin/bash
# Phase and per-wave segment clocks of the timing instantiation (KW_TILE_DEBUG=512) per config:
# where a tile's critical path goes (P1 / P2 item segments, each phase's busy time and barrier wait).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
TAG=${1:-seg}
for CFG in ${CFGS:-c4_64 c3_group c2_trusted}; do
  KW_TILE_DEBUG=512 timeout -k 10 300 python bench.py --config $CFG --steps 2 --warmup 1 --no-cpu-baseline --no-host-modes > /dev/null 2> gpurun_out/${TAG}_${CFG}.err || exit $?
  echo "[$CFG] $(grep -E 'kw phase' gpurun_out/${TAG}_${CFG}.err | tail -1)"
  echo "[$CFG] $(grep -E 'kw seg' gpurun_out/${TAG}_${CFG}.err | tail -1)"
done
echo "[seg] done"
