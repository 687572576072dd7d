#!/bin/bash
# Phase clocks (KW_TILE_DEBUG 512 + DEBUGS bits) for every library variant in policy-server_amd/variants.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
CFG=${CFG:-c4_64}
for v in policy-server_amd/variants/*.so; do
  n=$(basename "$v" .so)
  for d in ${DEBUGS:-0 7}; do
    KWGPU_LIB="$PWD/$v" KW_TILE_DEBUG=$((512 + d)) timeout -k 10 300 python bench.py --config $CFG --steps 2 --warmup 1 --no-cpu-baseline --no-host-modes > /dev/null 2> gpurun_out/phv_${n}_$d.err || exit $?
    echo "$n debug=$d $(grep -E 'kw phase' gpurun_out/phv_${n}_$d.err | tail -1 | sed 's/.*cycles.tile//')"
  done
done
