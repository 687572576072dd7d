#!/bin/bash
# Counter evidence per BASELINE config: phase clocks (KW_TILE_DEBUG 512) and the
# four PMC passes of scripts/pmc.sh, for each config in CFGS. Every GPU step under its own limit;
# a failing step ends the script.
set -u
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$ROOT"; mkdir -p gpurun_out
TAG=${1:-r03m}
for CFG in ${CFGS:-c4_64 c3_group c2_trusted c5_mixed}; do
  KW_TILE_DEBUG=768 timeout -k 10 300 python bench.py --config $CFG --steps 2 --warmup 1 --no-cpu-baseline --no-host-modes > /dev/null 2> gpurun_out/${TAG}_${CFG}_phase.err || exit $?
  echo "[$CFG] $(grep -E 'kw phase' gpurun_out/${TAG}_${CFG}_phase.err | tail -1)"
  CFG=$CFG bash scripts/pmc.sh ${TAG}_${CFG} || exit $?
  cd "$ROOT"
done
echo "[measure] done"
