#!/bin/bash
# A/B of plan knobs on one box (diagnostic): each line = one bench run with the given environment.
#   KNOBS="KW_SLOT_ROWS=32|KW_GLOBAL_TABLES=1" CFG=c4_64 bash scripts/knob_sweep.sh TAG
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
TAG=${1:-knob}
CFG=${CFG:-c4_64}
IFS='|' read -ra KS <<< "${KNOBS:-}"
KS=("" "${KS[@]}")
for k in "${KS[@]}"; do
  env KW_TILE_DEBUG=${DBG:-256} $k timeout -k 10 300 python bench.py --config $CFG --steps 20 --warmup 3 --no-cpu-baseline --no-host-modes \
    > gpurun_out/${TAG}.json 2> gpurun_out/${TAG}.err
  rc=$?
  echo "[$k] rc=$rc $(grep -m1 'kw tile\] lds_tables' gpurun_out/${TAG}.err) $(python -c "import json;d=json.load(open('gpurun_out/${TAG}.json'));print('evaluate_ms=%.4f Mreq/s=%.0f' % (d['kernel_ms']['evaluate'], d['value']/1e6))" 2>/dev/null)"
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/${TAG}.err; exit $rc; fi
  grep -h "kw phase" gpurun_out/${TAG}.err | tail -1 || true  # phase clocks (DBG=768): the last launch
done
