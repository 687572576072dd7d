#!/bin/bash
# Bulk path in-flight depth by column kind: the default (3 staged, 2 page-locked) against depth 2
# everywhere (KW_BULK_DEPTH=2), alternating, three times (C4 1M).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
TAG=${1:-r04d3}
timeout -k 10 300 python -u -m pytest tests/test_bulk_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_tests.log
for rep in 1 2 3; do
  for v in default d2; do
    case $v in default) E="";; d2) E="KW_BULK_DEPTH=2";; esac
    env $E KW_BULK_DEBUG=1 timeout -k 10 240 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/${TAG}_$v.json 2> gpurun_out/${TAG}_$v.err || exit $?
    python3 - gpurun_out/${TAG}_$v.json "$rep $v" <<'PY' | tee -a gpurun_out/${TAG}_summary.txt
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); t = d['timing_modes']
print('rep %s staged_ms=%.2f pinned_cols_ms=%.2f pageable_ms=%.2f' % (sys.argv[2], t['end_to_end']['ms'], t['end_to_end_pinned_columns']['ms'], t['end_to_end_pageable']['ms']))
PY
  done
done
