#!/bin/bash
# Bulk path chunk size and in-flight depth, staged and with page-locked columns: one bench run per
# variant, alternating, twice (C4 1M).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
TAG=${1:-r04bs}
for rep in 1 2; do
  for v in base c64k c256k d1 d3; do
    case $v in base) E="";; c64k) E="KW_BULK_CHUNK=65536";; c256k) E="KW_BULK_CHUNK=262144";; d1) E="KW_BULK_DEPTH=1";; d3) E="KW_BULK_DEPTH=3";; esac
    env $E KW_BULK_DEBUG=1 timeout -k 10 240 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/${TAG}_$v.json 2> gpurun_out/${TAG}_$v.err || exit $?
    python3 - gpurun_out/${TAG}_$v.json "$rep $v" <<'PY' | tee -a gpurun_out/${TAG}_summary.txt
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); t = d['timing_modes']
print('rep %s staged_ms=%.2f pinned_cols_ms=%.2f pageable_ms=%.2f' % (sys.argv[2], t['end_to_end']['ms'], t['end_to_end_pinned_columns']['ms'], t['end_to_end_pageable']['ms']))
PY
    grep -h "kw bulk" gpurun_out/${TAG}_$v.err | sed "s/^/rep $rep $v /" >> gpurun_out/${TAG}_stages.txt
  done
done
