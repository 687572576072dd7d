#!/bin/bash
# Bulk path (kw_validate_host) A/B on one box: packed chunk uploads (one H2D + scatter kernel per
# chunk, default) against one H2D per column range (KW_BULK_PACK=0), the default bench's host modes,
# alternating, three times each; then C5's line once per mode.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
TAG=${1:-r05pack}
timeout -k 10 300 python -u -m pytest tests/test_bulk_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; tail -1 gpurun_out/${TAG}_tests.log; if [ $rc -ne 0 ]; then exit $rc; fi
summ() {
  python3 -c "
import json;d=json.loads(open('$1').read().strip().splitlines()[-1]);t=d['timing_modes']
print('$2 staged_ms=%.2f (%.1f M/s) pinned_cols_ms=%.2f pageable_ms=%.2f serial_ms=%.2f' % (t['end_to_end']['ms'], t['end_to_end']['value']/1e6, t['end_to_end_pinned_columns']['ms'], t['end_to_end_pageable']['ms'], t['end_to_end_serial']['ms']))" | tee -a gpurun_out/${TAG}_summary.txt
}
for v in pack percol pack percol pack percol; do
  if [ $v = percol ]; then export KW_BULK_PACK=0; else unset KW_BULK_PACK; fi
  KW_BULK_DEBUG=1 timeout -k 10 240 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/${TAG}_$v.json 2> gpurun_out/${TAG}_$v.err || exit $?
  summ gpurun_out/${TAG}_$v.json "c4 $v"
  grep -h "kw bulk" gpurun_out/${TAG}_$v.err >> gpurun_out/${TAG}_stages_$v.txt
done
for v in pack percol; do
  if [ $v = percol ]; then export KW_BULK_PACK=0; else unset KW_BULK_PACK; fi
  timeout -k 10 400 python bench.py --config c5_mixed --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/${TAG}_c5_$v.json 2> gpurun_out/${TAG}_c5_$v.err || exit $?
  summ gpurun_out/${TAG}_c5_$v.json "c5 $v"
done
