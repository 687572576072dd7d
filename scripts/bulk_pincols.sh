#!/bin/bash
# Bulk path with the batch's columns page-locked in place (kw_batch_pin_host) beside the staged
# default: the bulk GPU tests, then the bench's timing modes three times with per-stage timings.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
TAG=${1:-r04pc}
timeout -k 10 300 python -u -m pytest tests/test_bulk_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_tests.log
for rep in 1 2 3; do
  KW_BULK_DEBUG=1 timeout -k 10 240 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/${TAG}_$rep.json 2> gpurun_out/${TAG}_$rep.err || exit $?
  python3 - gpurun_out/${TAG}_$rep.json $rep <<'PY' | tee -a gpurun_out/${TAG}_summary.txt
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); t = d['timing_modes']; p = t['pcie']
print('rep %s staged_ms=%.2f pinned_cols_ms=%.2f pin_host_ms=%.1f pageable_ms=%.2f h2d=%.1f d2h=%.1f bidir=%.1f GB/s bound=%.1fM bound_bidir=%.1fM' % (
    sys.argv[2], t['end_to_end']['ms'], t['end_to_end_pinned_columns']['ms'], t['end_to_end_pinned_columns']['pin_host_ms'],
    t['end_to_end_pageable']['ms'], p['h2d_GB_per_s'], p['d2h_GB_per_s'], p['bidir_GB_per_s'],
    p['bulk_bound_requests_per_s'] / 1e6, p['bulk_bound_bidir_requests_per_s'] / 1e6))
PY
  grep -h "kw bulk" gpurun_out/${TAG}_$rep.err | sed "s/^/rep $rep /" >> gpurun_out/${TAG}_stages.txt
done
