#!/bin/bash
# Bulk path (kw_validate_host) A/B on one box: its GPU tests, then the default bench's host modes for
# the in-tree build and variants/bulk_old.so (the pre-r04 chunk loop), alternating, twice.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
TAG=${1:-r04bulk}
timeout -k 10 300 python -u -m pytest tests/test_bulk_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; tail -1 gpurun_out/${TAG}_tests.log; if [ $rc -ne 0 ]; then exit $rc; fi
for v in new old new old; do
  if [ $v = old ]; then export KWGPU_LIB=$PWD/policy-server_amd/variants/bulk_old.so; else unset KWGPU_LIB; fi
  KW_BULK_DEBUG=1 timeout -k 10 240 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/${TAG}_$v.json 2> gpurun_out/${TAG}_$v.err || exit $?
  python3 -c "
import json;d=json.loads(open('gpurun_out/${TAG}_$v.json').read().strip().splitlines()[-1]);t=d['timing_modes'];print('$v pinned_ms=%.2f pageable_ms=%.2f serial_ms=%.2f' % (t['end_to_end']['ms'], t['end_to_end_pageable']['ms'], t['end_to_end_serial']['ms']))" | tee -a gpurun_out/${TAG}_summary.txt
  grep -h "kw bulk" gpurun_out/${TAG}_$v.err >> gpurun_out/${TAG}_stages_$v.txt
done
