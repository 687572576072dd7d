#!/bin/bash
# Bulk path with a pinned output: chunks in flight (KW_BULK_DEPTH) 2 / 3 / 4, alternating, twice.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
TAG=${1:-r04bd}
for rep in 1 2; do
  for dp in 2 3 4; do
    KW_BULK_DEPTH=$dp KW_BULK_DEBUG=1 timeout -k 10 240 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/${TAG}_$dp.json 2> gpurun_out/${TAG}_$dp.err || exit $?
    python3 -c "
import json;d=json.loads(open('gpurun_out/${TAG}_$dp.json').read().strip().splitlines()[-1]);t=d['timing_modes'];print('rep $rep depth $dp pinned_ms=%.2f pageable_ms=%.2f' % (t['end_to_end']['ms'], t['end_to_end_pageable']['ms']))" | tee -a gpurun_out/${TAG}_summary.txt
    grep -h "kw bulk" gpurun_out/${TAG}_$dp.err | sed "s/^/rep $rep depth $dp /" >> gpurun_out/${TAG}_stages.txt
  done
done
