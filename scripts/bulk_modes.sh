#!/bin/bash
# Bulk path output modes on one box: straight into the caller's pinned buffer (default), the same
# with at most 2 chunks in flight (KW_BULK_DEPTH=2), and through the pinned bounce blocks
# (KW_BULK_DIRECT=0); each twice, alternating.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
TAG=${1:-r04bm}
for rep in 1 2; do
  for m in direct depth2 bounce; do
    case $m in direct) E="";; depth2) E="KW_BULK_DEPTH=2";; bounce) E="KW_BULK_DIRECT=0";; esac
    env $E KW_BULK_DEBUG=1 timeout -k 10 240 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/${TAG}_$m.json 2> gpurun_out/${TAG}_$m.err || exit $?
    python3 -c "
import json;d=json.loads(open('gpurun_out/${TAG}_$m.json').read().strip().splitlines()[-1]);t=d['timing_modes'];print('rep $rep $m pinned_ms=%.2f pageable_ms=%.2f' % (t['end_to_end']['ms'], t['end_to_end_pageable']['ms']))" | tee -a gpurun_out/${TAG}_summary.txt
    grep -h "kw bulk" gpurun_out/${TAG}_$m.err | sed "s/^/rep $rep $m /" >> gpurun_out/${TAG}_stages.txt
  done
done
