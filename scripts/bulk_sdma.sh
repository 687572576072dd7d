#!/bin/bash
# Copy engines vs blit kernels for the bulk path: the bench's PCIe rates (one way and both ways at
# once) and bulk timing modes with the default SDMA copies and with HSA_ENABLE_SDMA=0, alternating.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
TAG=${1:-r04sd}
for rep in 1 2; do
  for m in sdma blit; do
    case $m in sdma) E="";; blit) E="HSA_ENABLE_SDMA=0";; esac
    env $E KW_BULK_DEBUG=1 timeout -k 10 240 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/${TAG}_$m$rep.json 2> gpurun_out/${TAG}_$m$rep.err || exit $?
    python3 - gpurun_out/${TAG}_$m$rep.json "$rep $m" <<'PY' | tee -a gpurun_out/${TAG}_summary.txt
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); t = d['timing_modes']; p = t['pcie']
print('rep %s staged_ms=%.2f pinned_cols_ms=%.2f pageable_ms=%.2f h2d=%.1f d2h=%.1f bidir=%.1f GB/s bound_bidir=%.1fM kernel_ms=%.4f' % (
    sys.argv[2], t['end_to_end']['ms'], t['end_to_end_pinned_columns']['ms'],
    t['end_to_end_pageable']['ms'], p['h2d_GB_per_s'], p['d2h_GB_per_s'], p['bidir_GB_per_s'],
    p['bulk_bound_bidir_requests_per_s'] / 1e6, d['ms_per_step']))
PY
    grep -h "kw bulk" gpurun_out/${TAG}_$m$rep.err | sed "s/^/rep $rep $m /" >> gpurun_out/${TAG}_stages.txt
  done
done
