#!/bin/bash
# r06: tile heights just under 64 rows (round-filling: the fewest rows that keep the number of
# tile rounds per workgroup) against 64, alternating, at the strong-scaling shard and the 1M pass.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
for rep in 1 2 3; do
  for r in ${ROWS_LIST:-125000 1000000}; do
    for sr in ${SR_LIST:-64 62 63}; do
      KW_SLOT_ROWS=$sr timeout -k 10 200 python bench.py --rows $r --steps ${STEPS:-300} --warmup 20 --no-cpu-baseline --no-host-modes > gpurun_out/ra_${r}_${sr}.json 2>/dev/null || exit $?
      python3 -c "import json;d=json.load(open('gpurun_out/ra_${r}_${sr}.json'));print('[rows] rep=$rep rows=$r slot_rows=$sr kernel_ms=%.4f step_ms=%.4f G req/s=%.3f' % (d['kernel_ms']['evaluate'], d['ms_per_step'], d['value']/1e9))"
    done
  done
done
