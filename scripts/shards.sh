#!/bin/bash
# C4 at strong-scaling shard sizes on one GPU (1M over 8 / 4 / 2 GPUs): kernel and step time per pass.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
for r in ${ROWS_LIST:-125000 250000 500000}; do
  timeout -k 10 200 python bench.py --rows $r --steps 300 --warmup 20 --no-cpu-baseline --no-host-modes > gpurun_out/shard_$r.json 2>/dev/null || exit $?
  python3 -c "import json;d=json.load(open('gpurun_out/shard_$r.json'));print('[shard] rows=$r kernel_ms=%.4f step_ms=%.4f G req/s=%.3f' % (d['kernel_ms']['evaluate'], d['ms_per_step'], d['value']/1e9))"
done
