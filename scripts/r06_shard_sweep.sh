#!/bin/bash
# r06: strong-scaling shard sizes of C4 under tile heights (KW_SLOT_ROWS) and the
# two tile schedules (KW_SCHED): kernel (HIP events) and step time per pass.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
for r in ${ROWS_LIST:-125000 250000}; do
  for sr in ${SR_LIST:-64 48 40 32}; do
    for sc in ${SCHED_LIST:-auto}; do
      envs="KW_SLOT_ROWS=$sr"; [ "$sc" != auto ] && envs="$envs KW_SCHED=$sc"
      env $envs timeout -k 10 200 python bench.py --rows $r --steps 300 --warmup 20 --no-cpu-baseline --no-host-modes > gpurun_out/sw_${r}_${sr}_${sc}.json 2>/dev/null || exit $?
      python3 -c "import json;d=json.load(open('gpurun_out/sw_${r}_${sr}_${sc}.json'));print('[sweep] rows=$r slot_rows=$sr sched=$sc kernel_ms=%.4f step_ms=%.4f G req/s=%.3f' % (d['kernel_ms']['evaluate'], d['ms_per_step'], d['value']/1e9))"
    done
  done
done
# phase clocks of one pass at 125k and 1M (the timing instantiation: table staging per workgroup,
# cycles per tile, workgroup start spread)
for r in 125000 1000000; do
  KW_TILE_DEBUG=512 timeout -k 10 200 python bench.py --rows $r --steps 2 --warmup 1 --no-cpu-baseline --no-host-modes > /dev/null 2> gpurun_out/ph_$r.err || exit $?
  echo "[phases] rows=$r"; grep -E "^\[kw (phase|start|seg)\]" gpurun_out/ph_$r.err | tail -n 3
done
