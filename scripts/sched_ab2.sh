#!/bin/bash
# Tile schedule A/B (r05): the per-XCD dynamic counters against the strided static schedule
# (KW_SCHED=static), every config, alternating, twice; kernel ms and step ms.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
for rep in 1 2; do
  for cfg in c4_64 c5_mixed c2_trusted c3_group c6_256 c1_namespace; do
    for s in dyn static; do
      if [ $s = static ]; then export KW_SCHED=static; else unset KW_SCHED; fi
      timeout -k 10 300 python bench.py --config $cfg --steps 20 --warmup 3 --no-cpu-baseline --no-host-modes > gpurun_out/sab_${cfg}_$s.json 2>/dev/null || exit $?
      python3 -c "import json;d=json.load(open('gpurun_out/sab_${cfg}_$s.json'));print('[sab] $cfg $s kernel_ms=%.4f step_ms=%.4f' % (d['kernel_ms']['evaluate'], d['ms_per_step']))"
    done
  done
done
