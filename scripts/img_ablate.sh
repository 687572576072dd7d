#!/bin/bash
# C2 / C3 image-chain ablations (KW_TILE_DEBUG, diagnostics only: the verdicts are wrong): the kernel
# time with the image DFA walks skipped (32768), the literal probes skipped (65536), both, and no
# classification at all (1) — the most any specialisation of the globs or probes could save.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
for rep in 1 2; do
for cfg in c3_group c2_trusted; do
  for dbg in 0 32768 65536 98304 1; do
    KW_TILE_DEBUG=$dbg timeout -k 10 300 python bench.py --config $cfg --steps 10 --no-cpu-baseline --no-host-modes > gpurun_out/imgab_${cfg}_$dbg.json 2> /dev/null || exit $?
    echo "[img] $cfg debug=$dbg kernel_ms=$(python -c "import json;print('%.4f' % json.load(open('gpurun_out/imgab_${cfg}_$dbg.json'))['kernel_ms']['evaluate'])")"
  done
done
done
