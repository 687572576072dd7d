#!/bin/bash
# Kernel time of every library variant (policy-server_amd/variants/*.so) on each config in CFGS,
# same box; no tests (run ab_variants.sh for parity first).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
TAG=${1:-abc}
for c in ${CFGS:-c2_trusted c3_group c4_64}; do
  for v in policy-server_amd/variants/*.so; do
    n=$(basename "$v" .so)
    KW_TILE_DEBUG=${KW_TILE_DEBUG:-256} KWGPU_LIB="$PWD/$v" timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --no-host-modes > gpurun_out/${TAG}_${c}_${n}.json 2> gpurun_out/${TAG}_${c}_${n}.err
    rc=$?; echo "[abc] $c $n rc=$rc $(python -c "import json;d=json.load(open('gpurun_out/${TAG}_${c}_${n}.json'));print('evaluate_ms=%.4f' % d['kernel_ms']['evaluate'])" 2>/dev/null)"
    if [ $rc -ne 0 ]; then exit $rc; fi
  done
done
