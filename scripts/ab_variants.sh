#!/bin/bash
# A/B of library variants (policy-server_amd/variants/*.so): per variant a parity subset on the
# GPU (the same tests, KWGPU_LIB selecting the variant), then a C4 bench. Stops at any failure.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
TAG=${1:-abv}
for v in policy-server_amd/variants/*.so; do
  n=$(basename "$v" .so)
  KWGPU_LIB="$PWD/$v" timeout -k 10 300 python -u -m pytest tests/test_parity_gpu.py -x -q -p no:cacheprovider --timeout 120 \
    --timeout-method thread -k "${PARITY_K:-(c4_64 or parity) and not stream}" > gpurun_out/${TAG}_${n}_tests.log 2>&1
  rc=$?; echo "[abv] $n tests rc=$rc $(tail -1 gpurun_out/${TAG}_${n}_tests.log)"
  if [ $rc -ne 0 ]; then exit $rc; fi
  KW_TILE_DEBUG=256 KWGPU_LIB="$PWD/$v" timeout -k 10 300 python bench.py --config ${CFG:-c4_64} --no-cpu-baseline --no-host-modes > gpurun_out/${TAG}_${n}.json 2> gpurun_out/${TAG}_${n}.err
  rc=$?; echo "[abv] $n bench rc=$rc $(python -c "import json;d=json.load(open('gpurun_out/${TAG}_${n}.json'));print('evaluate_ms=%.4f' % d['kernel_ms']['evaluate'])" 2>/dev/null) grid=$(grep -o 'grid [0-9]*' gpurun_out/${TAG}_${n}.err | head -1)"
  if [ $rc -ne 0 ]; then tail -3 gpurun_out/${TAG}_${n}.err; exit $rc; fi
  if [ -n "${PHASE:-}" ]; then  # phase clocks of the diagnostics instantiation
    KW_TILE_DEBUG=512 KWGPU_LIB="$PWD/$v" timeout -k 10 300 python bench.py --config ${CFG:-c4_64} --steps 2 --warmup 1 --no-cpu-baseline --no-host-modes > /dev/null 2> gpurun_out/${TAG}_${n}_phase.err || exit $?
    grep "kw phase" gpurun_out/${TAG}_${n}_phase.err | tail -1
  fi
done
echo "[abv] done"
