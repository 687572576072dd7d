#!/bin/bash
# A/B of the slot kernel's tile height (KW_SLOT_ROWS): kernel time and LDS / occupancy per setting.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
TAG=${1:-rows}
for r in ${ROWS:-64 56 48 40 32}; do
  KW_SLOT_ROWS=$r KW_TILE_DEBUG=${KW_TILE_DEBUG:-0} timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/${TAG}_r$r.json 2> gpurun_out/${TAG}_r$r.err
  rc=$?; echo "rows=$r rc=$rc $(python -c "import json;d=json.load(open('gpurun_out/${TAG}_r$r.json'));print(round(d['kernel_ms']['evaluate'],4), round(d['value']/1e6,1))" 2>/dev/null) $(grep -m1 'fused=' gpurun_out/${TAG}_r$r.err)"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
if [ -n "${PARITY_ROWS:-}" ]; then
  KW_SLOT_ROWS=$PARITY_ROWS timeout -k 10 600 python -u -m pytest tests/test_parity_gpu.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/${TAG}_parity.log 2>&1
  rc=$?; echo "parity rows=$PARITY_ROWS rc=$rc"; tail -2 gpurun_out/${TAG}_parity.log
fi
