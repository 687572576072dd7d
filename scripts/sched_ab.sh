#!/bin/bash
# GPU parity tests, then A/B of the slot kernel's tile schedule (KW_SCHED=static vs the default).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
TAG=${1:-sched}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -1 gpurun_out/${TAG}_tests.log; [ $rc -eq 0 ] || exit $rc
for k in 1 2; do
  for s in static dynamic; do
    KW_SCHED=$s timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/${TAG}_${s}$k.json 2>/dev/null || exit $?
    echo "$s: $(python -c "import json;d=json.load(open('gpurun_out/${TAG}_${s}$k.json'));print(round(d['kernel_ms']['evaluate'],4), round(d['value']/1e6,1))")"
  done
done
