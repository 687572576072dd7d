#!/bin/bash
# After the per-region schedule rule: GPU suite, then every config's kernel / step ms and C4 shards.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 500 --timeout-method thread > gpurun_out/sc_tests.log 2>&1
rc=$?; tail -1 gpurun_out/sc_tests.log; [ $rc -eq 0 ] || exit $rc
for a in "--config c4_64 --steps 20" "--config c5_mixed --steps 10" "--config c2_trusted --steps 20" "--config c3_group --steps 20" "--config c6_256 --steps 10" "--config c1_namespace --steps 50" "--rows 125000 --steps 300" "--rows 250000 --steps 300" "--rows 500000 --steps 200"; do
  timeout -k 10 300 python bench.py $a --no-cpu-baseline --no-host-modes > gpurun_out/sc.json 2>/dev/null || exit $?
  python3 -c "import json;d=json.load(open('gpurun_out/sc.json'));print('[sc] $a kernel_ms=%.4f step_ms=%.4f value=%.1fM' % (d['kernel_ms']['evaluate'], d['ms_per_step'], d['value']/1e6))"
done
