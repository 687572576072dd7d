#!/bin/bash
# Strided schedule within each XCD's range (r05): GPU suite, benches, and C4's FETCH_SIZE.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 500 --timeout-method thread > gpurun_out/xc_tests.log 2>&1
rc=$?; tail -1 gpurun_out/xc_tests.log; [ $rc -eq 0 ] || exit $rc
for a in "--config c4_64 --steps 20" "--config c2_trusted --steps 20" "--config c3_group --steps 20" "--config c1_namespace --steps 50" "--config c5_mixed --steps 10" "--config c6_256 --steps 10" "--rows 125000 --steps 300"; do
  timeout -k 10 300 python bench.py $a --no-cpu-baseline --no-host-modes > gpurun_out/xc.json 2>/dev/null || exit $?
  python3 -c "import json;d=json.load(open('gpurun_out/xc.json'));print('[xc] $a kernel_ms=%.4f step_ms=%.4f value=%.1fM' % (d['kernel_ms']['evaluate'], d['ms_per_step'], d['value']/1e6))"
done
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/xc_fetch -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-host-modes > $GRAFT_REPO_ROOT/gpurun_out/xc_fetch.log 2>&1 || exit $?
cd $GRAFT_REPO_ROOT && python3 scripts/pmc_summary.py gpurun_out/xc_fetch | head -2
