#!/bin/bash
# r06 closing record, part A: the GPU suite, smoke(), the default bench line (C4: HBM-resident value,
# roofline, CPU baseline, timing modes), then every other BASELINE config's line.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
TAG=${1:-r06f}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/${TAG}_gpu_tests.log 2>&1
rc=$?; tail -1 gpurun_out/${TAG}_gpu_tests.log; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || exit $?
echo "[final] smoke ok"
timeout -k 10 600 python bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || exit $?
tail -c 300 gpurun_out/${TAG}_bench.json
for cfg in c2_trusted c3_group c5_mixed c6_256 c1_namespace; do
  timeout -k 10 400 python bench.py --config $cfg --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/${TAG}_${cfg}_bench.json 2> gpurun_out/${TAG}_${cfg}_bench.err || exit $?
  python3 -c "import json;d=json.load(open('gpurun_out/${TAG}_${cfg}_bench.json'));print('[final] $cfg', round(d['value']/1e6,1), 'M req/s kernel', round(d['kernel_ms']['evaluate'],4), 'ms frac', round(d['roofline']['frac'],4))"
done
