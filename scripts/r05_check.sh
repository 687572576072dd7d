#!/bin/bash
# r05 GPU check: the GPU test suite, smoke, the default bench (C4) and C5's bench line.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
TAG=${1:-r05c}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 600 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/${TAG}_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || exit $?
echo smoke ok
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.log || exit $?
cat gpurun_out/${TAG}_bench.json
timeout -k 10 400 python bench.py --config c5_mixed --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/${TAG}_c5_bench.json 2> gpurun_out/${TAG}_c5_bench.log || exit $?
cat gpurun_out/${TAG}_c5_bench.json
