#!/bin/bash
# r04 closing record of the final build: the GPU suite, smoke(), then C4 (with its HBM traffic passes)
# and C5 bench lines, rocprofv3 kernel stats and LDS counters.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
TAG=${1:-r04y}
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_gpu_tests.log 2>&1
rc=$?; tail -1 gpurun_out/${TAG}_gpu_tests.log; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || exit $?
echo "[final] smoke ok"
CFGS="c4_64 c5_mixed" bash scripts/r04_measure.sh $TAG
