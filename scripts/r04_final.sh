#!/bin/bash
# r04 closing check on one box: the GPU suite, smoke(), then C6 (the global-table instantiation) and
# C4 bench lines with rocprofv3 kernel stats.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
TAG=${1:-r04z}
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_gpu_tests.log 2>&1
rc=$?; tail -1 gpurun_out/${TAG}_gpu_tests.log; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || exit $?
echo "[final] smoke ok"
CFGS="c6_256 c4_64" NO_TRAFFIC=1 bash scripts/r04_measure.sh $TAG
