#!/bin/bash
# The GPU suite on the in-tree build (L2 prefetch on), then C5 / C6 / C4 with (cur) and without (nopf) it.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
TAG=${1:-r04pfc}
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_gpu_tests.log 2>&1
rc=$?; tail -1 gpurun_out/${TAG}_gpu_tests.log; if [ $rc -ne 0 ]; then exit $rc; fi
REPS=2 CFGS="c5_mixed c6_256 c4_64" VARIANTS="cur nopf" bash scripts/ab_quick.sh $TAG
