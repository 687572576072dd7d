#!/bin/bash
# r06 GPU pass A: the GPU suite on the current build, then the C4 LDS-conflict ablations and the
# C2 / C3 PMC passes (scripts/r06_lds_ablate.sh).
set -u
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$ROOT"; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06a_gpu_tests.log 2>&1
rc=$?; echo "[r06a] gpu tests exit $rc"; tail -n 3 gpurun_out/r06a_gpu_tests.log
[ $rc -ne 0 ] && exit $rc
bash scripts/r06_lds_ablate.sh r06lds > gpurun_out/r06lds.log 2>&1
rc=$?; echo "[r06a] ablate exit $rc"; tail -n 5 gpurun_out/r06lds.log
exit $rc
