#!/bin/bash
# r06 GPU pass B: kwhost (incl. --devices 0,0), \p{..} patterns and the rhai forms on the device,
# then the 125k / 1M shard kernel traces (scripts/r06_shard_trace.sh).
set -u
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_kwhost_gpu.py tests/test_patterns_gpu.py tests/test_rhai_forms_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06b_gpu_tests.log 2>&1
rc=$?; echo "[r06b] gpu tests exit $rc"; tail -n 3 gpurun_out/r06b_gpu_tests.log
[ $rc -ne 0 ] && exit $rc
bash scripts/r06_shard_trace.sh > gpurun_out/r06tr.log 2>&1
rc=$?; echo "[r06b] trace exit $rc"; tail -n 20 gpurun_out/r06tr.log
exit $rc
