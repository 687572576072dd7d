#!/bin/bash
# r06 GPU pass C: the whole GPU suite on the current build, then the deep sweeps: random group
# scripts in the bytecode form (KW_SCRIPT_SEEDS) and random policy sets (KW_FUZZ_SEEDS).
set -u
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$ROOT"; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06c_gpu_tests.log 2>&1
rc=$?; echo "[r06c] gpu tests exit $rc"; tail -n 3 gpurun_out/r06c_gpu_tests.log
[ $rc -ne 0 ] && exit $rc
KW_SCRIPT_SEEDS=${KW_SCRIPT_SEEDS:-40} timeout -k 10 600 python -u -m pytest tests/test_rhai_forms_gpu.py -m gpu -x -q -k random_scripts --timeout 300 --timeout-method thread > gpurun_out/r06c_script_fuzz.log 2>&1
rc=$?; echo "[r06c] script fuzz exit $rc"; tail -n 2 gpurun_out/r06c_script_fuzz.log
[ $rc -ne 0 ] && exit $rc
KW_FUZZ_SEEDS=${KW_FUZZ_SEEDS:-60} timeout -k 10 600 python -u -m pytest tests/test_fuzz_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06c_fuzz.log 2>&1
rc=$?; echo "[r06c] policy fuzz exit $rc"; tail -n 2 gpurun_out/r06c_fuzz.log
exit $rc
