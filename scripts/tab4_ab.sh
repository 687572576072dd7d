#!/bin/bash
# Capability-mutation rows four loads a round (slots.hpp tab_or): variants/tab4.so against the r05
# final build (variants/cur.so, lib 700c76f3): parity subset on tab4, then C4 / C5 kernel times, twice.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
KWGPU_LIB=$PWD/policy-server_amd/variants/tab4.so timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/test_parity_gpu.py tests/test_ctr_scan.py > gpurun_out/tab4_tests.log 2>&1; rc=$?
tail -1 gpurun_out/tab4_tests.log; [ $rc -eq 0 ] || exit $rc
run() {  # name lib args...
  local n=$1 lib=$2; shift 2
  KWGPU_LIB=$PWD/policy-server_amd/variants/$lib.so timeout -k 10 300 python bench.py "$@" --no-cpu-baseline --no-host-modes > gpurun_out/tab4_ab.json 2>/dev/null || exit $?
  python3 -c "import json;d=json.load(open('gpurun_out/tab4_ab.json'));print('[tab4_ab] $n $* kernel_ms=%.4f step_ms=%.4f' % (d['kernel_ms']['evaluate'], d['ms_per_step']))"
}
for rep in 1 2; do
  for a in "--config c4_64 --steps 20" "--config c5_mixed --steps 10"; do
    run cur cur $a
    run tab4 tab4 $a
  done
done
