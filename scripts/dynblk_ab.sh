#!/bin/bash
# P1 / P2 item blocks from per-phase LDS counters (a wave that drew cheap blocks takes more; P2 order
# containers, requests, labels): variants/dyn.so against the r05 final build (variants/cur.so, lib
# 61d4cd9e): parity subset on dyn, then kernel times per config, alternating, twice.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
KWGPU_LIB=$PWD/policy-server_amd/variants/dyn.so timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/test_parity_gpu.py tests/test_ctr_scan.py tests/test_label_pairs.py tests/test_split_rows.py > gpurun_out/dyn_tests.log 2>&1; rc=$?
tail -2 gpurun_out/dyn_tests.log; [ $rc -eq 0 ] || exit $rc
run() {  # name lib args...
  local n=$1 lib=$2; shift 2
  KWGPU_LIB=$PWD/policy-server_amd/variants/$lib.so timeout -k 10 300 python bench.py "$@" --no-cpu-baseline --no-host-modes > gpurun_out/dyn_ab.json 2>/dev/null || exit $?
  python3 -c "import json;d=json.load(open('gpurun_out/dyn_ab.json'));print('[dyn_ab] $n $* kernel_ms=%.4f step_ms=%.4f' % (d['kernel_ms']['evaluate'], d['ms_per_step']))"
}
for rep in 1 2; do
  for a in "--config c4_64 --steps 20" "--config c5_mixed --steps 10" "--config c2_trusted --steps 20" "--config c3_group --steps 20" "--config c6_256 --steps 10"; do
    run cur cur $a
    run dyn dyn $a
  done
done
