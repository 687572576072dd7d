#!/bin/bash
# Second label-value DFAs walked by idle lanes (helper lanes through a per-wave mailbox): the GPU
# suite on the in-tree build (= variants/pairs.so), then kernel times of variants/fold.so (before,
# acef07b) and pairs.so, alternating, twice, per config.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/pairs_tests.log 2>&1; rc=$?
tail -3 gpurun_out/pairs_tests.log; [ $rc -eq 0 ] || exit $rc
run() {  # name lib args...
  local n=$1 lib=$2; shift 2
  KWGPU_LIB=$PWD/policy-server_amd/variants/$lib.so timeout -k 10 300 python bench.py "$@" --no-cpu-baseline --no-host-modes > gpurun_out/pairs_ab.json 2>/dev/null || exit $?
  python3 -c "import json;d=json.load(open('gpurun_out/pairs_ab.json'));print('[pairs_ab] $n $* kernel_ms=%.4f step_ms=%.4f' % (d['kernel_ms']['evaluate'], d['ms_per_step']))"
}
for rep in 1 2; do
  for a in "--config c4_64 --steps 20" "--config c5_mixed --steps 10" "--config c6_256 --steps 10"; do
    run before fold $a
    run pairs pairs $a
  done
done
