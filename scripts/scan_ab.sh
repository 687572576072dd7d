#!/bin/bash
# P2 container predecessor sets: or_range loops (variants/base.so) vs the segmented wave OR-scan
# (variants/rng.so, the kFeatRng instantiation): the GPU suite on the in-tree build (= rng.so) first, then C5 and C4
# kernel times, alternating, twice.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/scan_tests.log 2>&1; rc=$?
tail -3 gpurun_out/scan_tests.log; [ $rc -eq 0 ] || exit $rc
run() {  # name lib args...
  local n=$1 lib=$2; shift 2
  KWGPU_LIB=$PWD/policy-server_amd/variants/$lib.so timeout -k 10 300 python bench.py "$@" --no-cpu-baseline --no-host-modes > gpurun_out/scan_ab.json 2>/dev/null || exit $?
  python3 -c "import json;d=json.load(open('gpurun_out/scan_ab.json'));print('[scan_ab] $n $* kernel_ms=%.4f step_ms=%.4f' % (d['kernel_ms']['evaluate'], d['ms_per_step']))"
}
for rep in 1 2; do
  for a in "--config c5_mixed --steps 10" "--config c4_64 --steps 20"; do
    run base base $a
    run rng rng $a
  done
done
