#!/bin/bash
# r06 same-box A/B of the in-tree library against variants (policy-server_amd/variants/*.so) at
# the strong-scaling shard sizes and at 1M (C4), two alternating repetitions; a parity subset of
# the in-tree build first.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
TAG=${1:-abs}
timeout -k 10 300 python -u -m pytest tests/test_parity_gpu.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
  -k "${PARITY_K:-(c4_64 or parity) and not stream}" > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; echo "[ab] in-tree tests rc=$rc $(tail -1 gpurun_out/${TAG}_tests.log)"; [ $rc -ne 0 ] && exit $rc
LIBS="$PWD/policy-server_amd/libkwgpu.so $(ls $PWD/policy-server_amd/variants/*.so 2>/dev/null)"
for rep in 1 2; do
  for lib in $LIBS; do
    n=$(basename $lib .so)
    for r in ${ROWS_LIST:-125000 1000000}; do
      KWGPU_LIB=$lib timeout -k 10 200 python bench.py --rows $r --steps ${STEPS:-200} --warmup 20 --no-cpu-baseline --no-host-modes > gpurun_out/${TAG}_${n}_$r.json 2>/dev/null || exit $?
      python3 -c "import json;d=json.load(open('gpurun_out/${TAG}_${n}_$r.json'));print('[ab] rep=$rep lib=$n rows=$r kernel_ms=%.4f step_ms=%.4f G req/s=%.3f' % (d['kernel_ms']['evaluate'], d['ms_per_step'], d['value']/1e9))"
    done
  done
done
