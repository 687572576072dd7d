#!/bin/bash
# C5 bulk path stage clocks (KW_BULK_DEBUG=1) in both upload modes, and C4's once more.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
TAG=${1:-r05c5bulk}
timeout -k 10 300 python -u -m pytest tests/test_bulk_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; tail -1 gpurun_out/${TAG}_tests.log; if [ $rc -ne 0 ]; then exit $rc; fi
for v in pack percol; do
  if [ $v = percol ]; then export KW_BULK_PACK=0; else unset KW_BULK_PACK; fi
  KW_BULK_DEBUG=1 timeout -k 10 240 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/${TAG}_c4_$v.json 2> gpurun_out/${TAG}_c4_$v.err || exit $?
  grep -h "kw bulk" gpurun_out/${TAG}_c4_$v.err | tail -7
  KW_BULK_DEBUG=1 timeout -k 10 400 python bench.py --config c5_mixed --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/${TAG}_c5_$v.json 2> gpurun_out/${TAG}_c5_$v.err || exit $?
  grep -h "kw bulk" gpurun_out/${TAG}_c5_$v.err | tail -7
done
