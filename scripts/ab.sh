#!/bin/bash
# A/B of library variants (policy-server_amd/variants/*.so): GPU tests on the default build, then one
# bench per variant. Each GPU step is time-limited; a fault / timeout ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
TAG=${1:-ab}
stop() { local rc=$1 what=$2; echo "[ab] $what exit $rc"; if [ "$rc" -ge 124 ] || [ "$rc" -eq 134 ] || [ "$rc" -eq 139 ]; then exit "$rc"; fi; }
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 900 python -m pytest tests -m gpu -q -x -p no:cacheprovider > gpurun_out/${TAG}_gpu_tests.log 2>&1
  stop $? tests
fi
for v in policy-server_amd/variants/*.so; do
  n=$(basename "$v" .so)
  KW_TILE_DEBUG=${KW_TILE_DEBUG:-256} KWGPU_LIB="$PWD/$v" timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/${TAG}_${n}.json 2> gpurun_out/${TAG}_${n}.err
  stop $? "bench $n"
done
echo "[ab] done"
