#!/bin/bash
# One GPU-box session: parity tests, smoke, bench, kernel-trace profile. Every GPU step has its own
# time limit; a fault / abort / timeout (exit >= 124) ends the script before any further GPU step.
# Plain test failures (exit 1) do not stop the bench.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
TAG=${1:-r01}
STEPS=${STEPS:-tests,smoke,bench,prof}
stop_on_fault() { local rc=$1 what=$2; echo "[gpu_run] $what exit $rc"; if [ "$rc" -ge 124 ] || [ "$rc" -eq 134 ] || [ "$rc" -eq 139 ]; then echo "[gpu_run] stopping after $what"; exit "$rc"; fi; }
rocm-smi --showproductname > gpurun_out/${TAG}_smi.txt 2>&1 || true
if [[ $STEPS == *tests* ]]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/${TAG}_gpu_tests.log 2>&1
  stop_on_fault $? tests
fi
if [[ $STEPS == *smoke* ]]; then
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1
  stop_on_fault $? smoke
fi
if [[ $STEPS == *bench* ]]; then
  KW_TILE_DEBUG=${KW_TILE_DEBUG:-0} timeout -k 10 600 python bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
  stop_on_fault $? bench
fi
if [[ $STEPS == *prof* ]]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/${TAG}_prof" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 20 --no-cpu-baseline --no-host-modes > "$GRAFT_REPO_ROOT/gpurun_out/${TAG}_prof.log" 2>&1
  stop_on_fault $? prof
  cd "$GRAFT_REPO_ROOT"
fi
echo "[gpu_run] done"
