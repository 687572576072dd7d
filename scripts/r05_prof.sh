#!/bin/bash
# r05 closing record, part B: rocprofv3 kernel stats of the default bench (C4) and C5, the PMC passes
# of scripts/pmc.sh on C4 (HBM traffic -> gpurun_out/<tag>_traffic.json), and one C5 pass of wave
# counters per dispatch (the light and heavy regions' occupancy).
set -u
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$ROOT"; mkdir -p gpurun_out
TAG=${1:-r05p}
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/${TAG}_c4_stats" -o run --output-format csv -- python3 "$ROOT/bench.py" --steps 20 --warmup 3 --no-cpu-baseline --no-host-modes > "$ROOT/gpurun_out/${TAG}_c4_stats.json" 2> "$ROOT/gpurun_out/${TAG}_c4_stats.err" || exit $?
echo "[prof] c4 stats ok"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/${TAG}_c5_stats" -o run --output-format csv -- python3 "$ROOT/bench.py" --config c5_mixed --steps 10 --warmup 2 --no-cpu-baseline --no-host-modes > "$ROOT/gpurun_out/${TAG}_c5_stats.json" 2> "$ROOT/gpurun_out/${TAG}_c5_stats.err" || exit $?
echo "[prof] c5 stats ok"
timeout -s KILL 400 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace -d "$ROOT/gpurun_out/${TAG}_c5_waves" -o run --output-format csv -- python3 "$ROOT/bench.py" --config c5_mixed --steps 3 --warmup 1 --no-cpu-baseline --no-host-modes > "$ROOT/gpurun_out/${TAG}_c5_waves.log" 2>&1 || exit $?
echo "[prof] c5 waves ok"
cd "$ROOT" && bash scripts/pmc.sh ${TAG}_c4 || exit $?
