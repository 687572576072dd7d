#!/bin/bash
# r04 record per BASELINE config: one bench line, one rocprofv3 kernel-trace summary, and the LDS
# counter pass (SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE, calibrated in profiles/r04_lds_calib.txt)
# with the instruction mix, for each config in CFGS; then the HBM traffic passes for C4.
#   bash scripts/r04_measure.sh <tag>   -> gpurun_out/<tag>_<cfg>.json, <tag>_<cfg>_prof/, <tag>_<cfg>_lds/
# Every GPU step under its own limit; a failing step ends the script.
set -u
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$ROOT"; mkdir -p gpurun_out
TAG=${1:-r04m}
LDS="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
stop() { local rc=$1 what=$2; echo "[r04] $what exit $rc"; if [ "$rc" -ne 0 ]; then exit "$rc"; fi; }
for c in ${CFGS:-c4_64 c2_trusted c3_group c5_mixed c6_256}; do
  timeout -k 10 300 python bench.py --config $c > gpurun_out/${TAG}_$c.json 2> gpurun_out/${TAG}_$c.err
  stop $? "bench $c"
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/${TAG}_${c}_prof" \
     -o run --output-format csv -- python3 "$ROOT/bench.py" --config $c --steps 10 --no-cpu-baseline --no-host-modes \
     > "$ROOT/gpurun_out/${TAG}_${c}_prof.log" 2>&1)
  stop $? "prof $c"
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --pmc $LDS --kernel-trace -d "$ROOT/gpurun_out/${TAG}_${c}_lds" \
     -o run --output-format csv -- python3 "$ROOT/bench.py" --config $c --steps 5 --warmup 2 --no-cpu-baseline --no-host-modes \
     > "$ROOT/gpurun_out/${TAG}_${c}_lds.log" 2>&1)
  stop $? "lds pmc $c"
done
if [ -z "${NO_TRAFFIC:-}" ]; then
  CFG=c4_64 bash scripts/pmc.sh ${TAG}_c4traffic
  stop $? "traffic c4"
fi
echo "[r04] done"
