#!/bin/bash
# Diagnostic: instruction mix of the tile kernel per ablation (KW_TILE_DEBUG bits: 1 no classification,
# 2 no first-violation walk, 4 no verdict words, 1024 no mandatory labels, 2048 no value DFAs, 4096 no
# predecessor OR). One rocprofv3 --pmc pass (SQ counters only) per setting; the summary is one line each.
#   DBGS="0 4 2" bash scripts/pmc_ablate.sh TAG
set -u
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-abl}
CFG=${CFG:-c4_64}
CTRS=${CTRS:-"SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"}
cd /tmp && export TMPDIR=/tmp
for d in ${DBGS:-0 4 2 6 2048 1 1024 4096}; do
  KW_TILE_DEBUG=$d timeout -s KILL 120 rocprofv3 --pmc $CTRS --kernel-trace -d "$ROOT/gpurun_out/${TAG}_d$d" -o run --output-format csv -- python3 "$ROOT/bench.py" --config $CFG --steps 5 --warmup 2 --no-cpu-baseline --no-host-modes > "$ROOT/gpurun_out/${TAG}_d$d.log" 2>&1
  rc=$?; echo "[ablate] debug=$d exit $rc"
  if [ $rc -ne 0 ]; then tail -5 "$ROOT/gpurun_out/${TAG}_d$d.log"; exit $rc; fi
  python3 "$ROOT/scripts/pmc_summary.py" "$ROOT/gpurun_out/${TAG}_d$d" | tee -a "$ROOT/gpurun_out/${TAG}_summary.txt"
done
echo "[ablate] done"
