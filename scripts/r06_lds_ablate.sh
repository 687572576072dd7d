#!/bin/bash
# r06: where C4's LDS bank-conflict cycles and waits come from, one rocprofv3
# --pmc pass per KW_TILE_DEBUG ablation bit (capi.cpp), then the PMC passes of scripts/pmc.sh for C2
# and C3 (HBM traffic, waits, conflicts). Summaries under gpurun_out/<tag>_*.
set -u
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-r06lds}
cd "$ROOT"; mkdir -p gpurun_out
CTRS="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS"
CFG=${CFG:-c4_64} CTRS="$CTRS" DBGS="${DBGS:-0 1 2 4 2048 1024 4096 8192 16384}" bash scripts/pmc_ablate.sh ${TAG}_c4 || exit $?
if [ -z "${NO_C23:-}" ]; then
  CFG=c2_trusted bash scripts/pmc.sh ${TAG}_c2 || exit $?
  CFG=c3_group bash scripts/pmc.sh ${TAG}_c3 || exit $?
fi
echo "[r06lds] done"
