#!/bin/bash
# Deeper SQ counters of the tile kernel (diagnostics): issue activity per instruction type, LDS /
# SMEM instruction levels (in-flight count summed per cycle: / instructions = average latency),
# LDS FIFO and conflict stalls. Two passes (<= 8 SQ counters each), kernel-trace only.
set -u
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-deep}
CFG=${CFG:-c4_64}
cd /tmp && export TMPDIR=/tmp
PASSES=(
  "SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_SALU SQ_INST_LEVEL_LDS SQ_INSTS_LDS SQ_WAVE_CYCLES"
  "SQ_INSTS_BRANCH SQ_INST_LEVEL_SMEM SQ_INSTS_SMEM SQ_LDS_CMD_FIFO_FULL SQ_LDS_DATA_FIFO_FULL SQ_LDS_ADDR_CONFLICT SQ_BUSY_CU_CYCLES SQ_CYCLES"
  "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES"
  "SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VSKIPPED SQ_INSTS_VALU_INT SQ_INSTS_VALU_CVT SQ_INSTS_VMEM_RD SQ_INSTS_LDS_LOAD SQ_BUSY_CYCLES"
)
PASSES=("${PASSES[@]:${FIRST:-0}}")
i=${FIRST:-0}
for p in "${PASSES[@]}"; do
  timeout -k 10 -s KILL 200 rocprofv3 --pmc $p --kernel-trace -d "$ROOT/gpurun_out/${TAG}_pmc_$i" -o run --output-format csv -- python3 "$ROOT/bench.py" --config $CFG --steps 5 --warmup 2 --no-cpu-baseline --no-host-modes > "$ROOT/gpurun_out/${TAG}_pmc_$i.log" 2>&1
  rc=$?; echo "[deep] pass $i exit $rc"; if [ $rc -ne 0 ]; then tail -3 "$ROOT/gpurun_out/${TAG}_pmc_$i.log"; exit $rc; fi
  i=$((i+1))
done
cd "$ROOT" && python3 scripts/pmc_summary.py gpurun_out/${TAG}_pmc_*[0-9]
