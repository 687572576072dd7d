#!/bin/bash
# PMC passes over bench.py for the slot kernel, one counter group per rocprofv3 run (kernel-trace
# only, as the pool requires), then the HBM traffic summary profiles/traffic.json.
#   bash scripts/pmc.sh <tag>            -> gpurun_out/<tag>_pmc_<i>/ and profiles/traffic.json
#   CFG=c3_group bash scripts/pmc.sh <tag>   the same for another BASELINE config (bench.py --config)
# KWGPU_LIB=<variant .so> selects a library variant (default: the in-tree build).
set -u
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-pmc}
CFG=${CFG:-c4_64}
cd /tmp && export TMPDIR=/tmp
PASSES=(
  "FETCH_SIZE"
  "WRITE_SIZE"
  "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES"
  "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
)
i=0
for p in "${PASSES[@]}"; do
  timeout -k 10 300 rocprofv3 --pmc $p --kernel-trace -d "$ROOT/gpurun_out/${TAG}_pmc_$i" -o run --output-format csv -- python3 "$ROOT/bench.py" --config $CFG --steps 5 --warmup 2 --no-cpu-baseline --no-host-modes > "$ROOT/gpurun_out/${TAG}_pmc_$i.log" 2>&1
  rc=$?; echo "[pmc] pass $i ($p) exit $rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
  i=$((i+1))
done
cd "$ROOT"
ROWS=$(python3 -c "import sys; sys.path.insert(0, '.'); import bench; print(bench.CONFIGS['$CFG'][1])")
python3 scripts/pmc_summary.py --traffic "gpurun_out/${TAG}_pmc_0" "gpurun_out/${TAG}_pmc_1" "gpurun_out/${TAG}_traffic.json" "$TAG" "$CFG" "$ROWS" && \
python3 scripts/pmc_summary.py gpurun_out/${TAG}_pmc_0 gpurun_out/${TAG}_pmc_1 gpurun_out/${TAG}_pmc_2 gpurun_out/${TAG}_pmc_3 > "gpurun_out/${TAG}_pmc_summary.txt" && \
python3 scripts/pmc_summary.py --derived "$ROWS" gpurun_out/${TAG}_pmc_0 gpurun_out/${TAG}_pmc_1 gpurun_out/${TAG}_pmc_2 gpurun_out/${TAG}_pmc_3 >> "gpurun_out/${TAG}_pmc_summary.txt"
echo "[pmc] done"
