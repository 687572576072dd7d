#!/bin/bash
# PMC passes for the tiled kernel of each library variant (policy-server_amd/variants/*.so), one
# counter group per rocprofv3 run (kernel-trace only, as the pool requires). Output: gpurun_out/<tag>_pmc_<variant>_<pass>/
set -u
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-pmc}
cd /tmp && export TMPDIR=/tmp
PASSES=(
  "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES"
  "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
  "FETCH_SIZE"
  "WRITE_SIZE"
)
for v in "$ROOT"/policy-server_amd/variants/*.so; do
  n=$(basename "$v" .so)
  i=0
  for p in "${PASSES[@]}"; do
    KWGPU_LIB="$v" timeout -k 10 300 rocprofv3 --pmc $p --kernel-trace -d "$ROOT/gpurun_out/${TAG}_${n}_$i" -o run --output-format csv -- python3 "$ROOT/bench.py" --steps 5 --warmup 2 --no-cpu-baseline > "$ROOT/gpurun_out/${TAG}_${n}_$i.log" 2>&1
    rc=$?; echo "[pmc] $n pass $i exit $rc"
    if [ $rc -ne 0 ]; then exit $rc; fi
    i=$((i+1))
  done
done
echo "[pmc] done"
