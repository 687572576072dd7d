#!/bin/bash
# Phase ablation of the fused tile kernel (diagnostic): time with DFA / features / evaluation skipped.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
TAG=${1:-abl}
for d in 0 1 2 4 3 5 6 7; do
  KW_TILE_DEBUG=$d timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/${TAG}_d$d.json 2>/dev/null
  rc=$?; echo "debug=$d rc=$rc $(python -c "import json;d=json.load(open('gpurun_out/${TAG}_d$d.json'));print(d['kernel_ms'])" 2>/dev/null)"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES -d "$GRAFT_REPO_ROOT/gpurun_out/${TAG}_pmc1" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 2 --warmup 1 --no-cpu-baseline > "$GRAFT_REPO_ROOT/gpurun_out/${TAG}_pmc1.log" 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU -d "$GRAFT_REPO_ROOT/gpurun_out/${TAG}_pmc2" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 2 --warmup 1 --no-cpu-baseline > "$GRAFT_REPO_ROOT/gpurun_out/${TAG}_pmc2.log" 2>&1 || exit $?
echo done
