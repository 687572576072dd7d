#!/bin/bash
# Per-phase instruction mix of the slot kernel (diagnostic): one PMC pass per KW_TILE_DEBUG value
# (0 = full kernel; 1 / 2 / 4 skip classification / walk / verdict output), so the differences
# attribute VALU / SALU / LDS / SMEM instructions and wait cycles to each phase.
set -u
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-ph}
cd /tmp && export TMPDIR=/tmp
for d in ${DEBUGS:-0 1 2 4}; do
  KW_TILE_DEBUG=$d timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT --kernel-trace -d "$ROOT/gpurun_out/${TAG}_d$d" -o run --output-format csv -- python3 "$ROOT/bench.py" --steps 3 --warmup 1 --no-cpu-baseline > "$ROOT/gpurun_out/${TAG}_d$d.log" 2>&1
  rc=$?; if [ $rc -ne 0 ]; then echo "pass d=$d exit $rc"; exit $rc; fi
  (cd "$ROOT" && python3 scripts/pmc_summary.py "gpurun_out/${TAG}_d$d")
done
