#!/bin/bash
# Instruction-cache counters of the tile kernel (diagnostics): list the SQC counters, then one pass.
set -u
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-ic}
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > "$ROOT/gpurun_out/${TAG}_counters.txt" 2>&1
grep -o "SQC_[A-Z_]*\|SQ_IFETCH[A-Z_]*\|SQ_INSTS_[A-Z_]*" "$ROOT/gpurun_out/${TAG}_counters.txt" | sort -u | tr '\n' ' '; echo
timeout -k 10 -s KILL 200 rocprofv3 --pmc ${PMC:-SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH} --kernel-trace -d "$ROOT/gpurun_out/${TAG}_pmc" -o run --output-format csv -- python3 "$ROOT/bench.py" --config ${CFG:-c4_64} --steps 5 --warmup 2 --no-cpu-baseline --no-host-modes > "$ROOT/gpurun_out/${TAG}_pmc.log" 2>&1
rc=$?; echo "[ic] pmc exit $rc"; tail -3 "$ROOT/gpurun_out/${TAG}_pmc.log"
exit $rc
