#!/bin/bash
# Where the instructions go: per KW_TILE_DEBUG ablation bit (capi.cpp), the product kernel's time and
# its VALU / SALU / LDS instruction counts (one rocprofv3 --pmc pass each, kernel-trace only).
#   CFG=c4_64 DEBUGS="0 1 2 4" bash scripts/ablate_pmc.sh <tag>
set -u
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-abl}
CFG=${CFG:-c4_64}
cd /tmp && export TMPDIR=/tmp
ROWS=$(cd "$ROOT" && python3 -c "import bench; print(bench.CONFIGS['$CFG'][1])")
for d in ${DEBUGS:-0 1 2 4 1024 2048 4096 8192 16384}; do
  KW_TILE_DEBUG=$d timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY --kernel-trace -d "$ROOT/gpurun_out/${TAG}_d$d" -o run --output-format csv -- python3 "$ROOT/bench.py" --config $CFG --steps 5 --warmup 2 --no-cpu-baseline --no-host-modes > "$ROOT/gpurun_out/${TAG}_d$d.log" 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then echo "[abl] debug=$d exit $rc"; exit $rc; fi
  (cd "$ROOT" && python3 - "$ROOT/gpurun_out/${TAG}_d$d" "$ROWS" "$d" <<'PY'
import sys
sys.path.insert(0, "scripts")
from pmc_summary import summarise
s = summarise(sys.argv[1]); n = float(sys.argv[2])
print(f"debug={sys.argv[3]:>6} kernel_ms={s['dur_ns'] / 1e6:.4f} VALU/req={s['SQ_INSTS_VALU'] / n:6.1f} SALU/req={s['SQ_INSTS_SALU'] / n:5.1f} "
      f"LDS/req={s['SQ_INSTS_LDS'] / n:5.1f} wait={s['SQ_WAIT_ANY'] / s['SQ_WAVE_CYCLES']:.3f} active={s['SQ_ACTIVE_INST_ANY'] / s['SQ_WAVE_CYCLES']:.3f}")
PY
  )
done
echo "[abl] done"
