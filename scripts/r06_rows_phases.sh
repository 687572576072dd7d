#!/bin/bash
# r06: phase clocks and LDS layout of C4 1M at tile heights 64 / 63 / 62 (KW_TILE_DEBUG 512 + 256).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
for sr in 64 63 62; do
  KW_SLOT_ROWS=$sr KW_TILE_DEBUG=768 timeout -k 10 200 python bench.py --rows ${ROWS:-1000000} --steps 2 --warmup 1 --no-cpu-baseline --no-host-modes > /dev/null 2> gpurun_out/rp_$sr.err || exit $?
  echo "[rows $sr]"; grep -E "^\[kw (phase|seg|layout|tile|lds)" gpurun_out/rp_$sr.err | sort | uniq -c | sort -rn | head -n 8
done
