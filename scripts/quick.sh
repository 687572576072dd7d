#!/bin/bash
# Quick GPU check: parity tests, a short bench and one PMC pass (LDS / wave-state counters).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
TAG=${1:-q}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/${TAG}_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/${TAG}_bench.json 2>/dev/null || exit $?
python -c "import json;d=json.load(open('gpurun_out/${TAG}_bench.json'));print('bench', round(d['value']/1e6,1), 'Mreq/s', d['kernel_ms'])"
KW_TILE_DEBUG=256 timeout -k 10 300 python bench.py --steps 1 --warmup 0 --no-cpu-baseline > /dev/null 2> gpurun_out/${TAG}_tile.log || exit $?
grep -m10 "kw tile" gpurun_out/${TAG}_tile.log || true
[ -n "${NOPMC:-}" ] && exit 0
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY --kernel-trace -d "$GRAFT_REPO_ROOT/gpurun_out/${TAG}_pmc" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 3 --warmup 1 --no-cpu-baseline > "$GRAFT_REPO_ROOT/gpurun_out/${TAG}_pmc.log" 2>&1 || exit $?
cd "$GRAFT_REPO_ROOT" && python3 scripts/pmc_summary.py gpurun_out/${TAG}_pmc
