#!/bin/bash
# r04 serving and bulk record: kwhost under kwload at 16 / 64 / 256 connections with 4 pipeline
# workers, 256 connections with 8, then one default bench line (PCIe rates, bulk path).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
TAG=${1:-r04srv}
WORKERS=4 timeout -k 10 200 bash scripts/serve_bench.sh ${TAG}_w4 || exit $?
WORKERS=8 CONNS=256 timeout -k 10 120 bash scripts/serve_bench.sh ${TAG}_w8 || exit $?
timeout -k 10 300 python bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || exit $?
echo "[r04 serve] done"
