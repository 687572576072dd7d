#!/bin/bash
# Bulk knob sweep (scripts/bulk_knobs.py), each setting twice, interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
for rep in 1 2; do
  for s in "" "KW_BULK_DEPTH=4" "KW_BULK_DEPTH=6" "KW_BULK_CHUNK=131072" "KW_BULK_CHUNK=131072 KW_BULK_DEPTH=6" "KW_BULK_CHUNK=524288" "KW_BULK_CHUNK=65536 KW_BULK_DEPTH=8"; do
    env $s timeout -k 10 120 python scripts/bulk_knobs.py || exit $?
  done
done 2>&1 | tee gpurun_out/bulk_knobs.txt
