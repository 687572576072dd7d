#!/bin/bash
# LDS counter calibration on the GPU box: the lds_calib micro-kernels under one
# rocprofv3 --pmc pass (4 SQ counters), summarised per pattern against the bank rule's expectation.
#   scripts/lds_calib.sh > gpurun_out/lds_calib.txt
set -e
cd /tmp && export TMPDIR=/tmp
R="${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$R/gpurun_out/lds_calib"
rm -rf "$OUT" && mkdir -p "$OUT"
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT SQ_INSTS_LDS \
  --output-format csv -d "$OUT" -o calib -- "$R/scripts/lds_calib" >&2
python3 "$R/scripts/lds_calib_summary.py" "$OUT"
