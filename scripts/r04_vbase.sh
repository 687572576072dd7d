#!/bin/bash
# LDS region offsets in VGPRs (KW_VBASE) vs not, on C4 / C5 (the instantiation it changes) and C2
# (control, unchanged code); then the bulk path's in-flight depth sweep.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
REPS=2 CFGS="c4_64 c5_mixed c2_trusted" VARIANTS="vbase novbase" bash scripts/ab_quick.sh ${1:-r04vb} || exit $?
bash scripts/bulk_depth.sh ${1:-r04vb}_bd
