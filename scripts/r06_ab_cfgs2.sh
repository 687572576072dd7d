#!/bin/bash
# two alternating repetitions of scripts/ab_cfgs.sh (every variant on C2 / C3 / C4, same box)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash scripts/ab_cfgs.sh ${1:-ab2}a || exit $?
bash scripts/ab_cfgs.sh ${1:-ab2}b || exit $?
