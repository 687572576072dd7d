#!/bin/bash
# r06: the PMC passes of scripts/pmc.sh for the other single-launch BASELINE configs (C2, C3, C6), so their
# bench lines carry roofline.traffic (profiles/traffic_<config>.json).
set -u
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
for cfg in ${CFGS:-c2_trusted c3_group c6_256}; do
  CFG=$cfg bash "$ROOT/scripts/pmc.sh" ${1:-r06t}_$cfg || exit $?
done
