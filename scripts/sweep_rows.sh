set -u
for c in c3_group c5_mixed c6_256 c1_namespace; do
  echo "== $c"
  CFG=$c DBG=256 KNOBS="KW_SLOT_ROWS=96|KW_SLOT_ROWS=128" bash scripts/knob_sweep.sh r02_s35_$c || exit $?
done
