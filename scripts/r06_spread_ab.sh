#!/bin/bash
# r06: P0 copy jobs spread over the waves (KW_P0_SPREAD). Variants under policy-server_amd/variants
# (VARIANTS, default: spread spread0): C4 phase clocks of each, then kernel ms at C4, C5, C6 and at
# the 125k C4 shard, two alternating repetitions.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
VARIANTS=${VARIANTS:-spread spread0}
for v in $VARIANTS; do
  KWGPU_LIB=$PWD/policy-server_amd/variants/$v.so KW_TILE_DEBUG=512 timeout -k 10 200 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-host-modes > /dev/null 2> gpurun_out/sp_ph_$v.err || exit $?
  echo "[phases $v]"; grep -E "^\[kw (phase|seg)\]" gpurun_out/sp_ph_$v.err | tail -n 2
done
for rep in 1 2; do
  for v in $VARIANTS; do
    for c in ${CFGS:-c4_64 c5_mixed c6_256 c4_125k}; do
      args="--config $c --steps 20 --warmup 3"
      [ $c = c5_mixed ] && args="--config c5_mixed --steps 10 --warmup 2"
      [ $c = c4_125k ] && args="--rows 125000 --steps 300 --warmup 20"
      KWGPU_LIB=$PWD/policy-server_amd/variants/$v.so timeout -k 10 300 python bench.py $args --no-cpu-baseline --no-host-modes > gpurun_out/sp_${c}_$v.json 2>/dev/null || exit $?
      echo "[ab] rep=$rep $c $v $(python3 -c "import json;d=json.load(open('gpurun_out/sp_${c}_$v.json'));print('evaluate_ms=%.4f step_ms=%.4f' % (d['kernel_ms']['evaluate'], d['ms_per_step']))")"
    done
  done
done
