#!/bin/bash
# r04 A/B on one box: the GPU suite on the in-tree build, then kernel time per config for the
# in-tree build (variants/cur.so) against the previous commit (variants/bulk_old.so), alternating,
# twice; then the bulk path (kw_validate_host) for both.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
TAG=${1:-r04ab}
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_gpu_tests.log 2>&1
rc=$?; tail -2 gpurun_out/${TAG}_gpu_tests.log; if [ $rc -ne 0 ]; then exit $rc; fi
for rep in 1 2; do
  for c in ${CFGS:-c2_trusted c3_group c4_64}; do
    for n in ${VARIANTS:-cur bulk_old kvascii}; do
      KWGPU_LIB="$PWD/policy-server_amd/variants/$n.so" timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --no-host-modes > gpurun_out/${TAG}_${c}_${n}_$rep.json 2> gpurun_out/${TAG}_${c}_${n}_$rep.err
      rc=$?; echo "[ab] rep $rep $c $n rc=$rc $(python -c "import json;d=json.loads(open('gpurun_out/${TAG}_${c}_${n}_$rep.json').read().strip().splitlines()[-1]);print('evaluate_ms=%.4f' % d['kernel_ms']['evaluate'])" 2>/dev/null)" | tee -a gpurun_out/${TAG}_summary.txt
      if [ $rc -ne 0 ]; then exit $rc; fi
    done
  done
done
for n in cur bulk_old cur bulk_old; do
  KW_BULK_DEBUG=1 KWGPU_LIB="$PWD/policy-server_amd/variants/$n.so" timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/${TAG}_bulk_$n.json 2> gpurun_out/${TAG}_bulk_$n.err
  rc=$?; echo "[ab] bulk $n rc=$rc $(python -c "import json;d=json.loads(open('gpurun_out/${TAG}_bulk_$n.json').read().strip().splitlines()[-1]);t=d['timing_modes'];print('pinned_ms=%.2f pageable_ms=%.2f' % (t['end_to_end']['ms'], t['end_to_end_pageable']['ms']))" 2>/dev/null)" | tee -a gpurun_out/${TAG}_summary.txt
  if [ $rc -ne 0 ]; then exit $rc; fi
done
echo "[ab] done"
