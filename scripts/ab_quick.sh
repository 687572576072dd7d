#!/bin/bash
# Kernel time per config for the variants named in VARIANTS (policy-server_amd/variants/<name>.so),
# alternating, REPS times, same box; no tests.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
TAG=${1:-abq}
for rep in $(seq 1 ${REPS:-2}); do
  for c in ${CFGS:-c2_trusted c3_group c4_64}; do
    for n in ${VARIANTS:-cur}; do
      KWGPU_LIB="$PWD/policy-server_amd/variants/$n.so" timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --no-host-modes > gpurun_out/${TAG}_${c}_${n}_$rep.json 2> gpurun_out/${TAG}_${c}_${n}_$rep.err
      rc=$?; echo "[ab] rep $rep $c $n rc=$rc $(python -c "import json;d=json.loads(open('gpurun_out/${TAG}_${c}_${n}_$rep.json').read().strip().splitlines()[-1]);print('evaluate_ms=%.4f' % d['kernel_ms']['evaluate'])" 2>/dev/null)" | tee -a gpurun_out/${TAG}_summary.txt
      if [ $rc -ne 0 ]; then exit $rc; fi
    done
  done
done
