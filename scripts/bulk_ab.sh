set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_bulk_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r04_bulk_tests.log 2>&1 || exit $?
for v in new old new old; do
  if [ $v = old ]; then export KWGPU_LIB=$PWD/policy-server_amd/variants/bulk_old.so; else unset KWGPU_LIB; fi
  KW_BULK_DEBUG=1 timeout -k 10 240 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r04_bulk_$v.json 2> gpurun_out/r04_bulk_$v.err || exit $?
  python3 -c "
import json;d=json.loads(open('gpurun_out/r04_bulk_$v.json').read().strip().splitlines()[-1]);t=d['timing_modes'];print('$v', round(t['end_to_end']['ms'],2), round(t['end_to_end_pageable']['ms'],2))" | tee -a gpurun_out/r04_bulk_ab.txt
done
