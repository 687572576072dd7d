cd "${GRAFT_REPO_ROOT:-/root/repo}"
for r in 64 32 48; do
  KW_TILE_DEBUG=256 KW_SLOT_ROWS=$r timeout -k 10 300 python bench.py --config c5_mixed --no-cpu-baseline --no-host-modes > gpurun_out/s50_c5_r$r.json 2> gpurun_out/s50_c5_r$r.err || exit $?
  echo "c5 rows=$r $(python -c "import json;d=json.load(open('gpurun_out/s50_c5_r$r.json'));print('evaluate_ms=%.4f' % d['kernel_ms']['evaluate'])") $(grep -m1 'launch grid' gpurun_out/s50_c5_r$r.err)"
done
