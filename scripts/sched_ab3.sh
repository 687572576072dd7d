#!/bin/bash
# Schedule A/B (r05): old dynamic schedule (variants/old.so), the hybrid (first two tiles static,
# variants/new.so), and the static schedule (KW_SCHED=static) — every config plus C4 shards, twice.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
run() {  # name lib env args...
  local n=$1 lib=$2 ev=$3; shift 3
  env $ev KWGPU_LIB=$PWD/policy-server_amd/variants/$lib.so timeout -k 10 300 python bench.py "$@" --no-cpu-baseline --no-host-modes > gpurun_out/sab3.json 2>/dev/null || exit $?
  python3 -c "import json;d=json.load(open('gpurun_out/sab3.json'));print('[sab3] $n $* kernel_ms=%.4f step_ms=%.4f' % (d['kernel_ms']['evaluate'], d['ms_per_step']))"
}
for rep in 1 2; do
  for a in "--config c4_64 --steps 20" "--config c5_mixed --steps 10" "--config c2_trusted --steps 20" "--config c3_group --steps 20" "--config c6_256 --steps 10" "--config c1_namespace --steps 50" "--rows 125000 --steps 300" "--rows 65536 --steps 300"; do
    run old old KW_X=0 $a
    run hybrid new KW_X=0 $a
    run static new KW_SCHED=static $a
  done
done
