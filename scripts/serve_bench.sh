#!/bin/bash
# Serving measurement (SURVEY §8(d) mode 4): kwhost on one GPU driven by kwload over loopback.
# For each connection count: a fresh kwload run of DURATION s after WARMUP s; one JSON line each
# into gpurun_out/${TAG}_serve.jsonl. kwhost is started once and stopped by its PID.
#   scripts/serve_bench.sh TAG [CONFIG_YML] [POLICY] [SYNTH_CONFIG]
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
TAG=${1:-serve}
YML=${2:-configs/c4_64.yml}
POLICY=${3:-psp-capabilities-00}
SCFG=${4:-4}
CONNS=${CONNS:-"16 64 256"}
DURATION=${DURATION:-8}
WARMUP=${WARMUP:-2}
WORKERS=${WORKERS:-4}
MAXB=${MAXB:-512}
WAIT=${WAIT:-200}
PORT=$((20000 + RANDOM % 20000))
OUT=gpurun_out/${TAG}_serve.jsonl
: > "$OUT"; : > gpurun_out/${TAG}_serve_stats.jsonl
DEVARG="--device 0"; [ -n "${DEVICES:-}" ] && DEVARG="--devices $DEVICES"  # DEVICES=0,0: two pipelines on one GPU
policy-server_amd/kwhost --policies "$YML" --port $PORT $DEVARG --continue-on-errors \
  --always-accept-admission-reviews-on-namespace kubewarden --workers $WORKERS --max-batch $MAXB --max-wait-us $WAIT --stats-ms 1000 \
  2> gpurun_out/${TAG}_kwhost.err &
KW=$!
trap 'kill $KW 2>/dev/null; wait $KW 2>/dev/null' EXIT
for i in $(seq 1 600); do
  if curl -s -o /dev/null -w '%{http_code}' http://127.0.0.1:$PORT/readiness 2>/dev/null | grep -q 200; then break; fi
  if ! kill -0 $KW 2>/dev/null; then echo "[serve] kwhost exited"; cat gpurun_out/${TAG}_kwhost.err; exit 1; fi
  sleep 0.1
done
echo "[serve] kwhost ready on $PORT (workers=$WORKERS max-batch=$MAXB max-wait-us=$WAIT)"
for c in $CONNS; do
  timeout -k 5 $((DURATION + WARMUP + 60)) policy-server_amd/kwload --port $PORT --policy "$POLICY" --connections $c \
    --duration $DURATION --warmup $WARMUP --config $SCFG >> "$OUT" || { echo "[serve] kwload failed at $c"; exit 1; }
  tail -1 "$OUT"
  sleep 1.2  # kwhost's cumulative stage times (--stats-ms) after this run
  echo "{\"connections\": $c, $(grep kwhost_stats gpurun_out/${TAG}_kwhost.err | tail -1 | cut -c2-)" >> gpurun_out/${TAG}_serve_stats.jsonl
done
echo "[serve] done"
