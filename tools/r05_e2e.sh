#!/bin/bash
# live-shape e2e read models (batcher_e2e --reads submit|kcopy|zc), after the PCIe warm-up
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=$1
mkdir -p gpurun_out
E=tests/c/_build/batcher_e2e
for w in 1 2 3 4; do
  timeout -k 10 120 $E --conns 1024 --frames 4 --size 65536 --flushes 20 --device 0 --async 1 --cap 0.5 --pin 1 > /dev/null || exit 1
done
for r in 1 2; do
  for m in submit kcopy zc zc:clzero; do
    IFS=: read rm cz <<< "$m"
    cf=0; [ -n "$cz" ] && cf=1
    UVHTTP_WS_BATCHER_CLZERO=$cf timeout -k 10 120 $E --conns 1024 --frames 4 --size 65536 --flushes 20 --device 0 --async 1 --cap 0.5 --pin 1 --reads $rm \
      | sed "s/}\$/, \"clzero\": $cf}/" >> gpurun_out/${T}_e2e.jsonl || exit 1
  done
done
python3 - <<PY
import json
for l in open("gpurun_out/${T}_e2e.jsonl"):
    d=json.loads(l); print(d["reads"], "clzero", d.get("clzero"), d["value"], "submit_ms/flush", d["submit_ms_per_flush"], "copy", d["per_flush_ms"]["copy"], "p99", d["blocked_p99_ms"], "zc", d["zero_copy_reads"], "ok", d["messages_ok"])
PY
