#!/bin/bash
# The live-shape harness (tests/c/batcher_e2e.c) several times in a row on one box, to separate
# run-order effects (first processes slower) from the queue sizing: one JSON line per run.
# usage: tools/e2e_order.sh OUT "async cap" ["async cap" ...]
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/$1
shift
: > "$OUT"
for spec in "$@"; do
  set -- $spec
  timeout -k 10 120 tests/c/_build/batcher_e2e --conns 1024 --frames 4 --size 65536 --flushes 20 \
    --device 0 --async "$1" --cap "$2" --pin 1 | tail -1 | sed "s/^{/{\"spec\": \"$spec\", /" >> "$OUT" || exit 1
done
python3 - "$OUT" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    d = json.loads(l)
    print(f'{d["spec"]:10s} {d["value"]:6.1f} GiB/s  p50 {d["blocked_p50_ms"]:.2f}  p99 {d["blocked_p99_ms"]:.2f}  max {d["max_blocked_ms"]:.2f} ms  wait/flush {d["per_flush_ms"]["wait"]:.2f}  copy/flush {d["per_flush_ms"]["copy"]:.2f}')
PY
