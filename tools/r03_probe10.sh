#!/bin/bash
# Round-3 probe 10: live-shape e2e through the batcher, sync vs async, per-phase times.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r03p10
mkdir -p $OUT
for a in 0 1 0 1; do
  timeout -k 10 200 tests/c/_build/batcher_e2e --conns 1024 --frames 4 --size 65536 --flushes 20 --device 0 --async $a > $OUT/e2e.tmp 2>&1 || { cat $OUT/e2e.tmp; exit 1; }
  cat $OUT/e2e.tmp | tee -a $OUT/e2e.jsonl
done
