#!/bin/bash
# Round-3 probe 40: live-shape batcher timelines (tests/c/batcher_e2e --trace 1): async x3, sync x1,
# 20 rounds each, plus the box's PCIe ceiling
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r03p40
mkdir -p $OUT
timeout -k 10 60 tools/bin/pcie_probe 256 2 | tee $OUT/pcie.jsonl
for k in 1 2 3; do
  timeout -k 10 120 tests/c/_build/batcher_e2e --conns 1024 --frames 4 --size 65536 --flushes 20 --device 0 --async 1 --trace 1 > $OUT/e2e_async$k.json 2> $OUT/trace_async$k.txt || exit 1
  cut -c1-420 $OUT/e2e_async$k.json
done
timeout -k 10 120 tests/c/_build/batcher_e2e --conns 1024 --frames 4 --size 65536 --flushes 20 --device 0 --async 0 --trace 1 > $OUT/e2e_sync.json 2> $OUT/trace_sync.txt || exit 1
cut -c1-420 $OUT/e2e_sync.json
