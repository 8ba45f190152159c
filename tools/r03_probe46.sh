#!/bin/bash
# Round-3 probe 46: the async batcher when the loop outruns PCIe (AVX2 copy, pinned loop):
# loop timeline (--trace 1) and the copy / kernel trace
set -uo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/r03p46
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 120 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d "$OUT/trace" -o run \
  -- "$ROOT/tests/c/_build/batcher_e2e" --conns 1024 --frames 4 --size 65536 --flushes 12 --device 0 --async 1 --pin 1 --trace 1 \
  > "$OUT/e2e.json" 2> "$OUT/loop_trace.txt" || { echo "trace failed"; tail -5 "$OUT/loop_trace.txt"; exit 1; }
cut -c1-300 "$OUT/e2e.json"
