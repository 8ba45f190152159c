#!/bin/bash
# Round-3 probe 31: timeline of the live-shape batcher (async): kernels, memory copies and HIP
# API calls, to see what keeps a 256 MiB flush at ~11 ms when H2D + D2H together take 5.5 ms
# (tools/pcie_probe.hip)
set -uo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/r03p31
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 180 rocprofv3 --kernel-trace --memory-copy-trace --hip-runtime-trace --output-format csv -d "$OUT/async" -o run \
  -- "$ROOT/tests/c/_build/batcher_e2e" --conns 1024 --frames 4 --size 65536 --flushes 12 --device 0 --async 1 > "$OUT/async.json" 2> "$OUT/async.err" || { echo "async trace failed"; tail -5 "$OUT/async.err"; exit 1; }
timeout -k 10 180 rocprofv3 --kernel-trace --memory-copy-trace --hip-runtime-trace --output-format csv -d "$OUT/sync" -o run \
  -- "$ROOT/tests/c/_build/batcher_e2e" --conns 1024 --frames 4 --size 65536 --flushes 12 --device 0 --async 0 > "$OUT/sync.json" 2> "$OUT/sync.err" || { echo "sync trace failed"; exit 1; }
cat "$OUT/async.json" "$OUT/sync.json"
ls "$OUT/async"
