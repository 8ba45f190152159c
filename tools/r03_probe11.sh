#!/bin/bash
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r03p11
mkdir -p $OUT
UVHTTP_WS_BATCHER_TRACE=1 timeout -k 10 200 tests/c/_build/batcher_e2e --conns 1024 --frames 4 --size 65536 --flushes 6 --device 0 --async 1 > $OUT/e2e_async.txt 2>&1 || { tail $OUT/e2e_async.txt; exit 1; }
UVHTTP_WS_BATCHER_TRACE=1 timeout -k 10 200 tests/c/_build/batcher_e2e --conns 1024 --frames 4 --size 65536 --flushes 6 --device 0 --async 0 > $OUT/e2e_sync.txt 2>&1 || { tail $OUT/e2e_sync.txt; exit 1; }
tail -30 $OUT/e2e_async.txt; tail -12 $OUT/e2e_sync.txt
