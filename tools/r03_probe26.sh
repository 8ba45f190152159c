#!/bin/bash
# Round-3 probe 26: batcher end to end with the loop's uv_async modelled (on_ready -> poll
# between connections' reads), sync vs async, plus the batcher GPU tests
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r03p26
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_batcher_transitions.py tests/test_gpu_batcher_tls.py tests/test_gpu_batcher.py > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for a in 0 1 0 1 1; do
  timeout -k 10 200 tests/c/_build/batcher_e2e --conns 1024 --frames 4 --size 65536 --flushes 20 --device 0 --async $a > $OUT/e2e.tmp 2>&1 || { cat $OUT/e2e.tmp; exit 1; }
  cat $OUT/e2e.tmp | tee -a $OUT/e2e.jsonl
done
timeout -k 10 200 tests/c/_build/batcher_e2e --conns 1024 --frames 4 --size 65536 --flushes 3 --device -1 | tee -a $OUT/e2e.jsonl
