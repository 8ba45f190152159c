#!/bin/bash
# Round-3 probe 43: the batcher with AVX2 streaming copies in submit_read: host copy probe,
# batcher tests, e2e sync / async with traces (which regime when the loop outruns PCIe?)
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r03p43
mkdir -p $OUT
timeout -k 10 120 tools/bin/copy_probe 1 | tee $OUT/copy.jsonl
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_batcher.py tests/test_batcher_transitions.py tests/test_gpu_batcher_tls.py tests/test_c1_echo.py > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 60 tools/bin/pcie_probe 256 1 | tee $OUT/pcie.jsonl
for k in 1 2; do
  timeout -k 10 120 tests/c/_build/batcher_e2e --conns 1024 --frames 4 --size 65536 --flushes 20 --device 0 --async 1 --trace 1 > $OUT/e2e_async$k.json 2> $OUT/trace_async$k.txt || exit 1
  cut -c1-300 $OUT/e2e_async$k.json; cut -c300-700 $OUT/e2e_async$k.json
done
timeout -k 10 120 tests/c/_build/batcher_e2e --conns 1024 --frames 4 --size 65536 --flushes 20 --device 0 --async 0 > $OUT/e2e_sync.json 2>/dev/null || exit 1
cut -c1-300 $OUT/e2e_sync.json
