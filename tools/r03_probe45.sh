#!/bin/bash
# Round-3 probe 45: batcher with AVX2 copies, one fence per upload, loop pinned to the GPU's NUMA
# node: batcher GPU tests, copy probe, e2e async/sync pinned and unpinned
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r03p45
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_batcher.py tests/test_batcher_transitions.py tests/test_gpu_batcher_tls.py tests/test_c1_echo.py > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 120 tools/bin/copy_probe 1 | tee $OUT/copy.jsonl
timeout -k 10 60 tools/bin/pcie_probe 256 1 | tee $OUT/pcie.jsonl
for r in 1 2; do
  for pin in 1 0; do
    for a in 1 0; do
      timeout -k 10 120 tests/c/_build/batcher_e2e --conns 1024 --frames 4 --size 65536 --flushes 20 --device 0 --async $a --pin $pin > $OUT/e.json 2>/dev/null || exit 1
      cat $OUT/e.json >> $OUT/e2e.jsonl
      python3 -c "import json;d=json.load(open('$OUT/e.json'));print('pin=$pin async=$a', d['value'], d['ms_per_flush'], d['device_flushes'], d['per_flush_ms']['copy'], d['blocked_ms_per_flush'], d['max_blocked_ms'], d['gpu_numa_node'], d['pinned_node'])"
    done
  done
done
