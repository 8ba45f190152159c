#!/bin/bash
# Round-3 probe 2: batcher GPU tests (async), header-gather floor, timing-event A/B, e2e live.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r03p2
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_batcher.py tests/test_batcher_transitions.py > $OUT/pytest_batcher.log 2>&1
rc=$?
tail -3 $OUT/pytest_batcher.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 tools/bin/hdr_probe > $OUT/hdr_probe.txt 2>&1 || exit 1
cat $OUT/hdr_probe.txt
for cfg in c4 c2 c3; do
  for fence in 0 1; do
    UVHTTP_WS_TIMING_FENCE=$fence timeout -k 10 200 python bench.py --config $cfg --steps 100 --warmup 10 \
      --no-cpu-baseline --no-c5-base > $OUT/bench_${cfg}_fence$fence.json 2>>$OUT/bench.err || exit 1
    python3 -c "import json;d=json.load(open('$OUT/bench_${cfg}_fence$fence.json'));print('$cfg fence=$fence', d['value'], d['ms_per_step'], d['roofline']['avg_kernel_us'])"
  done
done
for a in 0 1; do
  timeout -k 10 200 tests/c/_build/batcher_e2e --conns 1024 --frames 4 --size 65536 --flushes 20 --device 0 --async $a > $OUT/e2e_async$a.json 2>&1 || exit 1
  cat $OUT/e2e_async$a.json
done
timeout -k 10 200 tests/c/_build/batcher_e2e --conns 1024 --frames 4 --size 65536 --flushes 3 --device -1 > $OUT/e2e_host.json 2>&1
cat $OUT/e2e_host.json
