#!/bin/bash
# Round-3 probe 37: k_fixup grid cap (UVHTTP_WS_FIXUP_BLOCKS) on C4 in place, interleaved runs;
# fused-path parity at the smallest cap first
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r03p37
mkdir -p $OUT
UVHTTP_WS_FIXUP_BLOCKS=16 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_fused.py > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for r in 1 2; do
  for fx in 1024 256 64 16; do
    UVHTTP_WS_FIXUP_BLOCKS=$fx timeout -k 10 200 python bench.py --config c4 --steps 200 --no-cpu-baseline --no-c5-base --no-ceiling > $OUT/b.json 2>>$OUT/bench.err || { tail -5 $OUT/bench.err; exit 1; }
    python3 -c "import json;d=json.load(open('$OUT/b.json'));print('fixup_blocks $fx', d['value'], d['ms_per_step'])" | tee -a $OUT/summary.txt
  done
done
