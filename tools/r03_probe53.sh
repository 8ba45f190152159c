#!/bin/bash
# Round-3 probe 53: cache-policy bits of the fused payload pass's stores (UVHTTP_WS_FUSED_AUX:
# 18 = default, 0, 2, 16), C4 in place, interleaved 200-step runs; fused parity at each
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r03p53
mkdir -p $OUT
for a in 0 2 16; do
  UVHTTP_WS_FUSED_AUX=$a timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_fused.py > $OUT/pytest_$a.log 2>&1 || { tail -20 $OUT/pytest_$a.log; exit 1; }
  echo "aux $a: $(tail -1 $OUT/pytest_$a.log)"
done
for r in 1 2; do
  for a in 18 0 2 16; do
    UVHTTP_WS_FUSED_AUX=$a timeout -k 10 200 python bench.py --config c4 --steps 200 --no-cpu-baseline --no-c5-base --no-ceiling > $OUT/b.json 2>>$OUT/err.txt || exit 1
    python3 -c "import json;d=json.load(open('$OUT/b.json'));print('aux $a', d['value'], d['ms_per_step'], d['roofline']['avg_kernel_us'])" | tee -a $OUT/summary.txt
  done
done
