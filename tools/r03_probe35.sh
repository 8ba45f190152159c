#!/bin/bash
# Round-3 probe 35: fused payload tile shapes (incl. the new 256x8 / 512x4 / 512x8) against the
# k_plan-first path, whole in-place step per frame size; fused-path parity first
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r03p35
mkdir -p $OUT
for t in 256x8 512x4 512x8; do
  UVHTTP_WS_FUSED_TILE=$t timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_gpu_fused.py > $OUT/pytest_$t.log 2>&1 || { echo "fused tests failed at $t"; tail -30 $OUT/pytest_$t.log; exit 1; }
  echo "$t: $(tail -1 $OUT/pytest_$t.log)"
done
FUSED_TILES=256x4,256x8,512x4,512x8 timeout -k 10 400 python -u tools/fused_sweep.py 120,250,1000,2000,3000,4000,8000,16000 3 > $OUT/sweep.txt 2>&1 || { tail -5 $OUT/sweep.txt; exit 1; }
cat $OUT/sweep.txt
