#!/bin/bash
# Round-3 probe 34: tile shapes of the fused payload pass (k_unmask_stride): C4 (fused by default)
# and C2 forced onto the fused path (UVHTTP_WS_FUSED_MAX=8192); payload-kernel medians per shape
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r03p34
mkdir -p $OUT
timeout -k 10 300 python tools/tile_sweep.py c4 inplace 5 > $OUT/c4.txt 2>&1 || { tail -5 $OUT/c4.txt; exit 1; }
cat $OUT/c4.txt
UVHTTP_WS_FUSED_MAX=8192 timeout -k 10 300 python tools/tile_sweep.py c2 inplace 5 > $OUT/c2_fused.txt 2>&1 || { tail -5 $OUT/c2_fused.txt; exit 1; }
cat $OUT/c2_fused.txt
for k in 1 2 3 4; do
  timeout -k 10 120 python3 bench.py --config c3 --mode streams --steps 30 --warmup 5 --no-cpu-baseline --no-c5-base --no-ceiling > $OUT/c3s.json 2>>$OUT/err.txt || exit 1
  python3 -c "import json;d=json.load(open('$OUT/c3s.json'));print('c3 streams', d['value'], d['ms_per_step'], d['roofline']['avg_kernel_us'])" | tee -a $OUT/c3s.txt
done
