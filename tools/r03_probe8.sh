#!/bin/bash
# Round-3 probe 8: C4/C2 after reverting the parse spread; fused sweep for the threshold.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r03p8
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_fused.py > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for k in 1 2; do
for cfg in c4 c2; do
  timeout -k 10 200 python bench.py --config $cfg --steps 200 --warmup 10 --no-cpu-baseline \
    --no-c5-base --no-ceiling > $OUT/bench_$cfg.json 2>>$OUT/bench.err || exit 1
  python3 -c "import json;d=json.load(open('$OUT/bench_$cfg.json'));r=d['roofline'];print('$cfg', d['value'], d['ms_per_step'], r['avg_kernel_us'])"
done
done
timeout -k 10 300 python -u tools/fused_sweep.py 250,500,1000,2000,3000,4000 > $OUT/fused_sweep.txt 2>&1 || { cat $OUT/fused_sweep.txt; exit 1; }
cat $OUT/fused_sweep.txt
