#!/bin/bash
# Round-3 probe 5: fused vs plan-first over frame sizes; default benches with sampled timing.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r03p5
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_fused.py > $OUT/pytest.log 2>&1 || { tail -20 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 300 python -u tools/fused_sweep.py > $OUT/fused_sweep.txt 2>&1 || { cat $OUT/fused_sweep.txt; exit 1; }
cat $OUT/fused_sweep.txt
for cfg in c4 c2 c3; do
  timeout -k 10 200 python bench.py --config $cfg --steps 100 --warmup 10 --no-cpu-baseline \
    --no-c5-base > $OUT/bench_$cfg.json 2>>$OUT/bench.err || exit 1
  python3 -c "import json;d=json.load(open('$OUT/bench_$cfg.json'));r=d['roofline'];print('$cfg', d['value'], d['ms_per_step'], r['avg_kernel_us'], r['launches_timed'], r['frac'])"
done
