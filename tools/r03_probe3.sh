#!/bin/bash
# Round-3 probe 3: the fused stride path (parity) + known answers + benches.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r03p3
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_fused.py tests/test_gpu_known_answers.py tests/test_batcher_transitions.py \
  tests/test_gpu_engine.py tests/test_gpu_parity.py > $OUT/pytest.log 2>&1
rc=$?
tail -5 $OUT/pytest.log
[ $rc -eq 0 ] || exit $rc
for cfg in c4 c2 c3; do
  for fused in 1 0; do
    UVHTTP_WS_FUSED=$fused timeout -k 10 200 python bench.py --config $cfg --steps 100 --warmup 10 \
      --no-cpu-baseline --no-c5-base > $OUT/bench_${cfg}_fused$fused.json 2>>$OUT/bench.err || exit 1
    python3 -c "import json;d=json.load(open('$OUT/bench_${cfg}_fused$fused.json'));r=d['roofline'];print('$cfg fused=$fused', d['value'], d['ms_per_step'], r['avg_kernel_us'], r['frac'], r['copy_ceiling'])"
  done
done
