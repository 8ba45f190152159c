#!/bin/bash
# Round-3 probe 36: fused path at 16 KiB tiles up to 6 KiB per frame (C2 now fused): parity
# (fused, parity, known answers, engine), then C2 / C4 / C3 in place
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r03p36
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_fused.py tests/test_gpu_parity.py tests/test_gpu_known_answers.py tests/test_gpu_engine.py tests/test_gpu_fuzz.py > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for cfg in c2 c4 c2 c4 c3; do
  timeout -k 10 200 python bench.py --config $cfg --no-cpu-baseline --no-c5-base > $OUT/bench_$cfg.json 2>>$OUT/bench.err || { tail -5 $OUT/bench.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/bench_$cfg.json'));r=d['roofline'];print('$cfg', d['value'], d['ms_per_step'], r['kernel'], r['avg_kernel_us'], r['copy_ceiling']['avg_us'])"
done
