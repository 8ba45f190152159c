#!/bin/bash
# Round-3 probe 54: compact stride batches on records (records-only pass + k_plan on records):
# parity (every test that runs decode_compact), then C4 / C2 compact A/B against
# UVHTTP_WS_COMPACT_RECS=0, interleaved
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r03p54
mkdir -p $OUT
UVHTTP_WS_COMPACT_RECS=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_config_digests.py tests/test_gpu_engine.py tests/test_gpu_fuzz.py tests/test_gpu_known_answers.py tests/test_gpu_fused.py > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for r in 1 2; do
  for cr in 1 0; do
    for cfg in c4 c2; do
      UVHTTP_WS_COMPACT_RECS=$cr timeout -k 10 200 python bench.py --config $cfg --mode compact --steps 100 --no-cpu-baseline --no-c5-base --no-ceiling > $OUT/b.json 2>>$OUT/err.txt || exit 1
      python3 -c "import json;d=json.load(open('$OUT/b.json'));print('$cfg compact recs=$cr', d['value'], d['ms_per_step'], d['roofline']['avg_kernel_us'])" | tee -a $OUT/summary.txt
    done
  done
done
