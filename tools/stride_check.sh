#!/bin/bash
# One GPU-box session for the one-launch stride decode: its parity tests, then C4 / C2 in place
# with the two-launch (UVHTTP_WS_STRIDE=0) and one-launch (=1) paths and a few tuning points.
# Every GPU step has its own time limit; the first failure ends the script.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p $OUT
TAG=${TAG:-stride}
if [[ ${SKIP_TESTS:-0} != 1 ]]; then
  timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_parity.py tests/test_gpu_engine.py -k "stride or config or plan_frames or give_up or graph or serialise" \
    > $OUT/${TAG}_pytest.log 2>&1 || { tail -30 $OUT/${TAG}_pytest.log; exit 1; }
  tail -2 $OUT/${TAG}_pytest.log
fi
: > $OUT/${TAG}_bench.jsonl
for cfg in c4 c2; do
  for v in "0 4" "1 4" "1 2" "1 8"; do
    set -- $v
    UVHTTP_WS_STRIDE=$1 UVHTTP_WS_STRIDE_U=$2 timeout -k 10 120 \
      python bench.py --config $cfg --steps 50 --warmup 5 --no-cpu-baseline --no-c5-base \
      2> $OUT/${TAG}_bench.err | python -c "import json,sys; d=json.loads(sys.stdin.readline()); print(json.dumps({'cfg': '$cfg', 'stride': '$1', 'u': $2, 'value': d['value'], 'ms': d['ms_per_step'], 'kernel_us': d['roofline']['avg_kernel_us'], 'frac': d['roofline']['frac']}))" \
      | tee -a $OUT/${TAG}_bench.jsonl
  done
done
