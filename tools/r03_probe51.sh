#!/bin/bash
# Round-3 probe 51: the lane walk two-pass by default: stream / fuzz / batcher parity, then
# C2 streams x10 and C3 / C4 streams x3 (chain-timed)
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r03p51
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_streams.py tests/test_gpu_fuzz.py tests/test_gpu_batcher.py tests/test_batcher_transitions.py tests/test_gpu_tls_ws_chain.py > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for cfg in c2 c2 c2 c2 c2 c2 c2 c2 c2 c2 c3 c3 c3 c4 c4 c4; do
  UVHTTP_WS_TIME_CHAIN=1 timeout -k 10 120 python3 bench.py --config $cfg --mode streams --steps 100 --warmup 10 \
    --no-cpu-baseline --no-c5-base --no-ceiling > $OUT/r.json 2>> $OUT/err.txt || exit 1
  python3 -c "import json;d=json.load(open('$OUT/r.json'));print('$cfg streams', d['value'], d['ms_per_step'], 'chain_us', d['roofline']['avg_kernel_us'])" | tee -a $OUT/summary.txt
done
