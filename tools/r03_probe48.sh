#!/bin/bash
# Round-3 probe 48: the batcher suite with the new async split-frame test (prefix_bound), then
# bench.py --e2e (pinned loop, AVX2 copies, PCIe ceiling)
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r03p48
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_batcher_transitions.py tests/test_gpu_batcher.py tests/test_gpu_batcher_tls.py tests/test_c1_echo.py > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 900 python bench.py --config c2 --e2e --no-cpu-baseline --no-c5-base > $OUT/bench_e2e.json 2> $OUT/bench_e2e.err || { tail -5 $OUT/bench_e2e.err; exit 1; }
python3 -c "
import json
d=json.load(open('$OUT/bench_e2e.json'))
print('e2e_pcie', json.dumps(d.get('e2e_pcie'))[:200])
for k,v in d['e2e_live'].items(): print('e2e_live', k, json.dumps(v)[:360])"
