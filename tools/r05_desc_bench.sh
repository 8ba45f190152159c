#!/bin/bash
# stream suite, then C4 streams bench lines (device timeline)
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=$1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_streams.py tests/test_gpu_streams_full.py tests/test_gpu_engine.py > gpurun_out/${T}_tests.log 2>&1 || { tail -30 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log
: > gpurun_out/${T}_bench.jsonl
for rep in 1 2 3; do
  timeout -k 10 300 python -u bench.py --config c4 --mode streams --steps 200 --warmup 20 \
    --no-cpu-baseline >> gpurun_out/${T}_bench.jsonl 2>> gpurun_out/${T}_bench.err || { tail gpurun_out/${T}_bench.err; exit 1; }
done
python3 - gpurun_out/${T}_bench.jsonl <<'PY'
import json, sys
for line in open(sys.argv[1]):
    d = json.loads(line)
    t = d.get("device_timeline") or {}
    print(d["value"], d["ms_per_step"], t.get("kernels_us"), t.get("gaps_us"))
PY
