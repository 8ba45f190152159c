#!/bin/bash
# k_swalk_fused: stream-decode tests, then C4 / C2 streams lines fused and apart
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=$1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_streams.py tests/test_gpu_stamps.py tests/test_gpu_engine.py tests/test_gpu_streams_full.py \
  > gpurun_out/${T}_tests.log 2>&1 || { tail -40 gpurun_out/${T}_tests.log; exit 1; }
tail -2 gpurun_out/${T}_tests.log
: > gpurun_out/${T}_bench.jsonl
for rep in 1 2; do
  for f in 1 0 1:0; do
    for cfg in c4; do
      IFS=: read fu tk <<< "$f"
      UVHTTP_WS_WALK_FUSE=$fu UVHTTP_WS_PLAN_TICKET=${tk:-1} timeout -k 10 300 python -u bench.py --config $cfg --mode streams --steps 200 --warmup 20 \
        --no-cpu-baseline >> gpurun_out/${T}_bench.jsonl 2>> gpurun_out/${T}_bench.err || { tail gpurun_out/${T}_bench.err; exit 1; }
    done
  done
done
python3 - gpurun_out/${T}_bench.jsonl <<'PY'
import json, sys
for line in open(sys.argv[1]):
    d = json.loads(line)
    t = d.get("timeline") or {}
    t = d.get("device_timeline") or {}
    print(d["config"]["workload"][:3], d["value"], d["ms_per_step"], t.get("kernels_us"), t.get("gaps_us"))
PY
