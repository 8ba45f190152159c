#!/bin/bash
# lane-path tile claims in k_stream_desc_lane (k_stream_claims gone): the stream, engine and
# parity suites, then C2 / C3 / C4 streams lines (device timeline)
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=$1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_streams.py tests/test_gpu_streams_full.py tests/test_gpu_engine.py tests/test_gpu_stamps.py \
  tests/test_gpu_parity.py tests/test_batcher_transitions.py tests/test_batcher_group.py \
  > gpurun_out/${T}_tests.log 2>&1 || { tail -30 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log
: > gpurun_out/${T}_bench.jsonl
for rep in 1 2; do
  for cfg in c2 c4 c3; do
    timeout -k 10 300 python -u bench.py --config $cfg --mode streams --steps 100 --warmup 10 \
      --no-cpu-baseline >> gpurun_out/${T}_bench.jsonl 2>> gpurun_out/${T}_bench.err || { tail gpurun_out/${T}_bench.err; exit 1; }
  done
done
python3 - gpurun_out/${T}_bench.jsonl <<'PY'
import json, sys
for line in open(sys.argv[1]):
    d = json.loads(line)
    t = d.get("device_timeline") or {}
    print(d["config"]["workload"][:3], d["value"], d["ms_per_step"], t.get("kernels_us"), t.get("gaps_us"))
PY
