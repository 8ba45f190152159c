#!/bin/bash
# k_stream_desc_lane's own first-frame scan (single-pass lane walk, <= 65536 connections): the
# stream and batcher suites, then C2 / C4 / C3 streams bench lines and a same-process A/B
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=$1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_streams.py tests/test_gpu_streams_full.py tests/test_gpu_engine.py tests/test_gpu_stamps.py \
  tests/test_batcher_transitions.py tests/test_batcher_group.py tests/test_gpu_batcher.py \
  > gpurun_out/${T}_tests.log 2>&1 || { tail -30 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log
{
AB_ENV_B=UVHTTP_WS_DESC_SCAN=0 timeout -k 10 300 python -u tools/ab_lib.py tree tree c2:streams c4:streams || exit 1
} 2>&1 | grep -v amdgpu.ids | tee gpurun_out/${T}_ab.txt
: > gpurun_out/${T}_bench.jsonl
for cfg in c2 c4 c3 c2; do
  timeout -k 10 300 python -u bench.py --config $cfg --mode streams --steps 100 --warmup 10 \
    --no-cpu-baseline >> gpurun_out/${T}_bench.jsonl 2>> gpurun_out/${T}_bench.err || { tail gpurun_out/${T}_bench.err; exit 1; }
done
python3 - gpurun_out/${T}_bench.jsonl <<'PY'
import json, sys
for line in open(sys.argv[1]):
    d = json.loads(line)
    t = d.get("device_timeline") or {}
    print(d["config"]["workload"][:3], d["value"], d["ms_per_step"], t.get("kernels_us"))
PY
