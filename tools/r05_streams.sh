#!/bin/bash
# stream-decode tests + C4/C2/C3 streams lines
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=$1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_stamps.py tests/test_gpu_streams.py tests/test_gpu_streams_full.py tests/test_gpu_fuzz.py \
  tests/test_batcher_transitions.py tests/test_gpu_batcher.py \
  > gpurun_out/${T}_pytest.log 2>&1 || { tail -40 gpurun_out/${T}_pytest.log; exit 1; }
tail -2 gpurun_out/${T}_pytest.log
for cm in c4 c2 c3; do
  IFS=: read c pv <<< "$cm"
  um=1; [ -n "$pv" ] && um=0
  UVHTTP_WS_WALK_UNMASK=$um timeout -k 10 300 python -u bench.py --config $c --mode streams --steps 100 --warmup 10 --no-cpu-baseline \
    >> gpurun_out/${T}_bench.jsonl 2>> gpurun_out/${T}_bench.err || { tail -20 gpurun_out/${T}_bench.err; exit 1; }
done
python - <<PY
import json
for l in open("gpurun_out/${T}_bench.jsonl"):
    d=json.loads(l); tl=d.get("device_timeline") or {}
    print(d["config"]["workload"][:3], d["config"]["mode"], d["roofline"]["kernel"][:14], d["value"], d["ms_per_step"], d["roofline"]["frac"], tl.get("kernels_us"), tl.get("gaps_us"))
PY
