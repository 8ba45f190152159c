#!/bin/bash
# send side: build tests with the fused size+scan launch and without, then a same-process A/B
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=$1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_build.py tests/test_gpu_stamps.py tests/test_gpu_engine.py \
  > gpurun_out/${T}_pytest.log 2>&1 || { tail -40 gpurun_out/${T}_pytest.log; exit 1; }
tail -2 gpurun_out/${T}_pytest.log
UVHTTP_WS_BUILD_FUSED_SCAN=0 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_build.py \
  > gpurun_out/${T}_pytest_nofuse.log 2>&1 || { tail -40 gpurun_out/${T}_pytest_nofuse.log; exit 1; }
tail -1 gpurun_out/${T}_pytest_nofuse.log
for cm in c4:build c4:build c2:build c3:build; do
  IFS=: read c m <<< "$cm"
  for fs in 1 0; do
    UVHTTP_WS_BUILD_FUSED_SCAN=$fs timeout -k 10 300 python -u bench.py --config $c --mode $m --steps 100 --warmup 10 --no-cpu-baseline \
      | sed "s/}\$/, \"fused_scan\": $fs}/" >> gpurun_out/${T}_bench.jsonl 2>> gpurun_out/${T}_bench.err || { tail -20 gpurun_out/${T}_bench.err; exit 1; }
  done
done
python3 - <<PY
import json
for l in open("gpurun_out/${T}_bench.jsonl"):
    d=json.loads(l); tl=d.get("device_timeline") or {}; r=d["roofline"]
    print(d["config"]["workload"][:3], d["config"]["mode"], "fused", d.get("fused_scan"), d["value"], d["ms_per_step"], r["frac"], tl.get("kernels_us"), tl.get("gaps_us"), tl.get("gap_between_calls_us"))
PY
