#!/bin/bash
# send side with device stamps: build tests, stamps tests, then build lines (kernel time off the device clock)
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=$1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_build.py tests/test_gpu_stamps.py \
  > gpurun_out/${T}_pytest.log 2>&1 || { tail -40 gpurun_out/${T}_pytest.log; exit 1; }
tail -2 gpurun_out/${T}_pytest.log
for cm in c4:build c4:build_masked c2:build c3:build; do
  IFS=: read c m <<< "$cm"
  timeout -k 10 300 python -u bench.py --config $c --mode $m --steps 100 --warmup 10 --no-cpu-baseline \
    >> gpurun_out/${T}_bench.jsonl 2>> gpurun_out/${T}_bench.err || { tail -20 gpurun_out/${T}_bench.err; exit 1; }
done
python3 - <<PY
import json
for l in open("gpurun_out/${T}_bench.jsonl"):
    d=json.loads(l); tl=d.get("device_timeline") or {}; r=d["roofline"]
    print(d["config"]["workload"][:3], d["config"]["mode"], d["value"], d["ms_per_step"], r["frac"], r["avg_kernel_source"][:20], r.get("event_kernel_us"), tl.get("kernels_us"), tl.get("gaps_us"))
PY
