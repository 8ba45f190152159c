#!/bin/bash
# summary-only compact decode: its tests (and the paths beside it), then C4 lines
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=$1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_summary_compact.py tests/test_gpu_summary_only.py tests/test_gpu_spec_compact.py \
  "tests/test_gpu_parity.py::test_config_full_summary_only" "tests/test_gpu_parity.py::test_pipeline_and_delivery" \
  tests/test_gpu_stamps.py \
  > gpurun_out/${T}_pytest.log 2>&1 || { tail -40 gpurun_out/${T}_pytest.log; exit 1; }
tail -3 gpurun_out/${T}_pytest.log
for cm in c4:compact c4:compact:nd c4:inplace:nd c4:compact c4:compact:nd; do
  IFS=: read c m nd <<< "$cm"
  timeout -k 10 300 python -u bench.py --config $c --mode $m ${nd:+--no-desc} --steps 100 --warmup 10 --no-cpu-baseline \
    >> gpurun_out/${T}_bench.jsonl 2>> gpurun_out/${T}_bench.err || { tail -20 gpurun_out/${T}_bench.err; exit 1; }
done
python - <<PY
import json
for l in open("gpurun_out/${T}_bench.jsonl"):
    d=json.loads(l); tl=d.get("device_timeline") or {}
    print(d["config"]["workload"][:3], d["config"]["mode"], d["value"], d["ms_per_step"], d["roofline"]["frac"], d["roofline"]["kernel"], tl.get("kernels_us"), tl.get("gaps_us"), tl.get("gap_between_calls_us"))
PY
