#!/bin/bash
# Round 5 check: GPU suite, the two-rank launcher on one GPU (readiness, not scaling), quick C4 lines.
# usage: tools/r05_check.sh TAG
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=$1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/${T}_pytest_gpu.log 2>&1 || { tail -30 gpurun_out/${T}_pytest_gpu.log; exit 1; }
tail -3 gpurun_out/${T}_pytest_gpu.log
timeout -k 10 300 python -u bench.py --gpus 2 --oversubscribe --config c5 --steps 2 --warmup 1 \
  > gpurun_out/${T}_bench_c5_2ranks.json 2> gpurun_out/${T}_bench_c5_2ranks.err || { tail -20 gpurun_out/${T}_bench_c5_2ranks.err; exit 1; }
cut -c1-400 gpurun_out/${T}_bench_c5_2ranks.json
for cm in c4:inplace c4:compact c4:streams c4:build; do
  c=${cm%%:*}; m=${cm##*:}
  timeout -k 10 300 python -u bench.py --config $c --mode $m --steps 100 --warmup 10 --no-cpu-baseline \
    >> gpurun_out/${T}_bench_matrix.jsonl 2>> gpurun_out/${T}_bench_matrix.err || exit 1
done
python - <<PY
import json
for l in open("gpurun_out/${T}_bench_matrix.jsonl"):
    d=json.loads(l); tl=d.get("device_timeline") or {}
    print(d["config"]["workload"][:3], d["config"]["mode"], d["value"], d["ms_per_step"], d["roofline"]["frac"], tl.get("kernels_us"), tl.get("gaps_us"))
PY
