#!/bin/bash
# C4 streams bench lines (device timeline) with and without streaming stores, alternating
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=$1
mkdir -p gpurun_out
: > gpurun_out/${T}_bench.jsonl
for rep in 1 2 3; do
  for nt in 1 0; do
    UVHTTP_WS_STREAM_NT=$nt timeout -k 10 300 python -u bench.py --config c4 --mode streams --steps 200 --warmup 20 \
      --no-cpu-baseline >> gpurun_out/${T}_bench.jsonl 2>> gpurun_out/${T}_bench.err || { tail gpurun_out/${T}_bench.err; exit 1; }
  done
done
python3 - gpurun_out/${T}_bench.jsonl <<'PY'
import json, sys
for i, line in enumerate(open(sys.argv[1])):
    d = json.loads(line)
    t = d.get("device_timeline") or {}
    print("nt" if i % 2 == 0 else "wb", d["value"], d["ms_per_step"], t.get("kernels_us"), t.get("gaps_us"))
PY
