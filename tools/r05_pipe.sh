#!/bin/bash
# pipeline depth 3 vs 4: rates, then a kernel + memory-copy trace of each
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=$1
export TMPDIR=/tmp
mkdir -p gpurun_out
for d in 3 4 3 4 2 5 8; do
  timeout -k 10 120 python3 tools/pipeline_trace.py $d 2048 1 >> gpurun_out/${T}_pipe.jsonl 2>/dev/null || exit 1
done
cat gpurun_out/${T}_pipe.jsonl
for d in 3 4; do
  timeout -k 10 180 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/${T}_trace$d -o run -- \
    python3 tools/pipeline_trace.py $d 2048 2 > gpurun_out/${T}_trace$d.json 2>/dev/null || exit 1
  cat gpurun_out/${T}_trace$d.json
done
