#!/bin/bash
# Round-3 probe 30: C2 stream decode with every call timed (UVHTTP_WS_TIMING_EVERY=1): whole
# chain (TIME_CHAIN=1) or payload kernel only; 10 runs each
set -uo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/r03p30
mkdir -p "$OUT"
one() {
  local tag=$1; shift
  env "$@" timeout -k 10 120 python3 bench.py --config c2 --mode streams --steps 100 --warmup 10 \
    --no-cpu-baseline --no-c5-base --no-ceiling > $OUT/r.json 2>> $OUT/err.txt || return 1
  python3 -c "import json;d=json.load(open('$OUT/r.json'));print('$tag', d['value'], d['ms_per_step'], 'timed_us', d['roofline']['avg_kernel_us'], d['roofline']['launches_timed'], 'host_us', d['host_issue_us_per_step'])" | tee -a $OUT/summary.txt
}
for k in $(seq 10); do one chain_all UVHTTP_WS_TIME_CHAIN=1 UVHTTP_WS_TIMING_EVERY=1 || exit 1; done
for k in $(seq 10); do one payload_all UVHTTP_WS_TIME_CHAIN=0 UVHTTP_WS_TIMING_EVERY=1 || exit 1; done
