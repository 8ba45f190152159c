#!/bin/bash
# Round-3 probe 56: does the stream-decode idle between calls need the sampled timing events?
# C2 streams, 8 processes with no event in the timed region (UVHTTP_WS_TIMING_EVERY=10^9)
# alternating with 8 at the default sampling (every 10th call).
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r03p56
mkdir -p $OUT
: > $OUT/summary.txt
for i in 1 2 3 4 5 6 7 8; do
  for every in 1000000000 10; do
    UVHTTP_WS_TIMING_EVERY=$every timeout -k 10 120 python3 bench.py --config c2 --mode streams --steps 100 --warmup 10 \
      --no-cpu-baseline --no-c5-base --no-ceiling > $OUT/r.json 2>> $OUT/err.txt || exit 1
    python3 -c "import json;d=json.load(open('$OUT/r.json'));print('c2 streams every=$every', d['value'], d['ms_per_step'], 'host_us', d.get('host_issue_us_per_step'), 'kernel_us', d['roofline']['avg_kernel_us'])" | tee -a $OUT/summary.txt
  done
done
