#!/bin/bash
# Round-3 probe 50: C2 stream-decode idle between calls vs the walk scratch: default (single-pass
# walk: 0.5 GB slices + 1 GB records), UVHTTP_WS_WALK_REC=0 (no record scratch), and
# UVHTTP_WS_WALK_SINGLE=0 (two-pass walk, no slice scratch); 10 runs each, interleaved
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r03p50
mkdir -p $OUT
for r in $(seq 10); do
  for v in "X=1" "UVHTTP_WS_WALK_REC=0" "UVHTTP_WS_WALK_SINGLE=0"; do
    env UVHTTP_WS_TIME_CHAIN=1 $v timeout -k 10 120 python3 bench.py --config c2 --mode streams --steps 100 --warmup 10 \
      --no-cpu-baseline --no-c5-base --no-ceiling > $OUT/r.json 2>> $OUT/err.txt || exit 1
    python3 -c "import json;d=json.load(open('$OUT/r.json'));print('$v', d['value'], d['ms_per_step'], 'chain_us', d['roofline']['avg_kernel_us'])" | tee -a $OUT/summary.txt
  done
done
