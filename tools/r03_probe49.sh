#!/bin/bash
# Round-3 probe 49: k_plan on records, frames per lane (UVHTTP_WS_PLAN_FPT 4 / 8 / 16) and the
# 512-thread variants (UVHTTP_WS_PLAN_WIDE=2: 8 frames per lane, =3: 16) on the final fused kernel, C4 in place, interleaved runs
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r03p49
mkdir -p $OUT
for r in 1 2; do
  for v in "UVHTTP_WS_PLAN_FPT=16" "UVHTTP_WS_PLAN_WIDE=2" "UVHTTP_WS_PLAN_WIDE=3"; do
    env $v timeout -k 10 200 python bench.py --config c4 --steps 200 --no-cpu-baseline --no-c5-base --no-ceiling > $OUT/b.json 2>>$OUT/err.txt || exit 1
    python3 -c "import json;d=json.load(open('$OUT/b.json'));print('$v', d['value'], d['ms_per_step'])" | tee -a $OUT/summary.txt
  done
done
