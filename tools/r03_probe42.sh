#!/bin/bash
# Round-3 probe 42: (1) C2 fused (UVHTTP_WS_FUSED_MAX=8192) vs k_plan-first after the 32-bit
# fused mask, interleaved runs; (2) host copy variants for submit_read (tools/copy_probe.hip)
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r03p42
mkdir -p $OUT
for r in 1 2 3; do
  for fm in 8192 2560; do
    UVHTTP_WS_FUSED_MAX=$fm timeout -k 10 200 python bench.py --config c2 --no-cpu-baseline --no-c5-base --no-ceiling > $OUT/b.json 2>>$OUT/err.txt || exit 1
    python3 -c "import json;d=json.load(open('$OUT/b.json'));print('c2 fused_max=$fm', d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['avg_kernel_us'])" | tee -a $OUT/c2.txt
  done
done
timeout -k 10 120 tools/bin/copy_probe 3 | tee $OUT/copy.jsonl
