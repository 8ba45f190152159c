#!/bin/bash
# Round-3 probe 29: C2 stream decode, 10 runs per runtime setting; the chain time (HIP events
# around walk .. payload) against the step time shows the device idle between calls.
set -uo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/r03p29
mkdir -p "$OUT"
one() {
  local tag=$1; shift
  env UVHTTP_WS_TIME_CHAIN=1 "$@" timeout -k 10 120 python3 bench.py --config c2 --mode streams --steps 100 --warmup 10 \
    --no-cpu-baseline --no-c5-base --no-ceiling > $OUT/r.json 2>> $OUT/err.txt || return 1
  python3 -c "import json;d=json.load(open('$OUT/r.json'));print('$tag', d['value'], d['ms_per_step'], 'chain_us', d['roofline']['avg_kernel_us'], 'host_us', d['host_issue_us_per_step'])" | tee -a $OUT/summary.txt
}
for k in $(seq 10); do one base X=1 || exit 1; done
for k in $(seq 10); do one devkarg0 HIP_FORCE_DEV_KERNARG=0 || exit 1; done
for k in $(seq 10); do one hwq1 GPU_MAX_HW_QUEUES=1 || exit 1; done
