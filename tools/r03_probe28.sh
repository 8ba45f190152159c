#!/bin/bash
# Round-3 probe 28: slow C2 stream-decode runs — is the device chain slow, or idle between steps?
# UVHTTP_WS_TIME_CHAIN=1 makes the sampled HIP-event timing bracket the whole kernel chain of a
# call (walk .. payload); ms_per_step - chain = device idle between calls.  4 runs, one PMC
# pass (as before the slow runs of r03p25), 4 more runs.
set -uo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/r03p28
mkdir -p "$OUT"
one() {
  UVHTTP_WS_TIME_CHAIN=1 timeout -k 10 120 python3 bench.py --config c2 --mode streams --steps 100 --warmup 10 \
    --no-cpu-baseline --no-c5-base --no-ceiling > $OUT/r.json 2>> $OUT/err.txt || return 1
  python3 -c "import json;d=json.load(open('$OUT/r.json'));print('$1', d['value'], d['ms_per_step'], 'chain_us', d['roofline']['avg_kernel_us'], 'host_us', d['host_issue_us_per_step'])" | tee -a $OUT/summary.txt
}
for k in 1 2 3 4; do one pre$k || exit 1; done
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run \
  -- python3 $ROOT/bench.py --config c2 --mode streams --steps 3 --warmup 1 --no-cpu-baseline --no-c5-base --no-ceiling > /dev/null 2> "$OUT/fetch.err" || exit 1
cd "$ROOT"
for k in 1 2 3 4 5 6; do one post$k || exit 1; done
