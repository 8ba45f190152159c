#!/bin/bash
# Round-3 probe 32: C2 stream decode issued per kernel (default) vs as one HIP graph per step
# (--graph): does the idle between calls (r03p28-30) belong to the per-dispatch submission?
set -uo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/r03p32
mkdir -p "$OUT"
one() {
  local tag=$1; shift
  timeout -k 10 120 python3 bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-c5-base --no-ceiling "$@" > $OUT/r.json 2>> $OUT/err.txt || return 1
  python3 -c "import json;d=json.load(open('$OUT/r.json'));print('$tag', d['value'], d['ms_per_step'], 'host_us', d['host_issue_us_per_step'])" | tee -a $OUT/summary.txt
}
for k in $(seq 10); do one graph_c2s --config c2 --mode streams --graph || exit 1; one plain_c2s --config c2 --mode streams || exit 1; done
for k in 1 2 3; do one graph_c4s --config c4 --mode streams --graph || exit 1; one plain_c4s --config c4 --mode streams || exit 1; done
for k in 1 2 3; do one graph_c2i --config c2 --graph || exit 1; one plain_c2i --config c2 || exit 1; done
for k in 1 2; do one graph_c4i --config c4 --graph || exit 1; one plain_c4i --config c4 || exit 1; done
