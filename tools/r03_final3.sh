#!/bin/bash
# Round-3 closing evidence on the final tree: full GPU suite + smoke + default bench, the all-mode
# matrix, bench.py --e2e
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r03f3
mkdir -p $OUT
bash tools/round_end.sh > $OUT/round_end.log 2>&1 || { echo "round_end failed"; tail -20 $OUT/round_end.log; exit 1; }
grep -E "passed|failed" gpurun_out/full_pytest.log | tail -1; tail -1 gpurun_out/smoke.log
python3 -c "import json;d=json.load(open('gpurun_out/bench_default.json'));print('bench', d['value'], d['ms_per_step'], d['roofline']['frac'])"
TAG=r03f3 bash tools/bench_matrix.sh > $OUT/matrix.log 2>&1 || { echo "matrix failed"; tail -5 $OUT/matrix.log; exit 1; }
tail -15 $OUT/matrix.log
timeout -k 10 900 python bench.py --config c2 --e2e --no-cpu-baseline --no-c5-base > $OUT/bench_e2e.json 2> $OUT/bench_e2e.err || { tail -5 $OUT/bench_e2e.err; exit 1; }
python3 -c "
import json
d=json.load(open('$OUT/bench_e2e.json'))
for k,v in d['e2e_live'].items(): print('e2e_live', k, v.get('value'), v.get('ms_per_flush'), v.get('blocked_ms_per_flush'), v.get('fallback_flushes'), v.get('ceiling_GiBs_for_this_payload'))"
