#!/bin/bash
# Round-3 probe 6: reduce-then-scan over records vs look-back k_plan (fused C4), parity first.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r03p6
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_fused.py tests/test_gpu_parity.py tests/test_gpu_engine.py > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for rs in 3pass lookback 3pass lookback; do
  for cfg in c4 c2; do
    UVHTTP_WS_REC_SCAN=$rs timeout -k 10 200 python bench.py --config $cfg --steps 200 --warmup 10 --no-cpu-baseline \
      --no-c5-base --no-ceiling > $OUT/bench_${cfg}_$rs.json 2>>$OUT/bench.err || exit 1
    python3 -c "import json;d=json.load(open('$OUT/bench_${cfg}_$rs.json'));r=d['roofline'];print('$cfg $rs', d['value'], d['ms_per_step'], r['avg_kernel_us'])"
  done
done
cd /tmp
export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/$OUT/trace" -o run \
  -- python3 $GRAFT_REPO_ROOT/bench.py --config c4 --steps 20 --warmup 5 --no-cpu-baseline --no-c5-base --no-ceiling > /dev/null 2>&1 || exit 1
python3 - "$GRAFT_REPO_ROOT/$OUT" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/trace/*kernel_stats.csv")[0]
for r in csv.DictReader(open(f)):
    n = r["Name"].replace("(anonymous namespace)::", "").split("(")[0]
    print(f'{n[:50]:50s} calls {r["Calls"]:>4s} avg {float(r["AverageNs"])/1e3:9.2f} us')
PY
