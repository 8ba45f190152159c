#!/bin/bash
# rocprofv3 kernel-trace stats for a list of "cfg:mode" pairs (no PMC).
set -euo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
export TMPDIR=/tmp
for pair in "$@"; do
  cfg=${pair%%:*}; mode=${pair##*:}
  OUT=$ROOT/gpurun_out/trace_${cfg}_${mode}
  mkdir -p "$OUT"
  cd /tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT" -o run \
    -- python3 "$ROOT/bench.py" --config "$cfg" --mode "$mode" --steps 10 --warmup 2 \
    --no-cpu-baseline > "$OUT/bench.json" 2> "$OUT/err.txt"
  cd "$ROOT"
  echo "== $cfg $mode"
  python3 - "$OUT" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    n = r["Name"].replace("(anonymous namespace)::", "").split("(")[0]
    print(f'{n[:60]:60s} calls {r["Calls"]:>4s} avg {float(r["AverageNs"])/1e3:9.2f} us')
PY
done
