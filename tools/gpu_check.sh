#!/bin/bash
# One GPU-box session: parity tests, smoke, bench, rocprofv3 kernel stats.
# Every GPU step has its own time limit; the first failure ends the script.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
TAG=${TAG:-r01}
STEP=${1:-all}

if [[ $STEP == all || $STEP == tests ]]; then
  timeout -k 10 900 python -m pytest tests -x -q -m gpu > "$OUT/pytest_gpu_$TAG.log" 2>&1
  tail -3 "$OUT/pytest_gpu_$TAG.log"
fi
if [[ $STEP == all || $STEP == smoke ]]; then
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke_$TAG.log" 2>&1
  tail -1 "$OUT/smoke_$TAG.log"
fi
if [[ $STEP == all || $STEP == bench ]]; then
  timeout -k 10 600 python bench.py --steps 20 --warmup 5 > "$OUT/bench_$TAG.json" 2> "$OUT/bench_$TAG.err"
  cat "$OUT/bench_$TAG.json"
fi
if [[ $STEP == all || $STEP == prof ]]; then
  cd /tmp
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$TAG" -o run \
    -- python3 "$ROOT/bench.py" --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/prof_bench_$TAG.json" 2> "$OUT/prof_$TAG.err"
  cd "$ROOT"
  find "$OUT/prof_$TAG" -name "*stats*" | head -5
fi
