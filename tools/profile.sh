#!/bin/bash
# rocprofv3 evidence for the payload kernel: kernel-trace stats, then FETCH_SIZE and
# WRITE_SIZE in separate PMC passes (they do not fit one pass on gfx950), then
# tools/pmc_traffic.py -> profiles/traffic_<cfg>_<mode>.json (HBM bytes per launch,
# FETCH_SIZE doubled per the gfx950 calibration in MI355X_MICROARCH.md §HBM).
set -euo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
CFG=${1:-c3}
MODE=${2:-inplace}
TAG=${TAG:-r01}
# XARGS: more bench arguments (e.g. --no-desc); MNAME: the mode's name in the output files
XARGS=${XARGS:-}
MNAME=${MNAME:-$MODE}
OUT=$ROOT/gpurun_out/prof_${TAG}_${CFG}_${MNAME}
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
ARGS="$ROOT/bench.py --config $CFG --mode $MODE --no-cpu-baseline --no-c5-base --no-ceiling $XARGS"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run \
  -- python3 $ARGS --steps 20 --warmup 5 > "$OUT/bench_trace.json" 2> "$OUT/trace.err"
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run \
  -- python3 $ARGS --steps 3 --warmup 1 > "$OUT/bench_fetch.json" 2> "$OUT/fetch.err"
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run \
  -- python3 $ARGS --steps 3 --warmup 1 > "$OUT/bench_write.json" 2> "$OUT/write.err"
cd "$ROOT"
python3 tools/pmc_traffic.py "$OUT" "$CFG" "$MNAME" "$TAG"
