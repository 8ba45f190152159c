#!/bin/bash
# rocprofv3 kernel stats of one bench config: tools/r05_prof.sh TAG CFG MODE [extra bench args]
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=$1; C=$2; M=$3; shift 3
export TMPDIR=/tmp
mkdir -p gpurun_out/${T}_prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_prof -o run -- \
  python3 bench.py --config $C --mode $M --steps 50 --warmup 5 --no-cpu-baseline --no-ceiling --no-stamps "$@" \
  > gpurun_out/${T}_prof/bench.json 2> gpurun_out/${T}_prof/bench.err || { tail -20 gpurun_out/${T}_prof/bench.err; exit 1; }
f=$(find gpurun_out/${T}_prof -name '*kernel_stats.csv' | head -1)
cp "$f" gpurun_out/${T}_kernel_stats.csv
cut -d, -f1-8 gpurun_out/${T}_kernel_stats.csv | head -12
