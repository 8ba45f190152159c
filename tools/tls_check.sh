#!/bin/bash
# TLS row on one GPU: bench line (+ CPU baselines) and a rocprofv3 kernel trace.
set -euo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$ROOT"
mkdir -p gpurun_out
TAG=${TAG:-r01}
timeout -k 10 300 python tools/bench_tls.py ${TLS_ARGS:-} > gpurun_out/bench_tls_$TAG.json 2> gpurun_out/bench_tls_$TAG.err
cat gpurun_out/bench_tls_$TAG.json
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/gpurun_out/prof_tls_$TAG" -o run \
  -- python3 "$ROOT/tools/bench_tls.py" --steps 5 --warmup 1 --no-cpu-baseline ${TLS_ARGS:-} > "$ROOT/gpurun_out/prof_tls_$TAG.json" 2> "$ROOT/gpurun_out/prof_tls_$TAG.err"
cd "$ROOT"
python3 - "$ROOT/gpurun_out/prof_tls_$TAG" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    n = r["Name"].replace("(anonymous namespace)::", "").split("(")[0]
    print(f'{n[:60]:60s} calls {r["Calls"]:>4s} avg {float(r["AverageNs"])/1e3:9.2f} us')
PY
